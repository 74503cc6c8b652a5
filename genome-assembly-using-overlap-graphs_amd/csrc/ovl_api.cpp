// ovl_api.cpp — the C ABI of include/ovl.h on top of the gfx950 kernels.
//
// A context (ovl_ctx) drives one or more HIP devices from one host thread.  Each
// device (Dev) owns: a compute stream and two copy streams (H2D, D2H), its copy
// of the resident read store (codes + bit-plane layouts in HBM), scratch for
// host-array calls, pinned staging rings and the device error flag.  Host-array
// scoring calls shard the pair list over the devices (contiguous ranges balanced
// by sum n*m) and run a chunked pipeline per device (run_pipeline).
// The kernels read host pair lists and store results through host mappings:
// packed (2 bytes per pair, Call::pack) into staging slots that the host pool
// expands into the caller's int32 arrays while the next chunk scores, with a
// last share of the pairs stored as int32 straight into pinned arrays; otherwise
// as int32 into the caller's pinned arrays or staging slots.  Only the compact
// in-place pair list (encode_chunk) crosses by copy-engine transfer.
// Kernel choice per call (ovl_plan): the ungapped popcount kernel whenever gaps
// provably cannot win and the read store has a bit-plane layout, else a DP kernel.
// Never falls back to the CPU.
#include <hip/hip_runtime.h>

#include <emmintrin.h>
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <new>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ovl.h"
#include "ovl_encode.h"
#include "ovl_scan.h"
#include "ovl_expand.h"
#include "ovl_pool.h"
#include "ovl_kernels.h"
#include "ovl_resident.h"

#define OVL_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int32_t kFastMaxLen = 256;   // bit-plane layouts up to W = 8 words of 32 bases
constexpr int32_t kDpMaxLen = 8192;    // DP kernel: LDS row of the t read
constexpr int32_t kLaneMaxLen = 1024;  // lane-per-pair DP: hand-off column buffer per wavefront slot
constexpr int kSlots = 3;              // pipeline depth: staging slots / events per device
// Host memory that kernels store into and host code reads within one call (staging slots, the error
// flag): fine-grained, whose device stores snoop the CPU caches, so a line the host read in an earlier call
// is never returned stale.  (HIP's default for hipHostMalloc, with HIP_HOST_COHERENT unset, is the
// coarse-grained kind.)
constexpr unsigned kHostShared = hipHostMallocPortable | hipHostMallocCoherent;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool view = false;  // a part of another buffer (set_view): not freed, not grown
};

thread_local std::string g_err;

// Test knobs, read from the environment once per context: they force a kernel form or a transport that the
// planner would otherwise pick by size or scoring, so the tests reach every form on small inputs.  (The A/B
// knobs of rounds 1-3 -- lane split, copy-engine transfers, spin waits, ordinary-store expansion, grid cap, heavy
// tiles, lane strip width and hand-off forms, read packing, pool spin, coarse-grained host memory -- are gone
// with the forms they measured; DESIGN.md records each measurement.  Round 5 merged the pairs of switches over one
// choice into one knob each -- OVL_DP_FORM, OVL_LANE_FORM, OVL_PAIRS_FORM -- and dropped the settled vector-width
// knobs of the host expansion and encoding: both run the widest form the CPU has.)
struct Knobs {
    int32_t band_form = -1;       // OVL_BAND_FORM env (lane|diag|rows|fast|strip): band knob kernel (tests)
    // OVL_DP_FORM env, full-DP scoring (tests): auto (default: lane-per-pair from kLaneMinPairs pairs, else
    // dp_fast_kernel), lane (lane-per-pair forced), fast (dp_fast_kernel), classic (dp_kernel)
    int32_t dp_classic = 0;
    int32_t dp_lane = -1;         // -1 auto by list size, 0 off, 1 forced
    // OVL_LANE_FORM env, the lane kernels' inner form (tests), a bit mask, default 7: bit 0 scores by the byte
    // profile (else compare/select), bit 1 takes row symbols from the bit planes (else byte gathers), bit 2 lets
    // the full DP hold two pairs per lane as packed f16 cells (dp_lane_h2_kernel) where the scoring allows
    int32_t lane_prof = 1;
    int32_t lane_sfx = 1;
    int32_t lane_h2 = 1;
    int64_t pipe_chunk = 0;       // OVL_PIPE_CHUNK env: pairs per pipeline chunk (0 = automatic; tests)
    int32_t pack = 1;             // OVL_PACK: 0 host-array results cross the link as int32 pairs even when a packed
                                  // form holds; 1 (default) packed as 2 bytes per pair, expanded chunk by chunk
                                  // after each chunk's kernel, a last chunk stored as int32 meanwhile.  (Round 5's
                                  // streamed tile records, one launch whose records host threads expand while it
                                  // runs, were removed in round 6: target N = 1 / 2 / 8 0.144 / 0.081 / 0.050 ms
                                  // against 0.135 / 0.088 / 0.045, profiles/r05_stream_vs_packed_ab.json; its record
                                  // format lives on in the resident grid's ring)
    int64_t pack_min = 1 << 16;   // OVL_PACK_MIN: packed transport from this many pairs per call into pinned arrays
                                  // (64 K: a 250 K-pair shard -- N = 8 at the target point -- 0.057 -> 0.054 ms)
    int32_t pack_adapt = 1;       // the direct share follows the measured balance (pack_share); off when
                                  // OVL_PACK_DIRECT_PCT fixes it
    // OVL_PAIRS_FORM env, host pair lists over the link (tests): ix (default: the compact encoding, encode_chunk,
    // read in place by uniform_kernel as b16 + tile deltas where it can), decode (compact, always decoded into HBM
    // by the widen / runs kernels), plain (the caller's int32 arrays)
    int32_t compact = 1;
    int32_t pairs_ix = 1;
    // OVL_RESIDENT: scoring calls over the resident candidate list into host arrays go to the device's resident grid
    // (ovl_resident.h) -- 0 never (default: on the boxes measured it did not beat the launch pipeline, N = 1 or a
    // 1/8 shard -- profiles/r06_shard_steps.json), 1 from resident_min pairs up to resident_max, 2 at every size
    int32_t resident = 0;
    int64_t resident_min = 1;
    int64_t resident_max = int64_t(1) << 40;
    int32_t resident_blocks = 2;  // the grid's blocks of 256 threads per CU
    int32_t resident_pf = 1;      // its tiles software-pipelined (fewer, fatter wavefronts) or one at a time
    int32_t resident_sleep = 4;   // its non-lead blocks' pause between polls (~0.1 us units)
    int32_t resident_ring = 0;    // its ring's memory (ResidentGrid::ring_kind)
    int32_t pack_direct_pct = 18; // OVL_PACK_DIRECT_PCT: packed calls into pinned arrays store this share of the
                                  // pairs (the last chunk) as int32 straight into them, over the link while the
                                  // host expands the packed chunks (tools/pack_ab.py, target point, six
                                  // processes: 0 % 0.16-0.26 ms, 10 % 0.16-0.25, 18 % 0.157-0.226, 25 % 0.175-0.209)
};

// Lane-per-pair DP kernels from this many pairs per launch (one 64-pair tile per SIMD); below, a wavefront per pair
constexpr int64_t kLaneMinPairs = 65536;
// uniform_kernel grid cap, blocks of 256 per CU: ~1 tile per wavefront at the target point, the dispatcher
// balances the tail (measured -2.3 % against 8 per CU; 16 / 32 / 64: 69.2 / 68.6 / 68.4 us)
#ifndef OVL_BLOCKS_PER_CU
#define OVL_BLOCKS_PER_CU 32  // (a build macro for A/B builds, not a runtime knob)
#endif
constexpr int64_t kBlocksPerCu = OVL_BLOCKS_PER_CU;
// band knob: two lanes per pair (band_lane2_kernel) from this half-width.  Measured at cfg5 (tools/band_ab.py,
// profiles/r04_band_lane_ab.json, ms one lane / two lanes): 40: 6.07 / 6.99, 48: 7.13 / 8.04, 56: 8.29 / 9.09,
// 64: 10.50 / 10.17 -- two lanes only pay where one lane's 129 band cells leave one wavefront per SIMD.  With
// the row table built once per row (profiles/r04_band_table_ab.json): 48: 6.60 / 7.59, 64: 10.52 / 9.63
constexpr int32_t kBandLane2Min = 64;
// uniform_kernel's latency mode (two wavefronts per tile) up to this many 64-pair tiles per CU in a launch: a
// rank's shard at N = 4 / 8 (0.5 M / 0.25 M pairs) 0.068 -> 0.062 / 0.051 -> 0.047 ms per step, the whole list's
// 0.87 M-pair chunks unchanged in throughput mode, 64 tiles per CU (those chunks too) slower: 0.141 -> 0.153 ms
// (tools/gpu_r04_lat.sh, profiles/r04_lat_mode_ab.json).  Host-encoded lists keep 8: only throughput mode reads
// them in place.
constexpr int64_t kLatTiles = 32;
constexpr int64_t kLatTilesIx = 8;
// compact host pair lists from this many pairs per call
constexpr int64_t kCompactMin = int64_t(1) << 16;
// host expansion of packed results: pairs per pool part at least (finer parts than 64 K: the expansion of a
// 250 K-pair shard 22.7 -> 9.4 us, the N = 4 step 0.085 -> 0.075 ms; tools/pool_probe.cpp,
// profiles/r04_pool_ab_*.json)
constexpr size_t kExpandPart = size_t(1) << 14;

}  // namespace

struct ovl_ctx;

#include "ovl_worker.h"
#include "ovl_digest.h"

// Per-device state.
struct Dev {
    ovl_ctx* owner = nullptr;
    int32_t device = 0;
    hipStream_t stream = nullptr;  // kernels
    hipStream_t s_in = nullptr;    // host-array calls: the pair list's copies and decodes, beside the kernels
    int32_t cu_count = 256;
    Knobs k;
    // knob aliases used by the launch code
    int32_t& band_form = k.band_form;
    int32_t& dp_classic = k.dp_classic;
    int32_t& dp_lane = k.dp_lane;
    int32_t& lane_prof = k.lane_prof;
    int32_t& lane_sfx = k.lane_sfx;
    int32_t& lane_h2 = k.lane_h2;
    // resident reads
    int32_t n_reads = -1;
    int32_t lmax = 0;
    int32_t planes = 2;
    int32_t wmax = 0;  // 0: no bit-plane layout (reads longer than kFastMaxLen)
    int32_t srow = 0;  // sfx row stride (words)
    int32_t trow = 0;  // pfx row stride (words)
    DevBuf codes, off, len, sfx, pfx, lut, full;  // full: bit r set iff len[r] == lmax
    DevBuf raw;                                   // the uploaded read bytes (raw or 2-bit packed)
    DevBuf rd;  // ovl_set_reads' upload block, the stage's layout; off, len, full, lut and raw are views into it
    // scratch
    DevBuf a, b, score, end, tb, err_flag;
    DevBuf lane_col;      // lane-per-pair DP: per-wavefront strip hand-off columns
    DevBuf seed_s, seed_e;  // band knob: the ungapped seed (score, j*) of each pair
    hipEvent_t scratch_evt = nullptr;     // last launch that used lane_col / seed_* ...
    hipEvent_t ev_last = nullptr;         // packed calls into pinned arrays: after the last (direct) chunk
    double pack_pct = -1.0;               // live direct share of packed calls into pinned arrays (pack_share)
    double pack_pct_h = -1.0;             // the same for calls with a compact host pair list (the host also
                                          // encodes the list, so its balance point differs)
    hipStream_t scratch_stream = nullptr; // ... and its stream (launches on other streams wait for it)
    bool scratch_used = false;
    int64_t codes_bytes = 0;
    // device candidate enumeration (ovl_candidates): per-read keys / groups and the pair list
    DevBuf k_pre, k_suf, k_sorted, k_iota, k_order, k_lo, k_hi, k_cnt, k_offs, k_temp, cand_a, cand_b;
    int64_t cand_n = -1;  // -1: no candidate list for the resident reads
    // heavy tiles of the candidate list (tiles holding side pairs, scheduled first: uniform_kernel), built on
    // the first throughput-mode launch over the list (ensure_heavy)
    DevBuf tile_flags, heavy_ids;
    std::vector<int32_t> h_heavy;
    int64_t heavy_for = -1;  // cand_n the heavy tiles were built for (-1: none)
    int64_t cand_tail[2] = {0, 0};
    DevBuf sh_cum, sh_temp, sh_cuts;  // shard bounds (ovl_candidates_shards)
    // local alignment (ovl_local_align): query / reference bytes, carried rows, progress, traceback
    DevBuf l_q, l_r, l_row, l_tb, l_best;
    uint32_t l_epoch = 0;  // tags this launch's row hand-off words (l_row is zeroed when allocated)
    // pinned host copy of the part of the traceback table the walk can reach (grown on demand)
    int8_t* l_tb_host = nullptr;
    size_t l_tb_host_bytes = 0;
    // host-array pipeline: events per slot and pinned staging (slots x cap pairs x {a, b} / {score, end})
    hipEvent_t ev_k[kSlots] = {};
    int32_t* st_in = nullptr;
    int32_t* st_out = nullptr;
    int32_t* st_in_dev = nullptr;   // device addresses of the staging rings (kernels read / store them)
    int32_t* st_out_dev = nullptr;
    int64_t st_cap = 0;
    uint32_t* h_flag = nullptr;      // pinned error flag of host-array calls (the kernels store into it)
    uint32_t* h_flag_dev = nullptr;  // its device address
    uint32_t* cur_flag = nullptr;    // the flag the next launches write: err_flag (device calls) or h_flag_dev
    int32_t out_mode = 0;            // result sink of the next ungapped launches (OvlUngappedArgs::host_out):
                                     // 0 HBM, 1 host-mapped int32 arrays, 2 host-mapped packed uint16
    std::vector<hipEvent_t> t_ev;  // timing: kernel start/end per chunk (recorded on the stream around the launch)
    std::vector<hipEvent_t> k_ev;  // timing: the same recorded by an ungapped launch itself (kernel start / end)
    hipEvent_t kev_start = nullptr, kev_stop = nullptr;  // the next ungapped launch records these (then cleared)
    // compact host pair lists (encode_chunk): pinned encoding buffer (8 bytes per pair + slack), its device
    // address, a decode event per chunk, and the encoded bytes of the last call
    char* cp_host = nullptr;
    char* cp_dev = nullptr;
    size_t cp_bytes = 0;
    DevBuf cp_hbm;  // the in-place encoding's chunks copied into HBM (same layout as cp_host)
    std::vector<hipEvent_t> dec_ev;
    int64_t cp_link = 0;
    // the next ungapped launch reads its pair list in the host encoding (OvlUngappedArgs::ix_*), or null
    const uint16_t* ix_b16 = nullptr;
    const uint8_t* ix_d8 = nullptr;
    const int32_t* ix_base = nullptr;
    ResidentGrid res;  // the resident scoring grid (ovl_resident.h), launched by the first call that uses it
    std::unique_ptr<DevWorker> worker;  // multi-device contexts: this device's host thread (run_pipeline)
};

// The host side of a read-set upload in one pinned block (grown on demand, kept by the context): offsets,
// lengths, the length bitmap, the code table and the bytes (stage_reads).
struct ReadStage {
    char* p = nullptr;
    size_t bytes = 0;
    size_t o_off = 0, o_len = 0, o_full = 0, o_lut = 0, o_raw = 0, o_pk = 0;
};

// The host-side facts of a read set (prep_reads); kept by the context so that its arrays are reused, without
// fresh pages to fault in, by the next ovl_set_reads.
struct HostReads {
    std::vector<int64_t> off;
    std::vector<int32_t> len;
    std::vector<uint32_t> full;
    uint8_t lut[256];
    const uint8_t* src = nullptr;  // the caller's bytes, then (stage_reads) their pinned copy
    int64_t total = 0;
    bool packed2 = false;          // every byte is A, C, G or T: the stage holds them 2-bit packed (o_pk)
    int32_t n_reads = 0, lmax = 0, planes = 2, wmax = 0, srow = 0, trow = 0;
};

struct ovl_ctx {
    std::vector<Dev*> devs;
    bool shared_slots = false;   // OVL_SHARE_DEVICES=1: a device listed more than once (tests); every call uses
                                 // every slot (no device cap, devices_for)
    ReadStage stage;             // pinned upload stage of ovl_set_reads
    HostReads hreads;            // ovl_set_reads' host arrays (reused)
    // the read set resident on every device after the last complete ovl_set_reads: its offsets relative to
    // offsets[0] and a digest of its bytes, so that a call with the same read set (a graph build per k over one read set,
    // the one-shot ovl_score_pairs per build) keeps it instead of uploading and packing it again
    std::vector<int64_t> res_off;
    int64_t res_total = 0;
    uint64_t res_hash[2] = {0, 0};  // reads_hash of its bytes
    bool res_valid = false;
    std::string err;
    std::vector<int32_t> h_len;  // read lengths (shard balance of host pair lists)
    int32_t timing = 0;          // ovl_set_timing
    double t_kernel_ms = 0.0, t_call_ms = 0.0;
    struct Launch {
        int32_t device, sink;
        int64_t pairs;
        double ms;
    };
    std::vector<Launch> t_launches;  // timing on: every scoring launch of the last host-array call
    int64_t x_link_bytes = 0, x_packed_pairs = 0;  // ovl_last_transfer
    int64_t x_res_bytes = 0, x_rec_pairs = 0, x_esc = 0;  // ovl_last_results
    int64_t x_ix_pairs = 0, x_dec_pairs = 0;       // ovl_last_pair_list
};

namespace {

int fail(const ovl_ctx* c, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(const ovl_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    if (c) const_cast<ovl_ctx*>(c)->err = buf;
    return code;
}

int fail(const Dev* d, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(const Dev* d, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    if (d && d->owner) d->owner->err = buf;
    return code;
}

#define HIPCHK(ctx, expr)                                                                           \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail((ctx), e_ == hipErrorOutOfMemory ? OVL_E_OOM : OVL_E_HIP, "%s: %s", #expr, \
                        hipGetErrorString(e_));                                                     \
    } while (0)

hipError_t ensure(DevBuf& b, size_t bytes) {
    if (bytes < 16) bytes = 16;
    if (b.view) return hipErrorInvalidValue;
    if (b.bytes >= bytes) return hipSuccess;
    if (b.p) {
        hipError_t e = hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e == hipSuccess) b.bytes = bytes;
    return e;
}

void release(DevBuf& b) {
    if (b.p && !b.view) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    b.view = false;
}

void set_view(DevBuf& v, DevBuf& whole, size_t offset, size_t bytes) {
    v.p = static_cast<char*>(whole.p) + offset;
    v.bytes = bytes;
    v.view = true;
}

template <typename T>
T* as(DevBuf& b) { return reinterpret_cast<T*>(b.p); }

int64_t iabs64(int64_t v) { return v < 0 ? -v : v; }

// aligners.py:40: diag is taken whenever diag >= up and diag >= left.  Every dp
// value is a sum of <= lmax diagonal terms when that always holds, so it does if
// indel <= min(0, lmax*min(match,mismatch)) - max(0, lmax*max(match,mismatch)).
bool gaps_cannot_win(int64_t match, int64_t mismatch, int64_t indel, int64_t lmax) {
    const int64_t lo = std::min<int64_t>(0, lmax * std::min(match, mismatch));
    const int64_t hi = std::max<int64_t>(0, lmax * std::max(match, mismatch));
    return indel <= lo - hi;
}

struct Plan {
    int kernel = OVL_KERNEL_NONE;
    bool key64 = false;
    bool wide = true;
    int32_t band = -1;       // OVL_KERNEL_BANDED: band half-width
    int seed_kernel = OVL_KERNEL_NONE;  // OVL_KERNEL_BANDED: how the seed end j* is computed
    bool seed_key64 = false;
    bool seed_wide = true;
};

int make_plan_full(const Dev* c, int32_t match, int32_t mismatch, int64_t indel, Plan* out);

// band >= 0: the build's seed-and-extend knob (oracle_overlap_banded), exact
// (== the reference) whenever gaps cannot win -- the seed cell (n, j*) is
// always in the band and nothing off the ungapped diagonals can beat it -- and
// whenever the band covers every diagonal (band >= 2 * lmax).
int make_plan(const Dev* c, int32_t match, int32_t mismatch, int64_t indel, int32_t band, Plan* out) {
    if (c->n_reads < 0) return fail(c, OVL_E_STATE, "no resident reads: call ovl_set_reads first");
    const int64_t L = std::max<int32_t>(c->lmax, 1);
    if (band < 0 || band >= 2 * L || gaps_cannot_win(match, mismatch, indel, L))
        return make_plan_full(c, match, mismatch, indel, out);
    // seed: the ungapped closed form (any kernel that evaluates it exactly)
    Plan seed;
    int rc = make_plan_full(c, match, mismatch, INT32_MIN, &seed);
    if (rc != OVL_OK) return rc;
    if (!gaps_cannot_win(match, mismatch, INT32_MIN, L))
        return fail(c, OVL_E_UNSUPPORTED, "banded: the ungapped seed cannot be evaluated exactly at these scores");
    Plan full;
    rc = make_plan_full(c, match, mismatch, indel, &full);
    if (rc != OVL_OK) return rc;
    if (full.kernel != OVL_KERNEL_DP || full.wide)
        return fail(c, OVL_E_UNSUPPORTED, "banded: scores too large for int32 cells (|score| * (2*lmax+1) >= 2^31)");
    Plan p;
    p.kernel = OVL_KERNEL_BANDED;
    p.wide = false;
    p.band = band;
    p.seed_kernel = seed.kernel;
    p.seed_key64 = seed.key64;
    p.seed_wide = seed.wide;
    *out = p;
    return OVL_OK;
}

int make_plan_full(const Dev* c, int32_t match, int32_t mismatch, int64_t indel, Plan* out) {
    const int64_t L = std::max<int32_t>(c->lmax, 1);
    const int64_t amax = std::max(iabs64(match), iabs64(mismatch));
    Plan p;
    // ungapped closed form: exact when gaps cannot win and no int32 store can wrap
    if (c->wmax > 0 && gaps_cannot_win(match, mismatch, indel, L) && amax * L < (int64_t(1) << 31)) {
        p.kernel = OVL_KERNEL_UNGAPPED;
        // 32-bit keys (score << 16) - j need |score| < 2^15 on both sides, and the
        // folded form X * ((mismatch - match) << 16) + ... a 24-bit multiplier
        const int64_t dms = (int64_t)mismatch - (int64_t)match;
        // (the uniform sweep compares keys without their block constant: |score| + 32*amax
        //  must stay below 2^15 as well)
        p.key64 = !(amax * (2 * L + 32) < (1 << 15) && iabs64(dms) < 128 && iabs64(match) < 128);
    } else {
        if (c->lmax > kDpMaxLen)
            return fail(c, OVL_E_UNSUPPORTED, "gapped DP supports reads up to %d bases (longest is %d)", kDpMaxLen,
                        c->lmax);
        p.kernel = OVL_KERNEL_DP;
        const int64_t M = std::max(amax, iabs64(indel));
        // |dp| <= 2*lmax*M; one more term for the candidates: int32 is exact below 2^31
        p.wide = !(indel > INT32_MIN && M < (int64_t(1) << 31) && (2 * L + 1) * M < (int64_t(1) << 31));
    }
    *out = p;
    return OVL_OK;
}

int launch_score_chunk(Dev* c, const Plan& pl, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs,
                       int32_t match, int32_t mismatch, int64_t indel, int32_t* d_score, int32_t* d_end,
                       hipStream_t s);

// Per-device scratch (lane_col, seed_*) is shared by every launch of the device.  A launch on stream s
// first waits for the previous user on another stream; growing a buffer first waits for that user.
struct ScratchNeed {
    DevBuf* buf;
    size_t bytes;
};

hipError_t scratch_acquire(Dev* c, hipStream_t s, std::initializer_list<ScratchNeed> needs) {
    hipError_t e = hipSuccess;
    for (const ScratchNeed& n : needs) {
        if (n.buf->bytes >= n.bytes) continue;
        if (c->scratch_used && (e = hipEventSynchronize(c->scratch_evt)) != hipSuccess) return e;
        if ((e = ensure(*n.buf, n.bytes)) != hipSuccess) return e;
    }
    if (c->scratch_used && c->scratch_stream != s) e = hipStreamWaitEvent(s, c->scratch_evt, 0);
    return e;
}

hipError_t scratch_release(Dev* c, hipStream_t s) {
    hipError_t e = hipEventRecord(c->scratch_evt, s);
    c->scratch_stream = s;
    c->scratch_used = true;
    return e;
}

// Lane-per-pair full DP (ovl_dp_lane.hip): one lane per pair, so it needs many pairs to fill the
// chip (below that the one-wavefront-per-pair dp_fast_kernel is faster), reads short enough for
// the per-wavefront hand-off columns, and G = dp - indel*(i+j) inside int32.
bool use_dp_lane(const Dev* c, int64_t match, int64_t mismatch, int64_t indel, int64_t n_pairs) {
    if (c->dp_lane == 0) return false;
    const int64_t L = std::max<int32_t>(c->lmax, 1);
    const int64_t M = std::max(std::max(iabs64(match), iabs64(mismatch)), iabs64(indel));
    if (L > kLaneMaxLen || (4 * L + 4) * M >= (int64_t(1) << 30) || c->codes_bytes + 64 >= (int64_t(1) << 32))
        return false;
    return c->dp_lane == 1 || n_pairs >= kLaneMinPairs;
}

// Kernels queue pair indices as int32 (LDS side ring); split huge lists.
int launch_score(Dev* c, const Plan& pl, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs,
                 int32_t match, int32_t mismatch, int64_t indel, int32_t* d_score, int32_t* d_end,
                 hipStream_t s) {
    constexpr int64_t kChunk = int64_t(1) << 30;
    for (int64_t lo = 0; lo < n_pairs; lo += kChunk) {
        const int64_t n = std::min(kChunk, n_pairs - lo);
        int rc = launch_score_chunk(c, pl, d_a + lo, d_b + lo, n, match, mismatch, indel, d_score + lo, d_end + lo, s);
        if (rc != OVL_OK) return rc;
    }
    return OVL_OK;
}

// The candidate list's heavy tiles (flags per list tile on the device, ascending ids on host and device),
// once per list; waits for the list's stream.
int ensure_heavy(Dev* c) {
    if (c->heavy_for == c->cand_n) return OVL_OK;
    const int64_t n_tiles = (c->cand_n + 63) / 64;
    HIPCHK(c, ensure(c->tile_flags, (size_t)std::max<int64_t>(n_tiles, 1)));
    HIPCHK(c, ovl_launch_tile_flags(as<int32_t>(c->cand_a), c->cand_n, as<uint32_t>(c->full), c->n_reads,
                                    as<uint8_t>(c->tile_flags), c->stream));
    std::vector<uint8_t> f((size_t)n_tiles);
    HIPCHK(c, hipMemcpyAsync(f.data(), c->tile_flags.p, (size_t)n_tiles, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->h_heavy.clear();
    for (int64_t t = 0; t < n_tiles; ++t)
        if (f[(size_t)t]) c->h_heavy.push_back((int32_t)t);
    HIPCHK(c, ensure(c->heavy_ids, sizeof(int32_t) * std::max<size_t>(c->h_heavy.size(), 1)));
    if (!c->h_heavy.empty())
        HIPCHK(c, hipMemcpy(c->heavy_ids.p, c->h_heavy.data(), sizeof(int32_t) * c->h_heavy.size(),
                            hipMemcpyHostToDevice));
    c->heavy_for = c->cand_n;
    return OVL_OK;
}

// rs_log2 of an ungapped launch over n pairs: bit shifts split over 1 << rs_log2 lanes (the general kernel),
// or (uniform kernel, 2 planes) latency mode when rs_log2 > 0: up to kLatTiles tiles per CU for device lists,
// up to kLatTilesIx for a host-encoded list (which only throughput mode reads in place)
int32_t ungapped_rs_log2(const Dev* c, int64_t n_pairs, bool ix = false) {
    int32_t rs_log2 = 0;
    const int64_t want_waves = (int64_t)c->cu_count * 4 * 4;
    while (rs_log2 < 2 && ((n_pairs << rs_log2) + 63) / 64 < want_waves) ++rs_log2;
    if (c->planes == 2)
        rs_log2 = ((n_pairs + 63) / 64 <= (int64_t)c->cu_count * (ix ? kLatTilesIx : kLatTiles)) ? 1 : 0;
    return rs_log2;
}

// An ungapped launch over n pairs runs uniform_kernel in throughput mode, the one that can read a
// host-encoded pair list in place (uniform_kernel IX)
bool ix_launch(const Dev* c, int64_t n_pairs) {
    return c->planes == 2 && c->lmax > 0 && c->wmax >= 1 && c->wmax <= 8 && ungapped_rs_log2(c, n_pairs, true) == 0;
}

int launch_score_chunk(Dev* c, const Plan& pl, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs,
                       int32_t match, int32_t mismatch, int64_t indel, int32_t* d_score, int32_t* d_end,
                       hipStream_t s) {
    if (n_pairs == 0) return OVL_OK;
    const int32_t* seed_end = nullptr;
    if (pl.kernel == OVL_KERNEL_BANDED) {
        // seed j* into device scratch (the outputs may be host memory), then the banded DP reads it
        const size_t sb = sizeof(int32_t) * (size_t)n_pairs;
        HIPCHK(c, scratch_acquire(c, s, {{&c->seed_s, sb}, {&c->seed_e, sb}}));
        Plan seed;
        seed.kernel = pl.seed_kernel;
        seed.key64 = pl.seed_key64;
        seed.wide = pl.seed_wide;
        const int32_t out_mode = c->out_mode;
        c->out_mode = 0;  // the seeds stay in HBM
        int rc = launch_score_chunk(c, seed, d_a, d_b, n_pairs, match, mismatch, INT32_MIN, as<int32_t>(c->seed_s),
                                    as<int32_t>(c->seed_e), s);
        c->out_mode = out_mode;
        if (rc != OVL_OK) return rc;
        seed_end = as<int32_t>(c->seed_e);
    }
    if (c->ix_b16 && (pl.kernel != OVL_KERNEL_UNGAPPED || pl.key64 || !ix_launch(c, n_pairs)))
        return fail(c, OVL_E_UNSUPPORTED, "host-encoded pair list on a launch that cannot read it");
    if (pl.kernel == OVL_KERNEL_UNGAPPED) {
        OvlUngappedArgs g{};
        g.sfx = as<uint32_t>(c->sfx);
        g.pfx = as<uint32_t>(c->pfx);
        g.len = as<int32_t>(c->len);
        g.n_reads = c->n_reads;
        g.a_idx = d_a;
        g.b_idx = d_b;
        g.n_pairs = n_pairs;
        // split a pair's 32 bit shifts over 1, 2 or 4 lanes until the grid has
        // enough wavefronts to fill every SIMD a few times
        // general kernel: split a pair's bit shifts over 1, 2 or 4 lanes until the grid
        // has enough wavefronts.  Uniform kernel: latency mode (two wavefronts per tile,
        // side pairs beside the sweep) when there is about one tile per wavefront slot.
        g.rs_log2 = ungapped_rs_log2(c, n_pairs, c->ix_b16 != nullptr);
        // uniform-length fast path (2 bit planes): pairs of two reads of length lmax;
        // uniform_kernel scores the other pairs through its LDS side ring
        g.lw = c->planes == 2 ? c->lmax : 0;
        g.full = as<uint32_t>(c->full);
        // (timing: this launch records the chunk's kernel events itself, once; issue_chunk checks they were taken)
        g.ev_start = c->kev_start;
        g.ev_stop = c->kev_stop;
        g.match = match;
        g.mismatch = mismatch;
        g.out_score = d_score;
        g.out_end = d_end;
        g.err_flag = c->cur_flag;
        g.planes = c->planes;
        g.wmax = c->wmax;
        g.key64 = pl.key64 ? 1 : 0;
        g.max_blocks = (int64_t)c->cu_count * kBlocksPerCu;
        g.host_out = c->out_mode;
        g.ix_b16 = c->ix_b16;
        g.ix_d8 = c->ix_d8;
        g.ix_base = c->ix_base;
        // a throughput-mode launch over (a 64-aligned part of) the resident candidate list: heavy tiles first
        const int32_t* ca = as<int32_t>(c->cand_a);
        if (!g.ix_b16 && g.lw > 0 && g.rs_log2 == 0 && c->cand_n > 0 && d_a >= ca &&
            d_a < ca + c->cand_n && d_b == as<int32_t>(c->cand_b) + (d_a - ca) && (d_a - ca) % 64 == 0) {
            int rc = ensure_heavy(c);
            if (rc != OVL_OK) return rc;
            const int64_t t0 = (d_a - ca) / 64, t1 = t0 + (n_pairs + 63) / 64;
            const auto k0 = std::lower_bound(c->h_heavy.begin(), c->h_heavy.end(), t0);
            const auto k1 = std::lower_bound(c->h_heavy.begin(), c->h_heavy.end(), t1);
            if (k1 > k0) {
                g.heavy_ids = as<int32_t>(c->heavy_ids) + (k0 - c->h_heavy.begin());
                g.heavy_n = (int32_t)(k1 - k0);
                g.tile_flags = as<uint8_t>(c->tile_flags);
                g.tile_base = t0;
            }
        }
        HIPCHK(c, ovl_launch_ungapped(&g, s));
        if (g.ev_start && g.lw > 0) c->kev_start = c->kev_stop = nullptr;  // (uniform_kernel recorded them)
    } else {
        OvlDpArgs g{};
        g.codes = as<uint8_t>(c->codes);
        g.off = as<int64_t>(c->off);
        g.len = as<int32_t>(c->len);
        g.n_reads = c->n_reads;
        g.a_idx = d_a;
        g.b_idx = d_b;
        g.n_pairs = n_pairs;
        g.mcap = std::max<int32_t>(c->lmax, 1);
        g.match = match;
        g.mismatch = mismatch;
        g.indel = indel;
        g.out_score = d_score;
        g.out_end = d_end;
        g.tb = nullptr;
        g.err_flag = c->cur_flag;
        g.wide = pl.wide ? 1 : 0;
        g.band = pl.kernel == OVL_KERNEL_BANDED ? pl.band : -1;
        g.seed = seed_end;
        g.classic = c->dp_classic;
        if (g.band < 0 && !g.wide && !g.classic && use_dp_lane(c, match, mismatch, indel, n_pairs)) {
            OvlLaneArgs k{};
            k.cw = 32;
            k.slots = (int64_t)c->cu_count * 4 * ovl_dp_lane_waves_per_simd(k.cw);
            const int64_t L = std::max<int32_t>(c->lmax, 1);
            const int64_t M = std::max(std::max(iabs64(match), iabs64(mismatch)), iabs64(indel));
            const int64_t sma = (int64_t)match - 2 * indel, smm = (int64_t)mismatch - 2 * indel;
            k.prof = c->lane_prof && c->planes == 2 && indel <= 0 && sma >= -128 && sma <= 127 && smm >= -128 &&
                     smm <= 127;
            k.ho = (4 * L + 4) * M < (int64_t(1) << 15) ? 1 : 0;
            k.sfx = k.prof && c->lane_sfx && c->wmax > 0;
            // column steps G[i][j] - G[i-1][j] lie in [0, max(match, mismatch) - 2*indel]: 4 bits in LDS
            const int64_t step_max = std::max<int64_t>(match, mismatch) - 2 * indel;
            if (k.sfx && indel <= 0 && std::max<int64_t>(match, mismatch) >= indel &&
                step_max <= 15 && g.mcap <= 256)
                k.ho = 2;
            k.h2 = k.ho == 2 && c->lane_h2 && ovl_dp_lane_h2_ok(match, mismatch, indel);
            // hand-off columns in HBM: one per resident slot (HO 0 / 1), per tile for the h2 form's HBM variant --
            // which launches at most kH2Slice pairs at a time over one reused column buffer (lcap / 2 bytes per
            // pair: 1 GiB at 256-base reads), and falls back to the int32 form (HO 2: no HBM column) when even that
            // cannot be allocated
            constexpr int64_t kH2Slice = int64_t(1) << 23;
            const int64_t slice = k.h2 ? std::min(n_pairs, kH2Slice) : n_pairs;
            size_t col_bytes =
                k.h2 ? (size_t)ovl_dp_lane_h2_col_bytes(slice, g.mcap)
                     : (k.ho == 2 ? 0 : (size_t)k.slots * ovl_dp_lane_rcap(g.mcap) * 64 * sizeof(uint32_t));
            hipError_t se = scratch_acquire(c, s, {{&c->lane_col, col_bytes}});
            if (se == hipErrorOutOfMemory && k.h2) {
                (void)hipGetLastError();
                k.h2 = 0;
                col_bytes = 0;
                se = scratch_acquire(c, s, {{&c->lane_col, col_bytes}});
            }
            HIPCHK(c, se);
            k.sfx_words = as<uint32_t>(c->sfx);
            k.pfx_words = as<uint32_t>(c->pfx);
            k.srow = c->srow;
            k.wsfx = c->wmax;
            k.colbuf = as<uint32_t>(c->lane_col);
            for (int64_t lo = 0; lo < n_pairs; lo += slice) {
                OvlDpArgs gs = g;
                gs.a_idx = d_a + lo;
                gs.b_idx = d_b + lo;
                gs.out_score = d_score + lo;
                gs.out_end = d_end + lo;
                gs.n_pairs = std::min(slice, n_pairs - lo);
                HIPCHK(c, ovl_launch_dp_lane(&gs, &k, s));
            }
            HIPCHK(c, scratch_release(c, s));
            return OVL_OK;
        }
        if (g.band >= 0) {
            // "-inf" (kBandNeg) must stay below every value: |values| <= (2*lmax + 1) * M and the row
            // form's scan adds up to 2*band*|indel|
            const int64_t Mx = std::max(std::max(iabs64(match), iabs64(mismatch)), iabs64(indel));
            const int64_t L = std::max<int32_t>(c->lmax, 1);
            const bool neg_ok = (4 * L + 2) * Mx < (int64_t(1) << 29);
            const int64_t lanes = 2 * (int64_t)g.band + 1;
            const bool diag_ok = neg_ok && ovl_band_diag_slots(g.band, c->lmax, nullptr) > 0;
            const bool rows_ok = neg_ok && lanes <= 192 && c->lmax <= 1024;
            // lane per pair: byte scores (match/mismatch - 2*indel, -2*indel, -indel in int8), indel <= 0,
            // <= 4 symbols, G = dp - indel*(i+j) in int32 with j down to -(2*lmax + band)
            const int64_t sma = (int64_t)match - 2 * indel, smm = (int64_t)mismatch - 2 * indel;
            auto i8 = [](int64_t v) { return v >= -128 && v <= 127; };
            const bool lane_ok = c->planes == 2 && ovl_band_lane_ok(g.band) && indel <= 0 && i8(sma) &&
                                 i8(smm) && i8(-2 * indel) && (6 * L + 2 * g.band + 8) * Mx < (int64_t(1) << 30) &&
                                 c->lmax <= kLaneMaxLen && c->codes_bytes + 64 < (int64_t(1) << 32);
            switch (c->band_form) {
                case OVL_BAND_FORM_ROWS: g.band_form = rows_ok ? OVL_BAND_FORM_ROWS : OVL_BAND_FORM_STRIP; break;
                case OVL_BAND_FORM_FAST: g.band_form = OVL_BAND_FORM_FAST; break;
                case OVL_BAND_FORM_STRIP: g.band_form = OVL_BAND_FORM_STRIP; break;
                case OVL_BAND_FORM_DIAG: g.band_form = diag_ok ? OVL_BAND_FORM_DIAG : OVL_BAND_FORM_FAST; break;
                case OVL_BAND_FORM_LANE:
                case OVL_BAND_FORM_LANE1:
                case OVL_BAND_FORM_LANE2:
                    g.band_form = lane_ok ? OVL_BAND_FORM_LANE : (diag_ok ? OVL_BAND_FORM_DIAG : OVL_BAND_FORM_FAST);
                    break;
                default:
                    g.band_form = (lane_ok && n_pairs >= kLaneMinPairs)
                                      ? OVL_BAND_FORM_LANE
                                      : (diag_ok ? OVL_BAND_FORM_DIAG : OVL_BAND_FORM_FAST);
                    break;
            }
            if (g.band_form == OVL_BAND_FORM_LANE) {
                OvlLaneArgs k{};
                k.slots = (int64_t)c->cu_count * 4 * 6;
                k.sfx = c->lane_sfx && c->wmax > 0;
                k.sfx_words = as<uint32_t>(c->sfx);
                k.pfx_words = as<uint32_t>(c->pfx);
                k.srow = c->srow;
                k.wsfx = c->wmax;
                k.split = c->band_form == OVL_BAND_FORM_LANE2 ||
                          (c->band_form != OVL_BAND_FORM_LANE1 && g.band >= kBandLane2Min);
                HIPCHK(c, ovl_launch_band_lane(&g, &k, s));
                HIPCHK(c, scratch_release(c, s));
                return OVL_OK;
            }
        }
        HIPCHK(c, ovl_launch_dp(&g, s));
        if (seed_end) HIPCHK(c, scratch_release(c, s));
    }
    return OVL_OK;
}

// ----------------------------------------------------------------------------- devices

// Restores the caller's current device when a public entry point returns.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

Knobs read_knobs() {
    Knobs k;
    if (const char* e = getenv("OVL_BAND_FORM")) {
        if (!strcmp(e, "diag")) k.band_form = OVL_BAND_FORM_DIAG;
        else if (!strcmp(e, "rows")) k.band_form = OVL_BAND_FORM_ROWS;
        else if (!strcmp(e, "fast")) k.band_form = OVL_BAND_FORM_FAST;
        else if (!strcmp(e, "strip")) k.band_form = OVL_BAND_FORM_STRIP;
        else if (!strcmp(e, "lane")) k.band_form = OVL_BAND_FORM_LANE;
        else if (!strcmp(e, "lane1")) k.band_form = OVL_BAND_FORM_LANE1;
        else if (!strcmp(e, "lane2")) k.band_form = OVL_BAND_FORM_LANE2;
    }
    if (const char* e = getenv("OVL_DP_FORM")) {
        if (!strcmp(e, "lane")) k.dp_lane = 1;
        else if (!strcmp(e, "fast")) k.dp_lane = 0;
        else if (!strcmp(e, "classic")) k.dp_classic = 1;
    }
    if (const char* e = getenv("OVL_LANE_FORM")) {
        const int v = atoi(e);
        k.lane_prof = v & 1;
        k.lane_sfx = (v >> 1) & 1;
        k.lane_h2 = (v >> 2) & 1;
    }
    if (const char* e = getenv("OVL_PACK")) k.pack = std::max(0, std::min(1, atoi(e)));
    if (const char* e = getenv("OVL_RESIDENT")) {  // mode[,blocks/CU[,pipelined[,poll sleep[,ring]]]] ("1x2x1x4x1")
        k.resident = std::max(0, std::min(2, atoi(e)));
        if (const char* c = strpbrk(e, ",x")) {
            k.resident_blocks = std::max(1, std::min(8, atoi(c + 1)));
            if (const char* c2 = strpbrk(c + 1, ",x")) {
                k.resident_pf = atoi(c2 + 1) != 0;
                if (const char* c3 = strpbrk(c2 + 1, ",x")) {
                    k.resident_sleep = std::max(0, std::min(1000, atoi(c3 + 1)));
                    if (const char* c4 = strpbrk(c3 + 1, ",x")) k.resident_ring = std::min(2, std::max(0, atoi(c4 + 1)));
                }
            }
        }
    }
    if (const char* e = getenv("OVL_PACK_MIN")) k.pack_min = std::max(0LL, atoll(e));
    if (const char* e = getenv("OVL_PACK_DIRECT_PCT")) {
        k.pack_direct_pct = std::max(0, std::min(100, atoi(e)));
        k.pack_adapt = 0;  // a fixed share
    }
    if (const char* e = getenv("OVL_PAIRS_FORM")) {
        if (!strcmp(e, "plain")) k.compact = 0;
        else if (!strcmp(e, "decode")) k.pairs_ix = 0;
    }
    if (const char* e = getenv("OVL_PIPE_CHUNK")) {
        const long long v = atoll(e);
        if (v >= 64) k.pipe_chunk = v;
    }
    return k;
}

void host_copy(void* dst, const void* src, size_t bytes) { CopyPool::get().copy(dst, src, bytes); }

// Packed results (ovl_kernels.hip put_pair, sink 2) into the caller's int32 arrays (ovl_expand.h), split
// over the host pool, at the widest vector width this CPU runs.
void host_expand(int32_t* s, int32_t* e, const uint16_t* pk, const int32_t* esc, int32_t match, int32_t mismatch,
                 bool nt, size_t n, size_t min_part) {
    static const ovl_expand::Fn f = ovl_expand::pick(nullptr);
    CopyPool::get().parallel(n, min_part,
                             [=](size_t lo, size_t hi) { f(s, e, pk, esc, match, mismatch, nt, lo, hi); });
}

// The pipeline's waits for a chunk: polled (a chunk is tens of microseconds away; a blocking wait can
// add its own wake-up latency per chunk, depending on the device's scheduling flags).
hipError_t wait_event(const Dev* d, hipEvent_t ev) {
    (void)d;
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        _mm_pause();
    }
}

void free_staging(int32_t*& p) {
    if (p) (void)hipHostFree(p);
    p = nullptr;
}

void destroy_dev(Dev* d) {
    if (!d) return;
    d->worker.reset();
    d->res.release();
    (void)hipSetDevice(d->device);
    for (hipStream_t s : {d->stream, d->s_in})
        if (s) (void)hipStreamSynchronize(s);
    for (DevBuf* b : {&d->codes, &d->off, &d->len, &d->sfx, &d->pfx, &d->lut, &d->full, &d->raw, &d->rd, &d->a, &d->b,
                      &d->score, &d->end, &d->tb, &d->err_flag, &d->k_pre, &d->k_suf, &d->k_sorted, &d->k_iota,
                      &d->k_order, &d->k_lo, &d->k_hi, &d->k_cnt, &d->k_offs, &d->k_temp, &d->cand_a, &d->cand_b,
                      &d->sh_cum, &d->sh_temp, &d->sh_cuts, &d->l_q, &d->l_r, &d->l_row, &d->l_tb, &d->l_best,
                      &d->lane_col, &d->seed_s, &d->seed_e, &d->tile_flags, &d->heavy_ids, &d->cp_hbm})
        release(*b);
    if (d->l_tb_host) (void)hipHostFree(d->l_tb_host);
    free_staging(d->st_in);
    free_staging(d->st_out);
    if (d->h_flag) (void)hipHostFree(d->h_flag);
    if (d->cp_host) (void)hipHostFree(d->cp_host);
    for (hipEvent_t e : d->dec_ev)
        if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < kSlots; ++i)
        if (d->ev_k[i]) (void)hipEventDestroy(d->ev_k[i]);
    for (hipEvent_t e : d->t_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : d->k_ev)
        if (e) (void)hipEventDestroy(e);
    if (d->scratch_evt) (void)hipEventDestroy(d->scratch_evt);
    if (d->ev_last) (void)hipEventDestroy(d->ev_last);
    for (hipStream_t s : {d->stream, d->s_in})
        if (s) (void)hipStreamDestroy(s);
    delete d;
}

hipError_t init_dev(Dev* d) {
    hipError_t e = hipSetDevice(d->device);
    if (e != hipSuccess) return e;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d->device) == hipSuccess && prop.multiProcessorCount > 0)
        d->cu_count = prop.multiProcessorCount;
    d->res.device = d->device;
    d->res.cu_count = d->cu_count;
    d->res.blocks_per_cu = d->k.resident_blocks;
    d->res.pipelined = d->k.resident_pf;
    d->res.poll_sleep = d->k.resident_sleep;
    d->res.ring_kind = d->k.resident_ring;
    for (hipStream_t* s : {&d->stream, &d->s_in}) {
        e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
        if (e != hipSuccess) return e;
    }
    for (int i = 0; i < kSlots; ++i) {
        e = hipEventCreateWithFlags(&d->ev_k[i], hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    e = hipEventCreateWithFlags(&d->scratch_evt, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    e = hipEventCreateWithFlags(&d->ev_last, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    e = hipHostMalloc((void**)&d->h_flag, 64, kHostShared);
    if (e != hipSuccess) return e;
    *d->h_flag = 0;
    e = hipHostGetDevicePointer((void**)&d->h_flag_dev, d->h_flag, 0);
    if (e != hipSuccess) return e;
    e = ensure(d->err_flag, 16);
    if (e != hipSuccess) return e;
    d->cur_flag = as<uint32_t>(d->err_flag);
    return hipMemset(d->err_flag.p, 0, 16);
}

int create_on(const int32_t* ids, int32_t n, ovl_ctx** out) {
    int count = 0;
    HIPCHK((ovl_ctx*)nullptr, hipGetDeviceCount(&count));
    if (count <= 0) return fail((ovl_ctx*)nullptr, OVL_E_HIP, "no HIP device visible");
    if (n <= 0) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "no devices requested");
    // OVL_SHARE_DEVICES=1 (tests on a one-GPU box): a device may be listed more than once; each entry is
    // an independent shard slot (own streams, buffers, staging and flag) on that GPU, so the N-device
    // sharding, per-device jobs and slice copies run for real
    const char* share = getenv("OVL_SHARE_DEVICES");
    const bool allow_dup = share && atoi(share) == 1;
    for (int32_t i = 0; i < n; ++i) {
        if (ids[i] < 0 || ids[i] >= count)
            return fail((ovl_ctx*)nullptr, OVL_E_ARG, "device %d outside [0, %d)", ids[i], count);
        for (int32_t j = 0; j < i && !allow_dup; ++j)
            if (ids[j] == ids[i]) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "device %d listed twice", ids[i]);
    }
    DeviceGuard guard;
    CpuShare::get().refresh(true);
    ovl_ctx* c = new ovl_ctx();
    c->shared_slots = allow_dup;
    const Knobs knobs = read_knobs();
    for (int32_t i = 0; i < n; ++i) {
        Dev* d = new Dev();
        d->owner = c;
        d->device = ids[i];
        d->k = knobs;
        c->devs.push_back(d);
        hipError_t e = init_dev(d);
        if (e != hipSuccess) {
            int rc = fail((ovl_ctx*)nullptr, e == hipErrorOutOfMemory ? OVL_E_OOM : OVL_E_HIP,
                          "context setup on device %d: %s", ids[i], hipGetErrorString(e));
            ovl_destroy(c);
            return rc;
        }
    }
    *out = c;
    return OVL_OK;
}

// ----------------------------------------------------------------------------- host-array pipeline

// True when [p, p + bytes) is pinned host memory (hipHostMalloc'd or registered), so DMA can
// read or write it in place.  hipPointerGetAttributes fails (or reports "unregistered") for
// pageable memory; its sticky error is cleared so later hipGetLastError callers (torch) see none.
bool host_pinned(const void* p, size_t bytes) {
    if (!p || bytes == 0) return false;
    const char* ends[2] = {(const char*)p, (const char*)p + bytes - 1};
    for (const char* q : ends) {
        hipPointerAttribute_t at;
        memset(&at, 0, sizeof(at));
        if (hipPointerGetAttributes(&at, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (at.type != hipMemoryTypeHost) return false;
    }
    return true;
}

// Pairs per pipeline chunk.  Measured on MI355X (tools/pipe_ab.py, profiles/r02_pipe_ab_*.json): every
// chunk's D2H copy costs ~0.1 ms of fixed overhead, which is more than the kernel time a chunk hides, so
// copies of pinned arrays run as one chunk; only pageable arrays, which go through pinned staging slots,
// are cut into chunks (the slot size): 512 K pairs, the kernels reading and storing the staging slots
// themselves (the host copy of chunk k+1 overlaps the kernel of chunk k).
// Direct kernel stores into pinned arrays need no chunks at all.  Packed results (pack_ok) are expanded
// on the host chunk by chunk while the next chunk is scored: 1 M pairs (tools/host_paths_ab.py at the
// target point: 128 K 0.53 ms, 256 K 0.38, 512 K 0.30, 1 M 0.25, one chunk 0.29).
int64_t pick_chunk(const Dev* d, int64_t n, bool staged, bool pack) {
    if (d->k.pipe_chunk > 0) return d->k.pipe_chunk;
    const int64_t cap = int64_t(1) << (pack ? 20 : 19);
    return std::max<int64_t>(1, staged ? std::min(n, cap) : n);
}

hipError_t alloc_staging(int32_t*& p, int32_t*& p_dev, int64_t cap) {
    hipError_t e = hipHostMalloc((void**)&p, (size_t)kSlots * 2 * (size_t)cap * sizeof(int32_t), kHostShared);
    if (e != hipSuccess) return e;
    return hipHostGetDevicePointer((void**)&p_dev, p, 0);
}

struct Call {
    const Plan* plan = nullptr;
    int32_t match = 0, mismatch = 0;
    int64_t indel = 0;
    const int32_t* h_a = nullptr;  // host pair list (global indexing), or null: device lists per job
    const int32_t* h_b = nullptr;
    bool in_pinned = false;
    int32_t* out_s = nullptr;      // host results; out_s[p - out_base] for global pair p
    int32_t* out_e = nullptr;
    int64_t out_base = 0;
    bool out_pinned = false;
    bool pack = false;             // results cross the link packed (2 bytes per pair) into the staging
                                   // slots and are expanded into the caller's arrays on the host (all chunks for
                                   // pageable arrays; for pinned ones all but a last direct chunk, Job::n_packed)
    bool compact = false;          // one device: the host pair list is encoded per chunk (encode_chunk)
                                   // and decoded into HBM by kernels reading it through the host mapping
    bool timing = false;
};

struct Job {
    Dev* d = nullptr;
    int64_t lo = 0, hi = 0;  // global pair range of this device
    int64_t chunk = 1;       // largest chunk (the staging slot capacity)
    std::vector<int64_t> cb; // chunk k: pairs [cb[k], cb[k + 1]) of the range (local indexing)
    int64_t nchunks = 0;
    int64_t n_packed = 0;    // C.pack: the first n_packed chunks are packed and staged
    int64_t st_in_cap = 0, st_out_cap = 0;
    const int32_t* dev_a = nullptr;  // device pair list (global indexing) when the call has no host list
    const int32_t* dev_b = nullptr;
    int32_t* ka = nullptr;  // device copies of the host list (local indexing)
    int32_t* kb = nullptr;
    const int32_t* za = nullptr;  // direct: device addresses of the caller's pinned pair arrays (local indexing)
    const int32_t* zb = nullptr;
    int32_t* d_score = nullptr;  // device results (local indexing)
    int32_t* d_end = nullptr;
    std::vector<uint8_t> ixk;    // C.compact: chunk k's list is read in place by uniform_kernel (encode_chunk)
    std::vector<uint8_t> kexact; // timing: chunk k's kernel recorded its own start / end (k_ev)
    std::vector<uint8_t> om;     // chunk k's result sink (OvlUngappedArgs::host_out): 1 int32, 2 packed
    std::vector<uint8_t> slot;   // chunk k's staging slot: k % kSlots
    int64_t drained = 0;         // chunks [0, drained) are drained (run_pipeline)
};

// Chunk k's results go through the staging slots (pageable caller arrays, or a packed chunk).
bool chunk_staged(const Call& C, const Job& J, int64_t k) { return !C.out_pinned || (C.pack && k < J.n_packed); }

int setup_job(const Call& C, Job& J) {
    Dev* d = J.d;
    const int64_t n = J.hi - J.lo;
    J.cb.assign(1, 0);
    J.nchunks = J.n_packed = 0;
    if (n <= 0) return OVL_OK;
    HIPCHK(d, hipSetDevice(d->device));
    const bool need_in = C.h_a && !C.in_pinned && !C.compact, need_out = !C.out_pinned || C.pack;
    J.chunk = pick_chunk(d, n, need_in || need_out, C.pack);
    // packed calls: the packed share in equal chunks of <= J.chunk, then (pinned arrays) the direct share
    int64_t packed = 0;
    if (C.pack) {
        double& share = C.compact ? d->pack_pct_h : d->pack_pct;
        if (share < 0.0) share = C.compact ? 2.0 * d->k.pack_direct_pct : d->k.pack_direct_pct;
        const int64_t pct = d->k.pack_adapt ? (int64_t)(share + 0.5) : d->k.pack_direct_pct;
        packed = C.out_pinned ? (n - n * pct / 100) & ~int64_t(63) : n;
        if (packed >= n - 64) packed = n;
        // (a ramp of growing chunks -- 196 K, x 1.5 each -- to start the host's expansion sooner measured slower:
        // 0.208 against 0.145 ms at the target point, each extra chunk costing an issue and a later direct
        // chunk; profiles/r04_pool_ab_*.json)
        const int64_t pieces = (packed + J.chunk - 1) / J.chunk;
        const int64_t step = pieces ? (((packed + pieces - 1) / pieces + 63) & ~int64_t(63)) : 0;
        for (int64_t o = step; o < packed; o += step) J.cb.push_back(o);
        if (packed > 0) J.cb.push_back(packed);
        J.n_packed = (int64_t)J.cb.size() - 1;
    }
    for (int64_t o = J.cb.back(); o < n;) {  // (the direct chunks)
        o = std::min(n, o + J.chunk);
        J.cb.push_back(o);
    }
    J.nchunks = (int64_t)J.cb.size() - 1;
    // sinks: packed chunks 2 bytes per pair; the rest int32
    J.om.assign((size_t)J.nchunks, 1);
    J.drained = 0;
    for (int64_t k = 0; k < J.n_packed; ++k) J.om[(size_t)k] = 2;
    J.slot.resize((size_t)J.nchunks);
    for (int64_t k = 0; k < J.nchunks; ++k) J.slot[(size_t)k] = (uint8_t)(k % kSlots);
    for (int64_t k = 0; k < J.nchunks; ++k) J.chunk = std::max(J.chunk, J.cb[(size_t)k + 1] - J.cb[(size_t)k]);
    const size_t bytes = sizeof(int32_t) * (size_t)n;
    if (C.compact) {
        // decoded pair list in HBM, the pinned encoding buffer (chunk k at align16(8 * cb[k] + 32 * k)) and
        // the chunks' decode events
        HIPCHK(d, ensure(d->a, bytes));
        HIPCHK(d, ensure(d->b, bytes));
        J.ka = as<int32_t>(d->a);
        J.kb = as<int32_t>(d->b);
        const size_t need = 8 * (size_t)n + 32 * (size_t)J.nchunks + 64;
        if (d->cp_bytes < need) {
            if (d->cp_host) (void)hipHostFree(d->cp_host);
            d->cp_host = d->cp_dev = nullptr;
            d->cp_bytes = 0;
            HIPCHK(d, hipHostMalloc((void**)&d->cp_host, need, kHostShared));
            HIPCHK(d, hipHostGetDevicePointer((void**)&d->cp_dev, d->cp_host, 0));
            d->cp_bytes = need;
        }
        if (d->k.pairs_ix) HIPCHK(d, ensure(d->cp_hbm, need));
        while ((int64_t)d->dec_ev.size() < J.nchunks) {
            hipEvent_t ev;
            HIPCHK(d, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            d->dec_ev.push_back(ev);
        }
        d->cp_link = 0;
    }
    if (C.h_a && C.in_pinned && !C.compact) {
        // the kernels read this device's slice of the caller's pinned pair arrays in place
        void* pa = nullptr;
        void* pb = nullptr;
        HIPCHK(d, hipHostGetDevicePointer(&pa, const_cast<int32_t*>(C.h_a + J.lo), 0));
        HIPCHK(d, hipHostGetDevicePointer(&pb, const_cast<int32_t*>(C.h_b + J.lo), 0));
        J.za = reinterpret_cast<const int32_t*>(pa);
        J.zb = reinterpret_cast<const int32_t*>(pb);
    }
    if (C.out_pinned) {
        // the device's address of this slice of the caller's pinned arrays
        void* ps = nullptr;
        void* pe = nullptr;
        HIPCHK(d, hipHostGetDevicePointer(&ps, C.out_s + (J.lo - C.out_base), 0));
        HIPCHK(d, hipHostGetDevicePointer(&pe, C.out_e + (J.lo - C.out_base), 0));
        J.d_score = reinterpret_cast<int32_t*>(ps);
        J.d_end = reinterpret_cast<int32_t*>(pe);
    }
    // pinned staging rings for pageable caller arrays, both allocated with capacity d->st_cap
    if ((need_in || need_out) && J.chunk > d->st_cap) {
        free_staging(d->st_in);
        free_staging(d->st_out);
        d->st_cap = (J.chunk + 63) & ~int64_t(63);  // (a slot's tile records start on 256 bytes)
    }
    if (need_in && !d->st_in) HIPCHK(d, alloc_staging(d->st_in, d->st_in_dev, d->st_cap));
    if (need_out && !d->st_out) {
        HIPCHK(d, alloc_staging(d->st_out, d->st_out_dev, d->st_cap));
    }
    if (C.timing && (int64_t)d->t_ev.size() < 2 * J.nchunks) {
        while ((int64_t)d->t_ev.size() < 2 * J.nchunks) {
            hipEvent_t ev;
            HIPCHK(d, hipEventCreate(&ev));
            d->t_ev.push_back(ev);
            HIPCHK(d, hipEventCreate(&ev));
            d->k_ev.push_back(ev);
        }
    }
    if (C.timing) J.kexact.assign((size_t)J.nchunks, 0);
    return OVL_OK;
}

// OVL_TRACE_PIPE=1 (diagnostics): one stderr line per host-array call with the microsecond offsets of its
// pipeline events (s setup, i<k> chunk k issued, w<k> its results ready on the host side, d<k> drained,
// y final synchronisation; streamed records: f<k> the calling thread's first record expanded, p<k> its part
// done, k<k> the chunk's kernel seen finished).
struct PipeTrace {
    bool on;
    std::chrono::steady_clock::time_point t0;
    std::string line;
    PipeTrace() : on(enabled()), t0(std::chrono::steady_clock::now()) {}
    static bool enabled() {
        static const bool e = [] {
            const char* v = getenv("OVL_TRACE_PIPE");
            return v && atoi(v) != 0;
        }();
        return e;
    }
    void mark(char what, int64_t k) {
        if (!on) return;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        char buf[48];
        snprintf(buf, sizeof(buf), " %c%lld=%.1f", what, (long long)k, us);
        line += buf;
    }
    ~PipeTrace() {
        if (on) fprintf(stderr, "ovl_pipe:%s\n", line.c_str());
    }
};
thread_local PipeTrace* g_trace = nullptr;

// Compact host pair list, chunk k (C.compact): the host pool encodes the caller's int32 pairs into the pinned
// encoding buffer and kernels on the device's second stream decode them into HBM (ovl_pairs.hip), reading the
// encoding through the host mapping; the chunk's scoring launch waits for dec_ev[k].  Encoding of chunk k:
//   b: uint16 when n_reads <= 65,535 (an index outside [0, n_reads) becomes 0xFFFF, decoded to -1, which the
//      scoring kernels report as OVL_E_INDEX like any bad index), else the int32 values;
//   a: runs (value, chunk-relative start; starts[R] = n) when 8 R + 4 < n * width -- the candidate lists of
//      overlapGraphs.py:43-52 are a-major, ~55 pairs per run at the target point --, else like b.
// At the target point 4.3 MB cross the link instead of 16 MB.
int issue_chunk(const Call& C, Job& J, int64_t k);

// `pre` (the previous chunk's issue, when given) runs on the calling thread while the pool encodes
int encode_chunk(const Call& C, Job& J, int64_t k, const std::function<int()>& pre = nullptr) {
    Dev* d = J.d;
    int pre_rc = OVL_OK;
    bool pre_done = !pre;
    const std::function<void()> run_pre = [&] {
        if (!pre_done) {
            pre_done = true;
            pre_rc = pre();
        }
    };
    const int64_t off = J.cb[(size_t)k];
    const int64_t n = J.cb[(size_t)k + 1] - off;
    const int64_t g = J.lo + off;
    const int32_t* A = C.h_a + g;
    const int32_t* B = C.h_b + g;
    const int32_t nr = d->n_reads;
    const int wd = nr <= 65535 ? 2 : 4;
    const size_t base = (8 * (size_t)off + 32 * (size_t)k + 15) & ~size_t(15);
    char* hb = d->cp_host + base;                  // b area
    const size_t b_bytes = ((size_t)n * wd + 15) & ~size_t(15);
    char* ha = hb + b_bytes;                       // a area: tile deltas + bases, runs, or a like b
    CopyPool& pool = CopyPool::get();
    const std::vector<size_t> parts = pool.cut((size_t)n, size_t(1) << 15);
    static const ovl_encode::Fns enc = ovl_encode::pick(nullptr);  // the widest this CPU runs
    J.ixk.resize((size_t)J.nchunks, 0);
    J.ixk[(size_t)k] = 0;
    // In place (uniform_kernel IX): b as uint16 and a as tile deltas (d8[p] = a[p] - a[64t], bases int32),
    // 3 bytes per pair and 4 per tile, copied into HBM by the copy engine on the second stream (large DMA
    // reads; the kernel's own 64-byte reads through the host mapping ran at ~25 GB/s) while the previous
    // chunk scores, and read by the scoring launch as they lie -- no decode launch.  Needs a-major tiles (a
    // within 255 of its tile's first, every a in range; the parts are cut at multiples of 64) and a
    // throughput-mode uniform launch; else the decode below.
    // (OVL_TRACE_PIPE: 'x' marks a chunk that cannot be read in place, with the first failed condition)
    const int ix_why = wd != 2 ? 1 : !d->k.pairs_ix ? 2 : C.plan->kernel != OVL_KERNEL_UNGAPPED ? 3
                       : C.plan->key64 ? 4 : !ix_launch(d, n) ? 5 : 0;
    if (g_trace && ix_why) g_trace->mark('x', ix_why);
    if (ix_why == 0) {
        uint8_t* d8 = reinterpret_cast<uint8_t*>(ha);
        int32_t* tb = reinterpret_cast<int32_t*>(ha + (((size_t)n + 15) & ~size_t(15)));
        std::vector<uint8_t> bad(parts.size(), 0);
        pool.parallel_parts(
            parts,
            [&](size_t i, size_t lo, size_t hi) {
                enc.narrow(B, nr, reinterpret_cast<uint16_t*>(hb), lo, hi);
                bad[i] = !enc.d8(A, nr, d8, tb, lo, hi);
            },
            run_pre);
        if (pre_rc != OVL_OK) return pre_rc;
        if (g_trace && std::find(bad.begin(), bad.end(), 1) != bad.end()) g_trace->mark('x', 6);
        if (std::find(bad.begin(), bad.end(), 1) == bad.end()) {
            J.ixk[(size_t)k] = 1;  // (issue_chunk copies the chunk into HBM and launches on it)
            if (g_trace) g_trace->mark('e', k);
            d->cp_link += 3 * (int64_t)n + 4 * ((n + 63) / 64);
            return OVL_OK;
        }
    }
    // one pass: b, and the runs of a (a[i] != a[i - 1], and i == 0) into part-local lists, given up (kept
    // short) once a part has more than 1 run per 16 pairs -- then a crosses like b
    std::vector<std::vector<int32_t>> pv(parts.size()), ps(parts.size());
    std::vector<uint8_t> many(parts.size(), 0);
    pool.parallel_parts(parts, [&](size_t i, size_t lo, size_t hi) {
        if (wd == 2) enc.narrow(B, nr, reinterpret_cast<uint16_t*>(hb), lo, hi);
        else memcpy(reinterpret_cast<int32_t*>(hb) + lo, B + lo, sizeof(int32_t) * (hi - lo));
        // (thread-local lists, handed over at the end: the parts' vector objects share cache lines)
        const size_t cap = (hi - lo) / 16 + 1;
        std::vector<int32_t> vv(cap + 1), ss(cap + 1);
        size_t r = enc.runs(A, lo ? A[lo - 1] : (int32_t)~A[0], lo, hi, vv.data(), ss.data(), cap);
        if (r > cap) {
            many[i] = 1;
            r = 0;
        }
        vv.resize(r);
        ss.resize(r);
        pv[i] = std::move(vv);
        ps[i] = std::move(ss);
    }, run_pre);
    if (pre_rc != OVL_OK) return pre_rc;
    int64_t R = 0;
    bool runs = n < (int64_t(1) << 31);
    for (size_t i = 0; i + 1 < parts.size(); ++i) {
        runs = runs && !many[i];
        R += (int64_t)pv[i].size();
    }
    runs = runs && 8 * R + 4 < n * wd;
    int32_t* vals = reinterpret_cast<int32_t*>(ha);
    int32_t* starts = vals + ((R + 3) & ~int64_t(3));  // 16-byte aligned
    if (runs) {
        int64_t r = 0;
        for (size_t i = 0; i + 1 < parts.size(); ++i) {
            memcpy(vals + r, pv[i].data(), sizeof(int32_t) * pv[i].size());
            memcpy(starts + r, ps[i].data(), sizeof(int32_t) * ps[i].size());
            r += (int64_t)pv[i].size();
        }
    } else {
        // a like b (a second pass, for lists that are not a-major)
        pool.parallel_parts(parts, [&](size_t, size_t lo, size_t hi) {
            if (wd == 2) {
                enc.narrow(A, nr, reinterpret_cast<uint16_t*>(ha), lo, hi);
            } else {
                memcpy(reinterpret_cast<int32_t*>(ha) + lo, A + lo, sizeof(int32_t) * (hi - lo));
            }
        });
    }
    if (runs) starts[R] = (int32_t)n;
    if (g_trace) g_trace->mark('e', k);
    // decode on the second stream (host-mapped reads) into this chunk's slice of the HBM list
    char* db = d->cp_dev + base;
    char* da = db + b_bytes;
    HIPCHK(d, hipSetDevice(d->device));
    HIPCHK(d, ovl_launch_widen(db, wd, n, J.kb + off, d->s_in));
    if (runs) {
        HIPCHK(d, ovl_launch_runs(reinterpret_cast<int32_t*>(da), reinterpret_cast<int32_t*>(da) + ((R + 3) & ~int64_t(3)),
                                  R, J.ka + off, d->s_in));
    } else {
        HIPCHK(d, ovl_launch_widen(da, wd, n, J.ka + off, d->s_in));
    }
    HIPCHK(d, hipEventRecord(d->dec_ev[(size_t)k], d->s_in));
    d->cp_link += (int64_t)n * wd + (runs ? 8 * R + 4 : (int64_t)n * wd);
    return OVL_OK;
}

// The kernels read the pair list and store the results through host mappings (no copy-engine transfers);
// pageable arrays are copied into / out of the pinned staging slots on the host.  (Round 1's copy-engine
// form -- H2D, kernel, D2H per chunk -- took 0.395 against 0.186 ms for the target point's step and is gone.)
int issue_chunk(const Call& C, Job& J, int64_t k) {
    Dev* d = J.d;
    HIPCHK(d, hipSetDevice(d->device));
    const int64_t off = J.cb[(size_t)k];
    const int64_t g = J.lo + off;
    const int64_t n = J.cb[(size_t)k + 1] - off;
    const bool staged_out = chunk_staged(C, J, k);
    const size_t nb = sizeof(int32_t) * (size_t)n;
    const int slot = J.slot[(size_t)k];
    const size_t so = (size_t)slot * 2 * (size_t)d->st_cap;
    const bool staged_in = C.h_a && !C.in_pinned && !C.compact;
    // the slot's previous user, chunk k - kSlots, must be done (its staged results were drained already)
    if (staged_in && k >= kSlots && !chunk_staged(C, J, k - kSlots)) HIPCHK(d, wait_event(d, d->ev_k[slot]));
    const int32_t* ka;
    const int32_t* kb;
    if (C.compact && J.ixk[(size_t)k]) {
        // read in place by uniform_kernel from its HBM copy (encode_chunk's layout of chunk k), copied by the
        // copy engine on the second stream
        const size_t base = (8 * (size_t)off + 32 * (size_t)k + 15) & ~size_t(15);
        const size_t b_bytes = ((size_t)n * 2 + 15) & ~size_t(15);
        const size_t bytes = b_bytes + (((size_t)n + 15) & ~size_t(15)) + 4 * (size_t)((n + 63) / 64);
        HIPCHK(d, hipMemcpyAsync(as<char>(d->cp_hbm) + base, d->cp_host + base, bytes, hipMemcpyHostToDevice,
                                 d->s_in));
        HIPCHK(d, hipEventRecord(d->dec_ev[(size_t)k], d->s_in));
        HIPCHK(d, hipStreamWaitEvent(d->stream, d->dec_ev[(size_t)k], 0));
        const char* hbm = as<char>(d->cp_hbm) + base;
        d->ix_b16 = reinterpret_cast<const uint16_t*>(hbm);
        d->ix_d8 = reinterpret_cast<const uint8_t*>(hbm + b_bytes);
        d->ix_base = reinterpret_cast<const int32_t*>(hbm + b_bytes + (((size_t)n + 15) & ~size_t(15)));
        ka = kb = nullptr;
    } else if (C.compact) {
        // decoded into HBM by encode_chunk's kernels on the second stream
        HIPCHK(d, hipStreamWaitEvent(d->stream, d->dec_ev[(size_t)k], 0));
        ka = J.ka + off;
        kb = J.kb + off;
    } else if (C.h_a) {
        if (staged_in) {
            host_copy(d->st_in + so, C.h_a + g, nb);
            host_copy(d->st_in + so + d->st_cap, C.h_b + g, nb);
            ka = d->st_in_dev + so;
            kb = d->st_in_dev + so + d->st_cap;
        } else {
            ka = J.za + off;
            kb = J.zb + off;
        }
    } else {
        ka = J.dev_a + g;
        kb = J.dev_b + g;
    }
    int32_t* os = staged_out ? d->st_out_dev + so : J.d_score + off;
    int32_t* oe = staged_out ? d->st_out_dev + so + d->st_cap : J.d_end + off;
    d->out_mode = J.om[(size_t)k];
    hipStream_t ks = d->stream;
    if (C.timing) {
        HIPCHK(d, hipEventRecord(d->t_ev[2 * k], ks));
        if (C.plan->kernel == OVL_KERNEL_UNGAPPED) {  // (a chunk of one ungapped launch: time the kernel itself)
            d->kev_start = d->k_ev[2 * k];
            d->kev_stop = d->k_ev[2 * k + 1];
        }
    }
    int rc = launch_score(d, *C.plan, ka, kb, n, C.match, C.mismatch, C.indel, os, oe, ks);
    if (C.timing) J.kexact[(size_t)k] = d->kev_start == nullptr && C.plan->kernel == OVL_KERNEL_UNGAPPED;
    d->kev_start = d->kev_stop = nullptr;
    d->ix_b16 = nullptr;
    d->ix_d8 = nullptr;
    d->ix_base = nullptr;
    if (rc != OVL_OK) return rc;
    if (C.timing) HIPCHK(d, hipEventRecord(d->t_ev[2 * k + 1], ks));
    if (staged_in || staged_out) HIPCHK(d, hipEventRecord(d->ev_k[slot], ks));
    if (C.pack && C.out_pinned && J.n_packed < J.nchunks && k == J.nchunks - 1)
        HIPCHK(d, hipEventRecord(d->ev_last, ks));
    return OVL_OK;
}

// Pageable outputs: copy chunk k out of its staging slot once its results are there (the kernel that stored
// them has finished).
int drain_chunk(const Call& C, Job& J, int64_t k) {
    Dev* d = J.d;
    const int64_t off = J.cb[(size_t)k];
    const int64_t g = J.lo + off;
    const int64_t n = J.cb[(size_t)k + 1] - off;
    const int slot = J.slot[(size_t)k];
    HIPCHK(d, wait_event(d, d->ev_k[slot]));
    if (g_trace) g_trace->mark('w', k);
    struct Drained {
        int64_t k;
        ~Drained() {
            if (g_trace) g_trace->mark('d', k);
        }
    } drained{k};
    const int32_t* ss = d->st_out + (size_t)slot * 2 * (size_t)d->st_cap;
    if (C.pack) {
        host_expand(C.out_s + (g - C.out_base), C.out_e + (g - C.out_base), reinterpret_cast<const uint16_t*>(ss),
                    ss + d->st_cap, C.match, C.mismatch, true, (size_t)n, kExpandPart);
        return OVL_OK;
    }
    host_copy(C.out_s + (g - C.out_base), ss, sizeof(int32_t) * (size_t)n);
    host_copy(C.out_e + (g - C.out_base), ss + d->st_cap, sizeof(int32_t) * (size_t)n);
    return OVL_OK;
}

void quiesce(std::vector<Job>& jobs) {
    for (Job& J : jobs) {
        (void)hipSetDevice(J.d->device);
        for (hipStream_t s : {J.d->stream, J.d->s_in}) (void)hipStreamSynchronize(s);
    }
}

// Host-array calls: the kernels flag a bad pair index by storing into the device's pinned host flag, which
// the host reads after the call's synchronisation (no flag copy behind the results).
struct HostFlag {
    std::vector<Job>& jobs;
    HostFlag(std::vector<Job>& j, int32_t out_mode) : jobs(j) {
        for (Job& J : jobs) {
            *(volatile uint32_t*)J.d->h_flag = 0;
            J.d->cur_flag = J.d->h_flag_dev;
            J.d->out_mode = out_mode;
        }
    }
    ~HostFlag() {
        for (Job& J : jobs) {
            J.d->cur_flag = as<uint32_t>(J.d->err_flag);
            J.d->out_mode = 0;
        }
    }
};

// One device's share of a host-array call: its chunks issued and drained in order.  A compact pair list (one device)
// has chunk k issued by this thread while the pool encodes chunk k + 1; staged chunks are drained kSlots - 1
// behind (a streamed record chunk once the chunk after it is queued: its kernel follows on the device while the
// host expands).  With `sync`, the job ends with its streams synchronised (device workers).
int run_job(const Call& C, Job& J, bool sync) {
    int rc = setup_job(C, J);
    if (rc != OVL_OK) return rc;
    if (g_trace) g_trace->mark('s', 0);
    if (C.compact && J.nchunks > 0 && (rc = encode_chunk(C, J, 0)) != OVL_OK) return rc;
    for (int64_t k = 0; k < J.nchunks && rc == OVL_OK; ++k) {
        const auto issue = [&]() -> int {
            const int r = issue_chunk(C, J, k);
            if (g_trace) g_trace->mark('i', k);
            return r;
        };
        if (C.compact && k + 1 < J.nchunks) rc = encode_chunk(C, J, k + 1, issue);
        else rc = issue();
        if (rc != OVL_OK) break;
        while (J.drained <= k) {
            const int64_t j = J.drained;
            if (chunk_staged(C, J, j) && k - j < kSlots - 1) break;
            if (chunk_staged(C, J, j) && (rc = drain_chunk(C, J, j)) != OVL_OK) break;
            ++J.drained;
        }
    }
    for (; rc == OVL_OK && J.drained < J.nchunks; ++J.drained)
        if (chunk_staged(C, J, J.drained)) rc = drain_chunk(C, J, J.drained);
    if (rc == OVL_OK && sync && J.nchunks > 0) {
        HIPCHK(J.d, hipSetDevice(J.d->device));
        HIPCHK(J.d, hipStreamSynchronize(J.d->stream));
    }
    return rc;
}

int run_pipeline(ovl_ctx* c, const Call& C, std::vector<Job>& jobs) {
    const auto t0 = std::chrono::steady_clock::now();
    PipeTrace trace;
    g_trace = &trace;
    struct Unset {
        ~Unset() { g_trace = nullptr; }
    } unset;
    int rc = OVL_OK;
    HostFlag host_flag(jobs, 1);  // (each chunk sets its own sink: issue_chunk)
    if (jobs.size() == 1) {
        rc = run_job(C, jobs[0], false);
    } else {
        // several devices: each device's job on its own host thread (DevWorker, on the GPU's NUMA node), so the
        // devices' launches, polls and synchronisations run side by side; this thread waits for all of them
        std::vector<int> rcs(jobs.size(), OVL_OK);
        std::atomic<int> left{(int)jobs.size()};
        std::mutex mu;
        std::condition_variable cv;
        for (size_t i = 0; i < jobs.size(); ++i) {
            Dev* d = jobs[i].d;
            if (!d->worker) d->worker.reset(new DevWorker(d->device));
            d->worker->post([&, i] {
                rcs[i] = run_job(C, jobs[i], true);
                if (left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                    std::lock_guard<std::mutex> lk(mu);
                    cv.notify_all();
                }
            });
        }
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return left.load(std::memory_order_acquire) == 0; });
        }
        for (size_t i = 0; i < jobs.size(); ++i)
            if (rcs[i] != OVL_OK) {
                rc = rcs[i];
                break;
            }
    }
    if (rc != OVL_OK) {
        quiesce(jobs);
        return rc;
    }
    #ifndef OVL_SHARE_WAIT_US
#define OVL_SHARE_WAIT_US 8.0  // (build macro for A/B builds: the host's wait for the direct chunk that counts)
#endif
// pack_share: the direct share of packed calls into pinned arrays follows which side finished last.  The
    // host pool has expanded every packed chunk now; if the direct chunk is already done, the link idled
    // while the host worked (more direct), if the host still waits for it, the host idles (more packed).
    for (Job& J : jobs) {
        Dev* d = J.d;
        if (!C.pack || !C.out_pinned || J.n_packed >= J.nchunks || !d->k.pack_adapt) continue;
        const auto tw = std::chrono::steady_clock::now();
        const hipError_t q = hipEventQuery(d->ev_last);
        if (q == hipSuccess) {
            double& share = C.compact ? d->pack_pct_h : d->pack_pct;
            share = std::min(C.compact ? 80.0 : 50.0, share + 1.0);
        } else if (q == hipErrorNotReady) {
            HIPCHK(c, wait_event(d, d->ev_last));
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw).count();
            double& share = C.compact ? d->pack_pct_h : d->pack_pct;
            if (us > OVL_SHARE_WAIT_US) share = std::max(2.0, share - 1.0);
        }
    }
    for (Job& J : jobs) {
        if (J.nchunks == 0) continue;
        HIPCHK(c, hipSetDevice(J.d->device));
        HIPCHK(c, hipStreamSynchronize(J.d->stream));
    }
    trace.mark('y', 0);
    double kms = 0.0;
    c->t_launches.clear();
    for (Job& J : jobs) {
        Dev* d = J.d;
        if (J.nchunks == 0) continue;
        if (*(volatile uint32_t*)d->h_flag) {
            *d->h_flag = 0;
            rc = fail(c, OVL_E_INDEX, "a pair index is outside [0, %d)", d->n_reads);
        }
        if (C.timing) {
            double s = 0.0;
            for (int64_t k = 0; k < J.nchunks; ++k) {
                float ms = 0.f;
                const bool exact = k < (int64_t)J.kexact.size() && J.kexact[(size_t)k];
                const hipEvent_t* ev = exact ? &d->k_ev[2 * (size_t)k] : &d->t_ev[2 * (size_t)k];
                if (hipEventElapsedTime(&ms, ev[0], ev[1]) == hipSuccess) s += ms;
                // the chunk's result sink (issue_chunk): packed staging, or int32 into host memory
                const int32_t sink = J.om[(size_t)k];
                c->t_launches.push_back({d->device, sink, J.cb[(size_t)k + 1] - J.cb[(size_t)k], (double)ms});
            }
            kms = std::max(kms, s);
        }
    }
    c->t_kernel_ms = kms;
    c->t_call_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    int64_t link = 0, packed = 0, ix = 0, dec = 0, res_all = 0;
    for (const Job& J : jobs) {
        const int64_t n = J.hi - J.lo;
        if (n <= 0) continue;
        const int64_t np = J.n_packed ? J.cb[(size_t)J.n_packed] : 0;
        packed += np;
        const int64_t res = 8 * (n - np) + 2 * np;  // results: int32 pairs, 2 bytes per packed pair
        res_all += res;
        link += (C.compact ? J.d->cp_link : (C.h_a ? 8 * n : 0)) + res;
        if (C.compact)
            for (int64_t k = 0; k < J.nchunks; ++k)
                (J.ixk[(size_t)k] ? ix : dec) += J.cb[(size_t)k + 1] - J.cb[(size_t)k];
    }
    c->x_link_bytes = link;
    c->x_packed_pairs = packed;
    c->x_res_bytes = res_all;
    c->x_rec_pairs = 0;  // (tile records: the resident grid's calls, resident_call)
    c->x_esc = 0;
    c->x_ix_pairs = ix;
    c->x_dec_pairs = dec;
    return rc;
}

// Host-side shard bounds of a host pair list over the context's devices (cost len[a]*len[b] + 1,
// the rule of ovl_shard_cut).  Indices are not trusted here: an out-of-range index costs 1.
std::vector<int64_t> host_cuts(const ovl_ctx* c, const int32_t* a, const int32_t* b, int64_t n, int32_t shards) {
    std::vector<int64_t> cuts((size_t)shards + 1, 0);
    cuts[(size_t)shards] = n;
    if (shards == 1 || n == 0) {
        for (int32_t r = 1; r < shards; ++r) cuts[(size_t)r] = 0;
        return cuts;
    }
    const int64_t nr = (int64_t)c->h_len.size();
    auto cost = [&](int64_t p) -> int64_t {
        const int32_t x = a[p], y = b[p];
        if (x < 0 || x >= nr || y < 0 || y >= nr) return 1;
        return (int64_t)c->h_len[(size_t)x] * c->h_len[(size_t)y] + 1;
    };
    int64_t total = 0;
    for (int64_t p = 0; p < n; ++p) total += cost(p);
    int64_t cum = 0, p = 0;
    for (int32_t r = 1; r < shards; ++r) {
        const int64_t want = total * r;
        while (p < n && (cum + cost(p)) * shards < want) cum += cost(p++);
        cuts[(size_t)r] = p;  // first p with cum[p] * shards >= want
    }
    return cuts;
}

// Shard bounds of [lo, hi) of device 0's resident candidate list over `shards` (ovl_shard_cut).
int device_cuts(Dev* d, int64_t lo, int64_t hi, int32_t shards, std::vector<int64_t>& cuts) {
    cuts.assign((size_t)shards + 1, lo);
    cuts[(size_t)shards] = hi;
    if (shards == 1 || hi <= lo) return OVL_OK;
    HIPCHK(d, hipSetDevice(d->device));
    const int64_t n = d->cand_n;
    size_t temp = 0;
    HIPCHK(d, ovl_shard_temp_bytes(n, &temp));
    HIPCHK(d, ensure(d->sh_temp, temp));
    HIPCHK(d, ensure(d->sh_cum, (size_t)n * sizeof(int64_t)));
    HIPCHK(d, ensure(d->sh_cuts, ((size_t)shards + 1) * sizeof(int64_t)));
    HIPCHK(d, ovl_shard_scan(d->sh_temp.p, d->sh_temp.bytes, as<int32_t>(d->cand_a), as<int32_t>(d->cand_b),
                             as<int32_t>(d->len), n, as<int64_t>(d->sh_cum), d->stream));
    HIPCHK(d, ovl_shard_cut(as<int64_t>(d->sh_cum), lo, hi, shards, as<int64_t>(d->sh_cuts), d->stream));
    HIPCHK(d, hipMemcpyAsync(cuts.data(), d->sh_cuts.p, ((size_t)shards + 1) * sizeof(int64_t), hipMemcpyDeviceToHost,
                             d->stream));
    HIPCHK(d, hipStreamSynchronize(d->stream));
    return OVL_OK;
}

// Direct host-array calls move results packed (ovl_kernels.hip put_pair, sink 2: end and mismatch count
// in a uint16) when the uniform kernel scores them with int32 keys and reads are at most 254 bases (ends
// and mismatch counts below the 0xFF marker).  One-device contexts only: the calling thread's host pool
// expands every packed chunk, so N devices would funnel N links' results through one pool, where int32
// results take N links in parallel (one process per GPU packs per process).
//   From OVL_PACK_MIN pairs into pinned arrays (256 K: tools/pack_size_ab.py, first n pairs of the target
// list, int32 / packed ms: 131 K 0.040 / 0.041, 262 K 0.065 / 0.057, 524 K 0.099 / 0.082, 1 M 0.182 / 0.100),
// from a quarter of that into pageable arrays, which need a host pass anyway (cfg2, 122 K pairs: 0.052-0.065
// against 0.065-0.079 ms; profiles/r02_pack_ab_cfg2_*.json, profiles/r02_pack_size_*.json).
bool pack_ok(const ovl_ctx* c, const Plan& p, int64_t n_pairs, bool out_pinned, int32_t n_devices) {
    const Dev* d = c->devs[0];
    const int64_t min_pairs = out_pinned ? d->k.pack_min : d->k.pack_min / 4;
    // (the expansion needs the host pool: with fewer than 6 threads -- several processes on one CPU set, e.g.
    // joblib workers or many ranks on one quota (CpuShare) -- the int32 stores over the link are faster)
    return n_devices == 1 && d->k.pack && n_pairs >= min_pairs && CopyPool::threads() >= 6 &&
           p.kernel == OVL_KERNEL_UNGAPPED && !p.key64 &&
           d->planes == 2 &&
           d->wmax > 0 && d->lmax > 0 && d->lmax <= 254;  // (lmax 0: the general kernel scores the list)
}

int check_scoring_args(ovl_ctx* c, int32_t match, int32_t mismatch, int64_t indel, int32_t band, Plan* p) {
    // every device holds the same read set, so device 0 plans for all
    return make_plan(c->devs[0], match, mismatch, indel, band, p);
}

// Devices (the context's first S) a host-array call over n pairs uses.  Calls over several devices store int32
// results over each device's own link (no packing: one host pool would expand every link's results), ~145 us per
// M pairs per link at 55 GB/s, against ~70 us per M pairs for one device with packed results and its resident grid
// or packed launches: several devices pay only from 3 of them, each with >= kMinPairsPerDevice
// pairs (their fixed per-call cost, ~15 us, against 36 us of link time).  Fewer -> one device, the single-device
// paths.  A context whose slots share a GPU (OVL_SHARE_DEVICES=1, tests) uses every slot.
constexpr int64_t kMinPairsPerDevice = int64_t(1) << 18;
int32_t devices_for(const ovl_ctx* c, int64_t n_pairs) {
    const int32_t k = (int32_t)c->devs.size();
    if (k <= 1) return 1;
    const int32_t s = (int32_t)std::min<int64_t>(k, n_pairs / kMinPairsPerDevice);
    return s >= 3 ? s : 1;
}
int32_t devices_used(const ovl_ctx* c, int64_t n_pairs) {
    return c->shared_slots ? (int32_t)c->devs.size() : devices_for(c, n_pairs);
}

// Stops the context's resident grids (ovl_resident.h) before other work on its devices: a grid's stream would hold
// a device synchronisation or a free until its idle deadline, and its blocks hold CU slots during other launches.
void quiet(ovl_ctx* c) {
    if (c)
        for (Dev* d : c->devs) (void)d->res.stop();
}

}  // namespace

// ----------------------------------------------------------------------------- context

OVL_API int ovl_version(void) { return OVL_ABI_VERSION; }

OVL_API const char* ovl_last_error(const ovl_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

OVL_API int ovl_device_count(int32_t* out_count) {
    if (!out_count) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "out_count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *out_count = 0;
        return fail((ovl_ctx*)nullptr, OVL_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *out_count = n;
    return OVL_OK;
}

OVL_API int ovl_create(int32_t n_devices, ovl_ctx** out_ctx) {
    if (!out_ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "out_ctx is NULL");
    *out_ctx = nullptr;
    if (n_devices < 0) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "n_devices < 0 (0 = all visible devices)");
    int count = 0, cur = 0;
    HIPCHK((ovl_ctx*)nullptr, hipGetDeviceCount(&count));
    if (count <= 0) return fail((ovl_ctx*)nullptr, OVL_E_HIP, "no HIP device visible");
    if (n_devices == 0) n_devices = count;
    if (n_devices > count)
        return fail((ovl_ctx*)nullptr, OVL_E_ARG, "n_devices %d > visible devices %d", n_devices, count);
    HIPCHK((ovl_ctx*)nullptr, hipGetDevice(&cur));
    std::vector<int32_t> ids((size_t)n_devices);
    for (int32_t i = 0; i < n_devices; ++i) ids[(size_t)i] = (cur + i) % count;
    return create_on(ids.data(), n_devices, out_ctx);
}

OVL_API int ovl_create_on_devices(const int32_t* devices, int32_t n_devices, ovl_ctx** out_ctx) {
    if (!out_ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "out_ctx is NULL");
    *out_ctx = nullptr;
    if (!devices || n_devices <= 0) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "empty device list");
    return create_on(devices, n_devices, out_ctx);
}

OVL_API int ovl_ctx_devices(const ovl_ctx* c, int32_t* ids, int32_t cap, int32_t* out_n) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    if (out_n) *out_n = (int32_t)c->devs.size();
    for (int32_t i = 0; ids && i < cap && i < (int32_t)c->devs.size(); ++i) ids[i] = c->devs[(size_t)i]->device;
    return OVL_OK;
}

OVL_API int ovl_destroy(ovl_ctx* c) {
    if (!c) return OVL_OK;
    DeviceGuard guard;
    for (Dev* d : c->devs) destroy_dev(d);
    if (c->stage.p) (void)hipHostFree(c->stage.p);
    delete c;
    return OVL_OK;
}

// ----------------------------------------------------------------------------- pinned host memory

OVL_API int ovl_host_alloc(int64_t bytes, void** out_ptr) {
    if (!out_ptr) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "out_ptr is NULL");
    *out_ptr = nullptr;
    if (bytes < 0) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "bytes < 0");
    // fine-grained (coherent): kernels store results into it while host code may hold cached copies of the
    // same lines (a caller reusing its arrays); the coarse-grained kind made no difference in step time
    // (profiles/r02_pack_ab_target.json)
    HIPCHK((ovl_ctx*)nullptr, hipHostMalloc(out_ptr, (size_t)std::max<int64_t>(bytes, 64), kHostShared));
    return OVL_OK;
}

OVL_API int ovl_host_free(void* ptr) {
    if (ptr) HIPCHK((ovl_ctx*)nullptr, hipHostFree(ptr));
    return OVL_OK;
}

OVL_API int ovl_host_register(void* ptr, int64_t bytes) {
    if (!ptr || bytes <= 0) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "NULL pointer or empty range");
    HIPCHK((ovl_ctx*)nullptr, hipHostRegister(ptr, (size_t)bytes, hipHostRegisterPortable));
    return OVL_OK;
}

OVL_API int ovl_host_unregister(void* ptr) {
    if (!ptr) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "NULL pointer");
    HIPCHK((ovl_ctx*)nullptr, hipHostUnregister(ptr));
    return OVL_OK;
}

OVL_API int ovl_host_pool(int32_t* threads, int32_t* sharers, int32_t* cpus, int32_t* packed) {
    CpuShare& cs = CpuShare::get();
    const int n = cs.refresh(true);
    const int t = CopyPool::threads();
    if (threads) *threads = t;
    if (sharers) *sharers = n;
    if (cpus) *cpus = cs.cpus();
    if (packed) *packed = t >= 6 ? 1 : 0;
    return OVL_OK;
}

OVL_API int32_t ovl_host_pool_rule(int32_t cpus, int32_t sharers, int32_t env_threads) {
    return pool_rule(cpus, sharers, env_threads);
}

OVL_API int ovl_set_timing(ovl_ctx* c, int32_t on) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    c->timing = on ? 1 : 0;
    return OVL_OK;
}

OVL_API int ovl_last_transfer(const ovl_ctx* c, int64_t* link_bytes, int64_t* packed_pairs) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    if (link_bytes) *link_bytes = c->x_link_bytes;
    if (packed_pairs) *packed_pairs = c->x_packed_pairs;
    return OVL_OK;
}

OVL_API int ovl_last_results(const ovl_ctx* c, int64_t* result_bytes, int64_t* record_pairs, int64_t* escapes) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    if (result_bytes) *result_bytes = c->x_res_bytes;
    if (record_pairs) *record_pairs = c->x_rec_pairs;
    if (escapes) *escapes = c->x_esc;
    return OVL_OK;
}

OVL_API int ovl_last_pair_list(const ovl_ctx* c, int64_t* in_place_pairs, int64_t* decoded_pairs) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    if (in_place_pairs) *in_place_pairs = c->x_ix_pairs;
    if (decoded_pairs) *decoded_pairs = c->x_dec_pairs;
    return OVL_OK;
}

OVL_API int ovl_last_launches(const ovl_ctx* c, int32_t cap, int32_t* device, int32_t* sink, int64_t* pairs,
                              double* ms, int32_t* out_n) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    if (cap < 0) return fail(c, OVL_E_ARG, "cap < 0");
    const int32_t n = (int32_t)c->t_launches.size();
    if (out_n) *out_n = n;
    for (int32_t i = 0; i < n && i < cap; ++i) {
        const auto& L = c->t_launches[(size_t)i];
        if (device) device[i] = L.device;
        if (sink) sink[i] = L.sink;
        if (pairs) pairs[i] = L.pairs;
        if (ms) ms[i] = L.ms;
    }
    return OVL_OK;
}

OVL_API int ovl_last_timing(const ovl_ctx* c, double* kernel_ms, double* call_ms) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    if (kernel_ms) *kernel_ms = c->t_kernel_ms;
    if (call_ms) *call_ms = c->t_call_ms;
    return OVL_OK;
}

// ----------------------------------------------------------------------------- reads

namespace {

// Offsets, lengths, the length bitmap and the longest read (split over the host pool for large read sets).
int prep_reads(ovl_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads, HostReads& h) {
    const int64_t base = n_reads > 0 ? offsets[0] : 0;
    if (base < 0) return fail(c, OVL_E_ARG, "offsets[0] < 0");
    h.n_reads = n_reads;
    h.off.resize((size_t)n_reads + 1);
    h.len.resize((size_t)std::max(n_reads, 1));
    h.off[0] = 0;
    h.len[0] = 0;
    CopyPool& pool = CopyPool::get();
    // parts of whole 32-read words (the bitmap), each with its longest read and first bad read
    const std::vector<size_t> parts = pool.cut((size_t)n_reads, size_t(1) << 14);
    std::vector<int32_t> pmax(parts.size(), 0), pbad(parts.size(), -1), ptoo(parts.size(), -1);
    pool.parallel_parts(parts, [&](size_t i, size_t lo, size_t hi) {
        int32_t m = 0;
        for (size_t r = lo; r < hi; ++r) {
            const int64_t l = offsets[r + 1] - offsets[r];
            if (l < 0 || l > INT32_MAX / 2) {
                (l < 0 ? pbad[i] : ptoo[i]) = (int32_t)r;
                return;
            }
            h.off[r + 1] = offsets[r + 1] - base;
            h.len[r] = (int32_t)l;
            m = std::max(m, (int32_t)l);
        }
        pmax[i] = m;
    });
    h.lmax = 0;
    for (size_t i = 0; i < parts.size(); ++i) {
        if (pbad[i] >= 0) return fail(c, OVL_E_ARG, "offsets not non-decreasing at read %d", pbad[i]);
        if (ptoo[i] >= 0) return fail(c, OVL_E_UNSUPPORTED, "read %d is too long", ptoo[i]);
        h.lmax = std::max(h.lmax, pmax[i]);
    }
    h.total = n_reads > 0 ? h.off[(size_t)n_reads] : 0;
    h.full.assign(((size_t)std::max(n_reads, 1) + 31) / 32, 0u);
    pool.parallel_parts(parts, [&](size_t, size_t lo, size_t hi) {
        for (size_t r = lo; r < hi; ++r)
            if (h.len[r] == h.lmax) h.full[r >> 5] |= 1u << (r & 31);  // (parts cut at multiples of 64 reads)
    });
    if (h.total > 0 && !seqs) return fail(c, OVL_E_ARG, "seqs is NULL");
    h.src = seqs ? seqs + base : nullptr;
    return OVL_OK;
}

// The pinned upload stage: offsets, lengths, bitmap and code table, and the read bytes -- 2-bit packed by the
// host pool in the same pass that scans them for the alphabet when every byte is A, C, G or T (a quarter of
// the bytes to upload, expanded by unpack2_kernel), else copied as they are.  Sets the code table and the
// bit-plane layout (dense codes in byte order, equality-preserving).
int stage_reads(ovl_ctx* c, ReadStage& st, HostReads& h) {
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    st.o_off = 0;
    st.o_len = al(st.o_off + sizeof(int64_t) * h.off.size());
    st.o_full = al(st.o_len + sizeof(int32_t) * h.len.size());
    st.o_lut = al(st.o_full + sizeof(uint32_t) * h.full.size());
    st.o_pk = al(st.o_lut + 256);
    st.o_raw = al(st.o_pk + (size_t)h.total / 4 + 64);
    const size_t need = al(st.o_raw + (size_t)h.total + 1);
    if (st.bytes < need) {
        if (st.p) (void)hipHostFree(st.p);
        st.p = nullptr;
        st.bytes = 0;
        HIPCHK(c, hipHostMalloc((void**)&st.p, need, hipHostMallocPortable));
        st.bytes = need;
    }
    bool present[256] = {false};
    h.packed2 = false;
    if (h.total > 0) {
        CopyPool& pool = CopyPool::get();
        const std::vector<size_t> parts = pool.cut((size_t)h.total, size_t(1) << 18);  // (multiples of 64)
        std::vector<std::array<uint8_t, 256>> seen(parts.size(), std::array<uint8_t, 256>{});
        std::vector<uint8_t> ok(parts.size() - 1, 0);  // (cut gives parts + 1 bounds)
        const uint8_t* src = h.src;
        uint8_t* pk = reinterpret_cast<uint8_t*>(st.p + st.o_pk);
        pool.parallel_parts(parts, [&](size_t i, size_t lo, size_t hi) {
            ok[i] = ovl_scan::scan_pack(src, lo, hi, seen[i].data(), pk);
        });
        for (const auto& t : seen)
            for (int v = 0; v < 256; ++v) present[v] = present[v] || t[(size_t)v];
        h.packed2 = std::find(ok.begin(), ok.end(), 0) == ok.end();
        if (!h.packed2) host_copy(st.p + st.o_raw, h.src, (size_t)h.total);
    }
    memset(h.lut, 0, sizeof(h.lut));
    int k = 0;
    for (int v = 0; v < 256; ++v)
        if (present[v]) h.lut[v] = (uint8_t)k++;
    h.planes = k <= 4 ? 2 : (k <= 16 ? 4 : 8);
    // bit-plane layouts: W = ceil(lmax/32) words of 32 bases, rows padded to 16 bytes
    h.wmax = 0;
    if (h.lmax <= kFastMaxLen) h.wmax = std::max(1, (h.lmax + 31) / 32);
    h.srow = h.wmax ? ((h.wmax * h.planes + 3) & ~3) : 0;
    h.trow = h.srow;
    memcpy(st.p + st.o_off, h.off.data(), sizeof(int64_t) * h.off.size());
    memcpy(st.p + st.o_len, h.len.data(), sizeof(int32_t) * h.len.size());
    memcpy(st.p + st.o_full, h.full.data(), sizeof(uint32_t) * h.full.size());
    memcpy(st.p + st.o_lut, h.lut, 256);
    h.src = reinterpret_cast<const uint8_t*>(st.p + (h.packed2 ? st.o_pk : st.o_raw));
    return OVL_OK;
}

// Asynchronous upload + pack of one device's copy from the pinned stage; the caller synchronises d->stream.
hipError_t upload_reads(Dev* d, const HostReads& h, const ReadStage& st) {
    hipError_t e = hipSetDevice(d->device);
    if (e != hipSuccess) return e;
    d->n_reads = -1;  // invalid until fully built
    d->cand_n = -1;
    d->heavy_for = -1;
    const int32_t n_reads = h.n_reads;
    // one copy of the stage's block (offsets, lengths, bitmap, code table, then the packed or raw bytes), the
    // arrays used in place as views into it
    const size_t pk_bytes = (((size_t)h.total + 63) / 64) * 16;
    const size_t blk = h.packed2 ? st.o_pk + pk_bytes : st.o_raw + (size_t)h.total;
    for (DevBuf* v : {&d->off, &d->len, &d->full, &d->lut, &d->raw}) release(*v);
    if ((e = ensure(d->rd, blk + 64)) != hipSuccess) return e;
    set_view(d->off, d->rd, st.o_off, sizeof(int64_t) * h.off.size());
    set_view(d->len, d->rd, st.o_len, sizeof(int32_t) * h.len.size());
    set_view(d->full, d->rd, st.o_full, sizeof(uint32_t) * h.full.size());
    set_view(d->lut, d->rd, st.o_lut, 256);
    set_view(d->raw, d->rd, h.packed2 ? st.o_pk : st.o_raw, h.packed2 ? pk_bytes : (size_t)h.total);
    if ((e = ensure(d->codes, (size_t)h.total + 64)) != hipSuccess) return e;  // tail pad: clamped reads
    hipStream_t s = d->stream;
    if ((e = hipMemcpyAsync(d->rd.p, st.p, blk, hipMemcpyHostToDevice, s))) return e;
    if (h.total > 0 && h.packed2) {
        if ((e = ovl_launch_unpack2(as<uint8_t>(d->raw), as<uint8_t>(d->lut), as<uint8_t>(d->codes), h.total, s)))
            return e;
    } else if (h.total > 0) {
        if ((e = ovl_launch_map_codes(as<uint8_t>(d->raw), as<uint8_t>(d->lut), as<uint8_t>(d->codes), h.total, s)))
            return e;
    }
    if (h.wmax > 0) {
        const size_t rows = (size_t)std::max(n_reads, 1);
        if ((e = ensure(d->sfx, rows * h.srow * sizeof(uint32_t)))) return e;
        if ((e = ensure(d->pfx, rows * h.trow * sizeof(uint32_t)))) return e;
        if ((e = ovl_launch_pack(h.planes, as<uint8_t>(d->codes), as<int64_t>(d->off), as<int32_t>(d->len), n_reads,
                                 h.wmax, h.srow, h.trow, as<uint32_t>(d->sfx), as<uint32_t>(d->pfx), s)))
            return e;
    }
    return hipSuccess;
}

}  // namespace

namespace {

// The caller's read set equals the resident one: the same offsets relative to offsets[0] (compared over the host
// pool, a part stops at its first difference) and the same 128-bit digest of the bytes.
bool same_reads(const ovl_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads) {
    if (!c->res_valid || (int64_t)c->res_off.size() != (int64_t)n_reads + 1) return false;
    for (const Dev* d : c->devs)
        if (d->n_reads != n_reads) return false;
    const int64_t base = n_reads > 0 ? offsets[0] : 0;
    if (n_reads > 0 && offsets[n_reads] - base != c->res_total) return false;
    CopyPool& pool = CopyPool::get();
    std::atomic<bool> differ{false};
    pool.parallel((size_t)n_reads + 1, size_t(1) << 14, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi && !differ.load(std::memory_order_relaxed); ++i)
            if (offsets[i] - base != c->res_off[i]) differ.store(true, std::memory_order_relaxed);
    });
    if (differ.load()) return false;
    if (c->res_total == 0) return true;
    if (!seqs) return false;
    uint64_t h[2];
    ovl_digest::reads_hash(seqs + base, c->res_total, h);
    return h[0] == c->res_hash[0] && h[1] == c->res_hash[1];
}

// ovl_set_reads; sync = false (ovl_score_pairs) leaves the uploads running on each device's kernel stream --
// the scoring launches queue behind them there -- and the caller synchronises those streams before it returns
// (the pinned stage must outlive the copy)
int set_reads(ovl_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads, bool sync) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(c);
    if (n_reads < 0) return fail(c, OVL_E_ARG, "n_reads < 0");
    if (n_reads > 0 && !offsets) return fail(c, OVL_E_ARG, "offsets is NULL");
    if (n_reads > 0 && offsets[0] < 0) return fail(c, OVL_E_ARG, "offsets[0] < 0");
    if (n_reads > 0 && offsets[n_reads] > offsets[0] && !seqs) return fail(c, OVL_E_ARG, "seqs is NULL");
    DeviceGuard guard;
    if (same_reads(c, seqs, offsets, n_reads)) {
        // already resident on every device: only the candidate list goes, as after an upload (and the sharer
        // count is refreshed as an upload would, when it is older than its interval)
        CpuShare::get().refresh();
        for (Dev* d : c->devs) {
            d->cand_n = -1;
            d->heavy_for = -1;
        }
        return OVL_OK;
    }
    c->res_valid = false;
    PipeTrace trace;  // OVL_TRACE_PIPE: r recount, p prepared, s staged, u uploads issued, y synchronised
    CpuShare::get().refresh();
    trace.mark('r', 0);
    HostReads& h = c->hreads;
    h.lmax = 0;
    int rc = prep_reads(c, seqs, offsets, n_reads, h);
    if (rc != OVL_OK) return rc;
    trace.mark('p', 0);
    c->h_len.clear();
    hipError_t e = hipSuccess;
    for (Dev* d : c->devs) {
        d->n_reads = -1;
        d->cand_n = -1;
        d->heavy_for = -1;
    }
    // the pinned stage (the previous upload from it is complete: every caller synchronised it), then the
    // upload to every device, then wait for all (the uploads and packs overlap across devices)
    rc = stage_reads(c, c->stage, h);
    if (rc != OVL_OK) return rc;
    trace.mark('s', 0);
    for (Dev* d : c->devs)
        if ((e = upload_reads(d, h, c->stage)) != hipSuccess) break;
    trace.mark('u', 0);
    for (Dev* d : c->devs) {
        if (!sync && e == hipSuccess) break;
        (void)hipSetDevice(d->device);
        hipError_t e2 = hipStreamSynchronize(d->stream);
        if (e == hipSuccess) e = e2;
    }
    trace.mark('y', 0);
    if (e != hipSuccess)
        return fail(c, e == hipErrorOutOfMemory ? OVL_E_OOM : OVL_E_HIP, "ovl_set_reads: %s", hipGetErrorString(e));
    for (Dev* d : c->devs) {
        d->lmax = h.lmax;
        d->codes_bytes = h.total;
        d->planes = h.planes;
        d->wmax = h.wmax;
        d->srow = h.srow;
        d->trow = h.trow;
        d->n_reads = n_reads;
    }
    c->h_len.assign(h.len.begin(), h.len.begin() + n_reads);
    // what is resident now (for same_reads)
    const int64_t base = n_reads > 0 ? offsets[0] : 0;
    c->res_off.resize((size_t)n_reads + 1);
    for (int32_t i = 0; i <= n_reads; ++i) c->res_off[(size_t)i] = n_reads > 0 ? offsets[i] - base : 0;
    // (a digest of the bytes, not a copy: the host memory a resident set costs is its offsets)
    c->res_total = h.total;
    c->res_hash[0] = c->res_hash[1] = 0;
    if (h.total > 0) ovl_digest::reads_hash(seqs + base, h.total, c->res_hash);
    c->res_valid = true;
    return OVL_OK;
}

}  // namespace

OVL_API int ovl_set_reads(ovl_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads) {
    return set_reads(c, seqs, offsets, n_reads, true);
}

OVL_API int ovl_reads_info(const ovl_ctx* c, int32_t* n_reads, int32_t* lmax, int32_t* planes, int64_t* device_bytes) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    const Dev* d = c->devs[0];
    if (n_reads) *n_reads = d->n_reads;
    if (lmax) *lmax = d->lmax;
    if (planes) *planes = d->planes;
    if (device_bytes)
        *device_bytes = (int64_t)(d->codes.bytes + d->off.bytes + d->len.bytes + d->sfx.bytes + d->pfx.bytes);
    return OVL_OK;
}

OVL_API int ovl_plan(const ovl_ctx* c, int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                     int32_t* out_kernel) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    if (!out_kernel) return fail(c, OVL_E_ARG, "out_kernel is NULL");
    Plan p;
    int rc = make_plan(c->devs[0], match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    *out_kernel = p.kernel;
    return OVL_OK;
}

// ----------------------------------------------------------------------------- scoring

OVL_API int ovl_score_device(ovl_ctx* c, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs, int32_t match,
                             int32_t mismatch, int64_t indel, int32_t band, int32_t* d_score, int32_t* d_end,
                             void* stream) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(c);
    if (n_pairs < 0) return fail(c, OVL_E_ARG, "n_pairs < 0");
    if (n_pairs > 0 && (!d_a || !d_b || !d_score || !d_end)) return fail(c, OVL_E_ARG, "NULL device pointer");
    Dev* d = c->devs[0];
    Plan p;
    int rc = make_plan(d, match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    if (n_pairs > 0 && d->n_reads == 0) return fail(c, OVL_E_INDEX, "pairs given but the read set is empty");
    DeviceGuard guard;
    HIPCHK(c, hipSetDevice(d->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = the default (null) stream
    return launch_score(d, p, d_a, d_b, n_pairs, match, mismatch, indel, d_score, d_end, s);
}

OVL_API int ovl_check_device_errors(ovl_ctx* c) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(c);
    DeviceGuard guard;
    int rc = OVL_OK;
    for (Dev* d : c->devs) {
        HIPCHK(c, hipSetDevice(d->device));
        HIPCHK(c, hipDeviceSynchronize());
        uint32_t flag = 0;
        HIPCHK(c, hipMemcpy(&flag, d->err_flag.p, sizeof(flag), hipMemcpyDeviceToHost));
        if (flag) {
            HIPCHK(c, hipMemset(d->err_flag.p, 0, sizeof(uint32_t)));
            rc = fail(c, OVL_E_INDEX, "a device scoring call saw a pair index outside [0, n_reads)");
        }
    }
    return rc;
}

OVL_API int ovl_score_host(ovl_ctx* c, const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs, int32_t match,
                           int32_t mismatch, int64_t indel, int32_t band, int32_t* out_score, int32_t* out_end) {
    if (!c) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(c);
    if (n_pairs < 0) return fail(c, OVL_E_ARG, "n_pairs < 0");
    if (n_pairs > 0 && (!a_idx || !b_idx || !out_score || !out_end))
        return fail(c, OVL_E_ARG, "NULL host pointer");
    Plan p;
    int rc = check_scoring_args(c, match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    if (n_pairs == 0) return OVL_OK;
    if (c->devs[0]->n_reads == 0) return fail(c, OVL_E_INDEX, "pairs given but the read set is empty");
    DeviceGuard guard;
    const size_t bytes = sizeof(int32_t) * (size_t)n_pairs;
    Call C;
    C.plan = &p;
    C.match = match;
    C.mismatch = mismatch;
    C.indel = indel;
    C.h_a = a_idx;
    C.h_b = b_idx;
    C.in_pinned = host_pinned(a_idx, bytes) && host_pinned(b_idx, bytes);
    C.out_s = out_score;
    C.out_e = out_end;
    C.out_pinned = host_pinned(out_score, bytes) && host_pinned(out_end, bytes);
    C.timing = c->timing != 0;
    const int32_t S = devices_used(c, n_pairs);
    C.pack = pack_ok(c, p, n_pairs, C.out_pinned, S);
    C.compact = S == 1 && c->devs[0]->k.compact && n_pairs >= kCompactMin;
    const std::vector<int64_t> cuts = host_cuts(c, a_idx, b_idx, n_pairs, S);
    std::vector<Job> jobs((size_t)S);
    for (int32_t r = 0; r < S; ++r) {
        jobs[(size_t)r].d = c->devs[(size_t)r];
        jobs[(size_t)r].lo = cuts[(size_t)r];
        jobs[(size_t)r].hi = cuts[(size_t)r + 1];
    }
    return run_pipeline(c, C, jobs);
}

OVL_API int ovl_score_pairs(ovl_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                            const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs, int32_t match,
                            int32_t mismatch, int64_t indel, int32_t band, int32_t* out_score, int32_t* out_end) {
    // the read upload runs on the devices while the host encodes the pair list's first chunk; the scoring
    // launches queue behind it on the same streams
    int rc = set_reads(c, seqs, offsets, n_reads, false);
    if (rc != OVL_OK) return rc;
    rc = ovl_score_host(c, a_idx, b_idx, n_pairs, match, mismatch, indel, band, out_score, out_end);
    DeviceGuard guard;
    for (Dev* d : c->devs) {  // (the stage outlives the copy; an upload error surfaces here if nothing else did)
        (void)hipSetDevice(d->device);
        const hipError_t e = hipStreamSynchronize(d->stream);
        if (rc == OVL_OK && e != hipSuccess)
            rc = fail(c, OVL_E_HIP, "ovl_score_pairs: read upload: %s", hipGetErrorString(e));
    }
    return rc;
}

OVL_API int ovl_align_one(ovl_ctx* ctx, int32_t a, int32_t b, int32_t match, int32_t mismatch, int64_t indel,
                          int32_t* out_score, int32_t* out_end, int8_t* traceback) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(ctx);
    Dev* c = ctx->devs[0];
    if (!out_score || !out_end) return fail(c, OVL_E_ARG, "NULL output pointer");
    if (c->n_reads < 0) return fail(c, OVL_E_STATE, "no resident reads: call ovl_set_reads first");
    if (a < 0 || a >= c->n_reads || b < 0 || b >= c->n_reads)
        return fail(c, OVL_E_INDEX, "pair (%d, %d) outside [0, %d)", a, b, c->n_reads);
    if (c->lmax > kDpMaxLen) return fail(c, OVL_E_UNSUPPORTED, "DP supports reads up to %d bases", kDpMaxLen);
    DeviceGuard guard;
    HIPCHK(c, hipSetDevice(c->device));
    // lengths from the host-visible offsets copy
    int64_t offs[2][2];
    HIPCHK(c, hipMemcpy(offs[0], as<int64_t>(c->off) + a, 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(offs[1], as<int64_t>(c->off) + b, 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
    const int64_t n = offs[0][1] - offs[0][0], m = offs[1][1] - offs[1][0];
    const size_t cells = (size_t)(n + 1) * (size_t)(m + 1);
    int32_t idx[2] = {a, b};
    HIPCHK(c, ensure(c->a, sizeof(int32_t) * 2));
    HIPCHK(c, ensure(c->score, sizeof(int32_t) * 2));
    if (traceback) {
        HIPCHK(c, ensure(c->tb, cells));
        HIPCHK(c, hipMemsetAsync(c->tb.p, 0, cells, c->stream));
    }
    HIPCHK(c, hipMemcpyAsync(c->a.p, idx, sizeof(idx), hipMemcpyHostToDevice, c->stream));
    const int64_t amax = std::max(iabs64(match), iabs64(mismatch));
    const int64_t M = std::max(amax, iabs64(indel));
    const int64_t L = std::max<int32_t>(c->lmax, 1);
    OvlDpArgs g{};
    g.codes = as<uint8_t>(c->codes);
    g.off = as<int64_t>(c->off);
    g.len = as<int32_t>(c->len);
    g.n_reads = c->n_reads;
    g.a_idx = as<int32_t>(c->a);
    g.b_idx = as<int32_t>(c->a) + 1;
    g.n_pairs = 1;
    g.mcap = (int32_t)std::max<int64_t>(m, 1);
    g.match = match;
    g.mismatch = mismatch;
    g.indel = indel;
    g.out_score = as<int32_t>(c->score);
    g.out_end = as<int32_t>(c->score) + 1;
    g.tb = traceback ? as<int8_t>(c->tb) : nullptr;
    g.err_flag = as<uint32_t>(c->err_flag);
    g.wide = !(indel > INT32_MIN && M < (int64_t(1) << 31) && (2 * L + 1) * M < (int64_t(1) << 31));
    g.band = -1;
    HIPCHK(c, ovl_launch_dp(&g, c->stream));
    int32_t res[2];
    HIPCHK(c, hipMemcpyAsync(res, c->score.p, sizeof(res), hipMemcpyDeviceToHost, c->stream));
    if (traceback) HIPCHK(c, hipMemcpyAsync(traceback, c->tb.p, cells, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *out_score = res[0];
    *out_end = res[1];
    return OVL_OK;
}

// ----------------------------------------------------------------------------- candidate enumeration

namespace {

// Keys, sort, per-read groups and their offsets; the list length comes back in d->cand_tail.
int cand_count(Dev* c, int32_t k) {
    HIPCHK(c, hipSetDevice(c->device));
    c->cand_n = -1;
    c->heavy_for = -1;
    const int32_t n = c->n_reads;
    const size_t nr = (size_t)std::max(n, 1);
    const int all = k == 0 ? 1 : 0;
    const int32_t bits = c->planes;  // symbol codes are dense: < 2^planes
    hipStream_t s = c->stream;
    HIPCHK(c, ensure(c->k_lo, nr * sizeof(int64_t)));
    HIPCHK(c, ensure(c->k_hi, nr * sizeof(int64_t)));
    HIPCHK(c, ensure(c->k_cnt, nr * sizeof(int64_t)));
    HIPCHK(c, ensure(c->k_offs, nr * sizeof(int64_t)));
    size_t temp = 0;
    HIPCHK(c, ovl_cand_temp_bytes(n, &temp));
    HIPCHK(c, ensure(c->k_temp, temp));
    if (!all) {
        HIPCHK(c, ensure(c->k_pre, nr * sizeof(uint64_t)));
        HIPCHK(c, ensure(c->k_suf, nr * sizeof(uint64_t)));
        HIPCHK(c, ensure(c->k_sorted, nr * sizeof(uint64_t)));
        HIPCHK(c, ensure(c->k_iota, nr * sizeof(int32_t)));
        HIPCHK(c, ensure(c->k_order, nr * sizeof(int32_t)));
        HIPCHK(c, ovl_cand_keys(as<uint8_t>(c->codes), as<int64_t>(c->off), as<int32_t>(c->len), n, k, bits,
                                as<uint64_t>(c->k_pre), as<uint64_t>(c->k_suf), as<int32_t>(c->k_iota), s));
        HIPCHK(c, ovl_cand_sort(c->k_temp.p, c->k_temp.bytes, as<uint64_t>(c->k_pre), as<uint64_t>(c->k_sorted),
                                as<int32_t>(c->k_iota), as<int32_t>(c->k_order), n, s));
    }
    HIPCHK(c, ovl_cand_count(as<uint64_t>(c->k_sorted), as<uint64_t>(c->k_pre), as<uint64_t>(c->k_suf), n, all,
                             as<int64_t>(c->k_lo), as<int64_t>(c->k_hi), as<int64_t>(c->k_cnt), s));
    HIPCHK(c, ovl_cand_scan(c->k_temp.p, c->k_temp.bytes, as<int64_t>(c->k_cnt), as<int64_t>(c->k_offs), n, s));
    c->cand_tail[0] = c->cand_tail[1] = 0;
    if (n > 0) {
        HIPCHK(c, hipMemcpyAsync(&c->cand_tail[0], as<int64_t>(c->k_offs) + (n - 1), sizeof(int64_t),
                                 hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(&c->cand_tail[1], as<int64_t>(c->k_cnt) + (n - 1), sizeof(int64_t),
                                 hipMemcpyDeviceToHost, s));
    }
    return OVL_OK;
}

int cand_emit(Dev* c, int32_t k) {
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t total = c->cand_tail[0] + c->cand_tail[1];
    HIPCHK(c, ensure(c->cand_a, (size_t)total * sizeof(int32_t)));
    HIPCHK(c, ensure(c->cand_b, (size_t)total * sizeof(int32_t)));
    if (total > 0)
        HIPCHK(c, ovl_cand_emit(as<int32_t>(c->k_order), as<int64_t>(c->k_lo), as<int64_t>(c->k_hi),
                                as<int64_t>(c->k_offs), c->n_reads, k == 0 ? 1 : 0, as<int32_t>(c->cand_a),
                                as<int32_t>(c->cand_b), c->stream));
    return OVL_OK;
}

}  // namespace

OVL_API int ovl_candidates(ovl_ctx* ctx, int32_t k, int64_t* out_n_pairs) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(ctx);
    if (!out_n_pairs) return fail(ctx, OVL_E_ARG, "out_n_pairs is NULL");
    if (k < 0) return fail(ctx, OVL_E_ARG, "k-mer length must be non-negative (k=%d)", k);
    Dev* d0 = ctx->devs[0];
    if (d0->n_reads < 0) return fail(ctx, OVL_E_STATE, "no resident reads: call ovl_set_reads first");
    const int32_t bits = d0->planes;
    if (k > 0 && (int64_t)k * bits > 58)
        return fail(ctx, OVL_E_UNSUPPORTED, "k=%d with %d-bit symbols does not fit a 64-bit key (k * bits <= 58)", k,
                    bits);
    DeviceGuard guard;
    CpuShare::get().refresh();
    // every device enumerates the same list from its own copy of the reads (no list broadcast); the
    // phases overlap across devices
    int rc = OVL_OK;
    for (Dev* d : ctx->devs)
        if ((rc = cand_count(d, k)) != OVL_OK) break;
    for (Dev* d : ctx->devs) {
        (void)hipSetDevice(d->device);
        hipError_t e = hipStreamSynchronize(d->stream);
        if (rc == OVL_OK && e != hipSuccess) rc = fail(ctx, OVL_E_HIP, "ovl_candidates: %s", hipGetErrorString(e));
    }
    if (rc != OVL_OK) return rc;
    for (Dev* d : ctx->devs)
        if ((rc = cand_emit(d, k)) != OVL_OK) break;
    for (Dev* d : ctx->devs) {
        (void)hipSetDevice(d->device);
        hipError_t e = hipStreamSynchronize(d->stream);
        if (rc == OVL_OK && e != hipSuccess) rc = fail(ctx, OVL_E_HIP, "ovl_candidates: %s", hipGetErrorString(e));
    }
    if (rc != OVL_OK) return rc;
    const int64_t total = d0->cand_tail[0] + d0->cand_tail[1];
    for (Dev* d : ctx->devs) {
        d->cand_n = total;
        d->heavy_for = -1;  // a new list: heavy tiles rebuilt on its first launch
    }
    *out_n_pairs = total;
    return OVL_OK;
}

OVL_API int ovl_candidates_copy(ovl_ctx* ctx, int32_t* a_idx, int32_t* b_idx) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    Dev* c = ctx->devs[0];
    if (c->cand_n < 0) return fail(c, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    if (c->cand_n == 0) return OVL_OK;
    if (!a_idx || !b_idx) return fail(c, OVL_E_ARG, "NULL host pointer");
    DeviceGuard guard;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t bytes = (size_t)c->cand_n * sizeof(int32_t);
    HIPCHK(c, hipMemcpyAsync(a_idx, c->cand_a.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(b_idx, c->cand_b.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return OVL_OK;
}

OVL_API int ovl_candidates_device(const ovl_ctx* ctx, const int32_t** d_a_idx, const int32_t** d_b_idx,
                                  int64_t* n_pairs) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    const Dev* c = ctx->devs[0];
    if (c->cand_n < 0) return fail(c, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    if (d_a_idx) *d_a_idx = reinterpret_cast<const int32_t*>(c->cand_a.p);
    if (d_b_idx) *d_b_idx = reinterpret_cast<const int32_t*>(c->cand_b.p);
    if (n_pairs) *n_pairs = c->cand_n;
    return OVL_OK;
}

OVL_API int ovl_candidates_shards(ovl_ctx* ctx, int32_t n_shards, int64_t* bounds) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(ctx);
    if (n_shards <= 0 || !bounds) return fail(ctx, OVL_E_ARG, "n_shards <= 0 or bounds is NULL");
    Dev* d = ctx->devs[0];
    if (d->cand_n < 0) return fail(ctx, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    DeviceGuard guard;
    std::vector<int64_t> cuts;
    int rc = device_cuts(d, 0, d->cand_n, n_shards, cuts);
    if (rc != OVL_OK) return rc;
    std::copy(cuts.begin(), cuts.end(), bounds);
    return OVL_OK;
}

namespace {

constexpr int kResidentFellBack = 1000;  // (resident_call: the call goes through the launch pipeline instead)

// A call over the resident candidate list that the resident grid scores: one device, the uniform kernel's form with
// int32 keys and 2-byte record codes (ends <= 254), timing off (its launch events time the launch pipeline), and a
// host pool of at least 6 threads to expand the records (fewer: several processes share the CPUs, pack_ok)
bool resident_ok(const ovl_ctx* c, const Plan& p, int64_t n) {
    if (devices_used(c, n) != 1 || c->timing || CopyPool::threads() < 6) return false;
    const Dev* d = c->devs[0];
    if (d->k.resident == 0 || d->res.broken) return false;
    if (d->k.resident == 1 && (n < d->k.resident_min || n > d->k.resident_max)) return false;
    return p.kernel == OVL_KERNEL_UNGAPPED && !p.key64 && d->planes == 2 && d->wmax >= 1 && d->wmax <= 8 &&
           d->lmax >= 1 && d->lmax <= 254 && d->cand_n >= 0;
}

int resident_call(ovl_ctx* ctx, int64_t lo, int64_t hi, int32_t match, int32_t mismatch, int32_t* out_s,
                  int32_t* out_e) {
    Dev* d = ctx->devs[0];
    HIPCHK(d, hipSetDevice(d->device));
    // heavy tiles first when the range starts on a list tile (uniform_kernel's order); built once per list, with the
    // grid stopped (ensure_heavy may reallocate)
    ResidentCall rc_;
    if (lo % 64 == 0) {
        if (d->heavy_for != d->cand_n) {
            (void)d->res.stop();
            const int r = ensure_heavy(d);
            if (r != OVL_OK) return r;
        }
        const int64_t t0 = lo / 64, t1 = t0 + (hi - lo + 63) / 64;
        const auto k0 = std::lower_bound(d->h_heavy.begin(), d->h_heavy.end(), t0);
        const auto k1 = std::lower_bound(d->h_heavy.begin(), d->h_heavy.end(), t1);
        if (k1 > k0) {
            rc_.heavy_ids = as<int32_t>(d->heavy_ids) + (k0 - d->h_heavy.begin());
            rc_.heavy_n = (int64_t)(k1 - k0);
            rc_.tile_base = t0;
        }
    }
    ResidentReads rd;
    rd.sfx = as<uint32_t>(d->sfx);
    rd.pfx = as<uint32_t>(d->pfx);
    rd.len = as<int32_t>(d->len);
    rd.n_reads = d->n_reads;
    rd.lw = d->lmax;
    rd.wmax = d->wmax;
    rd.full = as<uint32_t>(d->full);
    rd.tile_flags = rc_.heavy_n > 0 ? as<uint8_t>(d->tile_flags) : nullptr;
    rc_.d_a = as<int32_t>(d->cand_a) + lo;
    rc_.d_b = as<int32_t>(d->cand_b) + lo;
    rc_.n = hi - lo;
    rc_.match = match;
    rc_.mismatch = mismatch;
    rc_.out_s = out_s;
    rc_.out_e = out_e;
    const auto t0 = std::chrono::steady_clock::now();
    int64_t n_bad = 0;
    hipError_t e = hipSuccess;
    const int r = d->res.score(rd, rc_, &n_bad, &e);
    if (r == ResidentGrid::kFallback) return kResidentFellBack;
    if (r != ResidentGrid::kOk)
        return fail(ctx, OVL_E_HIP, "resident grid: %s", hipGetErrorString(e));
    ctx->t_launches.clear();
    ctx->t_kernel_ms = 0.0;
    ctx->t_call_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const int64_t n = hi - lo, nt = (n + 63) / 64;
    ctx->x_res_bytes = 128 * nt + 8 * d->res.last_specials;
    ctx->x_link_bytes = ctx->x_res_bytes;
    ctx->x_packed_pairs = n;
    ctx->x_rec_pairs = n;
    ctx->x_esc = d->res.last_specials;
    ctx->x_ix_pairs = ctx->x_dec_pairs = 0;
    if (n_bad > 0) return fail(ctx, OVL_E_INDEX, "a pair index is outside [0, %d)", d->n_reads);
    return OVL_OK;
}

}  // namespace

OVL_API int ovl_devices_for(const ovl_ctx* ctx, int64_t n_pairs, int32_t* out_devices) {
    if (!ctx || !out_devices) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx or out_devices is NULL");
    if (n_pairs < 0) return fail(ctx, OVL_E_ARG, "n_pairs < 0");
    *out_devices = devices_for(ctx, n_pairs);
    return OVL_OK;
}

OVL_API int ovl_quiesce(ovl_ctx* ctx) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    DeviceGuard guard;
    for (Dev* d : ctx->devs) HIPCHK(ctx, d->res.stop());
    return OVL_OK;
}

OVL_API int ovl_resident_stats(const ovl_ctx* ctx, int32_t* alive, int64_t* launches, int64_t* relaunches,
                               int32_t* broken) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    int32_t al = 0, br = 0;
    int64_t l = 0, rl = 0;
    for (const Dev* d : ctx->devs) {
        al += d->res.alive() ? 1 : 0;
        br += d->res.broken ? 1 : 0;
        l += d->res.n_launches;
        rl += d->res.n_relaunches;
    }
    if (alive) *alive = al;
    if (launches) *launches = l;
    if (relaunches) *relaunches = rl;
    if (broken) *broken = br;
    return OVL_OK;
}

OVL_API int ovl_score_candidates_range(ovl_ctx* ctx, int64_t lo, int64_t hi, int32_t match, int32_t mismatch,
                                       int64_t indel, int32_t band, int32_t* out_score, int32_t* out_end) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    Dev* d0 = ctx->devs[0];
    if (d0->cand_n < 0) return fail(ctx, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    if (lo < 0 || hi < lo || hi > d0->cand_n)
        return fail(ctx, OVL_E_ARG, "range [%lld, %lld) outside the candidate list [0, %lld)", (long long)lo,
                    (long long)hi, (long long)d0->cand_n);
    Plan p;
    int rc = check_scoring_args(ctx, match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    if (hi == lo) return OVL_OK;
    if (!out_score || !out_end) return fail(ctx, OVL_E_ARG, "NULL host pointer");
    DeviceGuard guard;
    if (resident_ok(ctx, p, hi - lo)) {
        rc = resident_call(ctx, lo, hi, match, mismatch, out_score, out_end);
        if (rc != kResidentFellBack) return rc;
    }
    quiet(ctx);
    const size_t bytes = sizeof(int32_t) * (size_t)(hi - lo);
    Call C;
    C.plan = &p;
    C.match = match;
    C.mismatch = mismatch;
    C.indel = indel;
    C.out_s = out_score;
    C.out_e = out_end;
    C.out_base = lo;
    C.out_pinned = host_pinned(out_score, bytes) && host_pinned(out_end, bytes);
    C.timing = ctx->timing != 0;
    const int32_t S = devices_used(ctx, hi - lo);
    C.pack = pack_ok(ctx, p, hi - lo, C.out_pinned, S);
    std::vector<int64_t> cuts;
    rc = device_cuts(d0, lo, hi, S, cuts);
    if (rc != OVL_OK) return rc;
    std::vector<Job> jobs((size_t)S);
    for (int32_t r = 0; r < S; ++r) {
        Job& J = jobs[(size_t)r];
        J.d = ctx->devs[(size_t)r];
        J.lo = cuts[(size_t)r];
        J.hi = cuts[(size_t)r + 1];
        J.dev_a = as<int32_t>(J.d->cand_a);
        J.dev_b = as<int32_t>(J.d->cand_b);
    }
    return run_pipeline(ctx, C, jobs);
}

OVL_API int ovl_score_candidates(ovl_ctx* ctx, int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                                 int32_t* out_score, int32_t* out_end) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    const int64_t n = ctx->devs[0]->cand_n;
    if (n < 0) return fail(ctx, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    return ovl_score_candidates_range(ctx, 0, n, match, mismatch, indel, band, out_score, out_end);
}

// ----------------------------------------------------------------------------- local alignment

OVL_API int ovl_local_align(ovl_ctx* ctx, const uint8_t* query, int32_t n, const uint8_t* ref, int32_t m,
                            int32_t match, int32_t mismatch, int64_t indel, int32_t* out_score, int32_t* out_end_i,
                            int32_t* out_end_j, int32_t* out_start_i, int32_t* out_start_j, int8_t* ops,
                            int64_t ops_cap, int64_t* out_n_ops) {
    if (!ctx) return fail((ovl_ctx*)nullptr, OVL_E_ARG, "ctx is NULL");
    quiet(ctx);
    Dev* c = ctx->devs[0];
    DeviceGuard guard;
    if (n < 0 || m < 0) return fail(c, OVL_E_ARG, "negative length");
    if ((n > 0 && !query) || (m > 0 && !ref)) return fail(c, OVL_E_ARG, "NULL sequence");
    if (!out_score || !out_end_i || !out_end_j || !out_start_i || !out_start_j || !out_n_ops)
        return fail(c, OVL_E_ARG, "NULL output pointer");
    if (ops && ops_cap < 0) return fail(c, OVL_E_ARG, "ops_cap < 0");
    // best-cell key: 24-bit score, 20-bit row and column
    const int64_t mn = std::min(n, m);
    const int64_t top = std::max<int64_t>(0, match) * mn;
    if (n > 0xFFFFF || m > 0xFFFFF || top >= (int64_t(1) << 24))
        return fail(c, OVL_E_UNSUPPORTED, "local alignment: lengths < 2^20 and match * min(n, m) < 2^24 required");
    *out_score = 0; *out_end_i = 0; *out_end_j = 0; *out_start_i = 0; *out_start_j = 0; *out_n_ops = 0;
    if (n == 0 || m == 0) return OVL_OK;
    const int64_t M = std::max(std::max(iabs64(match), iabs64(mismatch)), iabs64(indel));
    const int wide = (M >= (int64_t(1) << 30) || top + M >= (int64_t(1) << 31)) ? 1 : 0;
    const int32_t n_strips = (n + 63) / 64;
    const int64_t n_chunks = ((int64_t)m + 126) / 64;  // 64-step chunks covering tau = 0 .. m + 62
    const int64_t steps = n_chunks * 64;                // traceback pitch per strip
    const size_t tb_bytes = (size_t)n_strips * (size_t)steps * 64;
    const size_t row_bytes = (size_t)n_strips * (size_t)(steps + 64) * sizeof(uint64_t);
    if (ops && tb_bytes > (size_t(8) << 30))
        return fail(c, OVL_E_UNSUPPORTED, "local alignment traceback table would exceed 8 GiB");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    HIPCHK(c, ensure(c->l_q, (size_t)n));
    HIPCHK(c, ensure(c->l_r, (size_t)m));
    if (c->l_row.bytes < row_bytes) {
        // fresh words must not carry a live epoch: zero on (re)allocation, epochs start at 1
        HIPCHK(c, ensure(c->l_row, row_bytes));
        HIPCHK(c, hipMemsetAsync(c->l_row.p, 0, c->l_row.bytes, s));
        c->l_epoch = 0;
    }
    if (++c->l_epoch == 0) {  // 2^32 launches: start over from zeroed words
        HIPCHK(c, hipMemsetAsync(c->l_row.p, 0, c->l_row.bytes, s));
        c->l_epoch = 1;
    }
    HIPCHK(c, ensure(c->l_best, 16));
    if (ops) HIPCHK(c, ensure(c->l_tb, tb_bytes));
    HIPCHK(c, hipMemcpyAsync(c->l_q.p, query, (size_t)n, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->l_r.p, ref, (size_t)m, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemsetAsync(c->l_best.p, 0, 16, s));
    HIPCHK(c, hipMemsetAsync(c->err_flag.p, 0, sizeof(uint32_t), s));
    // strips round-robin over at most 8 one-wavefront blocks per CU: far below residency, so every
    // strip's producer is a resident wavefront (the hand-off polls would otherwise never end)
    const int32_t blocks = std::min<int32_t>(n_strips, c->cu_count * 8);
    HIPCHK(c, ovl_launch_local(as<uint8_t>(c->l_q), n, as<uint8_t>(c->l_r), m, match, mismatch, indel, wide,
                               as<uint64_t>(c->l_row), ops ? as<int8_t>(c->l_tb) : nullptr,
                               as<unsigned long long>(c->l_best), as<uint32_t>(c->err_flag), blocks, c->l_epoch, s));
    unsigned long long key = 0;
    uint32_t flag = 0;
    HIPCHK(c, hipMemcpyAsync(&key, c->l_best.p, sizeof(key), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&flag, c->err_flag.p, sizeof(flag), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (flag) {
        HIPCHK(c, hipMemset(c->err_flag.p, 0, sizeof(uint32_t)));
        return fail(c, OVL_E_HIP, "local alignment: a row hand-off timed out (flag %u)", flag);
    }
    int32_t bi = 0, bj = 0, score = 0;
    if (key) {
        score = (int32_t)(key >> 40);
        bi = (int32_t)(0xFFFFFu - (uint32_t)((key >> 20) & 0xFFFFF));
        bj = (int32_t)(0xFFFFFu - (uint32_t)(key & 0xFFFFF));
    }
    *out_score = score;
    *out_end_i = bi;
    *out_end_j = bj;
    int32_t i = bi, j = bj;
    int64_t k = 0;
    if (ops && bi > 0 && bj > 0) {
        // the walk moves up and left from (bi, bj): it reads strips 0 .. (bi-1)/64 and, in each,
        // steps j + L - 1 <= bj + 62.  Only that corner of the table comes back, as one strided copy
        // into a pinned buffer (the whole table is ~22 MB at contig x PhiX scale).
        const size_t n_st = (size_t)((bi - 1) >> 6) + 1;
        const size_t w = (size_t)(bj + 63) * 64;  // bytes of steps 0 .. bj + 62 in one strip
        const size_t need = n_st * w;
        if (c->l_tb_host_bytes < need) {
            if (c->l_tb_host) (void)hipHostFree(c->l_tb_host);
            c->l_tb_host = nullptr;
            c->l_tb_host_bytes = 0;
            HIPCHK(c, hipHostMalloc((void**)&c->l_tb_host, need, hipHostMallocDefault));
            c->l_tb_host_bytes = need;
        }
        HIPCHK(c, hipMemcpy2DAsync(c->l_tb_host, w, c->l_tb.p, (size_t)steps * 64, w, n_st, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        const int8_t* tb = c->l_tb_host;
        // aligners.py:133-153: walk while i > 0, j > 0 and dp[i][j] > 0
        while (i > 0 && j > 0) {
            const int32_t st = (i - 1) >> 6, L = (i - 1) & 63;
            const int8_t code = tb[(size_t)st * w + (size_t)(j + L - 1) * 64 + (size_t)L];
            if (!(code & 4)) break;
            const int8_t op = code & 3;
            if (op == 1) { --i; --j; }
            else if (op == 2) { --i; }
            else if (op == 3) { --j; }
            else break;
            if (k < ops_cap) ops[k] = op;
            ++k;
        }
    }
    *out_start_i = i;
    *out_start_j = j;
    *out_n_ops = k;
    if (ops && k > ops_cap) return fail(c, OVL_E_RANGE, "ops_cap %lld < walk length %lld", (long long)ops_cap,
                                        (long long)k);
    return OVL_OK;
}
