// ovl_api.cpp — the C ABI of include/ovl.h on top of the gfx950 kernels.
//
// Owns: the HIP stream, the resident read store (codes + bit-plane layouts in
// HBM), scratch for host-array calls and the device error flag.  Chooses the
// kernel per call (ovl_plan): the ungapped popcount kernel whenever gaps
// provably cannot win and the read store has a bit-plane layout, else the
// int64-exact DP kernel.  Never falls back to the CPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ovl.h"
#include "ovl_kernels.h"

#define OVL_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int32_t kFastMaxLen = 256;   // bit-plane layouts up to W = 8 words of 32 bases
constexpr int32_t kDpMaxLen = 8192;    // DP kernel: LDS row of the t read
constexpr int32_t kLaneMaxLen = 1024;  // lane-per-pair DP: hand-off column buffer per wavefront slot

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

thread_local std::string g_err;

}  // namespace

struct ovl_ctx {
    int32_t device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    int32_t cu_count = 256;
    int32_t split_override = -1;  // OVL_SPLIT env: force the lane split / latency mode, tuning only
    int32_t band_form = -1;       // OVL_BAND_FORM env (lane|diag|rows|fast|strip): band knob kernel (tests)
    int32_t dp_classic = 0;       // OVL_DP_CLASSIC=1 env: full-DP scoring through dp_kernel (tests)
    int32_t dp_lane = -1;         // OVL_DP_LANE env: lane-per-pair full DP (-1 auto by list size, 0 off, 1 forced)
    int32_t lane_cw = 32;         // OVL_LANE_CW env: lane kernel strip width (16 or 32 columns)
    int64_t lane_min_pairs = 65536;  // OVL_LANE_MIN_PAIRS env: auto threshold (one tile per SIMD)
    int32_t lane_prof = 1;        // OVL_LANE_PROF=0: compare/select scores instead of the byte profile (tests)
    int32_t lane_col16 = 1;       // OVL_LANE_COL16=0: int32 hand-off column even when int16 holds (tests)
    int32_t lane_sfx = 1;         // OVL_LANE_SFX=0: row symbols by byte gathers instead of the bit planes (tests)
    int32_t blocks_per_cu = 32;   // OVL_BLOCKS_PER_CU env: ungapped grid cap (blocks of 256 per CU); 32: ~1 tile per
                                  // wavefront at the target point, the dispatcher balances the tail (measured -2.3%)
    // resident reads
    int32_t n_reads = -1;
    int32_t lmax = 0;
    int32_t planes = 2;
    int32_t wmax = 0;  // 0: no bit-plane layout (reads longer than kFastMaxLen)
    int32_t srow = 0;  // sfx row stride (words)
    int32_t trow = 0;  // pfx row stride (words)
    DevBuf codes, off, len, sfx, pfx, lut, full;  // full: bit r set iff len[r] == lmax
    // scratch
    DevBuf a, b, score, end, tb, err_flag;
    DevBuf lane_col;      // lane-per-pair DP: per-wavefront strip hand-off columns
    int64_t codes_bytes = 0;
    // device candidate enumeration (ovl_candidates): per-read keys / groups and the pair list
    DevBuf k_pre, k_suf, k_sorted, k_iota, k_order, k_lo, k_hi, k_cnt, k_offs, k_temp, cand_a, cand_b;
    int64_t cand_n = -1;  // -1: no candidate list for the resident reads
    // local alignment (ovl_local_align): query / reference bytes, carried rows, progress, traceback
    DevBuf l_q, l_r, l_row, l_tb, l_best;
    uint32_t l_epoch = 0;  // tags this launch's row hand-off words (l_row is zeroed when allocated)
    // pinned host copy of the part of the traceback table the walk can reach (grown on demand)
    int8_t* l_tb_host = nullptr;
    size_t l_tb_host_bytes = 0;
};

namespace {

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

#define HIPCHK(ctx, expr)                                                                           \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail((ctx), e_ == hipErrorOutOfMemory ? OVL_E_OOM : OVL_E_HIP, "%s: %s", #expr, \
                        hipGetErrorString(e_));                                                     \
    } while (0)

hipError_t ensure(DevBuf& b, size_t bytes) {
    if (bytes < 16) bytes = 16;
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
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
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

int make_plan_full(const ovl_ctx* c, int32_t match, int32_t mismatch, int64_t indel, Plan* out);

// band >= 0: the build's seed-and-extend knob (oracle_overlap_banded), exact
// (== the reference) whenever gaps cannot win -- the seed cell (n, j*) is
// always in the band and nothing off the ungapped diagonals can beat it -- and
// whenever the band covers every diagonal (band >= 2 * lmax).
int make_plan(const ovl_ctx* c, int32_t match, int32_t mismatch, int64_t indel, int32_t band, Plan* out) {
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

int make_plan_full(const ovl_ctx* c, int32_t match, int32_t mismatch, int64_t indel, Plan* out) {
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

int launch_score_chunk(ovl_ctx* c, const Plan& pl, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs,
                       int32_t match, int32_t mismatch, int64_t indel, int32_t* d_score, int32_t* d_end,
                       hipStream_t s);

// Lane-per-pair full DP (ovl_dp_lane.hip): one lane per pair, so it needs many pairs to fill the
// chip (below that the one-wavefront-per-pair dp_fast_kernel is faster), reads short enough for
// the per-wavefront hand-off columns, and G = dp - indel*(i+j) inside int32.
bool use_dp_lane(const ovl_ctx* c, int64_t match, int64_t mismatch, int64_t indel, int64_t n_pairs) {
    if (c->dp_lane == 0) return false;
    const int64_t L = std::max<int32_t>(c->lmax, 1);
    const int64_t M = std::max(std::max(iabs64(match), iabs64(mismatch)), iabs64(indel));
    if (L > kLaneMaxLen || (4 * L + 4) * M >= (int64_t(1) << 30) || c->codes_bytes + 64 >= (int64_t(1) << 32))
        return false;
    return c->dp_lane == 1 || n_pairs >= c->lane_min_pairs;
}

// Kernels queue pair indices as int32 (LDS side ring); split huge lists.
int launch_score(ovl_ctx* c, const Plan& pl, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs,
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

int launch_score_chunk(ovl_ctx* c, const Plan& pl, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs,
                       int32_t match, int32_t mismatch, int64_t indel, int32_t* d_score, int32_t* d_end,
                       hipStream_t s) {
    if (n_pairs == 0) return OVL_OK;
    if (pl.kernel == OVL_KERNEL_BANDED) {
        // seed j* into d_end, then the banded DP reads it and overwrites (score, end)
        Plan seed;
        seed.kernel = pl.seed_kernel;
        seed.key64 = pl.seed_key64;
        seed.wide = pl.seed_wide;
        int rc = launch_score_chunk(c, seed, d_a, d_b, n_pairs, match, mismatch, INT32_MIN, d_score, d_end, s);
        if (rc != OVL_OK) return rc;
    }
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
        int32_t rs_log2 = 0;
        const int64_t want_waves = (int64_t)c->cu_count * 4 * 4;
        while (rs_log2 < 2 && ((n_pairs << rs_log2) + 63) / 64 < want_waves) ++rs_log2;
        if (c->planes == 2) rs_log2 = ((n_pairs + 63) / 64 <= (int64_t)c->cu_count * 8) ? 1 : 0;
        if (c->split_override >= 0) rs_log2 = c->split_override;  // OVL_SPLIT tuning knob
        g.rs_log2 = rs_log2;
        // uniform-length fast path (2 bit planes): pairs of two reads of length lmax;
        // uniform_kernel scores the other pairs through its LDS side ring
        g.lw = c->planes == 2 ? c->lmax : 0;
        g.full = as<uint32_t>(c->full);
        g.match = match;
        g.mismatch = mismatch;
        g.out_score = d_score;
        g.out_end = d_end;
        g.err_flag = as<uint32_t>(c->err_flag);
        g.planes = c->planes;
        g.wmax = c->wmax;
        g.key64 = pl.key64 ? 1 : 0;
        g.max_blocks = (int64_t)c->cu_count * c->blocks_per_cu;
        HIPCHK(c, ovl_launch_ungapped(&g, s));
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
        g.err_flag = as<uint32_t>(c->err_flag);
        g.wide = pl.wide ? 1 : 0;
        g.band = pl.kernel == OVL_KERNEL_BANDED ? pl.band : -1;
        g.classic = c->dp_classic;
        if (g.band < 0 && !g.wide && !g.classic && use_dp_lane(c, match, mismatch, indel, n_pairs)) {
            OvlLaneArgs k{};
            k.cw = c->lane_cw;
            k.slots = (int64_t)c->cu_count * 4 * ovl_dp_lane_waves_per_simd(k.cw);
            const size_t col_bytes = (size_t)k.slots * ovl_dp_lane_rcap(g.mcap) * 64 * sizeof(uint32_t);
            HIPCHK(c, ensure(c->lane_col, col_bytes));
            const int64_t L = std::max<int32_t>(c->lmax, 1);
            const int64_t M = std::max(std::max(iabs64(match), iabs64(mismatch)), iabs64(indel));
            const int64_t sma = (int64_t)match - 2 * indel, smm = (int64_t)mismatch - 2 * indel;
            k.prof = c->lane_prof && c->planes == 2 && indel <= 0 && sma >= -128 && sma <= 127 && smm >= -128 &&
                     smm <= 127;
            k.col16 = c->lane_col16 && (4 * L + 4) * M < (int64_t(1) << 15);
            k.sfx = k.prof && c->lane_sfx && c->wmax > 0;
            k.sfx_words = as<uint32_t>(c->sfx);
            k.pfx_words = as<uint32_t>(c->pfx);
            k.srow = c->srow;
            k.wsfx = c->wmax;
            k.colbuf = as<uint32_t>(c->lane_col);
            HIPCHK(c, ovl_launch_dp_lane(&g, &k, s));
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
                    g.band_form = lane_ok ? OVL_BAND_FORM_LANE : (diag_ok ? OVL_BAND_FORM_DIAG : OVL_BAND_FORM_FAST);
                    break;
                default:
                    g.band_form = (lane_ok && n_pairs >= c->lane_min_pairs)
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
                HIPCHK(c, ovl_launch_band_lane(&g, &k, s));
                return OVL_OK;
            }
        }
        HIPCHK(c, ovl_launch_dp(&g, s));
    }
    return OVL_OK;
}

int check_indices(const ovl_ctx* c, const int32_t* a, const int32_t* b, int64_t n) {
    for (int64_t p = 0; p < n; ++p) {
        if (a[p] < 0 || a[p] >= c->n_reads || b[p] < 0 || b[p] >= c->n_reads)
            return fail(c, OVL_E_INDEX, "pair %lld = (%d, %d) outside [0, %d)", (long long)p, a[p], b[p],
                        c->n_reads);
    }
    return OVL_OK;
}

}  // namespace

OVL_API int ovl_version(void) { return OVL_ABI_VERSION; }

OVL_API const char* ovl_last_error(const ovl_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

OVL_API int ovl_device_count(int32_t* out_count) {
    if (!out_count) return fail(nullptr, OVL_E_ARG, "out_count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *out_count = 0;
        return fail(nullptr, OVL_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *out_count = n;
    return OVL_OK;
}

OVL_API int ovl_create(int32_t device, ovl_ctx** out_ctx) {
    if (!out_ctx) return fail(nullptr, OVL_E_ARG, "out_ctx is NULL");
    *out_ctx = nullptr;
    int n = 0;
    HIPCHK(nullptr, hipGetDeviceCount(&n));
    if (n <= 0) return fail(nullptr, OVL_E_HIP, "no HIP device visible");
    if (device < 0) HIPCHK(nullptr, hipGetDevice(&device));
    if (device >= n) return fail(nullptr, OVL_E_ARG, "device %d >= device count %d", device, n);
    HIPCHK(nullptr, hipSetDevice(device));
    ovl_ctx* c = new ovl_ctx();
    c->device = device;
    if (const char* sp = getenv("OVL_SPLIT")) {
        const int v = atoi(sp);
        if (v >= 0 && v <= 2) c->split_override = v;
    }
    if (const char* e = getenv("OVL_BAND_FORM")) {
        if (!strcmp(e, "diag")) c->band_form = OVL_BAND_FORM_DIAG;
        else if (!strcmp(e, "rows")) c->band_form = OVL_BAND_FORM_ROWS;
        else if (!strcmp(e, "fast")) c->band_form = OVL_BAND_FORM_FAST;
        else if (!strcmp(e, "strip")) c->band_form = OVL_BAND_FORM_STRIP;
        else if (!strcmp(e, "lane")) c->band_form = OVL_BAND_FORM_LANE;
    }
    if (const char* e = getenv("OVL_DP_CLASSIC")) c->dp_classic = atoi(e) ? 1 : 0;
    if (const char* e = getenv("OVL_DP_LANE")) c->dp_lane = atoi(e) ? 1 : 0;
    if (const char* e = getenv("OVL_LANE_CW")) c->lane_cw = atoi(e) == 32 ? 32 : 16;
    if (const char* e = getenv("OVL_LANE_MIN_PAIRS")) c->lane_min_pairs = atoll(e);
    if (const char* e = getenv("OVL_LANE_PROF")) c->lane_prof = atoi(e) ? 1 : 0;
    if (const char* e = getenv("OVL_LANE_COL16")) c->lane_col16 = atoi(e) ? 1 : 0;
    if (const char* e = getenv("OVL_LANE_SFX")) c->lane_sfx = atoi(e) ? 1 : 0;
    if (const char* e = getenv("OVL_BLOCKS_PER_CU")) {
        const int v = atoi(e);
        if (v >= 1 && v <= 1024) c->blocks_per_cu = v;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->cu_count = prop.multiProcessorCount;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = ensure(c->err_flag, 16);
    if (e == hipSuccess) e = hipMemset(c->err_flag.p, 0, 16);
    if (e != hipSuccess) {
        int rc = fail(nullptr, OVL_E_HIP, "context setup: %s", hipGetErrorString(e));
        ovl_destroy(c);
        return rc;
    }
    *out_ctx = c;
    return OVL_OK;
}

OVL_API int ovl_destroy(ovl_ctx* c) {
    if (!c) return OVL_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (DevBuf* b : {&c->codes, &c->off, &c->len, &c->sfx, &c->pfx, &c->lut, &c->full, &c->a, &c->b, &c->score, &c->end,
                      &c->tb, &c->err_flag, &c->k_pre, &c->k_suf, &c->k_sorted, &c->k_iota, &c->k_order, &c->k_lo,
                      &c->k_hi, &c->k_cnt, &c->k_offs, &c->k_temp, &c->cand_a, &c->cand_b, &c->l_q, &c->l_r, &c->l_row,
                      &c->l_tb, &c->l_best, &c->lane_col})
        release(*b);
    if (c->l_tb_host) (void)hipHostFree(c->l_tb_host);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return OVL_OK;
}

OVL_API int ovl_set_reads(ovl_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (n_reads < 0) return fail(c, OVL_E_ARG, "n_reads < 0");
    if (n_reads > 0 && !offsets) return fail(c, OVL_E_ARG, "offsets is NULL");
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t base = n_reads > 0 ? offsets[0] : 0;
    if (base < 0) return fail(c, OVL_E_ARG, "offsets[0] < 0");
    std::vector<int64_t> off((size_t)n_reads + 1, 0);
    std::vector<int32_t> len((size_t)std::max(n_reads, 1), 0);
    int32_t lmax = 0;
    for (int32_t r = 0; r < n_reads; ++r) {
        const int64_t l = offsets[r + 1] - offsets[r];
        if (l < 0) return fail(c, OVL_E_ARG, "offsets not non-decreasing at read %d", r);
        if (l > INT32_MAX / 2) return fail(c, OVL_E_UNSUPPORTED, "read %d is too long", r);
        off[r + 1] = offsets[r + 1] - base;
        len[r] = (int32_t)l;
        lmax = std::max(lmax, (int32_t)l);
    }
    const int64_t total = n_reads > 0 ? off[n_reads] : 0;
    std::vector<uint32_t> full(((size_t)std::max(n_reads, 1) + 31) / 32, 0u);
    for (int32_t r = 0; r < n_reads; ++r)
        if (len[r] == lmax) full[(size_t)r >> 5] |= 1u << (r & 31);
    if (total > 0 && !seqs) return fail(c, OVL_E_ARG, "seqs is NULL");
    // alphabet: dense codes in byte order (equality-preserving)
    bool present[256] = {false};
    const uint8_t* src = seqs ? seqs + base : nullptr;
    for (int64_t i = 0; i < total; ++i) present[src[i]] = true;
    uint8_t lut[256] = {0};
    int k = 0;
    for (int v = 0; v < 256; ++v)
        if (present[v]) lut[v] = (uint8_t)k++;
    const int planes = k <= 4 ? 2 : (k <= 16 ? 4 : 8);
    // bit-plane layouts: W = ceil(lmax/32) words of 32 bases, rows padded to 16 bytes
    int32_t wmax = 0;
    if (lmax <= kFastMaxLen) wmax = std::max(1, (lmax + 31) / 32);
    const int32_t srow = wmax ? ((wmax * planes + 3) & ~3) : 0;
    const int32_t trow = wmax ? ((wmax * planes + 3) & ~3) : 0;

    c->n_reads = -1;  // invalid until fully built
    c->cand_n = -1;
    DevBuf raw;
    HIPCHK(c, ensure(c->off, sizeof(int64_t) * off.size()));
    HIPCHK(c, ensure(c->len, sizeof(int32_t) * len.size()));
    HIPCHK(c, ensure(c->codes, (size_t)total + 64));  // tail pad: clamped reads of empty last reads
    HIPCHK(c, ensure(c->lut, 256));
    hipError_t e = ensure(raw, (size_t)total);
    if (e != hipSuccess) return fail(c, OVL_E_OOM, "raw read buffer: %s", hipGetErrorString(e));
    int rc = OVL_OK;
    do {
        e = hipMemcpyAsync(c->off.p, off.data(), sizeof(int64_t) * off.size(), hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) break;
        e = hipMemcpyAsync(c->len.p, len.data(), sizeof(int32_t) * len.size(), hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) break;
        e = hipMemcpyAsync(c->lut.p, lut, 256, hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) break;
        e = ensure(c->full, sizeof(uint32_t) * full.size());
        if (e != hipSuccess) break;
        e = hipMemcpyAsync(c->full.p, full.data(), sizeof(uint32_t) * full.size(), hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) break;
        if (total > 0) {
            e = hipMemcpyAsync(raw.p, src, (size_t)total, hipMemcpyHostToDevice, c->stream);
            if (e != hipSuccess) break;
            e = ovl_launch_map_codes(as<uint8_t>(raw), as<uint8_t>(c->lut), as<uint8_t>(c->codes), total, c->stream);
            if (e != hipSuccess) break;
        }
        if (wmax > 0) {
            const size_t rows = (size_t)std::max(n_reads, 1);
            e = ensure(c->sfx, rows * srow * sizeof(uint32_t));
            if (e != hipSuccess) break;
            e = ensure(c->pfx, rows * trow * sizeof(uint32_t));
            if (e != hipSuccess) break;
            e = hipMemsetAsync(c->sfx.p, 0, rows * srow * sizeof(uint32_t), c->stream);
            if (e != hipSuccess) break;
            e = hipMemsetAsync(c->pfx.p, 0, rows * trow * sizeof(uint32_t), c->stream);
            if (e != hipSuccess) break;
            e = ovl_launch_pack(planes, as<uint8_t>(c->codes), as<int64_t>(c->off), as<int32_t>(c->len), n_reads,
                                wmax, srow, trow, as<uint32_t>(c->sfx), as<uint32_t>(c->pfx), c->stream);
            if (e != hipSuccess) break;
        }
        e = hipStreamSynchronize(c->stream);
    } while (false);
    release(raw);
    if (e != hipSuccess)
        return fail(c, e == hipErrorOutOfMemory ? OVL_E_OOM : OVL_E_HIP, "ovl_set_reads: %s", hipGetErrorString(e));
    c->lmax = lmax;
    c->codes_bytes = total;
    c->planes = planes;
    c->wmax = wmax;
    c->srow = srow;
    c->trow = trow;
    c->n_reads = n_reads;
    return rc;
}

OVL_API int ovl_reads_info(const ovl_ctx* c, int32_t* n_reads, int32_t* lmax, int32_t* planes, int64_t* device_bytes) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (n_reads) *n_reads = c->n_reads;
    if (lmax) *lmax = c->lmax;
    if (planes) *planes = c->planes;
    if (device_bytes)
        *device_bytes = (int64_t)(c->codes.bytes + c->off.bytes + c->len.bytes + c->sfx.bytes + c->pfx.bytes);
    return OVL_OK;
}

OVL_API int ovl_plan(const ovl_ctx* c, int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                     int32_t* out_kernel) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (!out_kernel) return fail(c, OVL_E_ARG, "out_kernel is NULL");
    Plan p;
    int rc = make_plan(c, match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    *out_kernel = p.kernel;
    return OVL_OK;
}

OVL_API int ovl_score_device(ovl_ctx* c, const int32_t* d_a, const int32_t* d_b, int64_t n_pairs, int32_t match,
                             int32_t mismatch, int64_t indel, int32_t band, int32_t* d_score, int32_t* d_end,
                             void* stream) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (n_pairs < 0) return fail(c, OVL_E_ARG, "n_pairs < 0");
    if (n_pairs > 0 && (!d_a || !d_b || !d_score || !d_end)) return fail(c, OVL_E_ARG, "NULL device pointer");
    Plan p;
    int rc = make_plan(c, match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    if (n_pairs > 0 && c->n_reads == 0) return fail(c, OVL_E_INDEX, "pairs given but the read set is empty");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = the default (null) stream
    return launch_score(c, p, d_a, d_b, n_pairs, match, mismatch, indel, d_score, d_end, s);
}

OVL_API int ovl_check_device_errors(ovl_ctx* c) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    uint32_t flag = 0;
    HIPCHK(c, hipMemcpy(&flag, c->err_flag.p, sizeof(flag), hipMemcpyDeviceToHost));
    if (flag) {
        HIPCHK(c, hipMemset(c->err_flag.p, 0, sizeof(uint32_t)));
        return fail(c, OVL_E_INDEX, "a device scoring call saw a pair index outside [0, n_reads)");
    }
    return OVL_OK;
}

OVL_API int ovl_score_host(ovl_ctx* c, const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs, int32_t match,
                           int32_t mismatch, int64_t indel, int32_t band, int32_t* out_score, int32_t* out_end) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (n_pairs < 0) return fail(c, OVL_E_ARG, "n_pairs < 0");
    if (n_pairs > 0 && (!a_idx || !b_idx || !out_score || !out_end)) return fail(c, OVL_E_ARG, "NULL host pointer");
    Plan p;
    int rc = make_plan(c, match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    if (n_pairs == 0) return OVL_OK;
    rc = check_indices(c, a_idx, b_idx, n_pairs);
    if (rc != OVL_OK) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t bytes = sizeof(int32_t) * (size_t)n_pairs;
    HIPCHK(c, ensure(c->a, bytes));
    HIPCHK(c, ensure(c->b, bytes));
    HIPCHK(c, ensure(c->score, bytes));
    HIPCHK(c, ensure(c->end, bytes));
    HIPCHK(c, hipMemcpyAsync(c->a.p, a_idx, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->b.p, b_idx, bytes, hipMemcpyHostToDevice, c->stream));
    rc = launch_score(c, p, as<int32_t>(c->a), as<int32_t>(c->b), n_pairs, match, mismatch, indel,
                      as<int32_t>(c->score), as<int32_t>(c->end), c->stream);
    if (rc != OVL_OK) return rc;
    HIPCHK(c, hipMemcpyAsync(out_score, c->score.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out_end, c->end.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return OVL_OK;
}

OVL_API int ovl_score_pairs(ovl_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                            const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs, int32_t match,
                            int32_t mismatch, int64_t indel, int32_t band, int32_t* out_score, int32_t* out_end) {
    int rc = ovl_set_reads(c, seqs, offsets, n_reads);
    if (rc != OVL_OK) return rc;
    return ovl_score_host(c, a_idx, b_idx, n_pairs, match, mismatch, indel, band, out_score, out_end);
}

OVL_API int ovl_align_one(ovl_ctx* c, int32_t a, int32_t b, int32_t match, int32_t mismatch, int64_t indel,
                          int32_t* out_score, int32_t* out_end, int8_t* traceback) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (!out_score || !out_end) return fail(c, OVL_E_ARG, "NULL output pointer");
    if (c->n_reads < 0) return fail(c, OVL_E_STATE, "no resident reads: call ovl_set_reads first");
    if (a < 0 || a >= c->n_reads || b < 0 || b >= c->n_reads)
        return fail(c, OVL_E_INDEX, "pair (%d, %d) outside [0, %d)", a, b, c->n_reads);
    if (c->lmax > kDpMaxLen) return fail(c, OVL_E_UNSUPPORTED, "DP supports reads up to %d bases", kDpMaxLen);
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

OVL_API int ovl_candidates(ovl_ctx* c, int32_t k, int64_t* out_n_pairs) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (!out_n_pairs) return fail(c, OVL_E_ARG, "out_n_pairs is NULL");
    if (k < 0) return fail(c, OVL_E_ARG, "k-mer length must be non-negative (k=%d)", k);
    if (c->n_reads < 0) return fail(c, OVL_E_STATE, "no resident reads: call ovl_set_reads first");
    const int32_t bits = c->planes;  // symbol codes are dense: < 2^planes
    if (k > 0 && (int64_t)k * bits > 58)
        return fail(c, OVL_E_UNSUPPORTED, "k=%d with %d-bit symbols does not fit a 64-bit key (k * bits <= 58)", k,
                    bits);
    HIPCHK(c, hipSetDevice(c->device));
    c->cand_n = -1;
    const int32_t n = c->n_reads;
    const size_t nr = (size_t)std::max(n, 1);
    const int all = k == 0 ? 1 : 0;
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
    int64_t tail[2] = {0, 0};
    if (n > 0) {
        HIPCHK(c, hipMemcpyAsync(&tail[0], as<int64_t>(c->k_offs) + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(&tail[1], as<int64_t>(c->k_cnt) + (n - 1), sizeof(int64_t), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, hipStreamSynchronize(s));
    const int64_t total = tail[0] + tail[1];
    HIPCHK(c, ensure(c->cand_a, (size_t)total * sizeof(int32_t)));
    HIPCHK(c, ensure(c->cand_b, (size_t)total * sizeof(int32_t)));
    if (total > 0)
        HIPCHK(c, ovl_cand_emit(as<int32_t>(c->k_order), as<int64_t>(c->k_lo), as<int64_t>(c->k_hi),
                                as<int64_t>(c->k_offs), n, all, as<int32_t>(c->cand_a), as<int32_t>(c->cand_b), s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->cand_n = total;
    *out_n_pairs = total;
    return OVL_OK;
}

OVL_API int ovl_candidates_copy(ovl_ctx* c, int32_t* a_idx, int32_t* b_idx) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (c->cand_n < 0) return fail(c, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    if (c->cand_n == 0) return OVL_OK;
    if (!a_idx || !b_idx) return fail(c, OVL_E_ARG, "NULL host pointer");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t bytes = (size_t)c->cand_n * sizeof(int32_t);
    HIPCHK(c, hipMemcpyAsync(a_idx, c->cand_a.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(b_idx, c->cand_b.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return OVL_OK;
}

OVL_API int ovl_candidates_device(const ovl_ctx* c, const int32_t** d_a_idx, const int32_t** d_b_idx,
                                  int64_t* n_pairs) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (c->cand_n < 0) return fail(c, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    if (d_a_idx) *d_a_idx = reinterpret_cast<const int32_t*>(c->cand_a.p);
    if (d_b_idx) *d_b_idx = reinterpret_cast<const int32_t*>(c->cand_b.p);
    if (n_pairs) *n_pairs = c->cand_n;
    return OVL_OK;
}

OVL_API int ovl_score_candidates(ovl_ctx* c, int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                                 int32_t* out_score, int32_t* out_end) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
    if (c->cand_n < 0) return fail(c, OVL_E_STATE, "no candidate list: call ovl_candidates first");
    Plan p;
    int rc = make_plan(c, match, mismatch, indel, band, &p);
    if (rc != OVL_OK) return rc;
    const int64_t n = c->cand_n;
    if (n == 0) return OVL_OK;
    if (!out_score || !out_end) return fail(c, OVL_E_ARG, "NULL host pointer");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t bytes = sizeof(int32_t) * (size_t)n;
    HIPCHK(c, ensure(c->score, bytes));
    HIPCHK(c, ensure(c->end, bytes));
    rc = launch_score(c, p, as<int32_t>(c->cand_a), as<int32_t>(c->cand_b), n, match, mismatch, indel,
                      as<int32_t>(c->score), as<int32_t>(c->end), c->stream);
    if (rc != OVL_OK) return rc;
    HIPCHK(c, hipMemcpyAsync(out_score, c->score.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(out_end, c->end.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return OVL_OK;
}

// ----------------------------------------------------------------------------- local alignment

OVL_API int ovl_local_align(ovl_ctx* c, const uint8_t* query, int32_t n, const uint8_t* ref, int32_t m,
                            int32_t match, int32_t mismatch, int64_t indel, int32_t* out_score, int32_t* out_end_i,
                            int32_t* out_end_j, int32_t* out_start_i, int32_t* out_start_j, int8_t* ops,
                            int64_t ops_cap, int64_t* out_n_ops) {
    if (!c) return fail(nullptr, OVL_E_ARG, "ctx is NULL");
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
