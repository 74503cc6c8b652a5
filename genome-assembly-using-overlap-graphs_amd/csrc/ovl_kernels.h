// ovl_kernels.h — launch interface between the C ABI (ovl_api.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Scoring kernels flag a pair index outside [0, n_reads): a relaxed system-scope store of 1 (idempotent,
// so no read-modify-write), because for host-array calls the flag is pinned host memory that the host
// reads after the call's synchronisation.
__device__ __forceinline__ void ovl_flag_error(uint32_t* flag) {
    __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct OvlUngappedArgs {
    const uint32_t* sfx;
    const uint32_t* pfx;
    const int32_t* len;
    int32_t n_reads;
    const int32_t* a_idx;
    const int32_t* b_idx;
    int64_t n_pairs;
    int32_t rs_log2;     // lanes per pair = 1 << rs_log2 (splits the bit shifts r)
    int32_t match;
    int32_t mismatch;
    int32_t* out_score;
    int32_t* out_end;
    uint32_t* err_flag;
    int32_t planes;      // 2, 4 or 8 bit planes per base
    int32_t wmax;        // W = 1..8 words of 32 bases (read length <= 32*W)
    int32_t key64;       // 64-bit (score, end) keys (else 32-bit folded keys)
    int32_t lw;          // dominant read length for uniform_kernel (0: general kernel only)
    const uint32_t* full; // bit r set iff len[r] == lw
    int64_t max_blocks;  // grid cap (grid-stride beyond it)
    const int32_t* heavy_ids;   // throughput mode over a resident candidate list: heavy tiles first (list tile
    const uint8_t* tile_flags;  // ids, ascending; per-list-tile flags); null: natural order
    int32_t heavy_n;            // heavy tiles of this launch: heavy_ids[0 .. heavy_n)
    int64_t tile_base;          // the launch's first pair / 64 within the list
    const uint16_t* ix_b16;  // non-null: uniform_kernel (throughput mode, int32 keys) reads a compact pair list
    const uint8_t* ix_d8;    // instead of a_idx / b_idx: b = ix_b16[p] (0xFFFF: a bad index), a = ix_base[p / 64]
    const int32_t* ix_base;  // + ix_d8[p]; the host pool encodes each chunk (ovl_api.cpp encode_chunk) and the
                             // copy engine moves it into HBM on the second stream, where the kernel reads it
    int32_t host_out;    // result sink of uniform_kernel (put_pair): 0 int32 arrays in HBM, 1 host-mapped int32
                         // arrays (non-temporal stores), 2 host-mapped packed (end, mismatches) per pair in
                         // out_score as uint16, the score of the few pairs that need it in out_end
    hipEvent_t ev_start; // non-null (timing): uniform_kernel's launch records these at the kernel's own start and
    hipEvent_t ev_stop;  // end (hipExtLaunchKernelGGL), without the dispatch wait that stream events include
};

// kernels of the band knob (ovl_launch_dp); OVL_BAND_FORM env picks one for tests
enum {
    OVL_BAND_FORM_STRIP = 0,  // dp_kernel<int32_t, true>: any length, one row per lane, masks per cell
    OVL_BAND_FORM_ROWS = 1,   // band_row_kernel: lanes on band diagonals, a row per step (<= 192 lanes)
    OVL_BAND_FORM_FAST = 2,   // dp_fast_kernel<int32_t, true>: chunked strips with band masks
    OVL_BAND_FORM_DIAG = 3,   // band_diag_kernel: lanes on band diagonals, an anti-diagonal per step
    OVL_BAND_FORM_LANE = 4,   // band_lane_kernel (a lane per pair, band diagonals in registers) or, from
                              // kBandLane2Min, band_lane2_kernel (two lanes per pair, one row apart)
    OVL_BAND_FORM_LANE1 = 5,  // band_lane_kernel at every width it has (tests, A/B)
    OVL_BAND_FORM_LANE2 = 6,  // band_lane2_kernel at every width it has (tests, A/B)
};

struct OvlDpArgs {
    const uint8_t* codes;
    const int64_t* off;
    const int32_t* len;
    int32_t n_reads;
    const int32_t* a_idx;
    const int32_t* b_idx;
    int64_t n_pairs;
    int32_t mcap;        // longest t read (LDS row capacity)
    int64_t match;
    int64_t mismatch;
    int64_t indel;
    int32_t* out_score;
    int32_t* out_end;
    int8_t* tb;          // optional traceback (single pair)
    uint32_t* err_flag;
    int32_t wide;        // int64 arithmetic (else int32, when magnitudes allow)
    int32_t band;        // < 0: full DP; >= 0: banded around the seed diagonal n - seed[pair]
    const int32_t* seed; // banded: the seed ends j* (device memory, never aliases out_*)
    int32_t band_form;   // banded: OVL_BAND_FORM_* -- the host checks each form's limits
    int32_t classic;     // full DP without traceback: use dp_kernel instead of dp_fast_kernel (tests)
};

// 2-bit packed ACGT bytes (base i at bits 2(i % 4) of byte i / 4; pk 16-byte aligned, readable up to the next
// 16-byte boundary) -> codes[i] = lut["ACGT"[code]]
extern "C" hipError_t ovl_launch_unpack2(const uint8_t* pk, const uint8_t* lut, uint8_t* codes, int64_t n,
                                         hipStream_t stream);
extern "C" hipError_t ovl_launch_map_codes(const uint8_t* raw, const uint8_t* lut, uint8_t* codes, int64_t n,
                                           hipStream_t stream);
extern "C" hipError_t ovl_launch_pack(int planes, const uint8_t* codes, const int64_t* off, const int32_t* len,
                                      int32_t n_reads, int32_t w, int32_t srow, int32_t trow, uint32_t* sfx,
                                      uint32_t* pfx, hipStream_t stream);
extern "C" hipError_t ovl_launch_ungapped(const OvlUngappedArgs* args, hipStream_t stream);
// flags[t] = 1 iff tile t of the pair list holds a pair whose read a is shorter than the dominant length
extern "C" hipError_t ovl_launch_tile_flags(const int32_t* a_idx, int64_t n_pairs, const uint32_t* full,
                                            int32_t n_reads, uint8_t* flags, hipStream_t stream);

extern "C" hipError_t ovl_launch_dp(const OvlDpArgs* args, hipStream_t stream);
// compact host pair lists (ovl_pairs.hip): dst[i] = src[i] from 2- or 4-byte elements (uint16 0xFFFF -> -1; src and
// dst 16-byte aligned), and runs: dst[starts[r] .. starts[r + 1]) = vals[r]
extern "C" hipError_t ovl_launch_widen(const void* src, int32_t width, int64_t n, int32_t* dst, hipStream_t stream);
extern "C" hipError_t ovl_launch_runs(const int32_t* vals, const int32_t* starts, int64_t n_runs, int32_t* dst,
                                      hipStream_t stream);
extern "C" int ovl_band_diag_slots(int32_t band, int32_t lcap, int32_t* nseg_out);
// lane-per-pair full DP (ovl_dp_lane.hip): colbuf holds slots x ovl_dp_lane_rcap(mcap) x 64 dwords
struct OvlLaneArgs {
    int32_t cw;                 // strip width: 16 or 32 columns
    int32_t prof;               // byte score profile (<= 4 symbols, diagonal scores in int8, indel <= 0)
    int32_t ho;                 // hand-off column: 0 int32 in HBM, 1 int16 in HBM (|G| < 2^15), 2 4-bit steps
                                // in LDS (sfx, cw 32, max(match, mismatch) - 2*indel <= 15, lmax <= 256)
    int32_t sfx;                // (prof) row symbols from the resident suffix bit planes
    const uint32_t* sfx_words;  // sfx / pfx layouts of ovl_set_reads (2 planes), srow words per read, wsfx words
    const uint32_t* pfx_words;
    int32_t srow;
    int32_t wsfx;
    uint32_t* colbuf;
    int64_t slots;              // resident wavefront slots (one hand-off column each)
    int32_t split;              // band knob: two lanes per pair (band_lane2_kernel) instead of one
    int32_t h2;                 // full DP (prof, sfx, ho 2): two pairs per lane as packed f16 cells
                                // (dp_lane_h2_kernel; the diagonal scores' f16 encodings end in a zero byte)
};
extern "C" int32_t ovl_dp_lane_rcap(int32_t lcap);
extern "C" int32_t ovl_dp_lane_waves_per_simd(int32_t cw);
extern "C" int32_t ovl_dp_lane_lds_bytes(int32_t lcap);
extern "C" int32_t ovl_dp_lane_h2_ok(int64_t match, int64_t mismatch, int64_t indel);
extern "C" int64_t ovl_dp_lane_h2_col_bytes(int64_t n_pairs, int32_t lcap);
extern "C" hipError_t ovl_launch_dp_lane(const OvlDpArgs* args, const OvlLaneArgs* lane, hipStream_t stream);
// band knob, a lane per pair (ovl_dp_lane.hip): ovl_band_lane_ok(band), <= 4 symbols, scores in int8;
// uses lane->slots, and lane->sfx (row symbols and t codes from the bit planes) with sfx/pfx_words
extern "C" int32_t ovl_band_lane_ok(int32_t band);
extern "C" hipError_t ovl_launch_band_lane(const OvlDpArgs* args, const OvlLaneArgs* lane, hipStream_t stream);

// candidate enumeration (ovl_candidates.hip)
extern "C" hipError_t ovl_cand_keys(const uint8_t* codes, const int64_t* off, const int32_t* len, int32_t n_reads,
                                    int32_t k, int32_t bits, uint64_t* pre_key, uint64_t* suf_key, int32_t* iota,
                                    hipStream_t stream);
extern "C" hipError_t ovl_cand_temp_bytes(int32_t n_reads, size_t* bytes);
extern "C" hipError_t ovl_cand_sort(void* temp, size_t temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                                    const int32_t* vals_in, int32_t* vals_out, int32_t n_reads, hipStream_t stream);
extern "C" hipError_t ovl_cand_count(const uint64_t* sorted, const uint64_t* pre_key, const uint64_t* suf_key,
                                     int32_t n_reads, int32_t all_pairs, int64_t* lo, int64_t* hi, int64_t* cnt,
                                     hipStream_t stream);
extern "C" hipError_t ovl_cand_scan(void* temp, size_t temp_bytes, const int64_t* cnt, int64_t* offs, int32_t n_reads,
                                    hipStream_t stream);
extern "C" hipError_t ovl_cand_emit(const int32_t* order, const int64_t* lo, const int64_t* hi, const int64_t* offs,
                                    int32_t n_reads, int32_t all_pairs, int32_t* out_a, int32_t* out_b,
                                    hipStream_t stream);

// local alignment (ovl_local.hip)
// rowbuf: n_strips x (64 * n_chunks + 64) words {value, epoch}, n_chunks = (m + 126) / 64; tb (nullable):
// n_strips x 64 * n_chunks x 64 bytes, [strip][tau][lane]
extern "C" hipError_t ovl_launch_local(const uint8_t* q, int32_t n, const uint8_t* r, int32_t m, int64_t match,
                                       int64_t mismatch, int64_t indel, int32_t wide, uint64_t* rowbuf, int8_t* tb,
                                       unsigned long long* best, uint32_t* err_flag, int32_t blocks, uint32_t epoch,
                                       hipStream_t stream);

// shard bounds of a pair list balanced by len[a]*len[b] + 1 (ovl_candidates.hip): ovl_shard_scan writes
// the inclusive prefix sum of the costs (n_pairs int64), ovl_shard_cut the shards + 1 cuts of [lo, hi)
extern "C" hipError_t ovl_shard_temp_bytes(int64_t n_pairs, size_t* bytes);
extern "C" hipError_t ovl_shard_scan(void* temp, size_t temp_bytes, const int32_t* a, const int32_t* b,
                                     const int32_t* len, int64_t n_pairs, int64_t* cum, hipStream_t stream);
extern "C" hipError_t ovl_shard_cut(const int64_t* cum, int64_t lo, int64_t hi, int32_t shards, int64_t* cuts,
                                    hipStream_t stream);
