// ovl_dp_lane.hip — lane-per-pair full DP for gapped scoring (scores only), gfx950.
//
// aligners.py:27-57 for a finite indel: the full (n+1) x (m+1) table with
// dp[i][j] = max(dp[i-1][j-1] + s(i,j), dp[i-1][j] + indel, dp[i][j-1] + indel),
// row 0 and column 0 zero, then the last row's first strict-'>' argmax.
//
// One lane owns one candidate pair (64 consecutive pairs per wavefront), so no
// cell waits on another lane and no lane idles on the table's corners (the
// anti-diagonal kernels do both).  The lane sweeps vertical strips of CW columns:
// the strip's current row sits in CW registers and the rows advance top to
// bottom; the strip's last column is handed to the next strip through a per-wave
// global column buffer ([row][lane], coalesced), the only memory traffic besides
// the read codes.
//
// Potential: G[i][j] = dp[i][j] - indel * (i + j).  Then
//   G[i][j] = max3(G[i-1][j-1] + s(i,j) - 2*indel, G[i-1][j], G[i][j-1])
// so a cell is compare, select, add, max3 -- no indel adds on the gap moves.
// Values are exact in int32 when the host's bound holds (|values| + |indel|*(n+m)
// < 2^30; otherwise the int64 anti-diagonal kernel runs).
//
// Rows are aligned at the END: lane row i = it - sk + 1 with sk = nmax - n (plus a
// pad making the row count a multiple of the 4-row body), so every lane reaches its
// row n on the last iteration and the row-n scan happens once per strip from
// registers.  Iterations with i <= 0 are "virtual": masked to the row-0 boundary
// (dp = 0), only in the leading iterations where some lane has them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "ovl_kernels.h"

namespace ovl {
namespace {

constexpr int32_t kLaneLdsMaxLen = 256;  // HO 2: 32 KiB of hand-off words per block, 4 blocks per CU

__device__ __forceinline__ int32_t wave_max(int32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ int32_t wave_min(int32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return __builtin_amdgcn_readfirstlane(v);
}

// band kernels, four rows at a time: bits b0..b3 of v4 into bit 0 of bytes 0..3 (the products' terms land on
// distinct bits, so no carries)
__device__ __forceinline__ uint32_t spread4(uint32_t v4) { return (v4 * 0x00204081u) & 0x01010101u; }

// rows r0..r0+3 of a 32-row block of two bit planes as bytes (codes 0..3)
__device__ __forceinline__ uint32_t codes4(uint32_t p0, uint32_t p1, uint32_t r0) {
    return spread4(__builtin_amdgcn_ubfe(p0, r0, 4)) | (spread4(__builtin_amdgcn_ubfe(p1, r0, 4)) << 1);
}

// the bytes k of c4 with u0 + k < 0 (t positions left of the read) replaced by the pad code 4
__device__ __forceinline__ uint32_t pad4(uint32_t c4, int32_t u0) {
    const int32_t np = min(max(-u0, 0), 4);
    const uint32_t mask = np >= 4 ? 0xFFFFFFFFu : ((1u << (8 * np)) - 1u);
    return (c4 & ~mask) | (0x04040404u & mask);
}

}  // namespace

// codes: dense symbol codes (ovl_set_reads), off/len per read.  colbuf: rcap dwords per lane for each
// resident wavefront slot ([row][lane], or [row pair][lane] with COL16), rcap >= lmax rounded to 32.
//   PROF   <= 4 symbols, diagonal scores within int8, indel <= 0: byte score profile + SDWA adds
//          (2 VALU per cell); virtual rows select an all-zero profile, which reproduces row 0
//          exactly (row 0 rises by -indel per column, so neither the diagonal nor the left move
//          can exceed it), so no cell needs a mask
//   HO     hand-off column: 0 = int32 in HBM; 1 = int16 in HBM, two rows per dword (|G| < 2^15);
//          2 = 4-bit row differences in LDS, eight rows per dword.  The column's steps
//          G[i][j] - G[i-1][j] lie in [0, max(match, mismatch) - 2*indel] (up move: >= 0; by
//          induction over j the diagonal and left moves stay below it), so when that is <= 15 a
//          lane's 256-row column is 128 bytes and a wavefront's fits LDS beside 15 others: no
//          hand-off traffic leaves the CU
//   SFX    (PROF) the row symbols come from the resident bit-plane rows (sfx, right-aligned):
//          with the row count a multiple of 32, row iteration `it` reads bit it % 32 of word
//          it / 32 + W - R / 32 on every lane, so a lane loads 8 bytes per 32 rows instead of
//          a byte gather per row
template <int CW, int OCC, bool PROF, int HO, bool SFX>
__global__ __launch_bounds__(256, OCC) void dp_lane_kernel(const uint8_t* __restrict__ codes,
                                                           const int64_t* __restrict__ off,
                                                           const int32_t* __restrict__ len, int32_t n_reads,
                                                           const uint32_t* __restrict__ sfx, int32_t srow,
                                                           int32_t wsfx, const int32_t* __restrict__ a_idx,
                                                           const int32_t* __restrict__ b_idx, int64_t n_pairs,
                                                           int32_t lcap, int32_t rcap, int32_t match,
                                                           int32_t mismatch, int32_t indel,
                                                           uint32_t* __restrict__ colbuf,
                                                           int32_t* __restrict__ out_score,
                                                           int32_t* __restrict__ out_end,
                                                           uint32_t* __restrict__ err_flag) {
    static_assert(!SFX || PROF, "bit-plane row symbols need the byte profile");
    static_assert(HO != 2 || SFX, "the LDS hand-off works on 8-row words (row count a multiple of 32)");
    constexpr bool COL16 = HO == 1;
    constexpr bool LH = HO == 2;
    const int lane = threadIdx.x & 63;
    extern __shared__ uint32_t lds_hand[];  // LH: [row / 8][wavefront in block][lane]
    uint32_t* __restrict__ hcol = lds_hand + (threadIdx.x >> 6) * 64 + lane;
    const int64_t wslot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nslots = (int64_t)gridDim.x * 4;
    uint32_t* __restrict__ col = colbuf + wslot * (int64_t)rcap * 64 + lane;
    const int64_t ntiles = (n_pairs + 63) >> 6;
    const int32_t g = indel;
    const int32_t s_ma = match - 2 * g;     // diagonal move, match, in G units
    const int32_t s_mm = mismatch - 2 * g;  // diagonal move, mismatch
    for (int64_t tile = wslot; tile < ntiles; tile += nslots) {
        const int64_t p = tile * 64 + lane;
        const bool live = p < n_pairs;
        int32_t a = live ? a_idx[p] : 0;
        int32_t b = live ? b_idx[p] : 0;
        bool bad = live && (a < 0 || a >= n_reads || b < 0 || b >= n_reads);
        if (!live || bad) { a = 0; b = 0; }
        int32_t n = (live && !bad) ? len[a] : 0;
        int32_t m = (live && !bad) ? len[b] : 0;
        if (n > lcap || m > lcap) { bad = true; n = 0; m = 0; }
        const uint32_t sa = (uint32_t)off[a];
        const uint32_t tb = (uint32_t)off[b];
        const int32_t nmax = wave_max(n);
        const int32_t nmin = wave_min(n);
        const int32_t mmax = wave_max(m);
        constexpr int RQ = SFX ? 32 : 4;
        const int32_t R = (nmax + RQ - 1) / RQ * RQ;  // row iterations (end-aligned rows)
        const int32_t sk = R - n;                      // this lane's virtual rows
        const int32_t mcut = R - nmin;                 // iterations in which some lane is virtual
        const uint32_t* __restrict__ srow_p = sfx + (int64_t)a * srow + 2 * (wsfx - R / 32);
        int32_t best = 0, bend = 0;                    // dp[n][0] = 0 is the j = 0 candidate

        // one strip of CW columns j0+1 .. j0+CW; FIRST: the left boundary is column 0 (no loads)
        auto strip = [&](int32_t j0, auto first_tag) {
            constexpr bool FIRST = decltype(first_tag)::value;
            uint32_t tc[CW];
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                // columns past m compute unread values: any symbol will do
                const int32_t jc = j0 + c < m ? j0 + c : 0;
                tc[c] = (uint32_t)codes[tb + (uint32_t)jc];
            }
            // PROF: a row's profile word w holds s(x, t[j0 + 4w + k]) in byte k (x = the row's symbol); a
            // cell adds its byte with a sign-extending SDWA add
            constexpr int PW = PROF ? CW / 4 : 1;
#ifdef OVL_LANE_MUX  // A/B reference: four byte profiles per strip, three bit muxes per word per row
            uint32_t PX[4][PW];
            if constexpr (PROF) {
#pragma unroll
                for (int x = 0; x < 4; ++x) {
#pragma unroll
                    for (int w = 0; w < PW; ++w) {
                        uint32_t word = 0;
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            word |= ((uint32_t)(tc[4 * w + k] == (uint32_t)x ? s_ma : s_mm) & 0xFFu) << (8 * k);
                        PX[x][w] = word;
                    }
                }
            }
#else
            // the strip's t codes as bytes (TW[w] byte k = t[j0 + 4w + k], codes 0..3); a row's profile
            // word is one v_perm_b32 of its 4-byte score table by these codes
            uint32_t TW[PW];
            if constexpr (PROF) {
#pragma unroll
                for (int w = 0; w < PW; ++w)
                    TW[w] = tc[4 * w] | (tc[4 * w + 1] << 8) | (tc[4 * w + 2] << 16) | (tc[4 * w + 3] << 24);
            }
            const uint32_t tbl_base = ((uint32_t)s_mm & 0xFFu) * 0x01010101u;   // every t mismatches
            const uint32_t tbl_diff = ((uint32_t)(s_ma ^ s_mm)) & 0xFFu;        // byte x -> match score
#endif
            int32_t A[CW], B[CW];
#pragma unroll
            for (int c = 0; c < CW; ++c) A[c] = -g * (j0 + 1 + c);  // row 0: G[0][j] = -indel * j
            int32_t prevL = -g * j0;                                 // G[i-1][j0] entering row 1

            // queue for rows it .. it+3: s codes (byte path) and the raw hand-off words
            constexpr int NCW = COL16 ? 2 : 4;
            constexpr int NQS = SFX ? 1 : 4;
            uint32_t qs[NQS], qc[NCW];
            // LH: the hand-off words of rows it..it+7 (read) and the next 8 (prefetched), the word being
            // written, and the running values the 4-bit steps start from: the left column's value of the
            // row before `it` and this strip's last column in that row (row 0's values carry through the
            // virtual rows, whose steps are 0)
            uint32_t hr = 0, hn = 0, hw = 0;
            int32_t lprev = -g * j0, vprev = -g * (j0 + CW);
            uint32_t S0 = 0, S1 = 0, S0n = 0, S1n = 0;  // SFX: bit planes of the current / next 32 rows
            auto fetch4 = [&](int32_t it4) {
                if constexpr (!SFX) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int32_t i0 = it4 + k - sk;  // s index i - 1
                        const int32_t ic = i0 < 0 ? 0 : (i0 >= n ? (n > 0 ? n - 1 : 0) : i0);
                        qs[k] = (uint32_t)codes[sa + (uint32_t)ic];
                    }
                }
                if constexpr (!FIRST && !LH) {
#pragma unroll
                    for (int k = 0; k < NCW; ++k) qc[k] = col[(int64_t)((COL16 ? it4 / 2 : it4) + k) * 64];
                }
            };
            auto fetch_planes = [&](int32_t kb) {
                const uint2 v = *reinterpret_cast<const uint2*>(srow_p + 2 * kb);
                S0n = v.x;
                S1n = v.y;
            };
            auto left = [&](int32_t it, const uint32_t(&cw)[NCW], int k) -> int32_t {
                if constexpr (FIRST) return -g * (it - sk + 1);  // G[i][0] = -indel * i
                else if constexpr (COL16) return (int32_t)(int16_t)(uint16_t)(cw[k >> 1] >> (16 * (k & 1)));
                else return (int32_t)cw[k];
            };
            // one row: O (row i-1) -> N (row i); returns N[CW-1], the hand-off value
            auto row = [&](int32_t it, int32_t(&O)[CW], int32_t(&N)[CW], uint32_t sc, int32_t lb,
                           auto masked_tag) -> int32_t {
                constexpr bool MASKED = decltype(masked_tag)::value;
                const bool virt = it < sk;
                int32_t d = prevL;
                int32_t l = lb;
                uint32_t P[PW];
                if constexpr (PROF) {
                    uint32_t m0, m1;  // bit 0 / bit 1 of the row symbol, as all-ones / all-zero masks
                    if constexpr (SFX) {
                        const uint32_t r = (uint32_t)it & 31u;
                        m0 = (uint32_t)__builtin_amdgcn_sbfe((int32_t)S0, r, 1);
                        m1 = (uint32_t)__builtin_amdgcn_sbfe((int32_t)S1, r, 1);
                    } else {
                        m0 = (uint32_t)(((int32_t)(sc << 31)) >> 31);
                        m1 = (uint32_t)(((int32_t)(sc << 30)) >> 31);
                    }
                    const uint32_t nv = (uint32_t)~((it - sk) >> 31);  // 0 on virtual rows
#ifdef OVL_LANE_MUX
#pragma unroll
                    for (int w = 0; w < PW; ++w) {
                        const uint32_t lo = __builtin_amdgcn_bitop3_b32(m0, PX[1][w], PX[0][w], 0xCA);  // m0 ? : mux
                        const uint32_t hi = __builtin_amdgcn_bitop3_b32(m0, PX[3][w], PX[2][w], 0xCA);
                        P[w] = __builtin_amdgcn_bitop3_b32(m1, hi, lo, 0xCA);
                        if constexpr (MASKED) P[w] &= nv;  // zero profile: the row repeats row 0
                    }
#else
                    // row symbol x = bit0 | bit1 << 1; its table: byte t = s(x, t) in G units
                    const uint32_t x8 = (m0 & 8u) | (m1 & 16u);          // 8 * x
                    uint32_t tbl = tbl_base ^ (tbl_diff << x8);
                    if constexpr (MASKED) tbl &= nv;                       // zero profile: the row repeats row 0
#pragma unroll
                    for (int w = 0; w < PW; ++w) P[w] = __builtin_amdgcn_perm(tbl, tbl, TW[w]);
#endif
                }
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    int32_t s2;
                    if constexpr (PROF) s2 = (int32_t)(int8_t)(uint8_t)(P[c >> 2] >> (8 * (c & 3)));
                    else s2 = sc == tc[c] ? s_ma : s_mm;
                    int32_t v = max(max(d + s2, O[c]), l);
                    if constexpr (MASKED && !PROF) v = virt ? __builtin_amdgcn_readfirstlane(-g * (j0 + 1 + c)) : v;
                    N[c] = v;
                    d = O[c];
                    l = v;
                }
                prevL = lb;
                return N[CW - 1];
            };
            auto body = [&](int32_t it, auto masked_tag) {
                // rows it .. it+3 (A -> B -> A -> B -> A); the queue refills 4 rows ahead
                uint32_t s4[NQS], c4[NCW];
#pragma unroll
                for (int k = 0; k < NQS; ++k) s4[k] = qs[k];
#pragma unroll
                for (int k = 0; k < NCW; ++k) c4[k] = qc[k];
                if constexpr (SFX) {
                    if ((it & 31) == 0) {  // next 32 rows: rotate the plane words, prefetch the block after
                        S0 = S0n;
                        S1 = S1n;
                        if (it + 32 < R) fetch_planes((it + 32) >> 5);
                    }
                }
                if (it + 4 < R) fetch4(it + 4);
                if constexpr (LH) {
                    const uint32_t sh = (uint32_t)(it & 4) * 4u;  // this body's half of the 8-row word
                    if constexpr (!FIRST) {
                        if ((it & 4) == 0) {
                            hr = hn;
                            if (it + 8 < R) hn = hcol[(int64_t)(it / 8 + 1) * 256];
                        }
                    }
                    int32_t lf[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if constexpr (FIRST) {
                            lf[k] = -g * (it + k - sk + 1);
                        } else {
                            lprev += (int32_t)__builtin_amdgcn_ubfe(hr, sh + 4u * k, 4u);
                            lf[k] = lprev;
                        }
                    }
                    const int32_t v0 = row(it, A, B, s4[0], lf[0], masked_tag);
                    const int32_t v1 = row(it + 1, B, A, s4[0], lf[1], masked_tag);
                    const int32_t v2 = row(it + 2, A, B, s4[0], lf[2], masked_tag);
                    const int32_t v3 = row(it + 3, B, A, s4[0], lf[3], masked_tag);
                    // steps of this strip's last column (also after the last strip: never read, no branch)
                    uint32_t h = (uint32_t)(v0 - vprev);
                    h |= (uint32_t)(v1 - v0) << 4;
                    h |= (uint32_t)(v2 - v1) << 8;
                    h |= (uint32_t)(v3 - v2) << 12;
                    vprev = v3;
                    if ((it & 4) == 0) {
                        hw = h;
                    } else {
                        hcol[(int64_t)(it / 8) * 256] = hw | (h << 16);
                    }
                    return;
                }
                const int32_t v0 = row(it, A, B, s4[0], left(it, c4, 0), masked_tag);
                const int32_t v1 = row(it + 1, B, A, s4[SFX ? 0 : 1], left(it + 1, c4, 1), masked_tag);
                const int32_t v2 = row(it + 2, A, B, s4[SFX ? 0 : 2], left(it + 2, c4, 2), masked_tag);
                const int32_t v3 = row(it + 3, B, A, s4[SFX ? 0 : 3], left(it + 3, c4, 3), masked_tag);
                // hand-off column for the next strip (also after the last strip: never read, no branch)
                if constexpr (COL16) {
                    col[(int64_t)(it / 2) * 64] = ((uint32_t)v0 & 0xFFFFu) | ((uint32_t)v1 << 16);
                    col[(int64_t)(it / 2 + 1) * 64] = ((uint32_t)v2 & 0xFFFFu) | ((uint32_t)v3 << 16);
                } else {
                    col[(int64_t)it * 64] = (uint32_t)v0;
                    col[(int64_t)(it + 1) * 64] = (uint32_t)v1;
                    col[(int64_t)(it + 2) * 64] = (uint32_t)v2;
                    col[(int64_t)(it + 3) * 64] = (uint32_t)v3;
                }
            };
            if constexpr (SFX) fetch_planes(0);
            fetch4(0);
            if constexpr (LH && !FIRST) hn = hcol[0];
            int32_t it = 0;
            for (; it < mcut; it += 4) body(it, std::true_type{});
            for (; it < R; it += 4) body(it, std::false_type{});
            // A holds row n of every lane: the strip's part of the last-row scan (strict '>', j ascending)
            const int32_t base = g * (n + j0 + 1);  // dp = G + indel * (n + j)
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const int32_t v = A[c] + base + g * c;
                const bool better = (j0 + 1 + c <= m) && v > best;
                best = better ? v : best;
                bend = better ? j0 + 1 + c : bend;
            }
        };
        if (mmax > 0) strip(0, std::true_type{});
        // the next strip reads this strip's hand-off column (same lane, program order)
        for (int32_t j0 = CW; j0 < mmax; j0 += CW) strip(j0, std::false_type{});
        if (live) {
            if (bad) {
                ovl_flag_error(err_flag);
                out_score[p] = -1;
                out_end[p] = -1;
            } else {
                out_score[p] = best;
                out_end[p] = bend;
            }
        }
    }
}

// ----------------------------------------------------------------------------- full DP, two pairs per lane
//
// dp_lane_kernel's recurrence (PROF, SFX, HO 2) with a lane holding two pairs -- p and p + 64 of a 128-pair
// tile -- as the low and high halves of packed f16 cells, so one v_pk_add_f16 and one v_pk_maximum3_f16
// advance two cells, and one v_perm_b32 makes both cells' scores: byte 1 of the selector picks the row
// symbol's score for t_p (from the pair's 4-byte row table), byte 3 the other pair's, bytes 0 and 2 select
// zero -- the diagonal scores' f16 encodings have a zero low byte (the host checks).  1.5 VALU per cell
// against 2.25.
//
// Exactness: f16 holds integers to 2048.  A strip's values are kept relative to a per-pair offset: it starts
// at row 0's value in column j0, and every 32 rows the previous row's left-column value (the row's minimum:
// G rises along rows and columns) moves into the offset.  Between two moves a cell lies within 32 row steps
// of the left column and 32 column steps of the moved value, each step in [0, smax], smax = max(match,
// mismatch) - 2*indel <= 15 (HO 2's bound), so every value and diagonal sum stays below 65*smax + 128
// (the host checks < 2048).  Virtual rows keep column 0 at 0 (any value <= row 0's works there).
//
// The hand-off column: 4-bit steps of both pairs, a dword per four rows (pair p in bits 0-15, p + 64 in bits
// 16-31), in HBM per tile ([tile][row / 4][lane], read two quads ahead; the next strip reads it soon after, from
// the caches).  In LDS (the OVL_H2_LDS build) its 16 KiB per wavefront capped residency at 2.5 wavefronts per
// SIMD: 13.0 ms against 11.1 for cfg5's full DP.  A step's f16 value plus 1024 has the step in its low mantissa
// bits, which is how steps move between f16 cells and nibbles in both directions.
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

namespace {
__device__ __forceinline__ half2_t as_h2(uint32_t v) { return __builtin_bit_cast(half2_t, v); }
__device__ __forceinline__ uint32_t h2_bits(half2_t v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ half2_t h2_splat(int32_t v) {
    const _Float16 h = (_Float16)(float)v;
    return half2_t{h, h};
}
__device__ __forceinline__ half2_t hmax3(half2_t a, half2_t b, half2_t c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
}  // namespace

constexpr uint32_t kH2Bias4 = 0x64006400u + (0x64006400u << 4) + (0x64006400u << 8) + (0x64006400u << 12);

template <int OCC>
__global__ __launch_bounds__(128, OCC) void dp_lane_h2_kernel(const int32_t* __restrict__ len, int32_t n_reads,
                                                              const uint32_t* __restrict__ sfx,
                                                              const uint32_t* __restrict__ pfx, int32_t srow,
                                                              int32_t wsfx, const int32_t* __restrict__ a_idx,
                                                              const int32_t* __restrict__ b_idx, int64_t n_pairs,
                                                              int32_t lcap, int32_t match, int32_t mismatch,
                                                              int32_t indel, int32_t* __restrict__ out_score,
                                                              int32_t* __restrict__ out_end,
                                                              uint32_t* __restrict__ err_flag,
                                                              uint32_t* __restrict__ colbuf, int32_t hq) {
    constexpr int CW = 32;
    const int lane = threadIdx.x & 63;
#ifndef OVL_H2_LDS  // the hand-off column per tile in HBM ([tile][row quad][lane], hq quads); A/B: LDS
    constexpr int HS = 64;
#else
    constexpr int HS = 128;  // hand-off dwords per row quad: [wavefront in block][lane]
    extern __shared__ uint32_t lds_hand[];
    uint32_t* __restrict__ hcol = lds_hand + (threadIdx.x >> 6) * 64 + lane;
    (void)colbuf;
    (void)hq;
#endif
    const int64_t wslot = (int64_t)blockIdx.x * 2 + (threadIdx.x >> 6);
    const int64_t nslots = (int64_t)gridDim.x * 2;
    const int64_t ntiles = (n_pairs + 127) >> 7;
    const int32_t g = indel;
    // the row tables' bytes: the high byte of the diagonal score's f16 (match / mismatch, in G units)
    const uint32_t hi_ma = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(float)(match - 2 * g)) >> 8;
    const uint32_t hi_mm = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(float)(mismatch - 2 * g)) >> 8;
    const uint32_t tbl_base = hi_mm * 0x01010101u;  // every t mismatches
    const uint32_t tbl_diff = hi_ma ^ hi_mm;         // byte x -> match
    const half2_t h1024 = h2_splat(1024);
    for (int64_t tile = wslot; tile < ntiles; tile += nslots) {
#ifndef OVL_H2_LDS
        uint32_t* __restrict__ hcol = colbuf + tile * (int64_t)hq * 64 + lane;
#endif
        int64_t p[2];
        bool live[2], bad[2];
        int32_t n[2], m[2], sk[2], best[2], bend[2];
        const uint32_t* __restrict__ srow_p[2];
        const uint32_t* __restrict__ tcol_p[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            p[h] = tile * 128 + h * 64 + lane;
            live[h] = p[h] < n_pairs;
            int32_t a = live[h] ? a_idx[p[h]] : 0;
            int32_t b = live[h] ? b_idx[p[h]] : 0;
            bad[h] = live[h] && (a < 0 || a >= n_reads || b < 0 || b >= n_reads);
            if (!live[h] || bad[h]) { a = 0; b = 0; }
            n[h] = (live[h] && !bad[h]) ? len[a] : 0;
            m[h] = (live[h] && !bad[h]) ? len[b] : 0;
            if (n[h] > lcap || m[h] > lcap) { bad[h] = true; n[h] = 0; m[h] = 0; }
            srow_p[h] = sfx + (int64_t)a * srow;
            tcol_p[h] = pfx + (int64_t)b * srow;  // (left-aligned: word pair q holds columns 32q + 1 .. 32q + 32)
            best[h] = 0;  // dp[n][0] = 0 is the j = 0 candidate
            bend[h] = 0;
        }
        const int32_t nmax = wave_max(max(n[0], n[1]));
        const int32_t nmin = wave_min(min(n[0], n[1]));
        const int32_t mmax = wave_max(max(m[0], m[1]));
        const int32_t R = (nmax + 31) / 32 * 32;  // row iterations (end-aligned rows)
        const int32_t mcut = R - nmin;            // iterations in which some pair is virtual
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            sk[h] = R - n[h];
            srow_p[h] += 2 * (wsfx - R / 32);
        }

        auto strip = [&](int32_t j0, auto first_tag) {
            constexpr bool FIRST = decltype(first_tag)::value;
            // selectors: byte 1 = t code of pair p (row table in src1), byte 3 = 4 + t code of pair p + 64
            // (columns past m compute unread values: any code will do)
            uint32_t SEL[CW];
            {
                const uint2 w0 = *reinterpret_cast<const uint2*>(tcol_p[0] + 2 * (j0 >> 5));
                const uint2 w1 = *reinterpret_cast<const uint2*>(tcol_p[1] + 2 * (j0 >> 5));
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const uint32_t t0 = ((w0.x >> c) & 1u) | (((w0.y >> c) & 1u) << 1);
                    const uint32_t t1 = ((w1.x >> c) & 1u) | (((w1.y >> c) & 1u) << 1);
                    SEL[c] = 0x040C000Cu | (t0 << 8) | (t1 << 24);
                }
            }
            half2_t A[CW];
#pragma unroll
            for (int c = 0; c < CW; ++c) A[c] = h2_splat(-g * (1 + c));  // row 0, relative to G[0][j0]
            int32_t offs[2] = {-g * j0, -g * j0};                          // G = cell + offs (per pair)
            half2_t prevL = h2_splat(0);                                   // G[i-1][j0], relative
            half2_t lprev = prevL;                                         // the left column's running value
            half2_t vprev = h2_splat(-g * CW);                             // this strip's last column, row before
            uint32_t hr = 0, hn = 0, hn2 = 0;
            uint32_t S[2][2], Sn[2][2];  // bit planes of the current / next 32 rows, per pair
            auto fetch_planes = [&](int32_t kb) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint2 v = *reinterpret_cast<const uint2*>(srow_p[h] + 2 * kb);
                    Sn[h][0] = v.x;
                    Sn[h][1] = v.y;
                }
            };
            // rows it .. it+3, skewed: step s advances row k at column s - k, so the four rows' cells of a
            // step are independent (row k reads row k-1's column c one step after it was written, in place)
            auto body = [&](int32_t it, auto masked_tag) {
                constexpr bool MASKED = decltype(masked_tag)::value;
                if ((it & 31) == 0) {
                    // next 32 rows: rotate the plane words, prefetch the block after; move the previous
                    // row's left value (its minimum) into the offsets
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        S[h][0] = Sn[h][0];
                        S[h][1] = Sn[h][1];
                    }
                    if (it + 32 < R) fetch_planes((it + 32) >> 5);
                    const half2_t C = prevL;
                    offs[0] += (int32_t)(float)C.x;
                    offs[1] += (int32_t)(float)C.y;
#pragma unroll
                    for (int c = 0; c < CW; ++c) A[c] -= C;
                    prevL -= C;
                    lprev -= C;
                    vprev -= C;
                }
                if constexpr (!FIRST) {
#ifndef OVL_H2_LDS  // two quads ahead
                    hr = hn;
                    hn = hn2;
                    if (it + 8 < R) hn2 = hcol[(int64_t)(it / 4 + 2) * HS];
#else
                    hr = hn;
                    if (it + 4 < R) hn = hcol[(int64_t)(it / 4 + 1) * HS];
#endif
                }
                half2_t d[4], l[4];
                uint32_t t0[4], t1[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    half2_t step;
                    if constexpr (FIRST) {
                        // column 0: -indel per real row, 0 on virtual rows
                        if constexpr (MASKED) {
                            const _Float16 s0 = (_Float16)(float)(it + k >= sk[0] ? -g : 0);
                            const _Float16 s1 = (_Float16)(float)(it + k >= sk[1] ? -g : 0);
                            step = half2_t{s0, s1};
                        } else {
                            step = h2_splat(-g);
                        }
                    } else {
                        step = as_h2(((hr >> (4 * k)) & 0x000F000Fu) | 0x64006400u) - h1024;
                    }
                    d[k] = k ? lprev : prevL;  // G[i-1][j0]
                    lprev += step;
                    l[k] = lprev;              // G[i][j0]
                    // the row's tables (byte t = the f16 high byte of s(x, t) - 2*indel; virtual rows: zero)
                    const uint32_t r = (uint32_t)(it + k) & 31u;
                    uint32_t tbl[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int32_t)S[h][0], r, 1);
                        const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int32_t)S[h][1], r, 1);
                        const uint32_t x8 = (m0 & 8u) | (m1 & 16u);  // 8 * the row symbol
                        tbl[h] = tbl_base ^ (tbl_diff << x8);
                        if constexpr (MASKED) tbl[h] &= (uint32_t)~((it + k - sk[h]) >> 31);
                    }
                    t0[k] = tbl[0];
                    t1[k] = tbl[1];
                }
                prevL = lprev;
#pragma unroll
                for (int st = 0; st < CW + 3; ++st) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int c = st - k;
                        if (c < 0 || c >= CW) continue;
                        const half2_t s2 = as_h2(__builtin_amdgcn_perm(t1[k], t0[k], SEL[c]));
                        const half2_t u = A[c];
                        A[c] = hmax3(d[k] + s2, u, l[k]);
                        d[k] = u;
                        l[k] = A[c];
                    }
                }
                // this strip's last column as steps (also after the last strip: never read, no branch)
                uint32_t hw = h2_bits((l[0] - vprev) + h1024);
                hw += h2_bits((l[1] - l[0]) + h1024) << 4;
                hw += h2_bits((l[2] - l[1]) + h1024) << 8;
                hw += h2_bits((l[3] - l[2]) + h1024) << 12;
                vprev = l[3];
                hcol[(int64_t)(it / 4) * HS] = hw - kH2Bias4;
            };
            fetch_planes(0);
            if constexpr (!FIRST) {
                hn = hcol[0];
                hn2 = hcol[HS];  // (R >= 32: quad 1 exists)
            }
            int32_t it = 0;
            for (; it < mcut; it += 4) body(it, std::true_type{});
            for (; it < R; it += 4) body(it, std::false_type{});
            // A holds row n of both pairs: the strip's part of the last-row scan (strict '>', j ascending)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int32_t base = offs[h] + g * (n[h] + j0 + 1);  // dp = G + indel * (n + j)
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const int32_t v = (int32_t)(float)(h ? A[c].y : A[c].x) + base + g * c;
                    const bool better = (j0 + 1 + c <= m[h]) && v > best[h];
                    best[h] = better ? v : best[h];
                    bend[h] = better ? j0 + 1 + c : bend[h];
                }
            }
        };
        if (mmax > 0) strip(0, std::true_type{});
        // the next strip reads this strip's hand-off column (same lane, program order)
        for (int32_t j0 = CW; j0 < mmax; j0 += CW) strip(j0, std::false_type{});
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (live[h]) {
                if (bad[h]) {
                    ovl_flag_error(err_flag);
                    out_score[p[h]] = -1;
                    out_end[p[h]] = -1;
                } else {
                    out_score[p[h]] = best[h];
                    out_end[p[h]] = bend[h];
                }
            }
        }
    }
}

// ----------------------------------------------------------------------------- band knob, lane per pair
//
// The build's seed-and-extend band (oracle_overlap_banded; not a reference mode): cells with
// |(i - j) - d*| <= W, d* = n - j*, j* the ungapped seed end already in out_end.  One lane owns a
// pair; its NB = 2W+1 band cells of the current row sit in registers indexed by diagonal
// k = j - i + d* + W, so a row needs no data from other lanes:
//   V[k] <- max3(V[k] + s2(i, k), V[k+1], V[k-1])          (in place, k ascending)
// diag is the same diagonal of the previous row, up is diagonal k+1 of the previous row (absent at
// k = 2W) and left is diagonal k-1 of this row (absent at k = 0) -- exactly the band edges of the
// oracle -- in G = dp - indel*(i+j) units (s2 = s - 2*indel).
//
// Scores: the t codes of the row's window sit as bytes in NBW words (byte k = t[j_k - 1]) and slide
// down one byte per row; the row's profile is P = perm(TBL_x, T) -- byte t of the row's 8-byte table:
// bytes 0..3 mismatch with the match at byte x (built once per row: tbl_mm ^ (tbl_dm << 8x)), byte 4 the
// pad code of positions left of t (s2 = -2*indel, i.e. s = 0, which keeps dp = 0 for every j <= 0 cell:
// column 0 and the band cells left of it).  (Round 4 took the per-word x ^ t out of the cell loop.)
// Virtual leading rows (end-aligned rows, i <= 0) use s2 = -indel, which maps row 0's G pattern
// (-indel * j, diagonals shifting one column per row) onto itself, edge cells included.
//
// PL: row symbols and the t codes entering the window come from the resident bit planes (sfx / pfx,
// W words of 32 bases, two planes per word) instead of a byte gather per row each: with the row count
// a multiple of 32 every lane reads bit it % 32 of its current 32-row words, 8 + 16 bytes per lane
// per 32 rows (the t words funnel-shifted once per block by the lane's window offset).
template <int NB, int OCC, bool PL>
__global__ __launch_bounds__(256, OCC) void band_lane_kernel(const uint8_t* __restrict__ codes,
                                                             const int64_t* __restrict__ off,
                                                             const int32_t* __restrict__ len, int32_t n_reads,
                                                             const uint32_t* __restrict__ sfx,
                                                             const uint32_t* __restrict__ pfx, int32_t prow,
                                                             int32_t wpl, const int32_t* __restrict__ a_idx,
                                                             const int32_t* __restrict__ b_idx, int64_t n_pairs,
                                                             int32_t lcap, int32_t match, int32_t mismatch,
                                                             int32_t indel, int32_t* __restrict__ out_score,
                                                             int32_t* __restrict__ out_end,
                                                             const int32_t* __restrict__ seed,
                                                             uint32_t* __restrict__ err_flag) {
    constexpr int W = (NB - 1) / 2;
    constexpr int NBW = (NB + 3) / 4;
    constexpr uint32_t PAD = 4;  // t code left of the read
    const int lane = threadIdx.x & 63;
    const int64_t wslot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nslots = (int64_t)gridDim.x * 4;
    const int64_t ntiles = (n_pairs + 63) >> 6;
    const int32_t g = indel;
    const uint32_t b_ma = (uint32_t)(match - 2 * g) & 0xFFu;
    const uint32_t b_mm = (uint32_t)(mismatch - 2 * g) & 0xFFu;
    const uint32_t b_pad = (uint32_t)(-2 * g) & 0xFFu;
    const uint32_t tbl_mm = b_mm * 0x01010101u;  // the row table's bytes t = 0..3 before byte x takes the match
    const uint32_t tbl_dm = b_ma ^ b_mm;
    const uint32_t tbl_hi = b_pad * 0x01010101u;  // bytes 4..7: the pad code
    const uint32_t p_virt = ((uint32_t)(-g) & 0xFFu) * 0x01010101u;
    for (int64_t tile = wslot; tile < ntiles; tile += nslots) {
        const int64_t p = tile * 64 + lane;
        const bool live = p < n_pairs;
        int32_t a = live ? a_idx[p] : 0;
        int32_t b = live ? b_idx[p] : 0;
        bool bad = live && (a < 0 || a >= n_reads || b < 0 || b >= n_reads);
        if (!live || bad) { a = 0; b = 0; }
        int32_t n = (live && !bad) ? len[a] : 0;
        int32_t m = (live && !bad) ? len[b] : 0;
        int32_t jstar = (live && !bad) ? seed[p] : 0;
        if (n > lcap || m > lcap || jstar < 0 || jstar > m) { bad = bad || live; n = 0; m = 0; jstar = 0; }
        const uint32_t sa = (uint32_t)off[a];
        const uint32_t tb = (uint32_t)off[b];
        const int32_t cc = n - jstar + W;  // j = i - cc + k
        const int32_t nmax = wave_max(n);
        const int32_t nmin = wave_min(n);
        constexpr int RQ = PL ? 32 : 4;
        const int32_t R = (nmax + RQ - 1) / RQ * RQ;  // row iterations (end-aligned rows)
        const int32_t sk = R - n;
        const int32_t mcut = R - nmin;
        // t code of 0-based position u (the cell column is u + 1)
        auto tcode = [&](int32_t u) -> uint32_t {
            const int32_t uc = u < 0 ? 0 : (u >= m ? (m > 0 ? m - 1 : 0) : u);
            const uint32_t v = (uint32_t)codes[tb + (uint32_t)uc];
            return u < 0 ? PAD : v;
        };
        // row i = it - sk + 1; its window holds t positions u = i - cc - 1 + k
        const int32_t u0 = -sk - cc;
        uint32_t T[NBW];
#pragma unroll
        for (int w = 0; w < NBW; ++w) {
            uint32_t word = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * w + q < NB) word |= tcode(u0 + 4 * w + q) << (8 * q);
            T[w] = word;
        }
        int32_t V[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) V[k] = -g * (u0 + k);  // row -sk (row 0 pattern): G = -indel * j
        // prefetch queues: s codes of rows it..it+3 and the t codes entering the window after each row
        // (the code entering after row it is at t position it + ub)
        const int32_t ub = NB - sk - cc;
        constexpr int NQ = PL ? 1 : 4;
        uint32_t qs[NQ], qt[NQ];
        auto fetch4 = [&](int32_t it4) {
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const int32_t i0 = it4 + k - sk;  // s index i - 1
                const int32_t ic = i0 < 0 ? 0 : (i0 >= n ? (n > 0 ? n - 1 : 0) : i0);
                qs[k] = (uint32_t)codes[sa + (uint32_t)ic];
                qt[k] = tcode(it4 + k + ub);  // top cell of row it4 + k + 1
            }
        };
        // PL: s planes of the 32-row block (sfx, right-aligned: block kb is word kb + wpl - R/32) and the
        // t planes of the positions entering in that block, funnel-shifted to bit 0 (pfx, left-aligned)
        const uint32_t* __restrict__ sp = sfx + (int64_t)a * prow + 2 * (wpl - R / 32);
        const uint32_t* __restrict__ tp = pfx + (int64_t)b * prow;
        const uint32_t tsh = (uint32_t)ub & 31u;
        uint32_t S0 = 0, S1 = 0, T0 = 0, T1 = 0;      // current block
        uint2 sn = make_uint2(0, 0), t0n = sn, t1n = sn;  // next block (raw words)
        auto fetch_planes = [&](int32_t kb) {
            sn = *reinterpret_cast<const uint2*>(sp + 2 * kb);
            const int32_t q = (32 * kb + ub) >> 5;  // floor
            const int32_t q0 = q < 0 ? 0 : (q >= wpl ? wpl - 1 : q);
            const int32_t q1 = q + 1 < 0 ? 0 : (q + 1 >= wpl ? wpl - 1 : q + 1);
            t0n = *reinterpret_cast<const uint2*>(tp + 2 * q0);
            t1n = *reinterpret_cast<const uint2*>(tp + 2 * q1);
        };
        // x8 = 8 * the row symbol, tnew = the t code entering after the row (both from body's four-row words)
        auto row = [&](int32_t it, uint32_t x8, uint32_t tnew, auto masked_tag) {
            constexpr bool MASKED = decltype(masked_tag)::value;
            // the row's 8-byte table (byte t = s2(x, t); virtual rows: s2 = -indel everywhere), built once per
            // row, so a profile word is one perm of it by the window word
            uint32_t tlo = tbl_mm ^ (tbl_dm << x8), thi = tbl_hi;
            if constexpr (MASKED) {
                const bool virt = it < sk;
                tlo = virt ? p_virt : tlo;
                thi = virt ? p_virt : thi;
            }
            // the profile word of cells 4w..4w+3, built just before its cells (one live word, not NBW: band 64
            // keeps 129 cells and 33 window words in registers)
            uint32_t P = 0;
#pragma unroll
            for (int k = 0; k < NB; ++k) {
                if ((k & 3) == 0) P = __builtin_amdgcn_perm(thi, tlo, T[k >> 2]);
                const int32_t d = V[k] + (int32_t)(int8_t)(uint8_t)(P >> (8 * (k & 3)));
                if constexpr (NB == 1) V[k] = d;
                else if (k == 0) V[k] = max(d, V[k + 1]);
                else if (k == NB - 1) V[k] = max(d, V[k - 1]);
                else V[k] = max(max(d, V[k + 1]), V[k - 1]);
            }
            // slide the window one position and append the next row's top t code
#pragma unroll
            for (int w = 0; w < NBW; ++w) T[w] = __builtin_amdgcn_alignbit(w + 1 < NBW ? T[w + 1] : 0u, T[w], 8);
            T[(NB - 1) >> 2] |= tnew << (8 * ((NB - 1) & 3));
        };
        // rows it..it+3: their symbols (times 8, the table shift) and entering t codes as the bytes of one word
        // each, extracted once per four rows
        auto body = [&](int32_t it, auto masked_tag) {
            uint32_t xs8, ts;
            if constexpr (PL) {
                if ((it & 31) == 0) {  // next 32 rows: rotate the block words, prefetch the block after
                    S0 = sn.x;
                    S1 = sn.y;
                    T0 = __builtin_amdgcn_alignbit(t1n.x, t0n.x, tsh);
                    T1 = __builtin_amdgcn_alignbit(t1n.y, t0n.y, tsh);
                    if (it + 32 < R) fetch_planes((it + 32) >> 5);
                }
                const uint32_t r0 = (uint32_t)it & 31u;
                xs8 = codes4(S0, S1, r0) << 3;
                ts = pad4(codes4(T0, T1, r0), it + ub);
            } else {
                xs8 = (qs[0] | (qs[1] << 8) | (qs[2] << 16) | (qs[3] << 24)) << 3;
                ts = qt[0] | (qt[1] << 8) | (qt[2] << 16) | (qt[3] << 24);
                if (it + 4 < R) fetch4(it + 4);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                row(it + k, __builtin_amdgcn_ubfe(xs8, 8 * k, 8), __builtin_amdgcn_ubfe(ts, 8 * k, 8), masked_tag);
        };
        if constexpr (PL) fetch_planes(0);
        else fetch4(0);
        int32_t it = 0;
        for (; it < mcut; it += 4) body(it, std::true_type{});
#ifndef OVL_BAND_UNROLL1  // eight rows per trip, as in band_lane2_kernel
        if (it < R && ((R - it) & 7)) {
            body(it, std::false_type{});
            it += 4;
        }
        for (; it < R; it += 8) {
            body(it, std::false_type{});
            body(it + 4, std::false_type{});
        }
#else
        for (; it < R; it += 4) body(it, std::false_type{});
#endif
        // row n: in-band cells with 0 <= j <= m, largest value, first j (the oracle's scan)
        int32_t best = INT32_MIN, bend = -1;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int32_t j = jstar - W + k;
            const int32_t v = V[k] + g * (n + j);
            const bool better = j >= 0 && j <= m && v > best;
            best = better ? v : best;
            bend = better ? j : bend;
        }
        if (live) {
            if (bad) {
                ovl_flag_error(err_flag);
                out_score[p] = -1;
                out_end[p] = -1;
            } else {
                out_score[p] = best;
                out_end[p] = bend;
            }
        }
    }
}


// ----------------------------------------------------------------------------- band knob, two lanes per pair
//
// band_lane_kernel keeps a pair's NB = 2W+1 band cells in one lane: at band 64 that is 129 cells plus 33
// window words, one wavefront per SIMD.  Here lanes 2q and 2q+1 share pair q, each with H = (NB + 1) / 2
// cells: lane 0 holds diagonals k = -1 .. H-2 (k = -1 a dummy held at -inf, the left edge of k = 0), lane 1
// holds k = H-1 .. NB-1.  A row's update is serial in k (the left move), and a row needs the previous row's
// k+1 (the up move), so the two halves of one row cannot run at once -- but lane 1 can run one row BEHIND
// lane 0: at step t lane 0 updates row iteration t and lane 1 row iteration t-1.  Then
//   * lane 1's first cell (k = H-1) takes as left lane 0's last cell (k = H-2) of iteration t-1, which
//     lane 0 finished in step t-1 (one DPP swap at the step's start);
//   * lane 0's last cell takes as up the value of cell k = H-1 after iteration t-1, which lane 1 computes
//     as the FIRST cell of this same step, before lane 0 reaches its last (one DPP swap after cell 0);
//   * the window slides one position per row, and the code entering lane 0's top is the one at lane 1's
//     bottom after lane 1's slide of the same step (one DPP swap); lane 1's top takes the code entering the
//     band, as in band_lane_kernel.
// Both lanes derive the row symbol and the entering code of iteration t; lane 1 uses the previous step's.
// Lane 1's extra first step (iteration -1) is a virtual row, which maps the row-0 pattern onto itself, so
// its cells start one iteration earlier; lane 0 is done after step R-1 (its row-n scan runs then) and lane
// 1 after step R.  The cells are the oracle's band edges exactly as in band_lane_kernel.
template <int NB, int OCC, bool PL>
__global__ __launch_bounds__(256, OCC) void band_lane2_kernel(const uint8_t* __restrict__ codes,
                                                              const int64_t* __restrict__ off,
                                                              const int32_t* __restrict__ len, int32_t n_reads,
                                                              const uint32_t* __restrict__ sfx,
                                                              const uint32_t* __restrict__ pfx, int32_t prow,
                                                              int32_t wpl, const int32_t* __restrict__ a_idx,
                                                              const int32_t* __restrict__ b_idx, int64_t n_pairs,
                                                              int32_t lcap, int32_t match, int32_t mismatch,
                                                              int32_t indel, int32_t* __restrict__ out_score,
                                                              int32_t* __restrict__ out_end,
                                                              const int32_t* __restrict__ seed,
                                                              uint32_t* __restrict__ err_flag) {
    static_assert(NB % 2 == 1 && NB >= 3, "NB = 2W + 1");
    constexpr int W = (NB - 1) / 2;
    constexpr int H = (NB + 1) / 2;   // cells per lane (lane 0: one dummy)
    constexpr int HW = (H + 3) / 4;   // window words per lane
    constexpr uint32_t PAD = 4;       // t code left of the read
    constexpr int32_t NEG = -(1 << 30);
    const int lane = threadIdx.x & 63;
    const int h = lane & 1;           // which half of its pair
    const int64_t wslot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nslots = (int64_t)gridDim.x * 4;
    const int64_t ntiles = (n_pairs + 31) >> 5;  // 32 pairs per wavefront
    const int32_t g = indel;
    const uint32_t b_ma = (uint32_t)(match - 2 * g) & 0xFFu;
    const uint32_t b_mm = (uint32_t)(mismatch - 2 * g) & 0xFFu;
    const uint32_t b_pad = (uint32_t)(-2 * g) & 0xFFu;
    const uint32_t tbl_mm = b_mm * 0x01010101u;  // the row table's bytes t = 0..3 before byte x takes the match
    const uint32_t tbl_dm = b_ma ^ b_mm;
    const uint32_t tbl_hi = b_pad * 0x01010101u;  // bytes 4..7: the pad code
    const uint32_t p_virt = ((uint32_t)(-g) & 0xFFu) * 0x01010101u;
    const int32_t kbase = h ? H - 1 : -1;  // diagonal of local cell 0
    // the partner lane's value (lanes 2q <-> 2q+1)
    auto swap = [](int32_t v) -> int32_t { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); };
    for (int64_t tile = wslot; tile < ntiles; tile += nslots) {
        const int64_t p = tile * 32 + (lane >> 1);
        const bool live = p < n_pairs;
        int32_t a = live ? a_idx[p] : 0;
        int32_t b = live ? b_idx[p] : 0;
        bool bad = live && (a < 0 || a >= n_reads || b < 0 || b >= n_reads);
        if (!live || bad) { a = 0; b = 0; }
        int32_t n = (live && !bad) ? len[a] : 0;
        int32_t m = (live && !bad) ? len[b] : 0;
        int32_t jstar = (live && !bad) ? seed[p] : 0;
        if (n > lcap || m > lcap || jstar < 0 || jstar > m) { bad = bad || live; n = 0; m = 0; jstar = 0; }
        const uint32_t sa = (uint32_t)off[a];
        const uint32_t tb = (uint32_t)off[b];
        const int32_t cc = n - jstar + W;  // j = i - cc + k
        const int32_t nmax = wave_max(n);
        const int32_t nmin = wave_min(n);
        constexpr int RQ = PL ? 32 : 4;
        const int32_t R = (nmax + RQ - 1) / RQ * RQ;  // row iterations (end-aligned rows)
        const int32_t sk = R - n;
        const int32_t mcut = R - nmin;
        auto tcode = [&](int32_t u) -> uint32_t {
            const int32_t uc = u < 0 ? 0 : (u >= m ? (m > 0 ? m - 1 : 0) : u);
            const uint32_t v = (uint32_t)codes[tb + (uint32_t)uc];
            return u < 0 ? PAD : v;
        };
        // the window of the lane's first iteration (-h): local cell j is diagonal kbase + j, t position
        // u0 - h + kbase + j; the cells start as the row pattern G = -indel * j before that iteration
        const int32_t u0 = -sk - cc;
        const int32_t uw = u0 - h + kbase;
        uint32_t T[HW];
#pragma unroll
        for (int w = 0; w < HW; ++w) {
            uint32_t word = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * w + q < H) word |= tcode(uw + 4 * w + q) << (8 * q);
            T[w] = word;
        }
        int32_t V[H];
#pragma unroll
        for (int j = 0; j < H; ++j) V[j] = -g * (uw + j);
        if (!h) V[0] = NEG;
        const int32_t ub = NB - sk - cc;  // the code entering after iteration it is at t position it + ub
        constexpr int NQ = PL ? 1 : 4;
        uint32_t qs[NQ], qt[NQ];
        auto fetch4 = [&](int32_t it4) {
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const int32_t i0 = it4 + k - sk;  // s index i - 1
                const int32_t ic = i0 < 0 ? 0 : (i0 >= n ? (n > 0 ? n - 1 : 0) : i0);
                qs[k] = (uint32_t)codes[sa + (uint32_t)ic];
                qt[k] = tcode(it4 + k + ub);
            }
        };
        const uint32_t* __restrict__ sp = sfx + (int64_t)a * prow + 2 * (wpl - R / 32);
        const uint32_t* __restrict__ tp = pfx + (int64_t)b * prow;
        const uint32_t tsh = (uint32_t)ub & 31u;
        uint32_t S0 = 0, S1 = 0, T0 = 0, T1 = 0;
        uint2 sn = make_uint2(0, 0), t0n = sn, t1n = sn;
        auto fetch_planes = [&](int32_t kb) {
            sn = *reinterpret_cast<const uint2*>(sp + 2 * kb);
            const int32_t q = (32 * kb + ub) >> 5;  // floor
            const int32_t q0 = q < 0 ? 0 : (q >= wpl ? wpl - 1 : q);
            const int32_t q1 = q + 1 < 0 ? 0 : (q + 1 >= wpl ? wpl - 1 : q + 1);
            t0n = *reinterpret_cast<const uint2*>(tp + 2 * q0);
            t1n = *reinterpret_cast<const uint2*>(tp + 2 * q1);
        };
        // the four-row words (body) of the previous group; before step 0 byte 3 is iteration -1's: a virtual row
        // (its symbol unused) whose entering code lane 1 appends in step 0
        uint32_t xs8_prev = 0, ts_prev = tcode(ub - 1) << 24;
        // step t: lane 0 runs iteration t, lane 1 iteration t - 1; x8 (8 * symbol) and tnew are the lane's own
        auto step = [&](int32_t t, uint32_t x8, uint32_t tnew, auto masked_tag) {
            constexpr bool MASKED = decltype(masked_tag)::value;
            const int32_t it = t - h;
            uint32_t tlo = tbl_mm ^ (tbl_dm << x8), thi = tbl_hi;  // the row's table (band_lane_kernel)
            if constexpr (MASKED) {
                const bool virt = it < sk;
                tlo = virt ? p_virt : tlo;
                thi = virt ? p_virt : thi;
            }
            // left of local cell 0: lane 1 takes lane 0's last cell of iteration t - 1 (finished last step); lane 0's
            // cell 0 is the dummy, set to -inf whatever its inputs
            int32_t left = swap(V[H - 1]);
            int32_t upin = NEG;
            uint32_t P = 0;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                if ((j & 3) == 0) P = __builtin_amdgcn_perm(thi, tlo, T[j >> 2]);
                const int32_t d = V[j] + (int32_t)(int8_t)(uint8_t)(P >> (8 * (j & 3)));
                const int32_t up = j + 1 < H ? V[j + 1] : upin;
                int32_t v = max(max(d, up), left);
                if (j == 0) {
                    if (!h) v = NEG;  // lane 0's dummy: the missing left of k = 0
                    // lane 0's last cell takes as up lane 1's cell 0 after iteration t - 1 (just computed); lane 1's
                    // receives lane 0's dummy, -inf: the missing up of k = 2W
                    upin = swap(v);
                }
                V[j] = v;
                left = v;
            }
            // slide the window one position; lane 0's top takes lane 1's new bottom code, lane 1's top the
            // code entering the band
#pragma unroll
            for (int w = 0; w < HW; ++w) T[w] = __builtin_amdgcn_alignbit(w + 1 < HW ? T[w + 1] : 0u, T[w], 8);
            const uint32_t bottom = (uint32_t)swap((int32_t)(T[0] & 0xFFu));
            T[(H - 1) >> 2] |= (h ? tnew : bottom) << (8 * ((H - 1) & 3));
        };
        // steps t..t+3: iterations t..t+3's symbols (times 8) and entering codes as the bytes of one word each,
        // extracted once per four steps; lane 1 takes them one iteration late (byte k - 1, byte 0 from the
        // previous group's byte 3)
        auto body = [&](int32_t t, auto masked_tag) {
            uint32_t xs8, ts;
            if constexpr (PL) {
                if ((t & 31) == 0) {  // next 32 rows: rotate the block words, prefetch the block after
                    S0 = sn.x;
                    S1 = sn.y;
                    T0 = __builtin_amdgcn_alignbit(t1n.x, t0n.x, tsh);
                    T1 = __builtin_amdgcn_alignbit(t1n.y, t0n.y, tsh);
                    if (t + 32 < R) fetch_planes((t + 32) >> 5);
                }
                const uint32_t r0 = (uint32_t)t & 31u;
                xs8 = codes4(S0, S1, r0) << 3;
                ts = pad4(codes4(T0, T1, r0), t + ub);
            } else {
                xs8 = (qs[0] | (qs[1] << 8) | (qs[2] << 16) | (qs[3] << 24)) << 3;
                ts = qt[0] | (qt[1] << 8) | (qt[2] << 16) | (qt[3] << 24);
                if (t + 4 < R) fetch4(t + 4);
            }
            const uint32_t xl = h ? __builtin_amdgcn_alignbyte(xs8, xs8_prev, 3) : xs8;
            const uint32_t tl = h ? __builtin_amdgcn_alignbyte(ts, ts_prev, 3) : ts;
            xs8_prev = xs8;
            ts_prev = ts;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                step(t + k, __builtin_amdgcn_ubfe(xl, 8 * k, 8), __builtin_amdgcn_ubfe(tl, 8 * k, 8), masked_tag);
        };
        // row n on this lane's cells: in-band cells with 0 <= j <= m, largest value, first j
        int32_t best = INT32_MIN, bend = -1;
        auto scan = [&]() {
#pragma unroll
            for (int jl = 0; jl < H; ++jl) {
                const int32_t j = jstar - W + kbase + jl;
                const int32_t v = V[jl] + g * (n + j);
                const bool better = (h || jl > 0) && j >= 0 && j <= m && v > best;
                best = better ? v : best;
                bend = better ? j : bend;
            }
        };
        if constexpr (PL) fetch_planes(0);
        else fetch4(0);
        int32_t t = 0;
        for (; t < mcut + 1 && t < R; t += 4) body(t, std::true_type{});
#ifndef OVL_BAND_UNROLL1
        // eight rows per trip: the window's one-word shift per four rows lands in place in the first body and
        // costs a register move per window word only at the trip's end (half the moves)
        if (t < R && ((R - t) & 7)) {
            body(t, std::false_type{});
            t += 4;
        }
        for (; t < R; t += 8) {
            body(t, std::false_type{});
            body(t + 4, std::false_type{});
        }
#else
        for (; t < R; t += 4) body(t, std::false_type{});
#endif
        if (!h) scan();  // lane 0 has finished iteration R - 1
        // step R: lane 1's last iteration (R - 1, byte 3 of the last group); lane 0's cells are no longer read
        step(R, xs8_prev >> 24, ts_prev >> 24, std::true_type{});
        if (h) scan();
        const int32_t ob = swap(best), oe = swap(bend);
        if (live && !h) {
            if (bad) {
                ovl_flag_error(err_flag);
                out_score[p] = -1;
                out_end[p] = -1;
            } else {
                const bool hi_wins = ob > best;  // lane 1's cells lie right of lane 0's: ties keep lane 0's
                out_score[p] = hi_wins ? ob : best;
                out_end[p] = hi_wins ? oe : bend;
            }
        }
    }
}

}  // namespace ovl

using ovl::dp_lane_kernel;

#ifndef OVL_H2_OCC
#define OVL_H2_OCC 3
#endif

extern "C" int32_t ovl_dp_lane_rcap(int32_t lcap) { return ((lcap + 31) & ~31) + 4; }

// waves per SIMD the strip width is compiled for: 32 columns at 4 (64 columns spill even at 3 waves per SIMD:
// the 4-row body keeps two rows of the strip live; 16 columns at 6 waves per SIMD were slower, round 1)
extern "C" int32_t ovl_dp_lane_waves_per_simd(int32_t cw) { return cw == 32 ? 4 : 0; }

// the LDS hand-off (HO 2): rows rounded to 32, 4 bits per row, a dword per 8 rows, per wavefront of the block
extern "C" int32_t ovl_dp_lane_lds_bytes(int32_t lcap) { return ((lcap + 31) & ~31) / 8 * 4 * 64 * 4; }

// dp_lane_h2_kernel: a diagonal score's f16 encoding ends in a zero byte when its odd part is <= 7 (at most three
// significant bits); the relative values stay below 65 * 15 + 128 < 2048 under HO 2's step bound
static bool h2_byte_score(int64_t v) {
    if (v == 0) return true;
    uint64_t u = (uint64_t)(v < 0 ? -v : v);
    while (!(u & 1)) u >>= 1;
    return u <= 7 && (v < 0 ? -v : v) <= 2048;
}

extern "C" int32_t ovl_dp_lane_h2_ok(int64_t match, int64_t mismatch, int64_t indel) {
    return indel <= 0 && h2_byte_score(match - 2 * indel) && h2_byte_score(mismatch - 2 * indel) &&
                   std::max(match, mismatch) - 2 * indel <= 15 ? 1 : 0;
}

// hand-off bytes dp_lane_h2_kernel needs in HBM (0: it hands off through LDS)
extern "C" int64_t ovl_dp_lane_h2_col_bytes(int64_t n_pairs, int32_t lcap) {
#ifndef OVL_H2_LDS
    return (n_pairs + 127) / 128 * (int64_t)(((lcap + 31) & ~31) / 4) * 64 * 4;
#else
    (void)n_pairs;
    (void)lcap;
    return 0;
#endif
}

extern "C" hipError_t ovl_launch_dp_lane(const OvlDpArgs* g, const OvlLaneArgs* k, hipStream_t stream) {
    if (g->n_pairs <= 0) return hipSuccess;
    if (k->h2) {
        const int32_t lcap = g->mcap;
        if (!k->sfx || !k->prof || k->ho != 2 || !k->sfx_words || !k->pfx_words || k->wsfx * 32 < lcap ||
            lcap > ovl::kLaneLdsMaxLen ||
            !ovl_dp_lane_h2_ok(g->match, g->mismatch, g->indel))
            return hipErrorInvalidValue;
        // a 128-pair tile per wavefront, two per block, all launched: the dispatcher places blocks as they free up
        // (resident slots looping over the tiles: 18.5 ms against 13.0, cfg5's full DP with the LDS hand-off)
        const int64_t tiles = (g->n_pairs + 127) / 128;
#ifdef OVL_LANE_GRID_SLOTS  // A/B: k->slots resident wavefronts looping over the tiles
        int64_t blocks = (std::min<int64_t>(k->slots, tiles) + 1) / 2;
#else
        int64_t blocks = (tiles + 1) / 2;
#endif
        if (blocks < 1) blocks = 1;
#ifndef OVL_H2_LDS
        const size_t shmem = 0;
        if (!k->colbuf) return hipErrorInvalidValue;
#else
        const size_t shmem = (size_t)((lcap + 31) & ~31) / 4 * 128 * 4;
#endif
        ovl::dp_lane_h2_kernel<OVL_H2_OCC><<<(unsigned)blocks, 128, shmem, stream>>>(
            g->len, g->n_reads, k->sfx_words, k->pfx_words, k->srow, k->wsfx, g->a_idx, g->b_idx, g->n_pairs,
            lcap, (int32_t)g->match, (int32_t)g->mismatch, (int32_t)g->indel, g->out_score, g->out_end,
            g->err_flag, k->colbuf, ((lcap + 31) & ~31) / 4);
        return hipGetLastError();
    }
    const int64_t tiles = (g->n_pairs + 63) / 64;
#ifndef OVL_LANE_GRID_SLOTS  // (the LDS hand-off only: the HBM hand-off columns are per resident slot)
    int64_t blocks = k->ho == 2 ? (tiles + 3) / 4 : (std::min<int64_t>(k->slots, tiles) + 3) / 4;
#else
    int64_t blocks = (std::min<int64_t>(k->slots, tiles) + 3) / 4;
#endif
    if (blocks < 1) blocks = 1;
    const int32_t lcap = g->mcap;
    const int32_t rcap = ovl_dp_lane_rcap(lcap);
    if (k->sfx && (!k->prof || !k->sfx_words || k->wsfx * 32 < lcap)) return hipErrorInvalidValue;
    if (k->cw != 32) return hipErrorInvalidValue;
    if (k->ho == 2 && (!k->sfx || lcap > ovl::kLaneLdsMaxLen)) return hipErrorInvalidValue;
    const size_t shmem = k->ho == 2 ? (size_t)ovl_dp_lane_lds_bytes(lcap) : 0;
#define OVL_LANE(CW, OCC, PR, HO, SX)                                                                         \
    dp_lane_kernel<CW, OCC, PR, HO, SX><<<(unsigned)blocks, 256, shmem, stream>>>(                           \
        g->codes, g->off, g->len, g->n_reads, k->sfx_words, k->srow, k->wsfx, g->a_idx, g->b_idx, g->n_pairs, \
        lcap, rcap, (int32_t)g->match, (int32_t)g->mismatch, (int32_t)g->indel, k->colbuf, g->out_score,     \
        g->out_end, g->err_flag)
    const int key = 1 << 5 | (k->prof ? 8 : 0) | (k->ho & 3) << 1 | (k->sfx ? 1 : 0);
    switch (key) {
        case 0x20: OVL_LANE(32, 4, false, 0, false); break;
        case 0x22: OVL_LANE(32, 4, false, 1, false); break;
        case 0x28: OVL_LANE(32, 4, true, 0, false); break;
        case 0x29: OVL_LANE(32, 4, true, 0, true); break;
        case 0x2A: OVL_LANE(32, 4, true, 1, false); break;
        case 0x2B: OVL_LANE(32, 4, true, 1, true); break;
        case 0x2D: OVL_LANE(32, 4, true, 2, true); break;
        default: return hipErrorInvalidValue;
    }
#undef OVL_LANE
    return hipGetLastError();
}

// band knob, lane per pair: one instantiation per band half-width 0..kBandLaneMax
namespace {
constexpr int kBandLaneMax = 64;

template <int W, bool PL>
hipError_t launch_band_lane_w(const OvlDpArgs* g, const OvlLaneArgs* k, int64_t blocks, hipStream_t stream) {
    constexpr int NB = 2 * W + 1;
    constexpr int OCC = NB <= 9 ? 8 : (NB <= 25 ? 6 : (NB <= 57 ? 4 : (NB <= 65 ? 3 : (NB <= 113 ? 2 : 1))));
    if constexpr (OCC == 8) {  // (the grid the caller sized for 6 wavefronts per SIMD, grown to 8)
        const int64_t tiles = (g->n_pairs + 63) / 64;
        blocks = std::max<int64_t>(1, (std::min<int64_t>(k->slots / 6 * 8, tiles) + 3) / 4);
    }
#ifndef OVL_LANE_GRID_SLOTS
    blocks = std::max<int64_t>(1, ((g->n_pairs + 63) / 64 + 3) / 4);
#endif
    ovl::band_lane_kernel<NB, OCC, PL><<<(unsigned)blocks, 256, 0, stream>>>(
        g->codes, g->off, g->len, g->n_reads, k->sfx_words, k->pfx_words, k->srow, k->wsfx, g->a_idx, g->b_idx,
        g->n_pairs, g->mcap, (int32_t)g->match, (int32_t)g->mismatch, (int32_t)g->indel, g->out_score, g->out_end,
        g->seed, g->err_flag);
    return hipGetLastError();
}

// two lanes per pair (band_lane2_kernel): H = W + 1 cells per lane, 32 pairs per wavefront
template <int W, bool PL>
hipError_t launch_band_lane2_w(const OvlDpArgs* g, const OvlLaneArgs* k, hipStream_t stream) {
    constexpr int NB = 2 * W + 1;
    constexpr int H = W + 1;
    constexpr int OCC = H <= 17 ? 6 : (H <= 33 ? 4 : 3);
    const int64_t tiles = (g->n_pairs + 31) / 32;
#ifndef OVL_LANE_GRID_SLOTS  // a tile per wavefront, the dispatcher places blocks as they free up
    int64_t blocks = (tiles + 3) / 4;
#else
    int64_t blocks = (std::min<int64_t>(k->slots / 6 * OCC, tiles) + 3) / 4;
#endif
    if (blocks < 1) blocks = 1;
    ovl::band_lane2_kernel<NB, OCC, PL><<<(unsigned)blocks, 256, 0, stream>>>(
        g->codes, g->off, g->len, g->n_reads, k->sfx_words, k->pfx_words, k->srow, k->wsfx, g->a_idx, g->b_idx,
        g->n_pairs, g->mcap, (int32_t)g->match, (int32_t)g->mismatch, (int32_t)g->indel, g->out_score, g->out_end,
        g->seed, g->err_flag);
    return hipGetLastError();
}

// every half-width up to 32, then 40, 48, 56, 64 (other widths above 32 take the anti-diagonal form)
constexpr int next_band_lane(int w) { return w < 32 ? w + 1 : w + 8; }

template <int W>
hipError_t dispatch_band_lane(int band, const OvlDpArgs* g, const OvlLaneArgs* k, int64_t blocks,
                              hipStream_t stream) {
    if (band == W) {
        if constexpr (W >= 1)
            if (k->split)
                return k->sfx ? launch_band_lane2_w<W, true>(g, k, stream)
                              : launch_band_lane2_w<W, false>(g, k, stream);
        return k->sfx ? launch_band_lane_w<W, true>(g, k, blocks, stream)
                      : launch_band_lane_w<W, false>(g, k, blocks, stream);
    }
    if constexpr (W < kBandLaneMax) return dispatch_band_lane<next_band_lane(W)>(band, g, k, blocks, stream);
    return hipErrorInvalidValue;
}
}  // namespace

extern "C" int32_t ovl_band_lane_ok(int32_t band) {
    return band >= 0 && (band <= 32 || (band <= kBandLaneMax && band % 8 == 0)) ? 1 : 0;
}

extern "C" hipError_t ovl_launch_band_lane(const OvlDpArgs* g, const OvlLaneArgs* k, hipStream_t stream) {
    if (g->n_pairs <= 0) return hipSuccess;
    if (g->band < 0 || g->band > kBandLaneMax) return hipErrorInvalidValue;
    if (k->sfx && (!k->sfx_words || !k->pfx_words || k->wsfx * 32 < g->mcap)) return hipErrorInvalidValue;
    const int64_t tiles = (g->n_pairs + 63) / 64;
    int64_t blocks = (std::min<int64_t>(k->slots, tiles) + 3) / 4;
    if (blocks < 1) blocks = 1;
    return dispatch_band_lane<0>(g->band, g, k, blocks, stream);
}
