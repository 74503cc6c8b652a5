// ovl_kernels.hip — gfx950 (CDNA4) kernels of the overlap-scoring engine.
//
// Hot path: aligners.py:27-57, the overlap DP and
// its last-row first-argmax, evaluated for every candidate pair of
// overlapGraphs.py:43-53.
//
// Kernels
//   map_codes     bytes -> dense symbol codes (LUT), one lane per byte.
//   pack_planes   codes -> bit-plane words in two layouts (prefix / suffix),
//                 one lane per (read, word).  HBM-bound byte work, run once per read set.
//   ungapped      THE hot kernel.  Exact whenever gaps cannot win (the reference's
//                 default indel = -2**31): dp[n][j] is the sum over
//                 the L=min(n,j) diagonal cells ending at (n, j), so
//                   score(j) = match*L + (mismatch-match)*X(j),  X = mismatch count.
//                 One wavefront per pair; lane l owns end positions j = 64*c + l.
//                 Bases are bit-planes (P planes, 32 bases per uint32 word); a
//                 mismatch word is OR_p(S_p ^ T_p) and X accumulates with v_bcnt.
//                 No MFMA: this is integer compare/popcount work (BASELINE north_star).
//   dp            anti-diagonal wavefront DP for any scoring (finite indel), int64
//                 arithmetic with int32 stores like Numba; lanes own rows, the row
//                 carried between 64-row strips and the t symbols are staged in LDS.
//
// Layouts (per read r, uint32 words, P planes interleaved per word):
//   sfx[r][k][p], k in [0, WMAX):   read right-aligned so that its last base is
//                                   bit 31 of word WMAX-1 (position 32*WMAX-n+i).
//   pfx[r][z][p], z in [0, ZS):     two zero words, then the read left-aligned
//                                   (base i at word 2 + i/32, bit i%32), zero tail.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ovl_kernels.h"

namespace ovl {

__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t r) {
    return __builtin_amdgcn_alignbit(hi, lo, r);
}

// ----------------------------------------------------------------------------- packing

__global__ void map_codes_kernel(const uint8_t* __restrict__ raw, const uint8_t* __restrict__ lut,
                                 uint8_t* __restrict__ codes, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) codes[i] = lut[raw[i]];
}

template <int P>
__global__ void pack_planes_kernel(const uint8_t* __restrict__ codes, const int64_t* __restrict__ off,
                                   const int32_t* __restrict__ len, int32_t n_reads, int32_t wmax,
                                   int32_t zs, uint32_t* __restrict__ sfx, uint32_t* __restrict__ pfx) {
    const int nw = wmax > zs ? wmax : zs;
    int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)n_reads * nw;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; gid < total; gid += stride) {
        const int32_t r = (int32_t)(gid / nw);
        const int32_t w = (int32_t)(gid % nw);
        const int32_t n = len[r];
        const uint8_t* s = codes + off[r];
        if (w < zs) {
            uint32_t pl[P];
#pragma unroll
            for (int p = 0; p < P; ++p) pl[p] = 0u;
            const int32_t d = w - 2;  // data word index
            if (d >= 0) {
                for (int b = 0; b < 32; ++b) {
                    const int32_t i = 32 * d + b;
                    if (i < n) {
                        const uint32_t c = s[i];
#pragma unroll
                        for (int p = 0; p < P; ++p) pl[p] |= ((c >> p) & 1u) << b;
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < P; ++p) pfx[((int64_t)r * zs + w) * P + p] = pl[p];
        }
        if (w < wmax) {
            uint32_t pl[P];
#pragma unroll
            for (int p = 0; p < P; ++p) pl[p] = 0u;
            const int32_t shift = 32 * wmax - n;  // position of base 0
            for (int b = 0; b < 32; ++b) {
                const int32_t i = 32 * w + b - shift;
                if (i >= 0 && i < n) {
                    const uint32_t c = s[i];
#pragma unroll
                    for (int p = 0; p < P; ++p) pl[p] |= ((c >> p) & 1u) << b;
                }
            }
#pragma unroll
            for (int p = 0; p < P; ++p) sfx[((int64_t)r * wmax + w) * P + p] = pl[p];
        }
    }
}

// ----------------------------------------------------------------------------- ungapped

template <typename KeyT>
struct KeyOps;

template <>
struct KeyOps<uint32_t> {
    // score in [1, 2^15), j in [0, 2^16): max key = max score, then min j
    __device__ static uint32_t make(int64_t score, int32_t j) {
        return ((uint32_t)score << 16) | (uint32_t)(0xFFFF - j);
    }
    __device__ static uint32_t wave_max(uint32_t v) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
            v = v > o ? v : o;
        }
        return v;
    }
    __device__ static void decode(uint32_t key, int32_t& score, int32_t& end) {
        score = key ? (int32_t)(key >> 16) : 0;
        end = key ? (int32_t)(0xFFFF - (key & 0xFFFF)) : 0;
    }
};

template <>
struct KeyOps<uint64_t> {
    __device__ static uint64_t make(int64_t score, int32_t j) {
        return ((uint64_t)(uint32_t)score << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)j);
    }
    __device__ static uint64_t wave_max(uint64_t v) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, off, 64);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), off, 64);
            const uint64_t o = ((uint64_t)hi << 32) | lo;
            v = v > o ? v : o;
        }
        return v;
    }
    __device__ static void decode(uint64_t key, int32_t& score, int32_t& end) {
        score = key ? (int32_t)(uint32_t)(key >> 32) : 0;
        end = key ? (int32_t)(0xFFFFFFFFu - (uint32_t)key) : 0;
    }
};

template <int P>
__device__ __forceinline__ void load_planes(const uint32_t* __restrict__ src, uint32_t (&dst)[P]) {
    if constexpr (P == 2) {
        const uint2 v = *reinterpret_cast<const uint2*>(src);
        dst[0] = v.x; dst[1] = v.y;
    } else if constexpr (P % 4 == 0) {
#pragma unroll
        for (int q = 0; q < P / 4; ++q) {
            const uint4 v = *reinterpret_cast<const uint4*>(src + 4 * q);
            dst[4 * q + 0] = v.x; dst[4 * q + 1] = v.y; dst[4 * q + 2] = v.z; dst[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int p = 0; p < P; ++p) dst[p] = src[p];
    }
}

// Score one pair; every lane returns the wave-wide best key.
//   s = read a (suffix layout, right-aligned in WMAX words), length n, WP = ceil(n/32)
//   t = read b (prefix layout), length m, nch = ceil((m+1)/64) chunks of 64 end positions.
// Lane l = 32h + r handles j = 64c + l.  With j = 32q + r (q = 2c + h), position x of the
// right-aligned s' (WP words) meets t position x + j - 32*WP; the t words it needs are
//   T_r[y] = t-bits [32y - 32 + r, 32y + r)  (y >= 0; t-bit < 0 is padding)
// and row q pairs s' word k = WP-1-(q-y) with T_r[y] for y in [max(0, q-WP+1), q].
// Half h keeps the array U[z] = T_r[z - 1 + h], so row q = 2c+h reads U[y - h + 1]
// with z = y' + 1, y' in [max(-1, 2c-WP+1), 2c]: a compile-time register index.
// Invalid bits: t padding only in T_r[0] (bits < 32-r), s padding only in word k=0
// (bits < 32*WP-n); both masked.  Everything else in the row is a real comparison.
template <int P, int WMAX, int WP, typename KeyT>
__device__ __forceinline__ KeyT score_pair_wp(const uint32_t* __restrict__ sfx_a,
                                              const uint32_t* __restrict__ pfx_b, int32_t n,
                                              int32_t m, int32_t match, int32_t mismatch,
                                              int lane) {
    constexpr int NCHMAX = (32 * WMAX + 64) / 64;  // ceil((32*WMAX + 1) / 64)
    constexpr int NZ = 2 * NCHMAX;                 // U words z in [0, NZ)
    const int nch = (m + 64) >> 6;
    const uint32_t h = (uint32_t)lane >> 5;
    const uint32_t r = (uint32_t)lane & 31u;

    // s words: wave-uniform (scalar loads / SGPR operands).
    uint32_t S[WP][P];
    const uint32_t* sp = sfx_a + (WMAX - WP) * P;
#pragma unroll
    for (int k = 0; k < WP; ++k) load_planes<P>(sp + k * P, S[k]);

    // t words for this half: Tw[y] = pfx word (y + h), y in [0, NZ].
    uint32_t Tw[NZ + 1][P];
    const uint32_t* tp = pfx_b + h * P;
#pragma unroll
    for (int y = 0; y <= NZ; ++y) load_planes<P>(tp + y * P, Tw[y]);

    const uint32_t vt = r ? (0xFFFFFFFFu << (32u - r)) : 0u;  // valid bits of T_r[0]
    const uint32_t vu0 = h ? vt : 0u;
    const uint32_t vu1 = h ? 0xFFFFFFFFu : vt;
    const uint32_t sv0 = 0xFFFFFFFFu << (uint32_t)(32 * WP - n);  // valid bits of s' word 0

    uint32_t U[NZ][P];
    KeyT best = 0;
    const int64_t dms = (int64_t)mismatch - (int64_t)match;
#pragma unroll
    for (int c = 0; c < NCHMAX; ++c) {
        if (c < nch) {  // wave-uniform
            constexpr int dummy = 0; (void)dummy;
            const int zlo = (2 * c - WP + 2) > 0 ? (2 * c - WP + 2) : 0;
#pragma unroll
            for (int z = 2 * c; z <= 2 * c + 1; ++z) {
                if (z >= zlo) {
#pragma unroll
                    for (int p = 0; p < P; ++p) U[z][p] = alignbit(Tw[z + 1][p], Tw[z][p], r);
                }
            }
            uint32_t X = 0;
#pragma unroll
            for (int z = zlo; z <= 2 * c + 1; ++z) {
                const int k = WP - 2 - 2 * c + z;  // s word paired with U[z]
                uint32_t mm = 0;
#pragma unroll
                for (int p = 0; p < P; ++p) mm |= S[k][p] ^ U[z][p];
                if (z == 0) mm &= vu0;
                if (z == 1) mm &= vu1;
                if (k == 0) mm &= sv0;
                X += (uint32_t)__builtin_popcount(mm);
            }
            const int32_t j = 64 * c + lane;
            const int32_t L = n < j ? n : j;
            const int64_t score = (int64_t)match * L + dms * (int64_t)X;
            const bool valid = (j >= 1) & (j <= m) & (score > 0);
            const KeyT key = valid ? KeyOps<KeyT>::make(score, j) : (KeyT)0;
            best = key > best ? key : best;
        }
    }
    return KeyOps<KeyT>::wave_max(best);
}

template <int P, int WMAX, typename KeyT, int WP = 1>
__device__ __forceinline__ KeyT score_pair(const uint32_t* __restrict__ sfx_a,
                                           const uint32_t* __restrict__ pfx_b, int32_t n, int32_t m,
                                           int32_t match, int32_t mismatch, int lane, int wp) {
    if constexpr (WP == WMAX) {
        return score_pair_wp<P, WMAX, WP, KeyT>(sfx_a, pfx_b, n, m, match, mismatch, lane);
    } else {
        if (wp == WP) return score_pair_wp<P, WMAX, WP, KeyT>(sfx_a, pfx_b, n, m, match, mismatch, lane);
        return score_pair<P, WMAX, KeyT, WP + 1>(sfx_a, pfx_b, n, m, match, mismatch, lane, wp);
    }
}

// Grid-stride over tiles of `tile` consecutive pairs; one wavefront per tile.
// Lane i of the wave owns pair base+i: it gathers the indices and lengths
// (coalesced) and keeps the result, stored once per tile (coalesced).
template <int P, int WMAX, typename KeyT>
__global__ __launch_bounds__(256) void ungapped_kernel(
    const uint32_t* __restrict__ sfx, const uint32_t* __restrict__ pfx, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx,
    int64_t n_pairs, int32_t tile, int32_t match, int32_t mismatch, int32_t* __restrict__ out_score,
    int32_t* __restrict__ out_end, uint32_t* __restrict__ err_flag) {
    constexpr int NCHMAX = (32 * WMAX + 64) / 64;
    constexpr int ZS = 2 * NCHMAX + 2;
    const int lane = threadIdx.x & 63;
    const int64_t waves_per_block = blockDim.x >> 6;
    const int64_t wave0 = (int64_t)blockIdx.x * waves_per_block + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * waves_per_block;
    const int64_t n_tiles = (n_pairs + tile - 1) / tile;
    for (int64_t t = wave0; t < n_tiles; t += n_waves) {
        const int64_t base = t * tile;
        const int64_t p = base + lane;
        const bool mine = (lane < tile) && (p < n_pairs);
        int32_t a = mine ? a_idx[p] : 0;
        int32_t b = mine ? b_idx[p] : 0;
        bool ok = mine && a >= 0 && a < n_reads && b >= 0 && b < n_reads;
        if (!ok) { a = 0; b = 0; }
        int32_t na = len[a], nb = len[b];
        ok = ok && na <= 32 * WMAX && nb <= 32 * WMAX;
        if (mine && !ok) atomicOr(err_flag, 1u);
        if (!ok) { na = 0; nb = 0; }
        int32_t res_s = ok ? 0 : -1, res_e = ok ? 0 : -1;
        const int64_t rem = n_pairs - base;
        const int cnt = rem < tile ? (int)rem : tile;
        for (int i = 0; i < cnt; ++i) {
            const int32_t A = __builtin_amdgcn_readlane(a, i);
            const int32_t B = __builtin_amdgcn_readlane(b, i);
            const int32_t n = __builtin_amdgcn_readlane(na, i);
            const int32_t m = __builtin_amdgcn_readlane(nb, i);
            KeyT key = 0;
            if (n > 0 && m > 0) {
                const int wp = (n + 31) >> 5;
                key = score_pair<P, WMAX, KeyT>(sfx + (int64_t)A * (WMAX * P), pfx + (int64_t)B * (ZS * P),
                                                n, m, match, mismatch, lane, wp);
            }
            if (lane == i && ok) KeyOps<KeyT>::decode(key, res_s, res_e);
        }
        if (mine) {
            out_score[p] = res_s;
            out_end[p] = res_e;
        }
    }
}

// ----------------------------------------------------------------------------- generic DP

__device__ __forceinline__ int32_t shr1_i32(int32_t v) {
    // wave_shr:1 — lane l receives lane l-1's value (lane 0 receives 0).
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
}

template <typename Acc>
__device__ __forceinline__ Acc shr1(Acc v);

template <>
__device__ __forceinline__ int32_t shr1<int32_t>(int32_t v) { return shr1_i32(v); }

template <>
__device__ __forceinline__ int64_t shr1<int64_t>(int64_t v) {
    const int32_t lo = shr1_i32((int32_t)(uint32_t)(uint64_t)v);
    const int32_t hi = shr1_i32((int32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// One wavefront (block of 64) per pair, grid-stride over pairs.  Strip of 64
// rows i = 64*st + 1 + lane; anti-diagonal step tau has lane l on column
// j = tau - l + 1.  up / t-symbol arrive from lane l-1 by DPP; lane 0 reads
// them from the staged LDS row (the previous strip's last row) and t codes.
// Cell rule of aligners.py:35-48 with Acc-width arithmetic; the stored value
// is narrowed to int32 as the reference's int32 table does.
template <typename Acc>
__global__ __launch_bounds__(64) void dp_kernel(
    const uint8_t* __restrict__ codes, const int64_t* __restrict__ off, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx,
    int64_t n_pairs, int32_t mcap, int64_t match, int64_t mismatch, int64_t indel,
    int32_t* __restrict__ out_score, int32_t* __restrict__ out_end, int8_t* __restrict__ tb,
    uint32_t* __restrict__ err_flag) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int32_t* row0 = reinterpret_cast<int32_t*>(smem);
    int32_t* row1 = row0 + (mcap + 1);
    uint8_t* tcodes = reinterpret_cast<uint8_t*>(row1 + (mcap + 1));
    const int lane = threadIdx.x;
    for (int64_t pair = blockIdx.x; pair < n_pairs; pair += gridDim.x) {
        const int32_t a = a_idx[pair];
        const int32_t b = b_idx[pair];
        if (a < 0 || a >= n_reads || b < 0 || b >= n_reads || len[b] > mcap) {
            if (lane == 0) {
                atomicOr(err_flag, 1u);
                out_score[pair] = -1;
                out_end[pair] = -1;
            }
            continue;
        }
        const int32_t n = len[a];
        const int32_t m = len[b];
        const uint8_t* s = codes + off[a];
        const uint8_t* t = codes + off[b];
        __syncthreads();  // previous pair's LDS readers are done
        for (int j = lane; j <= m; j += 64) row0[j] = 0;
        for (int j = lane; j < m; j += 64) tcodes[j] = t[j];
        __syncthreads();
        int32_t* rin = row0;
        int32_t* rout = row1;
        int32_t best = 0, bend = 0;  // tracked by the lane that owns row n
        const int nstrips = (n + 63) >> 6;
        for (int st = 0; st < nstrips; ++st) {
            const int32_t i = 64 * st + 1 + lane;
            const bool row_ok = i <= n;
            const uint32_t sc = row_ok ? (uint32_t)s[i - 1] : 0xFFFFFFFFu;
            int32_t cur = 0;      // dp[i][j-1] (starts as dp[i][0] = 0)
            int32_t uprev = 0;    // dp[i-1][j-1]
            uint32_t tch = 0;
            const bool last_strip_row = (lane == 63) && (st + 1 < nstrips);
            for (int tau = 0; tau < m + 63; ++tau) {
                const int32_t j = tau - lane + 1;
                // lane 0's inputs come from LDS (uniform address: broadcast)
                const int32_t jj = tau + 1 <= m ? tau + 1 : m;
                const int32_t lds_up = rin[jj];
                const uint32_t lds_t = tau < m ? (uint32_t)tcodes[tau] : 0u;
                int32_t upin = shr1<int32_t>(cur);
                uint32_t tin = (uint32_t)shr1<int32_t>((int32_t)tch);
                if (lane == 0) { upin = lds_up; tin = lds_t; }
                if (row_ok && j >= 1 && j <= m) {
                    const Acc diag = (Acc)uprev + (sc == tin ? (Acc)match : (Acc)mismatch);
                    const Acc up = (Acc)upin + (Acc)indel;
                    const Acc left = (Acc)cur + (Acc)indel;
                    int8_t dir;
                    Acc v;
                    if (diag >= up && diag >= left) { v = diag; dir = 0; }
                    else if (up >= left)            { v = up;   dir = 1; }
                    else                            { v = left; dir = 2; }
                    cur = (int32_t)v;
                    if (tb) tb[(int64_t)i * (m + 1) + j] = dir;
                    if (i == n && cur > best) { best = cur; bend = j; }
                    if (last_strip_row) rout[j] = cur;
                }
                uprev = upin;
                tch = tin;
            }
            __syncthreads();
            if (lane == 0 && st + 1 < nstrips) rout[0] = 0;
            __syncthreads();
            int32_t* tmp = rin; rin = rout; rout = tmp;
        }
        // row n lives in lane (n-1) % 64 of the last strip; dp[n][0] = 0 is the j = 0 candidate.
        const int owner = (n - 1) & 63;
        const int32_t bs = __shfl(best, owner, 64);
        const int32_t be = __shfl(bend, owner, 64);
        if (lane == 0) {
            out_score[pair] = n > 0 && m > 0 ? bs : 0;
            out_end[pair] = n > 0 && m > 0 ? be : 0;
        }
    }
}

}  // namespace ovl

// ----------------------------------------------------------------------------- launchers

using namespace ovl;

extern "C" hipError_t ovl_launch_map_codes(const uint8_t* raw, const uint8_t* lut, uint8_t* codes, int64_t n,
                                           hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    map_codes_kernel<<<(unsigned)blocks, 256, 0, stream>>>(raw, lut, codes, n);
    return hipGetLastError();
}

extern "C" hipError_t ovl_launch_pack(int planes, const uint8_t* codes, const int64_t* off, const int32_t* len,
                                      int32_t n_reads, int32_t wmax, int32_t zs, uint32_t* sfx, uint32_t* pfx,
                                      hipStream_t stream) {
    if (n_reads <= 0) return hipSuccess;
    const int64_t total = (int64_t)n_reads * (wmax > zs ? wmax : zs);
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    switch (planes) {
        case 2: pack_planes_kernel<2><<<(unsigned)blocks, 256, 0, stream>>>(codes, off, len, n_reads, wmax, zs, sfx, pfx); break;
        case 4: pack_planes_kernel<4><<<(unsigned)blocks, 256, 0, stream>>>(codes, off, len, n_reads, wmax, zs, sfx, pfx); break;
        case 8: pack_planes_kernel<8><<<(unsigned)blocks, 256, 0, stream>>>(codes, off, len, n_reads, wmax, zs, sfx, pfx); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int P, int WMAX, typename KeyT>
static void launch_ungapped_t(const OvlUngappedArgs& g, unsigned blocks, hipStream_t stream) {
    ungapped_kernel<P, WMAX, KeyT><<<blocks, 256, 0, stream>>>(
        g.sfx, g.pfx, g.len, g.n_reads, g.a_idx, g.b_idx, g.n_pairs, g.tile, g.match, g.mismatch,
        g.out_score, g.out_end, g.err_flag);
}

template <int P, typename KeyT>
static hipError_t launch_ungapped_p(const OvlUngappedArgs& g, unsigned blocks, hipStream_t stream) {
    switch (g.wmax) {
        case 2: launch_ungapped_t<P, 2, KeyT>(g, blocks, stream); break;
        case 4: launch_ungapped_t<P, 4, KeyT>(g, blocks, stream); break;
        case 8: launch_ungapped_t<P, 8, KeyT>(g, blocks, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" hipError_t ovl_launch_ungapped(const OvlUngappedArgs* g, hipStream_t stream) {
    if (g->n_pairs <= 0) return hipSuccess;
    const int64_t n_tiles = (g->n_pairs + g->tile - 1) / g->tile;
    int64_t blocks = (n_tiles + 3) / 4;  // 4 waves per block
    if (blocks > g->max_blocks) blocks = g->max_blocks;
    const unsigned nb = (unsigned)blocks;
    if (g->key64) {
        switch (g->planes) {
            case 2: return launch_ungapped_p<2, uint64_t>(*g, nb, stream);
            case 4: return launch_ungapped_p<4, uint64_t>(*g, nb, stream);
            case 8: return launch_ungapped_p<8, uint64_t>(*g, nb, stream);
        }
    } else {
        switch (g->planes) {
            case 2: return launch_ungapped_p<2, uint32_t>(*g, nb, stream);
            case 4: return launch_ungapped_p<4, uint32_t>(*g, nb, stream);
            case 8: return launch_ungapped_p<8, uint32_t>(*g, nb, stream);
        }
    }
    return hipErrorInvalidValue;
}

extern "C" hipError_t ovl_launch_dp(const OvlDpArgs* g, hipStream_t stream) {
    if (g->n_pairs <= 0) return hipSuccess;
    int64_t blocks = g->n_pairs;
    if (blocks > 16384) blocks = 16384;
    const size_t lds = (size_t)2 * (g->mcap + 1) * sizeof(int32_t) + (size_t)g->mcap + 16;
    if (g->wide) {
        dp_kernel<int64_t><<<(unsigned)blocks, 64, lds, stream>>>(
            g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx, g->n_pairs, g->mcap, g->match,
            g->mismatch, g->indel, g->out_score, g->out_end, g->tb, g->err_flag);
    } else {
        dp_kernel<int32_t><<<(unsigned)blocks, 64, lds, stream>>>(
            g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx, g->n_pairs, g->mcap, g->match,
            g->mismatch, g->indel, g->out_score, g->out_end, g->tb, g->err_flag);
    }
    return hipGetLastError();
}
