// ovl_kernels.hip — gfx950 (CDNA4) kernels of the overlap-scoring engine.
//
// Hot path: aligners.py:27-57, the overlap DP and
// its last-row first-argmax, evaluated for every candidate pair of
// overlapGraphs.py:43-53.
//
// Kernels
//   map_codes     bytes -> dense symbol codes (LUT), one lane per byte.
//   pack_planes   codes -> bit-plane words in two layouts (prefix / suffix),
//                 one lane per (read, word).  Byte work, run once per read set.
//   ungapped      THE hot kernel.  Exact whenever gaps cannot win (the reference's
//                 default indel = -2**31): dp[n][j] is the sum over
//                 the L=min(n,j) diagonal cells ending at (n, j), so
//                   score(j) = match*L + (mismatch-match)*X(j),  X = mismatch count.
//                 Lane-per-pair: a lane holds both reads as bit-planes (P planes, 32
//                 bases per uint32 word) and sweeps every end position j; a mismatch
//                 word is OR_p(S_p ^ T_p) and X accumulates with v_bcnt.  No MFMA:
//                 integer compare/popcount work (BASELINE north_star).
//   dp            anti-diagonal wavefront DP for any scoring (finite indel), int64
//                 arithmetic with int32 stores like Numba; lanes own rows, the row
//                 carried between 64-row strips and the t symbols are staged in LDS.
//
// Layouts (per read, W = ceil(lmax/32) words of 32 bases, P planes interleaved per
// word, rows padded to 16 bytes):
//   sfx[r][k*P + p], k < W:       read right-aligned: base i at position 32W - n + i
//   pfx[r][x*P + p], x < W:       read left-aligned: base i at position i (word W is implicitly zero)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include <hip/hip_ext.h>

#include "ovl_kernels.h"
#include "ovl_grid.h"

// uniform sweep: two shifts from one shifted row (sweep_uniform, keys_s2 / keys_t2); 0: one shifted row per shift
#ifndef OVL_SHIFT_PAIR
#define OVL_SHIFT_PAIR 1
#endif
// uniform sweep: rows of at most this many words shift s (W above: t; every W <= 8 by default)
#ifndef OVL_SHIFT_S_MAXW
#define OVL_SHIFT_S_MAXW 8
#endif

namespace ovl {

#ifdef OVL_TRACE  // diagnostic build only (make trace): per-wavefront timestamps of the uniform kernel
__device__ unsigned long long ovl_trace_buf[65536 * 8];
#define OVL_TR_CLOCK(k, dep)                                                                           \
    do {                                                                                               \
        unsigned long long t_;                                                                         \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)"            \
                     : "=s"(t_) : "v"(dep) : "memory");                                                \
        if (lane == 0 && tr_id < 65536) ovl_trace_buf[tr_id * 8 + (k)] = t_;                            \
    } while (0)
#define OVL_TR_VAL(k, v) \
    do { if (lane == 0 && tr_id < 65536) ovl_trace_buf[tr_id * 8 + (k)] = (unsigned long long)(v); } while (0)
#else
#define OVL_TR_CLOCK(k, dep) do {} while (0)
#define OVL_TR_VAL(k, v) do {} while (0)
#endif

__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t r) {
    return __builtin_amdgcn_alignbit(hi, lo, r);
}

// A result store: results that leave the GPU (host-mapped output arrays) go out as non-temporal stores, so
// they stream to the link without allocating in L2; device outputs are plain stores.
template <bool HOUT>
__device__ __forceinline__ void put_result(int32_t* p, int32_t v) {
    if constexpr (HOUT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// The (score, end) of pair p into the call's result sink (OvlUngappedArgs::host_out):
//   OM 0: the int32 arrays in HBM;  OM 1: the int32 arrays, host-mapped (non-temporal stores);
//   OM 2: packed, host-mapped into a pinned staging slot that the host expands into the int32 arrays
//         (2 instead of 8 link bytes per pair).  An end j <= n (the read a's length) has L = j compared
//         bases (aligners.py:27-48 with gaps that cannot win), so score = match*(j - X) + mismatch*X and the
//         pair is (j, X): one uint16 j << 8 | X.  X = 0xFF marks the rest: j << 8 | 0xFF with the score in
//         out_end[p] (j > n: a shorter read a inside b's window), or 0xFFFF for a bad pair.  The host asks
//         for it when lmax <= 254 (so j, X <= 254) and the keys are int32; inv = 1 / (match - mismatch),
//         or 0 when they are equal (X is then immaterial and 0).
template <int OM>
__device__ __forceinline__ void put_pair(int32_t* out_score, int32_t* out_end, int64_t p, int32_t sc, int32_t en,
                                         int32_t n = 0, int32_t match = 0, float inv = 0.f) {
    if constexpr (OM == 2) {
        uint32_t v;
        if (en < 0) {
            v = 0xFFFFu;
        } else if (en > n) {
            v = ((uint32_t)en << 8) | 0xFFu;
            __builtin_nontemporal_store(sc, out_end + p);
        } else {
            // X = (match*j - score) / (match - mismatch), an exact quotient below 2^8: float is exact
            const uint32_t x = (uint32_t)__builtin_rintf((float)(match * en - sc) * inv);
            v = ((uint32_t)en << 8) | x;
        }
        __builtin_nontemporal_store((uint16_t)v, reinterpret_cast<uint16_t*>(out_score) + p);
    } else {
        put_result<OM == 1>(out_score + p, sc);
        put_result<OM == 1>(out_end + p, en);
    }
}

__device__ __forceinline__ float pack_inv(int32_t match, int32_t mismatch) {
    return match != mismatch ? 1.0f / (float)(match - mismatch) : 0.f;
}

// popcount(v) + acc as one v_bcnt_u32_b32 with its accumulator operand; kept as a chain (the compiler
// would otherwise sum a block's word counts with an extra v_add3)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t v, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(acc));
    return r;
}

// ----------------------------------------------------------------------------- packing

__global__ void map_codes_kernel(const uint8_t* __restrict__ raw, const uint8_t* __restrict__ lut,
                                 uint8_t* __restrict__ codes, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) codes[i] = lut[raw[i]];
}

// 2-bit packed ACGT bytes (host-packed by ovl_set_reads: base i at bits 2(i % 4) of byte i / 4, A C G T =
// 0 1 2 3) -> dense symbol codes through the read set's LUT (codes[i] = lut["ACGT"[code]]); one lane per 16
// packed bytes (64 bases: one 16-byte load, four 16-byte stores), a 4-entry table in registers.
__global__ void unpack2_kernel(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ lut,
                               uint8_t* __restrict__ codes, int64_t n) {
    const uint32_t c0 = lut['A'], c1 = lut['C'], c2 = lut['G'], c3 = lut['T'];
    const int64_t groups = (n + 63) / 64;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride) {
        const uint4 v = reinterpret_cast<const uint4*>(pk)[g];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t out[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t x = w[k >> 2] >> (8 * (k & 3));  // packed byte k: bases 4k .. 4k + 3
            uint32_t o = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t c = (x >> (2 * b)) & 3u;
                const uint32_t m = c == 0 ? c0 : (c == 1 ? c1 : (c == 2 ? c2 : c3));
                o |= m << (8 * b);
            }
            out[k] = o;
        }
        const int64_t base = g * 64;
        if (base + 64 <= n) {
            uint4* d = reinterpret_cast<uint4*>(codes + base);
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = make_uint4(out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]);
        } else {
            for (int64_t i = base; i < n; ++i) codes[i] = (uint8_t)(out[(i - base) >> 2] >> (8 * ((i - base) & 3)));
        }
    }
}

// One lane per (read, word); the lane of a row's last word also zeroes the row padding (words W*P ..
// row stride), so the rows need no clearing beforehand.
template <int P>
__global__ void pack_planes_kernel(const uint8_t* __restrict__ codes, const int64_t* __restrict__ off,
                                   const int32_t* __restrict__ len, int32_t n_reads, int32_t w,
                                   int32_t srow, int32_t trow, uint32_t* __restrict__ sfx,
                                   uint32_t* __restrict__ pfx) {
    int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)n_reads * w;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (; gid < total; gid += stride) {
        const int32_t r = (int32_t)(gid / w);
        const int32_t k = (int32_t)(gid % w);
        const int32_t n = len[r];
        const uint8_t* s = codes + off[r];
        uint32_t pl[P], sl[P];
#pragma unroll
        for (int p = 0; p < P; ++p) { pl[p] = 0u; sl[p] = 0u; }
        const int32_t shift = 32 * w - n;  // suffix layout: base i sits at position shift + i
        for (int b = 0; b < 32; ++b) {
            const int32_t i = 32 * k + b;      // prefix layout
            if (i < n) {
                const uint32_t c = s[i];
#pragma unroll
                for (int p = 0; p < P; ++p) pl[p] |= ((c >> p) & 1u) << b;
            }
            const int32_t u = i - shift;       // suffix layout
            if (u >= 0 && u < n) {
                const uint32_t c = s[u];
#pragma unroll
                for (int p = 0; p < P; ++p) sl[p] |= ((c >> p) & 1u) << b;
            }
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
            pfx[(int64_t)r * trow + k * P + p] = pl[p];
            sfx[(int64_t)r * srow + k * P + p] = sl[p];
        }
        if (k == w - 1) {
            for (int32_t q = w * P; q < trow; ++q) pfx[(int64_t)r * trow + q] = 0u;
            for (int32_t q = w * P; q < srow; ++q) sfx[(int64_t)r * srow + q] = 0u;
        }
    }
}

// ----------------------------------------------------------------------------- ungapped

// (score, end) keys: key = score * 2^B - j, positive iff score > 0; the larger
// score wins, then the smaller j -- exactly the strict '>' first-argmax scan of
// aligners.py:54-57, which starts from dp[n][0] = 0 (so key <= 0 means (0, 0)).
template <int KM>
struct Key;

template <>
struct Key<0> {  // int32 keys, B = 16: needs |score| < 2^15 and j < 2^16
    using T = int32_t;
    __device__ static T make(int32_t score, int32_t j) { return (int32_t)((uint32_t)score << 16) - j; }
    // uniform pairs: key = X * (dms << 16) + j * ((match << 16) - 1), one v_mad_i32_i24
    __device__ static T make_folded(uint32_t X, int32_t d2, int32_t kj) {
        const int32_t xs = ((int32_t)X << 8) >> 8;   // both factors provably 24-bit:
        const int32_t ds = (d2 << 8) >> 8;           // one v_mad_i32_i24
        return xs * ds + kj;
    }
    __device__ static void decode(T key, int32_t& score, int32_t& end) {
        score = key > 0 ? (key + 0xFFFF) >> 16 : 0;
        end = key > 0 ? (int32_t)((uint32_t)score << 16) - key : 0;
    }
};

template <>
struct Key<1> {  // int64 keys, B = 32: any int32 score
    using T = int64_t;
    __device__ static T make(int32_t score, int32_t j) { return (int64_t)score * 4294967296ll - j; }
    __device__ static void decode(T key, int32_t& score, int32_t& end) {
        score = key > 0 ? (int32_t)((key + 0xFFFFFFFFll) >> 32) : 0;
        end = key > 0 ? (int32_t)((int64_t)score * 4294967296ll - key) : 0;
    }
};

template <int N>
__device__ __forceinline__ void load_words(const uint32_t* __restrict__ src, uint32_t (&dst)[N]) {
    static_assert(N % 4 == 0, "rows are padded to 16 bytes");
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + 4 * q);
        dst[4 * q + 0] = v.x; dst[4 * q + 1] = v.y; dst[4 * q + 2] = v.z; dst[4 * q + 3] = v.w;
    }
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

template <typename T>
__device__ __forceinline__ T group_max(T best, int ppw) {
    // combine the RS lanes of a pair (lanes slot, slot + ppw, ...): across rows (offsets 32, 16) with
    // ds_bpermute, inside a 16-lane row with DPP row rotations (offsets 8, 4, 2, 1 reach the same lanes
    // as xor for a max, as one VALU op each instead of an LDS round trip)
    auto xchg = [&](T v, auto off_tag) -> T {
        constexpr int OFF = decltype(off_tag)::value;
        auto one = [&](int x) -> int {
            if constexpr (OFF >= 16) return __shfl_xor(x, OFF, 64);
            else return __builtin_amdgcn_update_dpp(x, x, 0x120 + OFF, 0xF, 0xF, false);  // row_ror:OFF
        };
        if constexpr (sizeof(T) == 4) {
            return (T)one((int)v);
        } else {
            const uint32_t lo = (uint32_t)one((int)(uint32_t)v);
            const uint32_t hi = (uint32_t)one((int)(uint32_t)((uint64_t)v >> 32));
            return (T)(((uint64_t)hi << 32) | lo);
        }
    };
    auto step = [&](auto off_tag) {
        if (ppw <= decltype(off_tag)::value) {
            const T o = xchg(best, off_tag);
            best = o > best ? o : best;
        }
    };
    step(std::integral_constant<int, 32>{});
    step(std::integral_constant<int, 16>{});
    step(std::integral_constant<int, 8>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 1>{});
    return best;
}

// Bit-shift body shared by both ungapped kernels.
//
// Coordinates: s is right-aligned in W words (s' position 32W - n + i holds
// base i) and t is left-aligned behind W zero words (t'' position 32W + u holds
// base u).  For end position j (aligners.py:54 scans j = 0..m of the last row),
// s' position x meets t'' position x + j.  With j = 32q + r, s' word k meets the
// funnel-shifted t'' word T_r[k + q] = bits [32(k+q) + r, 32(k+q) + r + 32) of t''.
// Words k < W-1-q only meet t padding; T_r[W-1] is partly padding (bits < 32-r).
// X(j) = popcount of OR_p(S_p ^ T_p) over the valid bits, and
//   dp[n][j] = match * L + (mismatch - match) * X,   L = min(n, j)
// whenever gaps cannot win.  T_r is built once per r and
// reused for every q, so the inner loop is xor / bitop3 / popcount with
// compile-time register indices.
//
// UNI (uniform pairs, n = m = lw = lmax): j <= n always, so L = j, the window never
// reaches s padding (no per-lane mask) and the key folds to one mad24.
template <int P, int W, int KM, bool UNI, bool RS1 = false>
__device__ __forceinline__ typename Key<KM>::T sweep_shifts(const uint32_t* Sw, const uint32_t* Tw,
                                                            const uint32_t* SV, int32_t n, int32_t m,
                                                            int32_t jmax, int r0, int rs_log2,
                                                            int32_t match, int32_t dms) {
    using T = typename Key<KM>::T;
    constexpr int TW = W + 1;
    const int RS = RS1 ? 1 : 1 << rs_log2;
    const int32_t d2 = (int32_t)((uint32_t)dms << 16);
    const int32_t m2 = (int32_t)((uint32_t)match << 16) - 1;
    T best = 0;
    for (int it = 0; it < (RS1 ? 32 : (32 >> rs_log2)); ++it) {
        // RS1: one lane per pair, every lane of the wavefront is on the same bit
        // shift, so r and everything derived from it is scalar (SGPR)
        const uint32_t r = RS1 ? (uint32_t)it : (uint32_t)(r0 + it * RS);
        const int rmin = it * RS;                 // smallest / largest r in the wavefront
        const int rmax = rmin + RS - 1;
        if (rmin > jmax) break;                   // j = r > jmax for every lane
        const uint32_t vt = r ? (0xFFFFFFFFu << (32u - r)) : 0u;  // valid bits of T_r[W-1]
        // U[i] = T_r[W - 1 + i], i = 0..W   (T_r[W-1] takes its low word from zero padding)
        uint32_t U[TW][P];
#pragma unroll
        for (int i = 0; i < TW; ++i) {
#pragma unroll
            for (int c = 0; c < P; ++c) {
                const uint32_t hi = i < W ? Tw[i * P + c] : 0u;  // t word W is zero (m <= 32W)
                const uint32_t lo = i ? Tw[(i - 1) * P + c] : 0u;
                U[i][c] = alignbit(hi, lo, r);
            }
        }
        const int32_t kr = (int32_t)r * m2;
#pragma unroll
        for (int q = 0; q <= W; ++q) {
            if (32 * q + rmin > jmax) break;      // wave-uniform
            const int32_t j = 32 * q + (int32_t)r;
            uint32_t X = 0;
#pragma unroll
            for (int k = (W - 1 - q > 0 ? W - 1 - q : 0); k < W; ++k) {
                const int i = k + q - (W - 1);    // U index
                // mismatch word: OR over planes of (S ^ T); v_bitop3 LUT 0xBE = (a ^ b) | c
                uint32_t mm = Sw[k * P] ^ U[i][0];
#pragma unroll
                for (int c = 1; c < P; ++c) mm = __builtin_amdgcn_bitop3_b32(Sw[k * P + c], U[i][c], mm, 0xBE);
                if (i == 0) mm &= vt;
                if constexpr (!UNI) mm &= SV[k];
                X += (uint32_t)__builtin_popcount(mm);
            }
            T key;
            if constexpr (UNI && KM == 0) {
                key = Key<0>::make_folded(X, d2, kr + 32 * q * m2);
            } else if constexpr (KM == 0) {
                // key = L * (match << 16) + X * (dms << 16) - j with two v_mad_i32_i24
                // (v_mul_lo_u32 is quarter rate); host guarantees |match|, |dms| < 128
                const int32_t L = n < j ? n : j;
                const int32_t m16 = (int32_t)((uint32_t)match << 16);
                const int32_t xs = ((int32_t)X << 8) >> 8, ls = (L << 8) >> 8;
                key = ls * ((m16 << 8) >> 8) + (xs * ((d2 << 8) >> 8) - j);
            } else {
                const int32_t L = n < j ? n : j;
                key = Key<KM>::make(match * L + dms * (int32_t)X, j);
            }
            if constexpr (UNI && RS1) {
                if (j <= jmax) best = key > best ? key : best;   // scalar condition
            } else if (UNI && 32 * q + rmax <= jmax) {
                best = key > best ? key : best;   // every lane's j is in range
            } else {
                best = (j <= m && key > best) ? key : best;
            }
        }
    }
    return best;
}

// Sweep for uniform pairs (n = m = lw, P = 2, one lane per pair): every lane of
// the wavefront is on the same bit shift r, so r-derived values are scalar and
// no per-lane masking is needed (j <= lw = n means L = j and the window never
// reaches s padding).  Blocks q <= W-2 are always in range; block W-1 holds
// j = 32(W-1) + r <= lw iff r <= rcut = lw - 32(W-1); block W only j = 32W
// (r = 0, lw = 32W).  The r loop is split on rcut, so no end position needs a
// branch.  Per block q the running max is kept without its q-constant
// (key = keyq + 32q*M', M' = (match << 16) - 1), so an end position costs one
// v_mad_i32_i24 and one v_max.
//
// t-truncated pairs (n = lw, m < lw: read b cut at the genome end, generateErrorFreeReads.py:45-46) ride
// the same sweep: their end positions j <= m compare only real t bases, so their keys are the uniform
// keys, and only j > m must be dropped.  Blocks q < m/32 are always valid, blocks above m/32 never;
// block qm = m/32 is valid for r <= m % 32, so the lane snapshots best[qm] right after shift r = m % 32.
// tmask (scalar) has bit r set iff some lane of the wavefront snapshots at shift r, so a step takes the
// snapshot branch only on those shifts; tm = m for a t-truncated lane, -1 otherwise.
template <int W, int KM>
__device__ __forceinline__ typename Key<KM>::T sweep_uniform(const uint32_t* Sw, const uint32_t* Tw, int32_t lw,
                                                             int32_t match, int32_t dms, uint32_t r_lo,
                                                             uint32_t r_hi, uint32_t tmask = 0u,
                                                             int32_t tm = -1) {
    using T = typename Key<KM>::T;
    constexpr int P = 2;
    constexpr int TW = W + 1;
    const int32_t rcut = lw - 32 * (W - 1);  // 1..32
    T best[W + 1];
    T qoff[W + 1];
    T mq;  // M' as T
    if constexpr (KM == 0) {
        mq = (int32_t)((uint32_t)match << 16) - 1;
    } else {
        mq = (int64_t)match * 4294967296ll - 1;
    }
#pragma unroll
    for (int q = 0; q <= W; ++q) {
        qoff[q] = (T)(32 * q) * mq;
        best[q] = -qoff[q];  // "key <= 0" for block q
    }
    const int32_t d16 = (int32_t)((uint32_t)dms << 16);
    // the mismatch factor in a VGPR: v_mad_i32_i24 then reads only one SGPR (the scalar row offset
    // rm), within gfx9's one-scalar operand limit, and needs no per-shift v_mov of rm
    int32_t dv;
    {
        const int32_t ds = (__builtin_amdgcn_readfirstlane(d16) << 8) >> 8;
        asm volatile("v_mov_b32 %0, %1" : "=v"(dv) : "s"(ds));
    }
    // keys of one r over blocks [0, NQ) (NQ compile-time), r scalar
    auto keys = [&](uint32_t r, uint32_t vt, T rm, auto nq_tag, T (&kq)[W + 1]) {
        constexpr int NQ = decltype(nq_tag)::value;
        uint32_t U[TW][P];
#pragma unroll
        for (int i = 0; i < TW; ++i) {
            if (i < NQ || (NQ > W && i <= W)) {
#pragma unroll
                for (int c = 0; c < P; ++c) {
                    const uint32_t hi = i < W ? Tw[i * P + c] : 0u;  // t word W is zero (m <= 32W)
                    const uint32_t lo = i ? Tw[(i - 1) * P + c] : 0u;
                    U[i][c] = alignbit(hi, lo, r);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            uint32_t X = 0;
#pragma unroll
            for (int k = (W - 1 - q > 0 ? W - 1 - q : 0); k < W; ++k) {
                const int i = k + q - (W - 1);
                uint32_t mm = __builtin_amdgcn_bitop3_b32(Sw[k * P + 1], U[i][1], Sw[k * P] ^ U[i][0], 0xBE);
                if (i == 0) mm &= vt;
                X = k == (W - 1 - q > 0 ? W - 1 - q : 0) ? (uint32_t)__builtin_popcount(mm) : bcnt_acc(mm, X);
            }
            if constexpr (KM == 0) {
                kq[q] = ((((int32_t)X << 8) >> 8) * ((dv << 8) >> 8)) + rm;    // v_mad_i32_i24 (dv: 24-bit)
            } else {
                kq[q] = (int64_t)dms * 4294967296ll * (int64_t)X + rm;
            }
        }
    };
    // the same keys for r >= 1 with s shifted down by 32 - r instead of t up by it (the same base pairs
    // meet): the word shifted in from above is zero, so the top word of s is one v_lshrrev (fast class)
    // where t's bottom word needed a v_alignbit with zero (slow class).  Compared positions end inside
    // s word W-1 (its low r bits, mask vt = ~0 >> (32 - r)); block q pairs shifted s word k with t word
    // k - (W-1-q).  NQ <= W (block W only at r = 0).
    auto keys_s = [&](uint32_t r, uint32_t vt, T rm, auto nq_tag, T (&kq)[W + 1]) {
        constexpr int NQ = decltype(nq_tag)::value;
        static_assert(NQ <= W, "keys_s: r >= 1 has at most W blocks");
        const uint32_t sg = 32u - r;  // 1..31
        uint32_t V[W][P];
#pragma unroll
        for (int k = W - NQ; k < W; ++k) {
#pragma unroll
            for (int c = 0; c < P; ++c)
                V[k][c] = k < W - 1 ? alignbit(Sw[(k + 1) * P + c], Sw[k * P + c], sg) : Sw[k * P + c] >> sg;
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            uint32_t X = 0;
#pragma unroll
            for (int k = W - 1 - q; k < W; ++k) {
                const int i = k - (W - 1 - q);
                uint32_t mm = __builtin_amdgcn_bitop3_b32(V[k][1], Tw[i * P + 1], V[k][0] ^ Tw[i * P], 0xBE);
                if (k == W - 1) mm &= vt;
                X = k == W - 1 - q ? (uint32_t)__builtin_popcount(mm) : bcnt_acc(mm, X);
            }
            if constexpr (KM == 0) {
                kq[q] = ((((int32_t)X << 8) >> 8) * ((dv << 8) >> 8)) + rm;    // v_mad_i32_i24 (dv: 24-bit)
            } else {
                kq[q] = (int64_t)dms * 4294967296ll * (int64_t)X + rm;
            }
        }
    };
    // r = 0 (t unshifted, block W when lw = 32W) through keys; r >= 1 through keys_s for W <= 4 (A/B on
    // one box: cfg2 -0.7 %, target -0.4 %; at W = 5, cfg3, +1.3 %, so W >= 5 kept the t shift) -- and with
    // two shifts per shifted row for every W (cfg3, W = 5: 191 against 194-197 us with the t shift; cfg5's
    // default scoring, W = 8: 445-449 against 448-452 us, and W = 6 no longer spills; three interleaved passes
    // each, profiles/r03_shift_s_w5_ab.json, r03_shift_s_w8_ab.json)
    constexpr bool SHIFT_S = W <= OVL_SHIFT_S_MAXW;
    // Two shifts from one shifted s (keys_s2): s shifted down by 31 - r serves shift r + 1 against t as it
    // is and shift r against t moved up one bit (Tup, built once per pair), so a step of two shifts shifts
    // s once.  In Tup, bit 0 of word 0 is t position -1 (no base): that bit of a block's bottom word is
    // masked out (one v_and for blocks q >= 1; folded into the top-word mask for q = 0).
    constexpr bool PAIR = SHIFT_S && KM == 0 && OVL_SHIFT_PAIR;
    uint32_t Tup[PAIR ? W : 1][P];
    if constexpr (PAIR) {
#pragma unroll
        for (int i = 0; i < W; ++i) {
#pragma unroll
            for (int c = 0; c < P; ++c) Tup[i][c] = alignbit(Tw[i * P + c], i ? Tw[(i - 1) * P + c] : 0u, 31u);
        }
    }
    // The same for the t shift (W > OVL_SHIFT_S_MAXW, keys_t2): t shifted up by r + 1 serves shift r + 1
    // against s as it is and shift r against s moved down one bit (Sdn); bit 31 of Sdn's word W-1 is position
    // 32W (no base): that bit of a block's top word is masked out.
    constexpr bool PAIR_T = !SHIFT_S && KM == 0 && OVL_SHIFT_PAIR;
    uint32_t Sdn[PAIR_T ? W : 1][P];
    if constexpr (PAIR_T) {
#pragma unroll
        for (int k = 0; k < W; ++k) {
#pragma unroll
            for (int c = 0; c < P; ++c)
                Sdn[k][c] = k < W - 1 ? alignbit(Sw[(k + 1) * P + c], Sw[k * P + c], 1u) : Sw[k * P + c] >> 1;
        }
    }
    auto keys_t2 = [&](uint32_t r, T rm, auto nq_tag, T (&k0)[W + 1], T (&k1)[W + 1]) {
        constexpr int NQ = decltype(nq_tag)::value;
        static_assert(NQ <= W, "keys_t2: r >= 1 has at most W blocks");
        const uint32_t r1 = r + 1;                                // 2..31
        const uint32_t vt = (uint32_t)((int32_t)0x80000000 >> r);  // U[0]: its top r + 1 bits hold bases
        uint32_t U[W][P];
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
#pragma unroll
            for (int c = 0; c < P; ++c) U[i][c] = alignbit(Tw[i * P + c], i ? Tw[(i - 1) * P + c] : 0u, r1);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            uint32_t X0 = 0, X1 = 0;
#pragma unroll
            for (int k = W - 1 - q; k < W; ++k) {
                const int i = k + q - (W - 1);
                uint32_t m1 = __builtin_amdgcn_bitop3_b32(Sw[k * P + 1], U[i][1], Sw[k * P] ^ U[i][0], 0xBE);
                uint32_t m0 = __builtin_amdgcn_bitop3_b32(Sdn[k][1], U[i][1], Sdn[k][0] ^ U[i][0], 0xBE);
                if (i == 0) {
                    m1 &= vt;
                    m0 &= k == W - 1 ? (vt & 0x7FFFFFFFu) : vt;
                } else if (k == W - 1) {
                    m0 &= 0x7FFFFFFFu;
                }
                const bool first = k == W - 1 - q;
                X1 = first ? (uint32_t)__builtin_popcount(m1) : bcnt_acc(m1, X1);
                X0 = first ? (uint32_t)__builtin_popcount(m0) : bcnt_acc(m0, X0);
            }
            k0[q] = ((((int32_t)X0 << 8) >> 8) * ((dv << 8) >> 8)) + rm;
            k1[q] = ((((int32_t)X1 << 8) >> 8) * ((dv << 8) >> 8)) + (rm + mq);
        }
    };
    auto keys_s2 = [&](uint32_t r, T rm, auto nq_tag, T (&k0)[W + 1], T (&k1)[W + 1]) {
        constexpr int NQ = decltype(nq_tag)::value;
        static_assert(NQ <= W, "keys_s2: r >= 1 has at most W blocks");
        const uint32_t sg = 31u - r;                  // 1..30 (r + 1 <= 31)
        const uint32_t vt = 0xFFFFFFFFu >> sg;        // s word W-1: its low r + 1 bits hold bases
        uint32_t V[W][P];
#pragma unroll
        for (int k = W - NQ; k < W; ++k) {
#pragma unroll
            for (int c = 0; c < P; ++c)
                V[k][c] = k < W - 1 ? alignbit(Sw[(k + 1) * P + c], Sw[k * P + c], sg) : Sw[k * P + c] >> sg;
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            uint32_t X0 = 0, X1 = 0;
#pragma unroll
            for (int k = W - 1 - q; k < W; ++k) {
                const int i = k - (W - 1 - q);
                uint32_t m1 = __builtin_amdgcn_bitop3_b32(V[k][1], Tw[i * P + 1], V[k][0] ^ Tw[i * P], 0xBE);
                uint32_t m0 = __builtin_amdgcn_bitop3_b32(V[k][1], Tup[i][1], V[k][0] ^ Tup[i][0], 0xBE);
                if (k == W - 1) {
                    m1 &= vt;
                    m0 &= i == 0 ? (vt & ~1u) : vt;
                } else if (i == 0) {
                    m0 &= ~1u;
                }
                const bool first = k == W - 1 - q;
                X1 = first ? (uint32_t)__builtin_popcount(m1) : bcnt_acc(m1, X1);
                X0 = first ? (uint32_t)__builtin_popcount(m0) : bcnt_acc(m0, X0);
            }
            k0[q] = ((((int32_t)X0 << 8) >> 8) * ((dv << 8) >> 8)) + rm;
            k1[q] = ((((int32_t)X1 << 8) >> 8) * ((dv << 8) >> 8)) + (rm + mq);
        }
    };
    // t-truncated lanes: the best key of blocks 0..qm as they stand after shift m % 32 (block qm's last
    // valid end position).  A max under "q <= qm" masks, not a select on "q == qm": the compiler turns
    // an equality select chain into an indexed table, and the block maxima into an LDS array.
    T snap = 0;
    auto snapshot = [&](uint32_t r) {
        if (tm >= 0 && (uint32_t)(tm & 31) == r) {
            const int32_t qm = tm >> 5;
            T v = best[0] + qoff[0];
#pragma unroll
            for (int q = 1; q < W; ++q) {
                const T k = best[q] + qoff[q];
                v = q <= qm && k > v ? k : v;
            }
            snap = v;
        }
    };
    auto body = [&](uint32_t r, uint32_t vt, T rm, auto nq_tag) {
        constexpr int NQ = decltype(nq_tag)::value;
        T kq[W + 1];
        if constexpr (NQ > W || !SHIFT_S) {
            keys(r, vt, rm, nq_tag, kq);
        } else {
            if (r == 0) keys(r, vt, rm, nq_tag, kq);
            else keys_s(r, 0xFFFFFFFFu >> (32u - r), rm, nq_tag, kq);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) best[q] = kq[q] > best[q] ? kq[q] : best[q];
        if ((tmask >> r) & 1u) snapshot(r);  // scalar branch
    };
    // two consecutive r per step: per block one 3-way max (v_max3_i32) for both keys
    auto body2 = [&](uint32_t r, T rm, auto nq_tag) {
        constexpr int NQ = decltype(nq_tag)::value;
        T k0[W + 1], k1[W + 1];
        if constexpr (PAIR) {
            keys_s2(r, rm, nq_tag, k0, k1);
        } else if constexpr (PAIR_T) {
            keys_t2(r, rm, nq_tag, k0, k1);
        } else if constexpr (SHIFT_S) {
            keys_s(r, 0xFFFFFFFFu >> (32u - r), rm, nq_tag, k0);
            keys_s(r + 1, 0xFFFFFFFFu >> (31u - r), rm + mq, nq_tag, k1);
        } else {
            keys(r, (uint32_t)((int32_t)0x80000000 >> (r - 1)), rm, nq_tag, k0);
            keys(r + 1, (uint32_t)((int32_t)0x80000000 >> r), rm + mq, nq_tag, k1);
        }
        // scalar branch: a lane snapshots after r or r + 1, from the block maxima before this step's
        // update (kept apart from it, so the update stays one v_max3_i32 per block)
        if ((tmask >> r) & 3u) {
            const uint32_t d = (uint32_t)(tm & 31) - r;
            if (tm >= 0 && d <= 1u) {
                const int32_t qm = tm >> 5;
                T v = 0;
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    T k = best[q];
                    if (q < NQ) {
                        const T kk = d ? (k0[q] > k1[q] ? k0[q] : k1[q]) : k0[q];
                        k = kk > k ? kk : k;
                    }
                    k += qoff[q];
                    v = q <= qm && k > v ? k : v;
                }
                snap = v;
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const T m01 = k0[q] > k1[q] ? k0[q] : k1[q];
            best[q] = m01 > best[q] ? m01 : best[q];
        }
    };
    // r = 0: j = 32q (q >= 1); block W only when lw == 32W
    if (r_lo == 0) {
        T rm0 = 0;
        if (rcut == 32) {
            body(0u, 0u, rm0, std::integral_constant<int, W + 1>{});
        } else {
            body(0u, 0u, rm0, std::integral_constant<int, W>{});
        }
    }
    uint32_t r = r_lo > 1 ? r_lo : 1;
    T rm = (T)r * mq;
    const uint32_t rc = (uint32_t)(rcut < 31 ? rcut : 31);
    const uint32_t ra = rc < r_hi - 1 ? rc : r_hi - 1;
    // (int64 keys have no 3-way max and no registers to spare: one r per step)
    for (; KM == 0 && r + 1 <= ra; r += 2) {  // blocks 0..W-1, two r per step
        body2(r, rm, std::integral_constant<int, W>{});
        rm += 2 * mq;
    }
    for (; KM != 0 && r < ra; ++r) {
        body(r, (uint32_t)((int32_t)0x80000000 >> (r - 1)), rm, std::integral_constant<int, W>{});
        rm += mq;
    }
    if (r <= ra) {
        body(r, (uint32_t)((int32_t)0x80000000 >> (r - 1)), rm, std::integral_constant<int, W>{});
        ++r;
        rm += mq;
    }
    for (; KM == 0 && r + 1 < r_hi; r += 2) {  // blocks 0..W-2, two r per step
        body2(r, rm, std::integral_constant<int, W - 1>{});
        rm += 2 * mq;
    }
    for (; KM != 0 && r + 1 < r_hi; ++r) {
        body(r, (uint32_t)((int32_t)0x80000000 >> (r - 1)), rm, std::integral_constant<int, W - 1>{});
        rm += mq;
    }
    if (r < r_hi) {
        body(r, (uint32_t)((int32_t)0x80000000 >> (r - 1)), rm, std::integral_constant<int, W - 1>{});
        ++r;
        rm += mq;
    }
    T out = 0;
#pragma unroll
    for (int q = 0; q <= W; ++q) {
        const T k = best[q] + qoff[q];
        out = k > out ? k : out;
    }
    if (tm >= 0) {  // t-truncated: blocks below qm whole, block qm up to its snapshot
        const int32_t qm = tm >> 5;
        T t = snap > 0 ? snap : 0;
#pragma unroll
        for (int q = 0; q < W - 1; ++q) {
            const T k = best[q] + qoff[q];
            t = q < qm && k > t ? k : t;
        }
        out = t;
    }
    return out;
}

// Read a inside b's window (a lane of uniform_kernel's sweep whose read a is shorter than b, n < m): the end
// positions j in (n, m] compare all n bases of a with t[j - n, j) (L = n), which the sweep's shifts do not
// see.  j is wave-uniform -- the loop runs it from jhi down to jlo, the bounds over the wave's such lanes --
// and each lane keeps the keys of its own range.  In the rows, s base i sits at position 32W - n + i (suffix
// layout) and t base i at position i (prefix layout), so t shifted up by 32W - j puts t[j - n + i] on s base
// i; the shifted t moves up one bit per step (one v_alignbit per word and plane), and the s-padding
// positions below 32W - n are masked out.  Returns the best key of the lane's range (INT32_MIN if empty).
template <int W>
__device__ __forceinline__ int32_t window_keys(const uint32_t* Sw, const uint32_t* Tw, int32_t n, int32_t m,
                                            int32_t jlo, int32_t jhi, int32_t match, int32_t dms) {
    constexpr int P = 2;
    uint32_t SV[W];  // valid s bits: positions >= 32W - n
    const int32_t s0 = 32 * W - n;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const int32_t lo = 32 * k;
        SV[k] = s0 <= lo ? ~0u : (s0 >= lo + 32 ? 0u : (~0u << (uint32_t)(s0 - lo)));
    }
    // t shifted up by sh0 = 32W - jhi (wave-uniform: word shift ws, bit shift bs)
    const int32_t sh0 = 32 * W - jhi;
    const int ws = sh0 >> 5, bs = sh0 & 31;
    uint32_t U[W][P];
#pragma unroll
    for (int k = 0; k < W; ++k) {
#pragma unroll
        for (int c = 0; c < P; ++c) {
            uint32_t hi = 0u, lo = 0u;
#pragma unroll
            for (int q = 0; q < W; ++q) {  // (scalar select on ws: no dynamic register indexing)
                if (q == ws) {
                    hi = k - q >= 0 ? Tw[(k - q) * P + c] : 0u;
                    lo = k - q - 1 >= 0 ? Tw[(k - q - 1) * P + c] : 0u;
                }
            }
            U[k][c] = bs ? alignbit(hi, lo, 32u - (uint32_t)bs) : hi;
        }
    }
    const int32_t d16 = (int32_t)((uint32_t)dms << 16);
    const int32_t kn = (int32_t)((uint32_t)(match * n) << 16);
    int32_t best = INT32_MIN;
    for (int32_t j = jhi; j >= jlo; --j) {
        uint32_t X = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const uint32_t mm = __builtin_amdgcn_bitop3_b32(Sw[k * P + 1], U[k][1], Sw[k * P] ^ U[k][0], 0xBE) & SV[k];
            X = bcnt_acc(mm, X);
        }
        const int32_t key = (int32_t)X * d16 + (kn - j);
        if (j > n && j <= m && key > best) best = key;
        // j - 1: t one bit further up
#pragma unroll
        for (int k = W - 1; k >= 0; --k) {
#pragma unroll
            for (int c = 0; c < P; ++c) U[k][c] = alignbit(U[k][c], k ? U[k - 1][c] : 0u, 31u);
        }
    }
    return best;
}

// One general-path unit: up to 64/RS pairs, RS = 2^rs_log2 lanes per pair (lanes
// slot, slot + 64/RS, ...; lane group g sweeps r = g, g + RS, ...), any lengths
// <= 32W, per-lane masks.  Writes (score, end), or (-1, -1) for a bad index.
// score one pair per group of 2^rs_log2 lanes from its rows already in registers
// (n, m = lengths; ok = valid pair); returns the pair's best key on every lane of the group
template <int P, int W, int KM>
__device__ __forceinline__ typename Key<KM>::T general_core(bool ok, int32_t n, int32_t m, const uint32_t* Sw,
                                                            const uint32_t* Tw, int r0, int rs_log2, int32_t jbound,
                                                            int32_t match, int32_t mismatch) {
    if (!ok) { n = 0; m = 0; }
    uint32_t SV[W];  // valid bits of s' word k: positions >= 32W - n
    const int pad = 32 * W - n;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const int lo = pad - 32 * k;
        SV[k] = lo <= 0 ? 0xFFFFFFFFu : (lo >= 32 ? 0u : (0xFFFFFFFFu << lo));
    }
    // wave-uniform bound on end positions: the caller's (lmax) or the wave max of m
    const int jmax = jbound > 0 ? jbound : wave_max_i32(m);
    const auto best = sweep_shifts<P, W, KM, false>(Sw, Tw, SV, n, m, jmax, r0, rs_log2, match, mismatch - match);
    return group_max(best, 64 >> rs_log2);
}

template <int P, int W, int KM, int OM = 0>
__device__ __forceinline__ void general_unit(bool mine, int64_t p, int32_t a, int32_t b,
                                             const uint32_t* __restrict__ sfx, const uint32_t* __restrict__ pfx,
                                             const int32_t* __restrict__ len, int32_t n_reads, int r0,
                                             int rs_log2, int32_t jbound, int32_t match, int32_t mismatch,
                                             int32_t* __restrict__ out_score, int32_t* __restrict__ out_end,
                                             uint32_t* __restrict__ err_flag) {
    constexpr int SROW = (W * P + 3) & ~3;
    constexpr int TROW = (W * P + 3) & ~3;
    bool ok = mine && a >= 0 && a < n_reads && b >= 0 && b < n_reads;
    if (!ok) { a = 0; b = 0; }
    int32_t n = len[a], m = len[b];
    ok = ok && n <= 32 * W && m <= 32 * W;
    if (mine && !ok && r0 == 0) ovl_flag_error(err_flag);
    uint32_t Sw[SROW], Tw[TROW];
    load_words<SROW>(sfx + (int64_t)a * SROW, Sw);
    load_words<TROW>(pfx + (int64_t)b * TROW, Tw);
    const auto full = general_core<P, W, KM>(ok, n, m, Sw, Tw, r0, rs_log2, jbound, match, mismatch);
    if (mine && r0 == 0) {
        int32_t sc, en;
        Key<KM>::decode(full, sc, en);
        put_pair<OM>(out_score, out_end, p, ok ? sc : -1, ok ? en : -1, n, match, pack_inv(match, mismatch));
    }
}

// Uniform-pair kernel (P = 2 bit planes, reads of one length lw = lmax, the
// common case of simulated reads).  One lane per pair, so every lane of a
// wavefront sweeps the same bit shift r (scalar).  Pairs that are not (lw, lw)
// -- e.g. reads truncated at the genome end (generateErrorFreeReads.py:45-46) --
// are "side pairs", scored by the general path with 4, 8 or 16 lanes per pair:
//  - throughput mode (LAT = false): one wavefront per tile; side pairs are queued
//    as (p, a, b) in the wavefront's LDS ring and scored whenever 16 are waiting,
//    and once at the end;
//  - latency mode (LAT = true, about one tile per wavefront slot): two wavefronts
//    per tile running concurrently -- role 0 sweeps the uniform pairs, role 1
//    loads lengths and rows in the round trip after the indices, restages its
//    side pairs through LDS into the 4/8/16-lane layout and scores them -- so the
//    side work overlaps the sweep instead of trailing it.
// waves per SIMD the kernel is compiled for (VGPR budget 512 / occupancy): the
// most that fits without spilling
#ifndef OVL_UNI_OCC_W78
#define OVL_UNI_OCC_W78 4  // (build macro for A/B builds: int32-key waves per SIMD at W = 7, 8)
#endif
#define UNI_OCC(W, KM) ((KM) == 0 ? ((W) <= 4 ? 8 : ((W) <= 5 ? 7 : ((W) <= 6 ? 6 : OVL_UNI_OCC_W78))) \
                                  : ((W) <= 4 ? 7 : ((W) <= 5 ? 6 : ((W) <= 6 ? 5 : 4))))
// IX: the pair list is read in its compact encoding (b = ix_b16[p], 0xFFFF a bad index; a = ix_base[tile] +
// ix_d8[p]), which the copy engine moved into HBM beside the previous chunk's launch (3 bytes per pair plus 4 per
// tile over the link; ovl_api.cpp encode_chunk / issue_chunk): no decode launch before it.
template <int W, int KM, bool LAT, int OM, bool IX = false>
__global__ __launch_bounds__(256, UNI_OCC(W, KM)) void uniform_kernel(
    const uint32_t* __restrict__ sfx, const uint32_t* __restrict__ pfx, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx, int64_t n_pairs,
    int32_t lw, const uint32_t* __restrict__ full, int32_t match, int32_t mismatch,
    int32_t* __restrict__ out_score, int32_t* __restrict__ out_end, uint32_t* __restrict__ err_flag,
    const int32_t* __restrict__ heavy_ids, const uint8_t* __restrict__ tile_flags, int32_t heavy_n,
    int64_t tile_base, const uint16_t* __restrict__ ix_b16, const uint8_t* __restrict__ ix_d8,
    const int32_t* __restrict__ ix_base) {
    using T = typename Key<KM>::T;
    constexpr int P = 2;
    constexpr int SROW = (W * P + 3) & ~3;
    constexpr int TROW = (W * P + 3) & ~3;
    // t-truncated pairs in the sweep (snapshot): throughput mode with int32 keys.  Not in latency mode,
    // where the side wave scores them concurrently and the sweep is the critical path (A/B, cfg2:
    // 8.2 -> 9.0 us with them in the sweep)
    constexpr bool TT = KM == 0 && !LAT;
    constexpr int RING = 128;                      // >= 15 left over + 64 from one tile
    constexpr int ROWQ = (SROW + TROW) / 4;        // uint4 per staged side pair (latency mode)
    __shared__ int4 ring_all[LAT ? 1 : 4][RING];   // throughput mode: 8 KiB per block
    __shared__ int4 side_ent[LAT ? 2 : 1][64];     // latency mode: (p, -, n, m) per side pair
    __shared__ uint4 side_rows[LAT ? 2 * 64 * ROWQ : 1];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;              // wavefront in block
    // latency mode: 0 = sweep, 1 = side pairs; the side wave is the first of each pair in the block
    // (A/B with its drain at priority 1: cfg2 8.40 -> 8.33 us; without the priority 8.85 us)
    const int role = LAT ? ((wib & 1) ^ 1) : 0;
    constexpr int G = LAT ? 2 : 4;                 // tiles per block per iteration
    const int grp = LAT ? (wib >> 1) : wib;
    int4* ring = ring_all[LAT ? 0 : wib];
    const int64_t n_tiles = (n_pairs + 63) >> 6;
    int head = 0, tail = 0;                        // wave-uniform ring cursors
    // score ring[head .. head + count), count <= 16, with 64/count-ish lanes per pair:
    // 4 lanes (16 pairs), 8 lanes (<= 8), 16 lanes (<= 4) or 32 lanes (<= 2): shortest serial r loop
    auto drain = [&](int count) {
        const int rs = count > 8 ? 2 : (count > 4 ? 3 : (count > 2 ? 4 : 5));   // log2(lanes per pair)
        const int ppw = 64 >> rs;
        const int slot = lane & (ppw - 1);
        const bool mine = slot < count;
        int4 e = make_int4(0, 0, 0, 0);
        if (mine) e = ring[(head + slot) & (RING - 1)];
        general_unit<P, W, KM, OM>(mine, e.x, e.y, e.z, sfx, pfx, len, n_reads, lane >> (6 - rs), rs, lw, match,
                                   mismatch, out_score, out_end, err_flag);
        head += count;
    };
#ifdef OVL_TRACE
    const int64_t tr_id = (int64_t)blockIdx.x * 4 + wib;
    {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)" : "=s"(hw), "=s"(xcc));
        OVL_TR_VAL(5, hw);
        OVL_TR_VAL(6, xcc | (role << 8));
    }
    OVL_TR_CLOCK(0, lane);
#endif
    // Heavy tiles first (throughput mode, a resident candidate list): the tiles holding side pairs cost up to
    // ~2.6x a uniform tile (their ring drains), and one landing in the last round of wavefronts is the
    // launch's tail.  Work item i < heavy_n is heavy tile heavy_ids[i] (ids in list tiles, this launch's
    // tiles start at tile_base); item heavy_n + t is tile t, skipped when it is heavy (done already).
    const bool hf = !LAT && heavy_ids != nullptr;
    const int64_t n_items = hf ? n_tiles + heavy_n : n_tiles;
    for (int64_t base = (int64_t)blockIdx.x * G; base < n_items; base += (int64_t)gridDim.x * G) {
        const int64_t item = base + grp;  // wave-uniform
        int64_t tile = item;
        if (hf) {
            if (item < heavy_n) {
                tile = (int64_t)heavy_ids[item] - tile_base;
            } else {
                tile = item - heavy_n;
                if (tile < n_tiles && tile_flags[tile_base + tile]) continue;  // wave-uniform skip
            }
        }
        const int64_t p = tile * 64 + lane;
        const bool mine = item < n_items && tile < n_tiles && p < n_pairs;
        int32_t a = 0, b = 0;
        if constexpr (IX) {
            if (mine) {
                const uint32_t bv = ix_b16[p];
                b = bv == 0xFFFFu ? -1 : (int32_t)bv;
                a = ix_base[tile] + (int32_t)ix_d8[p];
            }
        } else {
            a = mine ? a_idx[p] : 0;
            b = mine ? b_idx[p] : 0;
        }
        const bool ok = mine && a >= 0 && a < n_reads && b >= 0 && b < n_reads;
        if (!ok) { a = 0; b = 0; }
        if (LAT && role == 1) {
            // lengths and rows in the round trip after the indices; side pairs
            // restaged through LDS and scored 16 at a time
            const int32_t n = len[a], m = len[b];
            uint32_t Sw[SROW], Tw[TROW];
            load_words<SROW>(sfx + (int64_t)a * SROW, Sw);
            load_words<TROW>(pfx + (int64_t)b * TROW, Tw);
            OVL_TR_CLOCK(1, Sw[0] ^ Tw[0]);
            if (mine && !ok) {
                ovl_flag_error(err_flag);
                put_pair<OM>(out_score, out_end, p, -1, -1);
            }
            // (n = lw, m <= lw) pairs are the sweeping wave's: uniform and (TT) t-truncated alike
            const bool push = ok && (TT ? n != lw : !(n == lw && m == lw));
            const uint64_t pm = __ballot(push);
            int4* ent = side_ent[LAT ? grp : 0];
            uint4* rows = side_rows + (LAT ? grp * 64 * ROWQ : 0);
            if (push) {
                const int s = __popcll(pm & ((1ull << lane) - 1ull));
                ent[s] = make_int4((int32_t)p, 0, n, m);
#pragma unroll
                for (int k = 0; k < SROW / 4; ++k)
                    rows[s * ROWQ + k] = make_uint4(Sw[4 * k], Sw[4 * k + 1], Sw[4 * k + 2], Sw[4 * k + 3]);
#pragma unroll
                for (int k = 0; k < TROW / 4; ++k)
                    rows[s * ROWQ + SROW / 4 + k] = make_uint4(Tw[4 * k], Tw[4 * k + 1], Tw[4 * k + 2], Tw[4 * k + 3]);
            }
            const int cnt = __popcll(pm);
#ifndef OVL_ABLATE_DRAIN  // diagnostic build only: side pairs left unscored
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            // issue priority over the co-resident sweeps while the side pairs drain: the drain's chain
            // (LDS restaging, a general sweep, the group max) is the launch's tail otherwise (A/B on one
            // box, cfg2: 8.87 -> 8.39 us with levels 1-3 alike; raised from the wave's start: 8.62 us)
            __builtin_amdgcn_s_setprio(1);
            for (int h = 0; h < cnt; h += 16) {
                const int count = cnt - h < 16 ? cnt - h : 16;
                const int rs = count > 8 ? 2 : (count > 4 ? 3 : (count > 2 ? 4 : 5));
                const int slot = lane & ((64 >> rs) - 1);
                const bool own = slot < count;
                const int s = own ? h + slot : 0;
                const int4 en = ent[s];
                uint32_t Sv[SROW], Tv[TROW];
#pragma unroll
                for (int k = 0; k < SROW / 4; ++k) {
                    const uint4 v = rows[s * ROWQ + k];
                    Sv[4 * k] = v.x; Sv[4 * k + 1] = v.y; Sv[4 * k + 2] = v.z; Sv[4 * k + 3] = v.w;
                }
#pragma unroll
                for (int k = 0; k < TROW / 4; ++k) {
                    const uint4 v = rows[s * ROWQ + SROW / 4 + k];
                    Tv[4 * k] = v.x; Tv[4 * k + 1] = v.y; Tv[4 * k + 2] = v.z; Tv[4 * k + 3] = v.w;
                }
                const int r0 = lane >> (6 - rs);
                const auto full = general_core<P, W, KM>(own, en.z, en.w, Sv, Tv, r0, rs, lw, match, mismatch);
                if (own && r0 == 0) {
                    int32_t sc, e2;
                    Key<KM>::decode(full, sc, e2);
                    put_pair<OM>(out_score, out_end, en.x, sc, e2, en.z, match, pack_inv(match, mismatch));
                }
            }
            __builtin_amdgcn_s_setprio(0);
#endif
            OVL_TR_CLOCK(2, cnt);
            OVL_TR_VAL(7, cnt);
            continue;
        }
        uint32_t Sw[SROW], Tw[TROW];
#ifdef OVL_ABLATE_LOADS  // diagnostic build only: rows made up from the indices (no row loads)
#pragma unroll
        for (int i = 0; i < SROW; ++i) Sw[i] = (uint32_t)a * 0x9E3779B9u + (uint32_t)i * 0x85EBCA6Bu;
#pragma unroll
        for (int i = 0; i < TROW; ++i) Tw[i] = (uint32_t)b * 0xC2B2AE35u + (uint32_t)i * 0x27D4EB2Fu;
#else
        load_words<SROW>(sfx + (int64_t)a * SROW, Sw);
        load_words<TROW>(pfx + (int64_t)b * TROW, Tw);
#endif
        // read a of length lw? one bit per read (L1-resident bitmap); b's length decides uniform (m = lw).
        // TT: every other pair is scored by this sweep too -- its keys for j <= min(n, m) are the uniform
        // keys (a snapshot of the block maxima after shift min(n, m) % 32), and a shorter read a (n < m) adds
        // its windows j in (n, m] after the sweep (window_keys); else a shorter read a is a side pair
        const bool fa = ok && ((full[a >> 5] >> (a & 31)) & 1u);
        const int32_t mb = len[b];
        int32_t na = lw;
        if (TT && ok && !fa) na = len[a];
        const bool uni = fa && mb == lw;
        const bool tt = TT && ok && !uni;
        const int32_t tm = tt ? (na < mb ? na : mb) : -1;
        uint32_t tmask = 0;
        for (uint64_t bm = __ballot(tt); bm; bm &= bm - 1)  // scalar loop over the truncated lanes
            tmask |= 1u << (__builtin_amdgcn_readlane(tm, (int)__builtin_ctzll(bm)) & 31);
        OVL_TR_CLOCK(1, Sw[0] ^ Tw[0]);
        if constexpr (!LAT) {
            if (mine && !ok) ovl_flag_error(err_flag);
            const bool push = ok && !uni && !tt;
            const uint64_t pm = __ballot(push);
            if (push)
                ring[(tail + __popcll(pm & ((1ull << lane) - 1ull))) & (RING - 1)] = make_int4((int32_t)p, a, b, 0);
            tail += __popcll(pm);
        }
#ifdef OVL_ABLATE_SWEEP  // diagnostic build only: keep the loads, skip the sweep
        T best = (T)(Sw[0] ^ Tw[0] ^ Sw[SROW - 1] ^ Tw[TROW - 1]) & 0;
        asm volatile("" ::"v"(Sw[0]), "v"(Tw[0]), "v"(Sw[SROW - 1]), "v"(Tw[TROW - 1]));
#else
        T best = sweep_uniform<W, KM>(Sw, Tw, lw, match, mismatch - match, 0u, 32u, tmask, tm);
#endif
        if constexpr (TT) {
            const bool win = tt && na < mb;
            uint64_t wm = __ballot(win);
            if (wm) {  // wave-uniform: j from the largest m down to the smallest n + 1 over the window lanes
                int32_t jlo = 1 << 30, jhi = 0;
                for (; wm; wm &= wm - 1) {
                    const int l = (int)__builtin_ctzll(wm);
                    jlo = min(jlo, __builtin_amdgcn_readlane(na, l) + 1);
                    jhi = max(jhi, __builtin_amdgcn_readlane(mb, l));
                }
                const int32_t wk = window_keys<W>(Sw, Tw, na, mb, jlo, jhi, match, mismatch - match);
                if (win && (T)wk > best) best = (T)wk;
            }
        }
        OVL_TR_CLOCK(3, (uint32_t)best);
        if (mine && (uni || tt || (!LAT && !ok))) {
            int32_t sc, en;
            Key<KM>::decode(best, sc, en);
            put_pair<OM>(out_score, out_end, p, ok ? sc : -1, ok ? en : -1, na, match, pack_inv(match, mismatch));
        }
        OVL_TR_CLOCK(4, (uint32_t)best);
#ifndef OVL_ABLATE_DRAIN
        if constexpr (!LAT) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            while (tail - head >= 16) drain(16);
        }
#endif
    }
#ifndef OVL_ABLATE_DRAIN
    if constexpr (!LAT) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (tail > head) drain(tail - head);
    }
#endif
}

// General kernel: any lengths <= 32W and P bit planes (used when the read set
// is not 2-plane-encodable or has no single dominant length), RS lanes per pair.
template <int P, int W, int KM>
__global__ __launch_bounds__(256) void general_kernel(
    const uint32_t* __restrict__ sfx, const uint32_t* __restrict__ pfx, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx, int64_t n_pairs,
    int32_t rs_log2, int32_t match, int32_t mismatch, int32_t* __restrict__ out_score,
    int32_t* __restrict__ out_end, uint32_t* __restrict__ err_flag) {
    const int lane = threadIdx.x & 63;
    const int ppw = 64 >> rs_log2;
    const int slot = lane & (ppw - 1);
    const int r0 = lane >> (6 - rs_log2);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t n_units = (n_pairs + ppw - 1) / ppw;
    for (int64_t u = wave; u < n_units; u += n_waves) {
        const int64_t p = u * ppw + slot;
        const bool mine = p < n_pairs;
        const int32_t a = mine ? a_idx[p] : 0;
        const int32_t b = mine ? b_idx[p] : 0;
        general_unit<P, W, KM>(mine, p, a, b, sfx, pfx, len, n_reads, r0, rs_log2, 0, match, mismatch, out_score,
                               out_end, err_flag);
    }
}

// ----------------------------------------------------------------------------- resident grid

// One tile's results as a ring record (ovl_grid.h OvlResidentBody), which host threads read while the grid runs
// (ovl_expand.h rec_tile_ready_scalar / rec_tile_scalar_t / rec_tile_avx512_t):
//   dword w (w < 32) = phase << 31 | c[w + 32] << 15 | c[w]   (c[l]: lane l's 15-bit code)
// The phase bit (the ring lap's) tells the host which dwords this request has written: every dword is one aligned
// 32-bit store, so a dword whose phase bit is the lap's holds this request's payload, and a record is complete
// when all 32 are.  Code c of a pair with end j <= n (read a's length; L = j compared bases, aligners.py:27-48
// with gaps that cannot win, so score = match*j + (mismatch - match)*X) is j(j + 1)/2 + X, X <= j <= 254
// (< 0x7FFF).  Every other pair has c = 0x7FFF and a special word, stored as one 8-byte {payload, seq}:
//   1 << 31 | j << 16 | X << 8 | n   a shorter read a inside b's window (j > n: L = n, score = match*n +
//                                    (mismatch - match)*X);
//   0xFFFFFFFF                       a bad pair (-1, -1).
// 2 link bytes per pair (+ 8 per special).  Every lane of the wavefront calls it (the cross-half exchange); lanes
// with !mine code 0, which the host never reads.  The
// stores are non-temporal 128-byte lines into fine-grained host memory, which the XCD's L2 keeps (write-back) until
// the wavefront's release fence after its last tile of the request (resident_kernel): a resident grid never reaches
// the end-of-kernel write-back.  (Measured against the alternatives, target point, N = 8 / N = 1 shards: write-through
// 16-byte sc1 stores 0.056 / 0.326 ms, 8-byte system-scope stores 0.071 / 0.344, non-temporal stores into uncached
// (MTYPE_UC) memory 0.062 / 0.340, this form 0.049 / 0.223; profiles/r06_resident_store_ab.json.)
__device__ __forceinline__ void put_ring_rec(uint32_t* rec, uint64_t* sp, int64_t ri, uint32_t phase, uint32_t seq,
                                             bool mine, int32_t sc, int32_t en, int32_t n, int32_t match, float inv,
                                             int lane) {
    uint32_t c = 0;
    if (mine) {
        uint32_t special = 0;
        if (en < 0) {
            special = 0xFFFFFFFFu;
        } else if (en > n) {
            const uint32_t x = (uint32_t)__builtin_rintf((float)(match * n - sc) * inv);
            special = 0x80000000u | (uint32_t)en << 16 | x << 8 | (uint32_t)n;
        } else {
            const uint32_t x = (uint32_t)__builtin_rintf((float)(match * en - sc) * inv);
            c = ((uint32_t)en * (uint32_t)(en + 1) >> 1) + x;
        }
        if (special) {
            c = 0x7FFFu;
            __builtin_nontemporal_store((uint64_t)seq << 32 | special, sp + 64 * ri + lane);
        }
    }
    const uint32_t hi = (uint32_t)__shfl_xor((int)c, 32, 64);
    if (lane < 32) __builtin_nontemporal_store(phase << 31 | hi << 15 | c, rec + 32 * ri + lane);
}

// One 64-pair tile of a resident request: uniform_kernel's throughput-mode sweep with every pair in it (TT: reads
// b cut at the genome end snapshot their block maxima, shorter reads a add their window keys), into the ring.
// Split in stages so a wavefront can have the next tiles' loads in flight during a sweep (resident_kernel):
// the indices (ResIdx), then the rows and lengths they select (ResRows), then the sweep (resident_sweep).
struct ResIdx {
    int32_t a, b;
    bool mine, ok;
};
template <int W>
struct ResRows {
    uint32_t Sw[(W * 2 + 3) & ~3], Tw[(W * 2 + 3) & ~3];
    uint32_t fw;  // read a's word of the length bitmap
    int32_t la, lb;
};

__device__ __forceinline__ ResIdx resident_idx(int64_t tile, const OvlResidentBody& q, int32_t n_reads, int lane) {
    ResIdx x;
    const int64_t p = tile * 64 + lane;
    x.mine = tile >= 0 && p < q.n_pairs;
    x.a = x.mine ? q.a_idx[p] : 0;
    x.b = x.mine ? q.b_idx[p] : 0;
    x.ok = x.mine && x.a >= 0 && x.a < n_reads && x.b >= 0 && x.b < n_reads;
    if (!x.ok) {
        x.a = 0;
        x.b = 0;
    }
    return x;
}

template <int W>
__device__ __forceinline__ void resident_rows(const ResIdx& x, ResRows<W>& r, const uint32_t* __restrict__ sfx,
                                              const uint32_t* __restrict__ pfx, const int32_t* __restrict__ len,
                                              const uint32_t* __restrict__ full) {
    constexpr int SROW = (W * 2 + 3) & ~3;
    load_words<SROW>(sfx + (int64_t)x.a * SROW, r.Sw);
    load_words<SROW>(pfx + (int64_t)x.b * SROW, r.Tw);
    r.fw = full[x.a >> 5];
    r.la = len[x.a];
    r.lb = len[x.b];
}

template <int W>
__device__ __forceinline__ void resident_sweep(int64_t tile, const ResIdx& x, const ResRows<W>& r,
                                               const OvlResidentBody& q, int32_t lw, int32_t match, int32_t mismatch,
                                               int lane) {
    const bool ok = x.ok;
    const bool fa = ok && ((r.fw >> (x.a & 31)) & 1u);
    const int32_t mb = r.lb;
    int32_t na = lw;
    if (ok && !fa) na = r.la;
    const bool uni = fa && mb == lw;
    const bool tt = ok && !uni;
    const int32_t tm = tt ? (na < mb ? na : mb) : -1;
    uint32_t tmask = 0;
    for (uint64_t bm = __ballot(tt); bm; bm &= bm - 1)
        tmask |= 1u << (__builtin_amdgcn_readlane(tm, (int)__builtin_ctzll(bm)) & 31);
    int32_t best = sweep_uniform<W, 0>(r.Sw, r.Tw, lw, match, mismatch - match, 0u, 32u, tmask, tm);
    const bool win = tt && na < mb;
    uint64_t wm = __ballot(win);
    if (wm) {
        int32_t jlo = 1 << 30, jhi = 0;
        for (; wm; wm &= wm - 1) {
            const int l = (int)__builtin_ctzll(wm);
            jlo = min(jlo, __builtin_amdgcn_readlane(na, l) + 1);
            jhi = max(jhi, __builtin_amdgcn_readlane(mb, l));
        }
        const int32_t wk = window_keys<W>(r.Sw, r.Tw, na, mb, jlo, jhi, match, mismatch - match);
        if (win && wk > best) best = wk;
    }
    int32_t sc, en;
    Key<0>::decode(best, sc, en);
    const int64_t g = q.pos + tile;
    const int64_t ri = g & ((int64_t(1) << q.ring_log2) - 1);
    const uint32_t phase = (uint32_t)((g >> q.ring_log2) + 1) & 1u;
    put_ring_rec(q.rec, q.sp, ri, phase, (uint32_t)q.seq, x.mine, ok ? sc : -1, ok ? en : -1, na, match,
                 pack_inv(match, mismatch), lane);
}

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The resident scoring grid: launched once, it serves requests posted by the host in pinned memory until the host
// asks it to leave or none comes for idle_ticks (the host relaunches it on its next request), so a call pays
// neither a launch nor a completion signal -- the results' ring records tell the host when it is done.
//   Block 0's thread 0 polls the host mailbox (a relaxed system-scope load per poll, s_sleep between), reads the
// request body, writes a device copy of it under a seqlock (8-byte agent-scope atomics, each group drained) and
// forwards the sequence number through one device word; the other blocks' thread 0 polls that word and reads the
// copy (the hand-off of MI355X_MICROARCH.md's first valid row: sc1 stores drained, one flag, sc1 loads).  Each
// block then scores tiles: wavefront w of the grid takes items w, w + waves, ... (heavy tiles first, as
// uniform_kernel orders them).  No fan-in across blocks: nothing is waited for on the device.  The records are
// non-temporal stores into fine-grained host memory, which stay in the XCD's L2 until written back: a release
// fence after a block's last tile (body.fence 2: the block's last wavefront, counted in LDS after each wavefront's
// stores drained; 1: every wavefront) -- each fence writes back the whole L2, and 2,048 of them per request queue
// behind each other (MI355X_MICROARCH.md: the write-back costs a few microseconds).
//   Every wait is bounded: block 0 leaves (and tells the others) after idle_ticks without a request; the other
// blocks leave after twice that without a new forward, so a grid whose block 0 never ran still ends.
// PF: tiles software-pipelined (fewer, fatter wavefronts: 2-4 per SIMD) or one tile at a time (UNI_OCC(W, 0)
// wavefronts per SIMD, uniform_kernel's register budget)
#ifndef OVL_RES_PF_OCC
#define OVL_RES_PF_OCC 2  // (build macro for A/B builds: the software-pipelined form's waves per SIMD at W >= 3)
#endif
#define RES_OCC(W, PF) ((PF) ? ((W) >= 3 ? OVL_RES_PF_OCC : 4) : UNI_OCC(W, 0))
template <int W, bool PF>
__global__ __launch_bounds__(256, RES_OCC(W, PF)) void resident_kernel(
    const uint32_t* __restrict__ sfx, const uint32_t* __restrict__ pfx, const int32_t* __restrict__ len,
    int32_t n_reads, int32_t lw, const uint32_t* __restrict__ full, const uint8_t* __restrict__ tile_flags,
    const OvlResidentCtl* mailbox, uint32_t* fwd, OvlResidentBody* dslot, uint32_t seq_base, uint64_t idle_ticks,
    uint64_t* status, uint32_t poll_sleep, uint64_t* tbuf) {
    __shared__ uint64_t s_body[kResidentBodyWords];
    __shared__ int s_go;
    __shared__ int s_done;  // (fence 2: wavefronts of this block done with the request)
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    uint32_t last = seq_base;  // (thread 0)
    for (;;) {
        if (threadIdx.x == 0) {
            int go = 0;
            uint64_t v[kResidentBodyWords];
            if (blockIdx.x == 0) {
                const uint64_t t_end = wall_clock64() + idle_ticks;
                uint32_t seq = 0;
                for (;;) {
                    const uint64_t c = __hip_atomic_load(&mailbox->ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (c >> 32) break;  // asked to leave
                    if ((uint32_t)c != last) {
                        seq = (uint32_t)c;
                        go = 1;
                        break;
                    }
                    if (wall_clock64() > t_end) break;
                    __builtin_amdgcn_s_sleep(2);
                }
                int why = go ? 0 : 2;  // (status: 1 asked to leave, 2 idle, 3 a body that is not the request's)
                if (!go && wall_clock64() <= t_end) why = 1;
                if (go) {
                    vm_drain();
                    const uint64_t* src = reinterpret_cast<const uint64_t*>(&mailbox->body[seq & 1]);
#pragma unroll
                    for (int k = 0; k < kResidentBodyWords; ++k)
                        v[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    go = (uint32_t)v[0] == seq;  // (the host writes the body before ctl: always)
                    if (!go) why = 3;
                }
                if (!go && status) {  // why block 0 left, for the host's trace (pinned, written only here)
                    __hip_atomic_store(status + 1, (uint64_t)last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(status + 2, (uint64_t)seq | (v[0] << 32), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(status + 3, idle_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    vm_drain();
                    __hip_atomic_store(status, (uint64_t)why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                if (go) {
                    uint64_t* ds = reinterpret_cast<uint64_t*>(&dslot[seq & 3]);
                    __hip_atomic_store(ds, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    vm_drain();
#pragma unroll
                    for (int k = 1; k < kResidentBodyWords; ++k)
                        __hip_atomic_store(ds + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    vm_drain();
                    __hip_atomic_store(ds, (uint64_t)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    vm_drain();
                    __hip_atomic_store(fwd, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    last = seq;
                    if (tbuf) __builtin_nontemporal_store(wall_clock64(), tbuf + 4 * (int64_t)gridDim.x * 4);
                } else {
                    __hip_atomic_store(fwd, kResidentLeave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                const uint64_t t_end = wall_clock64() + 2 * idle_ticks;
                for (;;) {
                    const uint32_t f = __hip_atomic_load(fwd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (f == kResidentLeave) break;
                    if (f != 0u && f != last) {
                        vm_drain();
                        const uint64_t* ds = reinterpret_cast<const uint64_t*>(&dslot[f & 3]);
                        const uint64_t s1 = __hip_atomic_load(ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        vm_drain();
#pragma unroll
                        for (int k = 1; k < kResidentBodyWords; ++k)
                            v[k] = __hip_atomic_load(ds + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        vm_drain();
                        const uint64_t s2 = __hip_atomic_load(ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (s1 == (uint64_t)f && s2 == (uint64_t)f) {  // (else rewritten meanwhile: poll again)
                            v[0] = s1;
                            last = f;
                            go = 1;
                            break;
                        }
                    }
                    if (wall_clock64() > t_end) break;
                    for (uint32_t z = 0; z < poll_sleep; ++z) __builtin_amdgcn_s_sleep(4);  // (~0.1 us each)
                }
                if (!go && status)  // (a block that left on its own deadline, not told to)
                    if (__hip_atomic_load(fwd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kResidentLeave)
                        __hip_atomic_store(status + 4, (uint64_t)blockIdx.x + 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (go) {
#pragma unroll
                for (int k = 0; k < kResidentBodyWords; ++k) s_body[k] = v[k];
            }
            s_go = go;
            s_done = 0;
        }
        __syncthreads();
        if (!s_go) return;
        // (trace, OVL_TRACE_PIPE: per wavefront the wall clock when it knew the request, finished its last tile
        // and had its records written back; block 0 stored when it saw the request)
        if (tbuf && lane == 0) __builtin_nontemporal_store(wall_clock64(), tbuf + 4 * wave);
        OvlResidentBody q;  // (wave-uniform: scalar registers, as kernel arguments would be)
        {
            uint64_t* d = reinterpret_cast<uint64_t*>(&q);
#pragma unroll
            for (int k = 0; k < kResidentBodyWords; ++k) {
                const uint64_t x = s_body[k];
                const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
                const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
                d[k] = (uint64_t)hi << 32 | lo;
            }
        }
        const int32_t match = (int32_t)(uint32_t)q.scoring, mismatch = (int32_t)(uint32_t)(q.scoring >> 32);
        const int64_t n_tiles = (q.n_pairs + 63) >> 6;
        const bool hf = q.heavy_ids != nullptr && q.heavy_n > 0;
        const int64_t n_items = hf ? n_tiles + q.heavy_n : n_tiles;
        // The wave's items w, w + waves, ... (heavy tiles first, as uniform_kernel orders them; an item whose tile
        // was done among the heavy ones is skipped): item -> tile, or -1 past the last.  Software-pipelined: while
        // tile i sweeps, the rows of tile i + 1 and the indices of tile i + 2 are in flight (a resident grid runs
        // a few wavefronts per SIMD, too few to hide a tile's two dependent loads by switching waves).
        if constexpr (!PF) {
            for (int64_t item = wave; item < n_items; item += n_waves) {  // (wave-uniform)
                int64_t tile = item;
                if (hf) {
                    if (item < q.heavy_n) {
                        tile = (int64_t)q.heavy_ids[item] - q.tile_base;
                    } else {
                        tile = item - q.heavy_n;
                        if (tile_flags[q.tile_base + tile]) continue;  // done among the heavy ones
                    }
                }
                const ResIdx x = resident_idx(tile, q, n_reads, lane);
                ResRows<W> r;
                resident_rows<W>(x, r, sfx, pfx, len, full);
                resident_sweep<W>(tile, x, r, q, lw, match, mismatch, lane);
            }
        }
        int64_t item = PF ? wave : n_items;
        const auto next_tile = [&]() -> int64_t {  // (wave-uniform; leaves `item` on the tile's item)
            for (; item < n_items; item += n_waves) {
                if (!hf) return item;
                if (item < q.heavy_n) return (int64_t)q.heavy_ids[item] - q.tile_base;
                const int64_t t = item - q.heavy_n;
                if (!tile_flags[q.tile_base + t]) return t;
            }
            return -1;
        };
        int64_t t0 = next_tile();
        ResIdx x0 = resident_idx(t0, q, n_reads, lane);
        ResRows<W> r0;
        if (t0 >= 0) resident_rows<W>(x0, r0, sfx, pfx, len, full);
        item += n_waves;
        int64_t t1 = t0 >= 0 ? next_tile() : -1;
        ResIdx x1 = resident_idx(t1, q, n_reads, lane);
        while (t0 >= 0) {
            ResRows<W> r1;
            if (t1 >= 0) resident_rows<W>(x1, r1, sfx, pfx, len, full);
            item += n_waves;
            const int64_t t2 = t1 >= 0 ? next_tile() : -1;
            const ResIdx x2 = resident_idx(t2, q, n_reads, lane);
            resident_sweep<W>(t0, x0, r0, q, lw, match, mismatch, lane);
            t0 = t1;
            x0 = x1;
            r0 = r1;
            t1 = t2;
            x1 = x2;
        }
        // this wavefront's records out of the XCD's L2 (system-scope release: an L2 write-back)
        if (tbuf && lane == 0) __builtin_nontemporal_store(wall_clock64(), tbuf + 4 * wave + 1);
        if (q.fence == 1) {
            if (wave < n_items) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        } else if (q.fence == 2 && (int64_t)blockIdx.x * 4 < n_items) {
            vm_drain();  // (this wavefront's records are in the L2: the fence of the block's last one covers them)
            int k = 0;
            if (lane == 0) k = atomicAdd(&s_done, 1);
            k = __builtin_amdgcn_readfirstlane(k);
            if (k == 3) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        if (tbuf && lane == 0) {
            __hip_atomic_store(tbuf + 4 * wave + 2, (uint64_t)wall_clock64(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(tbuf + 4 * wave + 3, q.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();  // (thread 0 rewrites s_body for the next request)
    }
}

extern "C" hipError_t ovl_launch_resident(const OvlResidentArgs* g, hipStream_t stream) {
    if (g->lw <= 0 || g->lw > 254 || g->blocks <= 0 || !g->mailbox || !g->fwd || !g->dslot) return hipErrorInvalidValue;
    const dim3 grid((unsigned)g->blocks), block(256);
#define OVL_RESIDENT_CASE(Wc)                                                                                       \
    case Wc:                                                                                                        \
        if (g->pipelined)                                                                                           \
            resident_kernel<Wc, true><<<grid, block, 0, stream>>>(g->sfx, g->pfx, g->len, g->n_reads, g->lw,        \
                                                                  g->full, g->tile_flags, g->mailbox, g->fwd,       \
                                                                  g->dslot, g->seq_base, g->idle_ticks, g->status,  \
                                                                  g->poll_sleep, g->tbuf);                          \
        else                                                                                                        \
            resident_kernel<Wc, false><<<grid, block, 0, stream>>>(g->sfx, g->pfx, g->len, g->n_reads, g->lw,       \
                                                                   g->full, g->tile_flags, g->mailbox, g->fwd,      \
                                                                   g->dslot, g->seq_base, g->idle_ticks, g->status, \
                                                                   g->poll_sleep, g->tbuf);                         \
        break;
    switch (g->wmax) {
        OVL_RESIDENT_CASE(1)
        OVL_RESIDENT_CASE(2)
        OVL_RESIDENT_CASE(3)
        OVL_RESIDENT_CASE(4)
        OVL_RESIDENT_CASE(5)
        OVL_RESIDENT_CASE(6)
        OVL_RESIDENT_CASE(7)
        OVL_RESIDENT_CASE(8)
        default: return hipErrorInvalidValue;
    }
#undef OVL_RESIDENT_CASE
    return hipGetLastError();
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
// BANDED (the build's band knob, oracle_overlap_banded; not a reference mode):
// seed[pair] holds the seed end j* (the ungapped closed form's first argmax,
// written by the launch before into a separate buffer, so out_* may be host memory); only cells with
// |(i - j) - d*| <= band, d* = n - j*, are filled, out-of-band predecessors
// count as -inf, and only strips and anti-diagonal steps that meet the band are
// swept.  A cell's diagonal predecessor is always in the band; "up" leaves it
// only at the row's last band cell and "left" only at its first.
template <typename Acc, bool BANDED>
__global__ __launch_bounds__(64) void dp_kernel(
    const uint8_t* __restrict__ codes, const int64_t* __restrict__ off, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx,
    int64_t n_pairs, int32_t mcap, int64_t match, int64_t mismatch, int64_t indel, int32_t band,
    int32_t* __restrict__ out_score, int32_t* __restrict__ out_end, const int32_t* __restrict__ seed,
    int8_t* __restrict__ tb, uint32_t* __restrict__ err_flag) {
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
                ovl_flag_error(err_flag);
                out_score[pair] = -1;
                out_end[pair] = -1;
            }
            continue;
        }
        const int32_t n = len[a];
        const int32_t m = len[b];
        const uint8_t* s = codes + off[a];
        const uint8_t* t = codes + off[b];
        // band: seed diagonal d* and the rows [rlo, rhi] that hold band cells
        const int32_t dstar = BANDED ? n - seed[pair] : 0;
        const int32_t W = BANDED ? band : 0;
        const int32_t rlo = BANDED ? (dstar - W + 1 > 1 ? dstar - W + 1 : 1) : 1;
        __syncthreads();  // previous pair's LDS readers are done
        for (int j = lane; j <= m; j += 64) row0[j] = 0;
        for (int j = lane; j < m; j += 64) tcodes[j] = t[j];
        __syncthreads();
        int32_t* rin = row0;
        int32_t* rout = row1;
        // tracked by the lane that owns row n; dp[n][0] = 0 is the j = 0 candidate
        // (in banded mode only when (n, 0) is in the band)
        int32_t best = (!BANDED || n - dstar - W <= 0) ? 0 : INT32_MIN, bend = 0;
        const int nstrips = (n + 63) >> 6;
        const int st0 = BANDED ? (rlo - 1) >> 6 : 0;
        for (int st = st0; st < nstrips; ++st) {
            const int32_t i = 64 * st + 1 + lane;
            const bool row_ok = i <= n;
            const uint32_t sc = row_ok ? (uint32_t)s[i - 1] : 0xFFFFFFFFu;
            // anti-diagonal steps: lane L is on column j = tau - L + 1
            int tau_lo = 0, tau_hi = m + 62;
            if (BANDED) {
                const int lmax = (n - 64 * st - 1) < 63 ? (n - 64 * st - 1) : 63;
                const int lo = 64 * st - dstar - W;
                const int hi = 64 * st + 2 * lmax - dstar + W;
                tau_lo = lo > 0 ? lo : 0;
                tau_hi = hi < tau_hi ? hi : tau_hi;
            }
            const int32_t jlo = i - dstar - W, jhi = i - dstar + W;  // unclamped band edges of row i
            int32_t cur = 0;      // dp[i][j-1] (starts as dp[i][0] = 0)
            // dp[i-1][j-1]; lane 0 starts mid-row in banded mode
            int32_t uprev = (BANDED && lane == 0) ? rin[tau_lo] : 0;
            uint32_t tch = 0;
            const bool last_strip_row = (lane == 63) && (st + 1 < nstrips);
            for (int tau = tau_lo; tau <= tau_hi; ++tau) {
                const int32_t j = tau - lane + 1;
                // lane 0's inputs come from LDS (uniform address: broadcast)
                const int32_t jj = tau + 1 <= m ? tau + 1 : m;
                const int32_t lds_up = rin[jj];
                const uint32_t lds_t = tau < m ? (uint32_t)tcodes[tau] : 0u;
                int32_t upin = shr1<int32_t>(cur);
                uint32_t tin = (uint32_t)shr1<int32_t>((int32_t)tch);
                if (lane == 0) { upin = lds_up; tin = lds_t; }
                const bool in_band = !BANDED || (j >= jlo && j <= jhi);
                if (row_ok && j >= 1 && j <= m && in_band) {
                    const Acc diag = (Acc)uprev + (sc == tin ? (Acc)match : (Acc)mismatch);
                    const Acc up = (Acc)upin + (Acc)indel;
                    const Acc left = (Acc)cur + (Acc)indel;
                    const bool up_ok = !BANDED || j != jhi;
                    const bool left_ok = !BANDED || j != jlo;
                    int8_t dir;
                    Acc v;
                    if ((!up_ok || diag >= up) && (!left_ok || diag >= left)) { v = diag; dir = 0; }
                    else if (up_ok && (!left_ok || up >= left))               { v = up;   dir = 1; }
                    else                                                      { v = left; dir = 2; }
                    cur = (int32_t)v;
                    if (!BANDED && tb) tb[(int64_t)i * (m + 1) + j] = dir;
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
        // row n lives in lane (n-1) % 64 of the last strip
        const int owner = (n - 1) & 63;
        const int32_t bs = __shfl(best, owner, 64);
        const int32_t be = __shfl(bend, owner, 64);
        __syncthreads();  // every lane is done with this pair's LDS rows
        if (lane == 0) {
            out_score[pair] = n > 0 && m > 0 ? bs : 0;
            out_end[pair] = n > 0 && m > 0 ? be : 0;
        }
    }
}

// Full DP, scores only (no traceback, no band): the scoring path for gapped parameters.
// Same strips and anti-diagonals as dp_kernel, restructured for issue: 64-step chunks with the step
// loop unrolled at compile time and branch-free; lane 0's inputs (the previous strip's last row and
// t) come from one LDS read per chunk and readlane per step; lane 63's values for the next strip are
// staged with v_writelane (inline-constant lane) and written once per chunk.  A cell's value is
// max(diag, up, left) whatever the tie order (aligners.py:40-48 keeps the maximum), and the int32
// store wraps like the reference's table.
template <int L>
__device__ __forceinline__ int32_t writelane_c(int32_t vec, int32_t s) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(vec) : "s"(s), "n"(L));
    return vec;
}

template <int B, int E, typename F>
__device__ __forceinline__ void unroll_steps(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        unroll_steps<B + 1, E>(f);
    }
}

template <typename Acc, bool BANDED>
__global__ __launch_bounds__(64) void dp_fast_kernel(
    const uint8_t* __restrict__ codes, const int64_t* __restrict__ off, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx,
    int64_t n_pairs, int32_t mcap, int64_t match, int64_t mismatch, int64_t indel, int32_t band,
    int32_t* __restrict__ out_score, int32_t* __restrict__ out_end, const int32_t* __restrict__ seed,
    uint32_t* __restrict__ err_flag) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // rows hold columns 0 .. 64*nch + 64 (hand-off chunks of 64 columns); t codes padded likewise
    const int32_t pitch = ((mcap + 126) / 64) * 64 + 64;
    int32_t* row0 = reinterpret_cast<int32_t*>(smem);
    int32_t* row1 = row0 + pitch;
    uint8_t* tcodes = reinterpret_cast<uint8_t*>(row1 + pitch);
    const int lane = threadIdx.x;
    for (int64_t pair = blockIdx.x; pair < n_pairs; pair += gridDim.x) {
        const int32_t a = a_idx[pair];
        const int32_t b = b_idx[pair];
        if (a < 0 || a >= n_reads || b < 0 || b >= n_reads || len[b] > mcap) {
            if (lane == 0) {
                ovl_flag_error(err_flag);
                out_score[pair] = -1;
                out_end[pair] = -1;
            }
            continue;
        }
        const int32_t n = len[a];
        const int32_t m = len[b];
        const uint8_t* s = codes + off[a];
        const uint8_t* t = codes + off[b];
        const int32_t nch = (m + 126) / 64;  // chunks covering tau = 0 .. m + 62
        // band: seed diagonal d* (seed holds the ungapped seed end j*) and the first row with
        // a band cell of column >= 1; the band of row i is columns [i - d* - W, i - d* + W]
        const int32_t W = BANDED ? band : 0;
        const int32_t dstar = BANDED ? n - seed[pair] : 0;
        const int32_t rlo = BANDED ? (dstar - W + 1 > 1 ? dstar - W + 1 : 1) : 1;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // previous pair's LDS readers are done
        for (int j = lane; j < pitch; j += 64) row0[j] = 0;
        for (int j = lane; j < 64 * nch; j += 64) tcodes[j] = j < m ? t[j] : 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        int32_t* rin = row0;
        int32_t* rout = row1;
        // tracked by the lane that owns row n; dp[n][0] = 0 is the j = 0 candidate when in the band
        int32_t best = (!BANDED || n - dstar - W <= 0) ? 0 : INT32_MIN, bend = 0;
        const int nstrips = (n + 63) >> 6;
        const int st0 = BANDED ? (rlo - 1) >> 6 : 0;
        for (int st = st0; st < nstrips; ++st) {
            const int32_t i = 64 * st + 1 + lane;
            const bool last_row = i == n;
            // rows past n (last strip only) compute unread values: no row mask is needed
            const uint32_t sc = i <= n ? (uint32_t)s[i - 1] : 0xFFFFFFFFu;
            const bool last = st + 1 == nstrips;  // last strip: track row n; else carry the last row
            const int32_t jlo = i - dstar - W, jhi = i - dstar + W;  // this lane's band (BANDED)
            // chunks whose steps meet the band (all chunks when not banded)
            int32_t c_lo = 0, c_hi = nch - 1;
            if constexpr (BANDED) {
                const int lmax = (n - 64 * st - 1) < 63 ? (n - 64 * st - 1) : 63;
                const int32_t tlo = 64 * st - dstar - W;                 // lane 0's first band step
                const int32_t thi = 64 * st + 2 * lmax - dstar + W;      // last lane's last band step
                c_lo = tlo > 0 ? tlo / 64 : 0;
                c_hi = thi / 64 < nch - 1 ? thi / 64 : nch - 1;
                if (c_hi < c_lo) c_hi = c_lo;
            }
            // state entering chunk c_lo: lane L used t[64 c_lo - 1 - L] at the step before, lane 0's
            // diagonal is dp[64 st][64 c_lo]; other lanes' carried values only meet masked cells
            int32_t cur = 0, uprev = 0, tch = 0;
            if (BANDED && c_lo > 0) {
                const int32_t tp = 64 * c_lo - 1 - lane;
                tch = tp >= 0 && tp < m ? (int32_t)tcodes[tp] : 0;
                uprev = lane == 0 ? rin[64 * c_lo] : 0;
            }
            int32_t out_a = 0, out_b = 0;
            // one chunk of 64 steps; EDGE: chunk 0 (lanes still left of column 1 keep dp[i][0] = 0);
            // LAST: best tracking of row n instead of the carry staging.
            auto chunk = [&](int32_t c, auto edge_tag, auto last_tag) {
                constexpr bool EDGE = decltype(edge_tag)::value;
                constexpr bool LAST = decltype(last_tag)::value;
                int32_t v_rin = rin[64 * c + 1 + lane];        // lane u: dp[64 st][64c+1+u]
                int32_t v_t = (int32_t)tcodes[64 * c + lane];  // lane u: t[64c+u]
                // the column as a running register: per-step lane masks built from constants would be
                // hoisted as 64 loop invariants (SGPR pairs spilled to VGPR lanes)
                int32_t jv = 64 * c - lane + 1;
                unroll_steps<0, 64>([&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    const int32_t j = jv;
                    // lane 0 takes its inputs from the chunk registers' lane 0, then they rotate down
                    const int32_t upin = __builtin_amdgcn_update_dpp(v_rin, cur, 0x138, 0xF, 0xF, false);
                    const int32_t tin = __builtin_amdgcn_update_dpp(v_t, tch, 0x138, 0xF, 0xF, false);
                    v_rin = __builtin_amdgcn_mov_dpp(v_rin, 0x130, 0xF, 0xF, true);  // wave_shl:1, lane 63 <- 0
                    v_t = __builtin_amdgcn_mov_dpp(v_t, 0x130, 0xF, 0xF, true);
                    const Acc diag = (Acc)uprev + ((uint32_t)tin == sc ? (Acc)match : (Acc)mismatch);
                    Acc up = (Acc)upin + (Acc)indel;
                    Acc left = (Acc)cur + (Acc)indel;
                    if constexpr (BANDED) {
                        // out-of-band predecessors: "up" leaves the band only at the row's last band
                        // cell, "left" only at its first; diag is always in the band, so substituting
                        // it leaves the maximum exact
                        up = j != jhi ? up : diag;
                        left = j != jlo ? left : diag;
                    }
                    const Acc mx = diag > up ? diag : up;
                    const int32_t nv = (int32_t)(mx > left ? mx : left);
                    if constexpr (EDGE) cur = j >= 1 ? nv : cur;
                    else cur = nv;
                    if constexpr (LAST) {
                        bool better = last_row && j >= 1 && j <= m && nv > best;
                        if constexpr (BANDED) better = better && j >= jlo && j <= jhi;
                        best = better ? nv : best;
                        bend = better ? j : bend;
                    } else {
                        const int32_t v63 = __builtin_amdgcn_readlane(cur, 63);
                        if constexpr (u <= 62) out_a = writelane_c<u + 1>(out_a, v63);
                        else out_b = writelane_c<0>(out_b, v63);
                    }
                    uprev = upin;
                    tch = tin;
                    jv += 1;
                    asm volatile("" : "+v"(jv), "+v"(v_rin), "+v"(v_t));
                });
                if constexpr (!LAST) {
                    if (c >= 1) rout[64 * (c - 1) + 1 + lane] = out_a;  // columns 64(c-1)+1 .. 64c
                    out_a = out_b;
                }
            };
            using T_ = std::true_type;
            using F_ = std::false_type;
            if (last) {
                if (c_lo == 0) chunk(0, T_{}, T_{});
                for (int32_t c = c_lo > 1 ? c_lo : 1; c <= c_hi; ++c) chunk(c, F_{}, T_{});
            } else {
                if (c_lo == 0) chunk(0, T_{}, F_{});
                for (int32_t c = c_lo > 1 ? c_lo : 1; c <= c_hi; ++c) chunk(c, F_{}, F_{});
                rout[64 * c_hi + 1 + lane] = out_a;  // the last processed hand-off chunk's first column
                if (lane == 0) rout[0] = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            int32_t* tmp = rin; rin = rout; rout = tmp;
        }
        // row n lives in lane (n-1) % 64 of the last strip
        const int owner = (n - 1) & 63;
        const int32_t bs = __shfl(best, owner, 64);
        const int32_t be = __shfl(bend, owner, 64);
        if (lane == 0) {
            out_score[pair] = n > 0 && m > 0 ? bs : 0;
            out_end[pair] = n > 0 && m > 0 ? be : 0;
        }
    }
}

// Banded knob, row form (used when 2*band+1 <= 192, lmax <= 1024 and magnitudes are small):
// lanes own band diagonals t = j - (i - d* - band) in [0, 2*band] and the sweep walks rows.
// diag = same lane of the previous row, up = lane t+1 of the previous row (wave_shl:1; out of the
// band at t = 2*band), and the row's left dependency H[t] = max(C[t], H[t-1] + indel) becomes an
// inclusive prefix maximum of C[t] - t*indel (DPP row_shr 1/2/4/8, row_bcast 15/31), segmented per
// pair: SEG = 16, 32 or 64 lanes (4, 2 or 1 pairs per wavefront), or NC = 2/3 chunks of 64 lanes
// carried left to right.  Same values as dp_kernel<int32_t, true> (only values matter: no traceback
// in band mode).  Column 0 is the boundary (value 0) inside the band; j < 0 and j > m are not cells.
constexpr int32_t kBandNeg = -(1 << 30);  // "-inf": host keeps (4*lmax + 2) * |score| < 2^29

template <int SEG>
__device__ __forceinline__ int32_t seg_scan_max(int32_t v) {
    // inclusive prefix max inside aligned SEG-lane segments (identity kBandNeg)
    v = max(v, __builtin_amdgcn_update_dpp(kBandNeg, v, 0x111, 0xF, 0xF, false));  // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(kBandNeg, v, 0x112, 0xF, 0xF, false));  // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(kBandNeg, v, 0x114, 0xF, 0xF, false));  // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(kBandNeg, v, 0x118, 0xF, 0xF, false));  // row_shr:8
    if constexpr (SEG >= 32) v = max(v, __builtin_amdgcn_update_dpp(kBandNeg, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    if constexpr (SEG >= 64) v = max(v, __builtin_amdgcn_update_dpp(kBandNeg, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return v;
}

template <int SEG, int NC>
__global__ __launch_bounds__(256) void band_row_kernel(
    const uint8_t* __restrict__ codes, const int64_t* __restrict__ off, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx, int64_t n_pairs,
    int32_t lcap, int32_t match, int32_t mismatch, int32_t indel, int32_t band, int32_t* __restrict__ out_score,
    int32_t* __restrict__ out_end, const int32_t* __restrict__ seed, uint32_t* __restrict__ err_flag) {
    constexpr int PPW = 64 / SEG;  // pairs per wavefront
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    const int seg = lane / SEG;      // pair slot in the wavefront
    const int t0 = lane % SEG;       // band lane inside the segment (chunk 0)
    uint8_t* sq = smem + (size_t)(wib * PPW + seg) * 2 * lcap;  // this pair's s, then t
    uint8_t* st = sq + lcap;
    const int64_t n_slots = (n_pairs + PPW - 1) / PPW;
    const int64_t wave0 = (int64_t)blockIdx.x * 4 + wib;
    for (int64_t slot = wave0; slot < n_slots; slot += (int64_t)gridDim.x * 4) {
        const int64_t p = slot * PPW + seg;
        const bool mine = p < n_pairs;
        int32_t a = mine ? a_idx[p] : 0, b = mine ? b_idx[p] : 0;
        bool ok = mine && a >= 0 && a < n_reads && b >= 0 && b < n_reads;
        if (!ok) { a = 0; b = 0; }
        const int32_t n = ok ? len[a] : 0, m = ok ? len[b] : 0;
        ok = ok && n <= lcap && m <= lcap;
        if (mine && !ok && t0 == 0) {
            ovl_flag_error(err_flag);
            out_score[p] = -1;
            out_end[p] = -1;
        }
        const int32_t jstar = ok ? seed[p] : 0;  // seed from the ungapped launch
        const int32_t dstar = n - jstar;
        // stage s and t of this pair in LDS (the segment's lanes copy them)
        if (ok) {
            const uint8_t* gs = codes + off[a];
            const uint8_t* gt = codes + off[b];
            for (int q = t0; q < n; q += SEG) sq[q] = gs[q];
            for (int q = t0; q < m; q += SEG) st[q] = gt[q];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // rows: from r0 (first row with a cell of column >= 1 in the band) to n
        const int32_t r0 = dstar - band + 1 > 1 ? dstar - band + 1 : 1;
        int32_t rows = ok && n > 0 && m > 0 ? n - r0 + 1 : 0;
        // previous row (r0 - 1) in band lanes: row 0 is all zero, otherwise only column 0 is a value
        int32_t hp[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int32_t t = t0 + 64 * c;
            const int32_t j = (r0 - 1) - dstar - band + t;
            hp[c] = (t <= 2 * band && (j == 0 || (r0 == 1 && j >= 0 && j <= m))) ? 0 : kBandNeg;
        }
        // segments of a wavefront run different pairs: iterate to the longest
        int32_t rows_max = rows;
#pragma unroll
        for (int o = SEG; o < 64; o <<= 1) rows_max = max(rows_max, __shfl_xor(rows_max, o, 64));
        int64_t bestkey = INT64_MIN;
        for (int32_t k = 0; k < rows_max; ++k) {
            const int32_t i = r0 + k;
            const bool live = k < rows;
            const int32_t jlo = i - dstar - band;
            const uint32_t sc = live ? (uint32_t)sq[i - 1] : 0xFFFFu;
            int32_t h[NC];
            int32_t carry = kBandNeg;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int32_t t = t0 + 64 * c;
                const int32_t j = jlo + t;
                const bool cell = live && t <= 2 * band && j >= 1 && j <= m;
                const uint32_t tc = cell ? (uint32_t)st[j - 1] : 0xFFFFFu;
                // up: lane t+1 of the previous row (wave_shl:1; chunk c+1's lane 0 for lane 63)
                int32_t upv = __builtin_amdgcn_update_dpp(kBandNeg, hp[c], 0x130, 0xF, 0xF, false);
                if constexpr (NC > 1) {
                    if (c + 1 < NC) {
                        const int32_t nxt = __builtin_amdgcn_readlane(hp[c + 1 < NC ? c + 1 : c], 0);
                        if (lane == 63) upv = nxt;
                    }
                }
                const bool up_ok = t < 2 * band;
                const int32_t dv = hp[c] + (sc == tc ? match : mismatch);
                int32_t cv = up_ok ? max(dv, upv + indel) : dv;
                cv = cell ? cv : ((live && j == 0 && t <= 2 * band) ? 0 : kBandNeg);
                const int32_t tind = t * indel;
                int32_t g = seg_scan_max<SEG>(cv - tind);
                if constexpr (NC > 1) {
                    g = max(g, carry);
                    carry = __builtin_amdgcn_readlane(g, 63);
                }
                int32_t hv = g + tind;
                hv = (cell || (live && j == 0 && t <= 2 * band)) ? hv : kBandNeg;
                h[c] = hv;
                if (live && i == n && t <= 2 * band && j >= 0 && j <= m) {
                    // last row: strict '>' first argmax = max value, then smallest j
                    const int64_t key = (int64_t)hv * 2048 + (2047 - j);
                    bestkey = key > bestkey ? key : bestkey;
                }
            }
#pragma unroll
            for (int c = 0; c < NC; ++c) hp[c] = h[c];
        }
        // reduce the segment's keys
#pragma unroll
        for (int o = 1; o < SEG; o <<= 1) {
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)bestkey, o, 64);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)bestkey >> 32), o, 64);
            const int64_t ok2 = (int64_t)(((uint64_t)hi << 32) | lo);
            bestkey = ok2 > bestkey ? ok2 : bestkey;
        }
        if (mine && ok && t0 == 0) {
            int32_t sc_out = 0, en_out = 0;
            if (n > 0 && m > 0 && bestkey != INT64_MIN) {
                // floor division of the packed key (value may be negative)
                const int64_t v = bestkey >= 0 ? bestkey / 2048 : -((-bestkey + 2047) / 2048);
                sc_out = (int32_t)v;
                en_out = 2047 - (int32_t)(bestkey - v * 2048);
            }
            out_score[p] = sc_out;
            out_end[p] = en_out;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // LDS reuse by the next slot
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

extern "C" hipError_t ovl_launch_unpack2(const uint8_t* pk, const uint8_t* lut, uint8_t* codes, int64_t n,
                                         hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if (reinterpret_cast<uintptr_t>(pk) & 15) return hipErrorInvalidValue;
    int64_t blocks = ((n + 63) / 64 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    unpack2_kernel<<<(unsigned)blocks, 256, 0, stream>>>(pk, lut, codes, n);
    return hipGetLastError();
}

extern "C" hipError_t ovl_launch_pack(int planes, const uint8_t* codes, const int64_t* off, const int32_t* len,
                                      int32_t n_reads, int32_t w, int32_t srow, int32_t trow, uint32_t* sfx,
                                      uint32_t* pfx, hipStream_t stream) {
    if (n_reads <= 0) return hipSuccess;
    const int64_t total = (int64_t)n_reads * w;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    switch (planes) {
        case 2: pack_planes_kernel<2><<<(unsigned)blocks, 256, 0, stream>>>(codes, off, len, n_reads, w, srow, trow, sfx, pfx); break;
        case 4: pack_planes_kernel<4><<<(unsigned)blocks, 256, 0, stream>>>(codes, off, len, n_reads, w, srow, trow, sfx, pfx); break;
        case 8: pack_planes_kernel<8><<<(unsigned)blocks, 256, 0, stream>>>(codes, off, len, n_reads, w, srow, trow, sfx, pfx); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int W, int KM, bool LAT, int OM, bool IX = false>
static void launch_uniform_4(const OvlUngappedArgs& g, unsigned blocks, hipStream_t stream) {
    if (g.ev_start) {
        hipExtLaunchKernelGGL(uniform_kernel<W, KM, LAT, OM, IX>, dim3(blocks), dim3(256), 0, stream, g.ev_start,
                              g.ev_stop, 0, g.sfx, g.pfx, g.len, g.n_reads, g.a_idx, g.b_idx, g.n_pairs, g.lw, g.full,
                              g.match, g.mismatch, g.out_score, g.out_end, g.err_flag, g.heavy_ids, g.tile_flags,
                              g.heavy_n, g.tile_base, g.ix_b16, g.ix_d8, g.ix_base);
        return;
    }
    uniform_kernel<W, KM, LAT, OM, IX><<<blocks, 256, 0, stream>>>(
        g.sfx, g.pfx, g.len, g.n_reads, g.a_idx, g.b_idx, g.n_pairs, g.lw, g.full, g.match, g.mismatch, g.out_score,
        g.out_end, g.err_flag, g.heavy_ids, g.tile_flags, g.heavy_n, g.tile_base, g.ix_b16, g.ix_d8, g.ix_base);
}

template <int W, int KM, bool LAT>
static bool launch_uniform_m(const OvlUngappedArgs& g, unsigned blocks, hipStream_t stream) {
    if (g.ix_b16) {
        // host-encoded pair lists: throughput mode, int32 keys, host-mapped results (the compact one-shot path)
        if constexpr (!LAT && KM == 0) {
            if (g.host_out == 1) {
                launch_uniform_4<W, KM, LAT, 1, true>(g, blocks, stream);
                return true;
            }
            if (g.host_out == 2) {
                launch_uniform_4<W, KM, LAT, 2, true>(g, blocks, stream);
                return true;
            }
        }
        return false;
    }
    switch (g.host_out) {
        case 0: launch_uniform_4<W, KM, LAT, 0>(g, blocks, stream); return true;
        case 1: launch_uniform_4<W, KM, LAT, 1>(g, blocks, stream); return true;
        case 2:
            if constexpr (KM == 0) {  // packed results: int32 keys only (the host asks for them only then)
                launch_uniform_4<W, KM, LAT, 2>(g, blocks, stream);
                return true;
            }
            return false;
    }
    return false;
}

template <int W, int KM>
static bool launch_uniform_t(const OvlUngappedArgs& g, unsigned blocks, hipStream_t stream) {
    // latency mode (two wavefronts per tile) when rs_log2 > 0; host-mapped outputs stream out non-temporally
    return g.rs_log2 > 0 ? launch_uniform_m<W, KM, true>(g, blocks, stream)
                         : launch_uniform_m<W, KM, false>(g, blocks, stream);
}

template <int P, int W, int KM>
static void launch_general_t(const OvlUngappedArgs& g, unsigned blocks, hipStream_t stream) {
    general_kernel<P, W, KM><<<blocks, 256, 0, stream>>>(g.sfx, g.pfx, g.len, g.n_reads, g.a_idx, g.b_idx,
                                                         g.n_pairs, g.rs_log2, g.match, g.mismatch, g.out_score,
                                                         g.out_end, g.err_flag);
}

template <int KM>
static bool dispatch_uniform(const OvlUngappedArgs& g, unsigned blocks, hipStream_t s) {
    switch (g.wmax) {
        case 1: return launch_uniform_t<1, KM>(g, blocks, s);
        case 2: return launch_uniform_t<2, KM>(g, blocks, s);
        case 3: return launch_uniform_t<3, KM>(g, blocks, s);
        case 4: return launch_uniform_t<4, KM>(g, blocks, s);
        case 5: return launch_uniform_t<5, KM>(g, blocks, s);
        case 6: return launch_uniform_t<6, KM>(g, blocks, s);
        case 7: return launch_uniform_t<7, KM>(g, blocks, s);
        case 8: return launch_uniform_t<8, KM>(g, blocks, s);
    }
    return false;
}

template <int P, int KM>
static bool dispatch_general_w(const OvlUngappedArgs& g, unsigned blocks, hipStream_t s) {
    switch (g.wmax) {
        case 1: launch_general_t<P, 1, KM>(g, blocks, s); return true;
        case 2: launch_general_t<P, 2, KM>(g, blocks, s); return true;
        case 3: launch_general_t<P, 3, KM>(g, blocks, s); return true;
        case 4: launch_general_t<P, 4, KM>(g, blocks, s); return true;
        case 5: launch_general_t<P, 5, KM>(g, blocks, s); return true;
        case 6: launch_general_t<P, 6, KM>(g, blocks, s); return true;
        case 7: launch_general_t<P, 7, KM>(g, blocks, s); return true;
        case 8: launch_general_t<P, 8, KM>(g, blocks, s); return true;
    }
    return false;
}

template <int KM>
static bool dispatch_general(const OvlUngappedArgs& g, unsigned blocks, hipStream_t s) {
    switch (g.planes) {
        case 2: return dispatch_general_w<2, KM>(g, blocks, s);
        case 4: return dispatch_general_w<4, KM>(g, blocks, s);
        case 8: return dispatch_general_w<8, KM>(g, blocks, s);
    }
    return false;
}

static unsigned grid_for(int64_t pairs, int rs_log2, int64_t max_blocks) {
    const int64_t ppw = 64 >> rs_log2;
    int64_t blocks = ((pairs + ppw - 1) / ppw + 3) / 4;  // 4 wavefronts per block
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    return (unsigned)blocks;
}

// Uniform path (P = 2 and a dominant read length lw): uniform_kernel, which also
// scores the other pairs through its LDS side ring.  Otherwise general_kernel.
// flags[t] = 1 iff tile t (pairs 64t .. 64t + 63) holds a pair whose read a is not of the dominant length
// (a side pair of uniform_kernel's ring); one wavefront per tile
__global__ __launch_bounds__(256) void tile_flags_kernel(const int32_t* __restrict__ a_idx, int64_t n_pairs,
                                                         const uint32_t* __restrict__ full, int32_t n_reads,
                                                         uint8_t* __restrict__ flags) {
    const int64_t n_tiles = (n_pairs + 63) >> 6;
    const int lane = threadIdx.x & 63;
    for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < n_tiles; t += (int64_t)gridDim.x * 4) {
        const int64_t p = t * 64 + lane;
        bool side = false;
        if (p < n_pairs) {
            const int32_t a = a_idx[p];
            side = a >= 0 && a < n_reads && !((full[a >> 5] >> (a & 31)) & 1u);
        }
        const uint64_t m = __ballot(side);
        if (lane == 0) flags[t] = m ? 1 : 0;
    }
}

extern "C" hipError_t ovl_launch_tile_flags(const int32_t* a_idx, int64_t n_pairs, const uint32_t* full,
                                            int32_t n_reads, uint8_t* flags, hipStream_t stream) {
    const int64_t n_tiles = (n_pairs + 63) >> 6;
    if (n_tiles <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n_tiles + 3) / 4, 8192);
    tile_flags_kernel<<<(unsigned)blocks, 256, 0, stream>>>(a_idx, n_pairs, full, n_reads, flags);
    return hipGetLastError();
}

extern "C" hipError_t ovl_launch_ungapped(const OvlUngappedArgs* g, hipStream_t stream) {
    if (g->n_pairs <= 0) return hipSuccess;
    bool ok;
    if (g->host_out >= 2 && (g->lw <= 0 || g->key64)) return hipErrorInvalidValue;  // packed: uniform, int32 keys
    if (g->host_out < 0 || g->host_out > 2) return hipErrorInvalidValue;
    if (g->ix_b16 && (g->lw <= 0 || g->key64 || g->rs_log2 > 0 || g->heavy_ids || !g->ix_d8 || !g->ix_base))
        return hipErrorInvalidValue;  // host-encoded lists: uniform throughput mode only
    if (g->lw > 0) {
        // rs_log2 > 0 here selects the latency mode
        const unsigned nb = grid_for((g->n_pairs << (g->rs_log2 > 0 ? 1 : 0)) +
                                         (g->heavy_ids && g->rs_log2 == 0 ? 64 * (int64_t)g->heavy_n : 0),
                                     0, g->max_blocks);
        ok = g->key64 ? dispatch_uniform<1>(*g, nb, stream) : dispatch_uniform<0>(*g, nb, stream);
    } else {
        const unsigned nb = grid_for(g->n_pairs, g->rs_log2, g->max_blocks);
        ok = g->key64 ? dispatch_general<1>(*g, nb, stream) : dispatch_general<0>(*g, nb, stream);
    }
    if (!ok) return hipErrorInvalidValue;
    return hipGetLastError();
}

// Banded knob, anti-diagonal form (default for bands up to 255 when values fit int32).
//
// Lanes sit on band diagonals and a step is one anti-diagonal a = i + j: every cell of the band
// depends only on anti-diagonals a-1 (up: diagonal d-1, left: diagonal d+1) and a-2 (diag: own
// diagonal), so no in-step scan is needed.  A cell of diagonal d exists on every second
// anti-diagonal; each lane therefore holds D consecutive diagonals (slots k = 0..D-1, relative
// band index r = D*lane + k) and updates the even slots on even steps and the odd slots on odd
// ones, which keeps every lane busy on every step.  A segment of P = ceil((2W+1)/D) lanes holds
// one pair; 64/P segments share a wavefront.  The slot holding r = 2W is KW = 2W - D(P-1) of the
// segment's last lane; the slots above it are padding.  Band-edge predecessors ("up" of r = 0,
// "left" of r = 2W) are -inf (kBandNeg), as in oracle_overlap_banded; cells left of column 1 or
// above row 1 are the table's zero boundary.
//
// Values are kept as w = dp + indel, so both gap moves are read as stored and a cell is
// w' = max3(w_diag + (score - indel), w_up, w_left) + indel (5 VALU per cell with the compare).
// The s and t codes of each segment's pair are staged in LDS; slot k of lane l at iteration kap
// (steps 2kap, 2kap+1) reads s[I0 + kap + ceil(k/2) - 1] and t[J0 + kap - floor(k/2) - 1].
template <int D, int KW>
__global__ __launch_bounds__(64, (D <= 4 ? 8 : 6)) void band_diag_kernel(
    const uint8_t* __restrict__ codes, const int64_t* __restrict__ off, const int32_t* __restrict__ len,
    int32_t n_reads, const int32_t* __restrict__ a_idx, const int32_t* __restrict__ b_idx, int64_t n_pairs,
    int32_t lcap, int32_t match, int32_t mismatch, int32_t indel, int32_t W, int32_t nseg,
    int32_t* __restrict__ out_score, int32_t* __restrict__ out_end, const int32_t* __restrict__ seed,
    uint32_t* __restrict__ err_flag) {
    constexpr int U = 8;       // iterations (2 anti-diagonal steps each) per unrolled block
    constexpr int H = D / 2;   // slots of one parity
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int64_t* keys = reinterpret_cast<int64_t*>(smem);  // per-lane row-n keys for the segment max
    const int front = W + D + 16;
    unsigned char* chars = smem + 512 + front;
    const int lane = threadIdx.x;
    const int P = (2 * W + D) / D;
    const int seg_raw = lane / P;
    const bool real = seg_raw < nseg;
    const int seg = real ? seg_raw : nseg - 1;
    const int sl = real ? lane - seg * P : 0;
    const bool first = sl == 0;
    const bool last = real && sl == P - 1;
    unsigned char* ss = chars + (size_t)seg * 2 * lcap;
    unsigned char* ts = ss + lcap;
    const int32_t wneg = kBandNeg;
    const int32_t sc_ma = match - indel, sc_mm = mismatch - indel;
    const int64_t n_tasks = (n_pairs + nseg - 1) / nseg;
    for (int64_t task = blockIdx.x; task < n_tasks; task += gridDim.x) {
        const int64_t pair = task * nseg + seg;
        const bool live = real && pair < n_pairs;
        int32_t n = 0, m = 0, jstar = 0;
        const uint8_t* sg = codes;
        const uint8_t* tg = codes;
        bool bad = false;
        if (live) {
            const int32_t a = a_idx[pair], b = b_idx[pair];
            bad = a < 0 || a >= n_reads || b < 0 || b >= n_reads;
            if (!bad) {
                n = len[a];
                m = len[b];
                jstar = seed[pair];
                bad = n > lcap || m > lcap || jstar < 0 || jstar > m;
                sg = codes + off[a];
                tg = codes + off[b];
            }
            if (bad) n = m = jstar = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // previous task's LDS readers are done
        if (live) {
#pragma unroll 4
            for (int x = sl; x < n; x += P) ss[x] = sg[x];
#pragma unroll 4
            for (int x = sl; x < m; x += P) ts[x] = tg[x];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // geometry: band diagonals d = dlo + r, first anti-diagonal amin (parity of dlo)
        const int32_t dstar = n - jstar, dlo = dstar - W, dhi = dstar + W;
        int32_t amin = (dlo <= 0 && dhi >= 0) ? 2 : (dlo > 0 ? dlo + 2 : 2 - dhi);
        amin -= (amin - dlo) & 1;
        const int32_t d0 = dlo + D * sl;
        const int32_t I0 = (amin + d0) >> 1, J0 = (amin - d0) >> 1;
        const int32_t KN = (2 * n - d0 - amin) >> 1;  // slot k meets row n at iteration KN - ceil(k/2)
        int32_t kend = 0, kpro = 0, ktlo = INT32_MAX, kthi = -1;
        if (live && !bad) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const int32_t r = D * sl + k, d = d0 + k;
                if (r > 2 * W) continue;
                const int32_t par = k & 1;
                const int32_t ast = (d < 0 ? -d : d) + 2;
                const int32_t aend = min(2 * n - d, 2 * m + d);
                kpro = max(kpro, (ast - amin - par) >> 1);
                if (ast > aend) continue;
                kend = max(kend, ((aend - amin - par) >> 1) + 1);
                const int32_t jn = n - d;
                if (jn >= 1 && jn <= m) {
                    const int32_t kn = KN - ((k + 1) >> 1);
                    ktlo = min(ktlo, kn);
                    kthi = max(kthi, kn);
                }
            }
        }
        for (int o = 32; o; o >>= 1) {
            kend = max(kend, __shfl_xor(kend, o, 64));
            kpro = max(kpro, __shfl_xor(kpro, o, 64));
            ktlo = min(ktlo, __shfl_xor(ktlo, o, 64));
            kthi = max(kthi, __shfl_xor(kthi, o, 64));
        }
        // wave-uniform block bounds (multiples of U): masks before KP, row-n capture in [TL, TH)
        kend = __builtin_amdgcn_readfirstlane(kend);
        kpro = __builtin_amdgcn_readfirstlane(kpro);
        ktlo = __builtin_amdgcn_readfirstlane(ktlo);
        kthi = __builtin_amdgcn_readfirstlane(kthi);
        const int32_t KE = (kend + U - 1) / U * U;
        const int32_t KP = min(KE, (kpro + U - 1) / U * U);
        const int32_t TL = kthi < 0 ? KE : ktlo / U * U;
        const int32_t TH = kthi < 0 ? KE : min(KE, (kthi + U) / U * U);

        int32_t w[D], cap[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            w[k] = indel;  // zero boundary (w = dp + indel)
            cap[k] = wneg;
        }
        const int32_t Ai = 1 - I0, Bj = 1 - J0;  // slot k valid once kap + ceil(k/2) >= Ai, kap - floor(k/2) >= Bj
        const unsigned char* sp = ss + I0 - 1;
        const unsigned char* tp = ts + J0 - H;
        auto block = [&](int32_t kb, auto pro_t, auto trk_t) {
            constexpr bool PRO = decltype(pro_t)::value;
            constexpr bool TRK = decltype(trk_t)::value;
            int32_t S[U + H], T[U + H];
            const unsigned char* spb = sp + kb;
            const unsigned char* tpb = tp + kb;
#pragma unroll
            for (int x = 0; x < U + H; ++x) {
                S[x] = spb[x];
                T[x] = tpb[x];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int32_t kap = kb + u;
                // even step: even slots read the odd slots of the previous step
                // wave_shr:1 (lane 0 is a segment's first lane: the mask covers it)
                int32_t upsh = __builtin_amdgcn_mov_dpp(w[D - 1], 0x138, 0xF, 0xF, true);
                upsh = first ? wneg : upsh;
#pragma unroll
                for (int k = 0; k < D; k += 2) {
                    const int32_t up = k == 0 ? upsh : w[k - 1];
                    const int32_t left = (k == KW) ? (last ? wneg : w[k + 1]) : w[k + 1];
                    const int32_t sc = S[u + k / 2] == T[u + H - 1 - k / 2] ? sc_ma : sc_mm;
                    int32_t nv = max(max(w[k] + sc, up), left) + indel;
                    if constexpr (PRO) nv = ((kap + k / 2 >= Ai) & (kap - k / 2 >= Bj)) ? nv : indel;
                    w[k] = nv;
                    if constexpr (TRK) cap[k] = kap + k / 2 == KN ? nv : cap[k];
                }
                // odd step: odd slots read the even slots just written
                // wave_shl:1 (lane 63 holds padding or an unused lane: its input is never read)
                const int32_t lsh = __builtin_amdgcn_mov_dpp(w[0], 0x130, 0xF, 0xF, true);
#pragma unroll
                for (int k = 1; k < D; k += 2) {
                    const int32_t up = w[k - 1];
                    const int32_t left = k == D - 1 ? lsh : w[k + 1];
                    const int32_t sc = S[u + (k + 1) / 2] == T[u + H - 1 - (k - 1) / 2] ? sc_ma : sc_mm;
                    int32_t nv = max(max(w[k] + sc, up), left) + indel;
                    if constexpr (PRO) nv = ((kap + (k + 1) / 2 >= Ai) & (kap - (k - 1) / 2 >= Bj)) ? nv : indel;
                    w[k] = nv;
                    if constexpr (TRK) cap[k] = kap + (k + 1) / 2 == KN ? nv : cap[k];
                }
            }
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        for (int32_t kb = 0; kb < KE;) {
            const bool pro = kb < KP, trk = kb >= TL && kb < TH;
            int32_t nx = KE;
            if (KP > kb) nx = min(nx, KP);
            if (TL > kb) nx = min(nx, TL);
            if (TH > kb) nx = min(nx, TH);
            if (pro && trk) for (; kb < nx; kb += U) block(kb, T_{}, T_{});
            else if (pro) for (; kb < nx; kb += U) block(kb, T_{}, F_{});
            else if (trk) for (; kb < nx; kb += U) block(kb, F_{}, T_{});
            else for (; kb < nx; kb += U) block(kb, F_{}, F_{});
        }
        // row-n keys: max value, ties to the smallest column (the reference's first strict '>')
        int64_t key = INT64_MIN;
        if (live && !bad) {
            if (first && jstar <= W) key = (int64_t)0xFFFFFFFFll;  // j = 0 inside the band: value 0
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const int32_t r = D * sl + k, d = d0 + k, jn = n - d;
                if (r <= 2 * W && jn >= 1 && jn <= m) {
                    const int64_t kk = ((int64_t)(cap[k] - indel) << 32) | (uint32_t)~jn;
                    key = kk > key ? kk : key;
                }
            }
        }
        keys[lane] = key;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (live && first) {
            for (int x = 1; x < P; ++x) {
                const int64_t kx = keys[lane + x];
                key = kx > key ? kx : key;
            }
            if (bad) {
                ovl_flag_error(err_flag);
                out_score[pair] = -1;
                out_end[pair] = -1;
            } else {
                out_score[pair] = (int32_t)(key >> 32);
                out_end[pair] = (int32_t)~(uint32_t)key;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

template <typename Acc, bool BANDED>
static void launch_dp_t(const OvlDpArgs* g, unsigned blocks, size_t lds, hipStream_t stream) {
    dp_kernel<Acc, BANDED><<<blocks, 64, lds, stream>>>(g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx,
                                                         g->n_pairs, g->mcap, g->match, g->mismatch, g->indel,
                                                         g->band, g->out_score, g->out_end, g->seed, g->tb, g->err_flag);
}

template <int SEG, int NC>
static void launch_band_row_t(const OvlDpArgs* g, hipStream_t stream) {
    constexpr int PPW = 64 / SEG;
    const int64_t slots = (g->n_pairs + PPW - 1) / PPW;
    int64_t blocks = (slots + 3) / 4;
    if (blocks > 16384) blocks = 16384;
    const size_t lds = (size_t)4 * PPW * 2 * g->mcap;
    band_row_kernel<SEG, NC><<<(unsigned)blocks, 256, lds, stream>>>(
        g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx, g->n_pairs, g->mcap, (int32_t)g->match,
        (int32_t)g->mismatch, (int32_t)g->indel, g->band, g->out_score, g->out_end, g->seed, g->err_flag);
}

template <int D, int KW>
static void launch_band_diag_t(const OvlDpArgs* g, int nseg, hipStream_t stream) {
    const int W = g->band;
    const int64_t lcap = g->mcap > 0 ? g->mcap : 1;
    // keys + front pad + one 2*lcap stride per segment (s then t) + the over-read tail
    const size_t lds = 512 + (size_t)(W + D + 16) + (size_t)(nseg + 1) * 2 * lcap + W + 64;
    int64_t blocks = (g->n_pairs + nseg - 1) / nseg;
    if (blocks > 32768) blocks = 32768;
    band_diag_kernel<D, KW><<<(unsigned)blocks, 64, lds, stream>>>(
        g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx, g->n_pairs, (int32_t)lcap, (int32_t)g->match,
        (int32_t)g->mismatch, (int32_t)g->indel, W, nseg, g->out_score, g->out_end, g->seed, g->err_flag);
}

// Slots per lane for the anti-diagonal form: the VALU cost per pair-iteration is about
// (5 D + 8) / segments-per-wave; the smallest wins.  Returns D (0: band too wide).
extern "C" int ovl_band_diag_slots(int32_t band, int32_t lcap, int32_t* nseg_out) {
    int bestD = 0, bestseg = 0;
    double bestc = 1e30;
    for (int D = 2; D <= 8; D *= 2) {
        const int P = (2 * band + D) / D;
        if (P > 64) continue;
        int nseg = 64 / P;
        // keep the per-wave LDS near 24 KiB (at least one segment)
        const int64_t per = 2 * (int64_t)(lcap > 0 ? lcap : 1);
        const int64_t fit = (24576 - 1024 - 2 * (int64_t)band) / per - 1;
        if (nseg > fit) nseg = fit > 1 ? (int)fit : 1;
        const double c = (5.0 * D + 8.0) / nseg;
        if (c < bestc - 1e-9) {
            bestc = c;
            bestD = D;
            bestseg = nseg;
        }
    }
    if (nseg_out) *nseg_out = bestseg;
    return bestD;
}

static hipError_t launch_band_diag(const OvlDpArgs* g, hipStream_t stream) {
    int nseg = 0;
    const int D = ovl_band_diag_slots(g->band, g->mcap, &nseg);
    if (D == 0) return hipErrorInvalidValue;
    const int P = (2 * g->band + D) / D;
    const int KW = 2 * g->band - D * (P - 1);
    switch (D * 16 + KW) {
        case 2 * 16 + 0: launch_band_diag_t<2, 0>(g, nseg, stream); break;
        case 4 * 16 + 0: launch_band_diag_t<4, 0>(g, nseg, stream); break;
        case 4 * 16 + 2: launch_band_diag_t<4, 2>(g, nseg, stream); break;
        case 8 * 16 + 0: launch_band_diag_t<8, 0>(g, nseg, stream); break;
        case 8 * 16 + 2: launch_band_diag_t<8, 2>(g, nseg, stream); break;
        case 8 * 16 + 4: launch_band_diag_t<8, 4>(g, nseg, stream); break;
        case 8 * 16 + 6: launch_band_diag_t<8, 6>(g, nseg, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" hipError_t ovl_launch_dp(const OvlDpArgs* g, hipStream_t stream) {
    if (g->n_pairs <= 0) return hipSuccess;
    int64_t blocks = g->n_pairs;
    if (blocks > 16384) blocks = 16384;
    const size_t lds = (size_t)2 * (g->mcap + 1) * sizeof(int32_t) + (size_t)g->mcap + 16;
    const unsigned nb = (unsigned)blocks;
    if (g->band >= 0) {
        // banded mode runs only where values fit int32 (the host checks) and never writes tb
        if (g->wide || g->tb) return hipErrorInvalidValue;
        const int lanes = 2 * g->band + 1;
        switch (g->band_form) {
            case OVL_BAND_FORM_DIAG:
                return launch_band_diag(g, stream);
            case OVL_BAND_FORM_ROWS:
                if (lanes <= 16) launch_band_row_t<16, 1>(g, stream);
                else if (lanes <= 32) launch_band_row_t<32, 1>(g, stream);
                else if (lanes <= 64) launch_band_row_t<64, 1>(g, stream);
                else if (lanes <= 128) launch_band_row_t<64, 2>(g, stream);
                else if (lanes <= 192) launch_band_row_t<64, 3>(g, stream);
                else return hipErrorInvalidValue;
                return hipGetLastError();
            case OVL_BAND_FORM_FAST: {
                const int32_t pitch = ((g->mcap + 126) / 64) * 64 + 64;
                const size_t lds2 = (size_t)2 * pitch * sizeof(int32_t) + (size_t)pitch;
                dp_fast_kernel<int32_t, true><<<nb, 64, lds2, stream>>>(
                    g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx, g->n_pairs, g->mcap, g->match,
                    g->mismatch, g->indel, g->band, g->out_score, g->out_end, g->seed, g->err_flag);
                return hipGetLastError();
            }
            default:
                break;
        }
        launch_dp_t<int32_t, true>(g, nb, lds, stream);
    } else if (!g->tb && !g->classic) {
        // scores only: the chunked kernel (LDS: two padded rows + padded t)
        const int32_t pitch = ((g->mcap + 126) / 64) * 64 + 64;
        const size_t lds2 = (size_t)2 * pitch * sizeof(int32_t) + (size_t)pitch;
        if (g->wide)
            dp_fast_kernel<int64_t, false><<<nb, 64, lds2, stream>>>(
                g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx, g->n_pairs, g->mcap, g->match,
                g->mismatch, g->indel, -1, g->out_score, g->out_end, g->seed, g->err_flag);
        else
            dp_fast_kernel<int32_t, false><<<nb, 64, lds2, stream>>>(
                g->codes, g->off, g->len, g->n_reads, g->a_idx, g->b_idx, g->n_pairs, g->mcap, g->match,
                g->mismatch, g->indel, -1, g->out_score, g->out_end, g->seed, g->err_flag);
    } else if (g->wide) {
        launch_dp_t<int64_t, false>(g, nb, lds, stream);
    } else {
        launch_dp_t<int32_t, false>(g, nb, lds, stream);
    }
    return hipGetLastError();
}

#ifdef OVL_TRACE
extern "C" __attribute__((visibility("default"))) int ovl_debug_trace_read(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ovl::ovl_trace_buf), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
