// ovl_encode.h — host encoding of a compact pair list (ovl_api.cpp encode_chunk, decoded on the device by
// ovl_pairs.hip).  Host code only (tests/c/encode_test.cpp checks every variant against the scalar form).
//
// Passes over a part [lo, hi) of one chunk, each reading one of the caller's int32 arrays once:
//   narrow: b[p] -> uint16 (an index outside [0, nr) becomes 0xFFFF), nr <= 65,535;
//   d8:     a as tile deltas (base[t] = a[64t], d8[p] = a[p] - base[t]), read by uniform_kernel in place;
//   runs:   the positions p where a[p] != a[p - 1] (and p == lo, against `prev`), as (a[p], p) into
//           vals / starts, decoded by runs_kernel; returns the count, or cap + 1 once more than `cap` runs
//           were found.
// The candidate lists of overlapGraphs.py:43-52 are a-major (~40-55 pairs per run), so the runs pass mostly
// compares 16 lanes and finds nothing.  The vector forms move the chunk at the host's memory rate where
// the scalar loops spend ~1 ns per pair (a compare-and-branch per element, a select per narrowed index).
#pragma once

#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace ovl_encode {

using NarrowFn = void (*)(const int32_t* B, int32_t nr, uint16_t* o, size_t lo, size_t hi);
using RunsFn = size_t (*)(const int32_t* A, int32_t prev, size_t lo, size_t hi, int32_t* vals, int32_t* starts,
                          size_t cap);

inline void narrow_scalar(const int32_t* B, int32_t nr, uint16_t* o, size_t lo, size_t hi) {
    for (size_t p = lo; p < hi; ++p) {
        const int32_t v = B[p];
        o[p] = (v >= 0 && v < nr) ? (uint16_t)v : (uint16_t)0xFFFF;
    }
}

inline size_t runs_scalar(const int32_t* A, int32_t prev, size_t lo, size_t hi, int32_t* vals, int32_t* starts,
                          size_t cap) {
    size_t r = 0;
    for (size_t p = lo; p < hi; ++p) {
        const int32_t v = A[p];
        if (v != prev) {
            if (r == cap) return cap + 1;
            vals[r] = v;
            starts[r] = (int32_t)p;
            ++r;
        }
        prev = v;
    }
    return r;
}

// 32 indices per step: two 64-byte loads, unsigned range compares, vpmovdw truncation, 0xFFFF blended in
__attribute__((target("avx512f,avx512bw,avx512vl"))) inline void narrow_avx512(const int32_t* B, int32_t nr,
                                                                               uint16_t* o, size_t lo, size_t hi) {
    size_t p = lo;
    const __m512i vnr = _mm512_set1_epi32(nr);
    const __m256i bad = _mm256_set1_epi16((int16_t)0xFFFF);
    for (; p + 32 <= hi; p += 32) {
        const __m512i v0 = _mm512_loadu_si512(B + p);
        const __m512i v1 = _mm512_loadu_si512(B + p + 16);
        const __mmask16 ok0 = _mm512_cmplt_epu32_mask(v0, vnr);
        const __mmask16 ok1 = _mm512_cmplt_epu32_mask(v1, vnr);
        const __m256i h0 = _mm256_mask_blend_epi16(ok0, bad, _mm512_cvtepi32_epi16(v0));
        const __m256i h1 = _mm256_mask_blend_epi16(ok1, bad, _mm512_cvtepi32_epi16(v1));
        _mm512_storeu_si512(o + p, _mm512_inserti64x4(_mm512_castsi256_si512(h0), h1, 1));
    }
    narrow_scalar(B, nr, o, p, hi);
}

// 32 positions per step against the same lanes shifted by one (an unaligned load at p - 1)
__attribute__((target("avx512f,avx512bw"))) inline size_t runs_avx512(const int32_t* A, int32_t prev, size_t lo,
                                                                      size_t hi, int32_t* vals, int32_t* starts,
                                                                      size_t cap) {
    if (lo >= hi) return 0;
    size_t r = runs_scalar(A, prev, lo, lo + 1, vals, starts, cap);
    if (r > cap) return cap + 1;
    size_t p = lo + 1;
    for (; p + 32 <= hi; p += 32) {
        const __mmask16 m0 = _mm512_cmpneq_epi32_mask(_mm512_loadu_si512(A + p), _mm512_loadu_si512(A + p - 1));
        const __mmask16 m1 =
            _mm512_cmpneq_epi32_mask(_mm512_loadu_si512(A + p + 16), _mm512_loadu_si512(A + p + 15));
        uint32_t m = (uint32_t)m0 | (uint32_t)m1 << 16;
        while (m) {
            const unsigned t = (unsigned)__builtin_ctz(m);
            if (r == cap) return cap + 1;
            vals[r] = A[p + t];
            starts[r] = (int32_t)(p + t);
            ++r;
            m &= m - 1;
        }
    }
    const size_t rest = runs_scalar(A, A[p - 1], p, hi, vals + r, starts + r, cap - r);
    return rest > cap - r ? cap + 1 : r + rest;
}

__attribute__((target("avx2"))) inline void narrow_avx2(const int32_t* B, int32_t nr, uint16_t* o, size_t lo,
                                                        size_t hi) {
    size_t p = lo;
    // v in [0, nr)  <=>  (v ^ INT_MIN) < (nr ^ INT_MIN) as signed (the unsigned compare AVX2 lacks)
    const __m256i flip = _mm256_set1_epi32(INT32_MIN);
    const __m256i vnr = _mm256_set1_epi32(nr ^ INT32_MIN);
    for (; p + 16 <= hi; p += 16) {
        __m256i v0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(B + p));
        __m256i v1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(B + p + 8));
        // bad lanes -> 0xFFFF (the all-ones lane truncates to it; good lanes are < 65,536)
        v0 = _mm256_or_si256(v0, _mm256_andnot_si256(_mm256_cmpgt_epi32(vnr, _mm256_xor_si256(v0, flip)),
                                                     _mm256_set1_epi32(-1)));
        v1 = _mm256_or_si256(v1, _mm256_andnot_si256(_mm256_cmpgt_epi32(vnr, _mm256_xor_si256(v1, flip)),
                                                     _mm256_set1_epi32(-1)));
        // keep the low 16 bits of each lane, then pack (unsigned saturation is exact on values <= 0xFFFF)
        const __m256i lo16 = _mm256_set1_epi32(0xFFFF);
        const __m256i pk = _mm256_packus_epi32(_mm256_and_si256(v0, lo16), _mm256_and_si256(v1, lo16));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(o + p), _mm256_permute4x64_epi64(pk, 0xD8));
    }
    narrow_scalar(B, nr, o, p, hi);
}

__attribute__((target("avx2"))) inline size_t runs_avx2(const int32_t* A, int32_t prev, size_t lo, size_t hi,
                                                        int32_t* vals, int32_t* starts, size_t cap) {
    if (lo >= hi) return 0;
    size_t r = runs_scalar(A, prev, lo, lo + 1, vals, starts, cap);
    if (r > cap) return cap + 1;
    size_t p = lo + 1;
    for (; p + 16 <= hi; p += 16) {
        const __m256i e0 = _mm256_cmpeq_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(A + p)),
                                              _mm256_loadu_si256(reinterpret_cast<const __m256i*>(A + p - 1)));
        const __m256i e1 = _mm256_cmpeq_epi32(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(A + p + 8)),
                                              _mm256_loadu_si256(reinterpret_cast<const __m256i*>(A + p + 7)));
        uint32_t m = ~((uint32_t)_mm256_movemask_ps(_mm256_castsi256_ps(e0)) |
                       (uint32_t)_mm256_movemask_ps(_mm256_castsi256_ps(e1)) << 8) &
                     0xFFFFu;
        while (m) {
            const unsigned t = (unsigned)__builtin_ctz(m);
            if (r == cap) return cap + 1;
            vals[r] = A[p + t];
            starts[r] = (int32_t)(p + t);
            ++r;
            m &= m - 1;
        }
    }
    const size_t rest = runs_scalar(A, A[p - 1], p, hi, vals + r, starts + r, cap - r);
    return rest > cap - r ? cap + 1 : r + rest;
}

// tile deltas: for each tile t of 64 pairs in [lo, hi) (lo a multiple of 64; the last tile may be short),
// base[t] = a[64t] and d8[p] = a[p] - base[t].  False when some a[p] is outside [0, nr) or more than 255
// above its tile's first (a list that is not a-major); d8 / base are then partly written.
inline bool d8_scalar(const int32_t* A, int32_t nr, uint8_t* d8, int32_t* base, size_t lo, size_t hi) {
    for (size_t t0 = lo; t0 < hi; t0 += 64) {
        const int32_t b0 = A[t0];
        base[t0 >> 6] = b0;
        const size_t t1 = t0 + 64 < hi ? t0 + 64 : hi;
        for (size_t p = t0; p < t1; ++p) {
            const int32_t v = A[p];
            const uint32_t dv = (uint32_t)v - (uint32_t)b0;
            if ((uint32_t)v >= (uint32_t)nr || dv > 255u) return false;
            d8[p] = (uint8_t)dv;
        }
    }
    return true;
}

// a tile per step: four 64-byte loads, unsigned range checks, vpmovdb into one 64-byte store
__attribute__((target("avx512f,avx512bw"))) inline bool d8_avx512(const int32_t* A, int32_t nr, uint8_t* d8,
                                                                  int32_t* base, size_t lo, size_t hi) {
    const __m512i vnr = _mm512_set1_epi32(nr), v255 = _mm512_set1_epi32(255);
    size_t t0 = lo;
    for (; t0 + 64 <= hi; t0 += 64) {
        const int32_t b0 = A[t0];
        base[t0 >> 6] = b0;
        const __m512i vb = _mm512_set1_epi32(b0);
        __mmask16 bad = 0;
        __m128i q[4];
        for (int k = 0; k < 4; ++k) {
            const __m512i v = _mm512_loadu_si512(A + t0 + 16 * k);
            const __m512i dv = _mm512_sub_epi32(v, vb);
            bad |= _mm512_cmpge_epu32_mask(v, vnr) | _mm512_cmpgt_epu32_mask(dv, v255);
            q[k] = _mm512_cvtepi32_epi8(dv);
        }
        if (bad) return false;
        const __m512i out = _mm512_inserti64x4(
            _mm512_castsi256_si512(_mm256_inserti128_si256(_mm256_castsi128_si256(q[0]), q[1], 1)),
            _mm256_inserti128_si256(_mm256_castsi128_si256(q[2]), q[3], 1), 1);
        _mm512_storeu_si512(d8 + t0, out);
    }
    return d8_scalar(A, nr, d8, base, t0, hi);
}

using D8Fn = bool (*)(const int32_t* A, int32_t nr, uint8_t* d8, int32_t* base, size_t lo, size_t hi);

struct Fns {
    NarrowFn narrow;
    RunsFn runs;
    D8Fn d8;
};

// isa: "scalar", "avx2", "avx512" or NULL / "" (the widest this CPU runs); all null if unsupported
inline Fns pick(const char* isa) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the device pass of a HIP translation unit parses host code too)
    const bool a512 = false, a2 = false;
#else
    __builtin_cpu_init();
    const bool a512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                      __builtin_cpu_supports("avx512vl");
    const bool a2 = __builtin_cpu_supports("avx2");
#endif
    const Fns scalar{narrow_scalar, runs_scalar, d8_scalar}, v2{narrow_avx2, runs_avx2, d8_scalar},
        v512{narrow_avx512, runs_avx512, d8_avx512}, none{nullptr, nullptr, nullptr};
    if (!isa || !*isa) return a512 ? v512 : (a2 ? v2 : scalar);
    if (!strcmp(isa, "scalar")) return scalar;
    if (!strcmp(isa, "avx2")) return a2 ? v2 : none;
    if (!strcmp(isa, "avx512")) return a512 ? v512 : none;
    return none;
}

}  // namespace ovl_encode
