// ovl_expand.h — host expansion of packed results (ovl_kernels.hip put_pair, sink 2) into the caller's
// int32 (score, end) arrays.  Host code only (ovl_api.cpp; tests/c/expand_test.cpp checks every variant
// against the scalar form).
//
// Per pair one uint16 v = j << 8 | X (end j, mismatch count X over the L = j compared bases):
//   score = match*(j - X) + mismatch*X,  end = j
//   X == 0xFF: the score travels separately in esc[i] (a shorter read a inside b's window)
//   v == 0xFFFF: a bad pair, (-1, -1)
// Every int32-key score fits int16 (|score| < 2^15, the planner's condition), so the vector forms compute
// match*j + (mismatch - match)*X in wrapping 16-bit lanes and sign-extend.  Non-temporal stores where the
// destination is aligned: the arrays are written once and not re-read here, so no read-for-ownership.
#pragma once

#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace ovl_expand {

using Fn = void (*)(int32_t* s, int32_t* e, const uint16_t* pk, const int32_t* esc, int32_t match,
                    int32_t mismatch, bool nt, size_t lo, size_t hi);

inline void one(int32_t* s, int32_t* e, const uint16_t* pk, const int32_t* esc, int32_t match, int32_t mismatch,
                size_t i) {
    const uint32_t v = pk[i], j = v >> 8, x = v & 0xFFu;
    if (v == 0xFFFFu) {
        s[i] = e[i] = -1;
        return;
    }
    s[i] = x == 0xFFu ? esc[i] : match * (int32_t)(j - x) + mismatch * (int32_t)x;
    e[i] = (int32_t)j;
}

inline void expand_scalar(int32_t* s, int32_t* e, const uint16_t* pk, const int32_t* esc, int32_t match,
                          int32_t mismatch, bool, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) one(s, e, pk, esc, match, mismatch, i);
}

// the escaped and bad pairs among w lanes of a vector step, fixed in the temporaries ts / te
inline void fix_spills(int32_t* ts, int32_t* te, const uint16_t* pk, const int32_t* esc, size_t i, int w) {
    for (int k = 0; k < w; ++k) {
        const uint32_t v = pk[i + k];
        if ((v & 0xFFu) != 0xFFu) continue;
        if (v == 0xFFFFu) {
            ts[k] = te[k] = -1;
        } else {
            ts[k] = esc[i + k];
        }
    }
}

inline void expand_sse2(int32_t* s, int32_t* e, const uint16_t* pk, const int32_t* esc, int32_t match,
                        int32_t mismatch, bool nt, size_t lo, size_t hi) {
    size_t i = lo;
    for (; i < hi && ((uintptr_t)(s + i) & 15); ++i) one(s, e, pk, esc, match, mismatch, i);
    const bool s_al = nt, e_al = nt && ((uintptr_t)(e + i) & 15) == 0;
    const __m128i lo8 = _mm_set1_epi16(0xFF), zero = _mm_setzero_si128();
    const __m128i vm = _mm_set1_epi16((int16_t)match), vd = _mm_set1_epi16((int16_t)(mismatch - match));
    auto put = [](int32_t* p, __m128i v, bool al) {
        if (al) _mm_stream_si128(reinterpret_cast<__m128i*>(p), v);
        else _mm_storeu_si128(reinterpret_cast<__m128i*>(p), v);
    };
    for (; i + 8 <= hi; i += 8) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(pk + i));
        const __m128i x = _mm_and_si128(v, lo8);
        const __m128i j = _mm_srli_epi16(v, 8);
        const __m128i sc = _mm_add_epi16(_mm_mullo_epi16(j, vm), _mm_mullo_epi16(x, vd));
        __m128i s0 = _mm_srai_epi32(_mm_unpacklo_epi16(zero, sc), 16);
        __m128i s1 = _mm_srai_epi32(_mm_unpackhi_epi16(zero, sc), 16);
        __m128i e0 = _mm_unpacklo_epi16(j, zero);
        __m128i e1 = _mm_unpackhi_epi16(j, zero);
        if (_mm_movemask_epi8(_mm_cmpeq_epi16(x, lo8))) {
            alignas(16) int32_t ts[8], te[8];
            _mm_store_si128(reinterpret_cast<__m128i*>(ts), s0);
            _mm_store_si128(reinterpret_cast<__m128i*>(ts + 4), s1);
            _mm_store_si128(reinterpret_cast<__m128i*>(te), e0);
            _mm_store_si128(reinterpret_cast<__m128i*>(te + 4), e1);
            fix_spills(ts, te, pk, esc, i, 8);
            s0 = _mm_load_si128(reinterpret_cast<const __m128i*>(ts));
            s1 = _mm_load_si128(reinterpret_cast<const __m128i*>(ts + 4));
            e0 = _mm_load_si128(reinterpret_cast<const __m128i*>(te));
            e1 = _mm_load_si128(reinterpret_cast<const __m128i*>(te + 4));
        }
        put(s + i, s0, s_al);
        put(s + i + 4, s1, s_al);
        put(e + i, e0, e_al);
        put(e + i + 4, e1, e_al);
    }
    for (; i < hi; ++i) one(s, e, pk, esc, match, mismatch, i);
    _mm_sfence();
}

__attribute__((target("avx2"))) inline void put256(int32_t* p, __m256i v, bool al) {
    if (al) _mm256_stream_si256(reinterpret_cast<__m256i*>(p), v);
    else _mm256_storeu_si256(reinterpret_cast<__m256i*>(p), v);
}

__attribute__((target("avx512f,avx512bw"))) inline void put512(int32_t* p, __m512i v, bool al) {
    if (al) _mm512_stream_si512(reinterpret_cast<__m512i*>(p), v);
    else _mm512_storeu_si512(p, v);
}

__attribute__((target("avx2"))) inline void expand_avx2(int32_t* s, int32_t* e, const uint16_t* pk,
                                                        const int32_t* esc, int32_t match, int32_t mismatch,
                                                        bool nt, size_t lo, size_t hi) {
    size_t i = lo;
    for (; i < hi && ((uintptr_t)(s + i) & 31); ++i) one(s, e, pk, esc, match, mismatch, i);
    const bool s_al = nt, e_al = nt && ((uintptr_t)(e + i) & 31) == 0;
    const __m256i lo8 = _mm256_set1_epi16(0xFF);
    const __m256i vm = _mm256_set1_epi16((int16_t)match), vd = _mm256_set1_epi16((int16_t)(mismatch - match));
    for (; i + 16 <= hi; i += 16) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(pk + i));
        const __m256i x = _mm256_and_si256(v, lo8);
        const __m256i j = _mm256_srli_epi16(v, 8);
        const __m256i sc = _mm256_add_epi16(_mm256_mullo_epi16(j, vm), _mm256_mullo_epi16(x, vd));
        __m256i s0 = _mm256_cvtepi16_epi32(_mm256_castsi256_si128(sc));
        __m256i s1 = _mm256_cvtepi16_epi32(_mm256_extracti128_si256(sc, 1));
        __m256i e0 = _mm256_cvtepu16_epi32(_mm256_castsi256_si128(j));
        __m256i e1 = _mm256_cvtepu16_epi32(_mm256_extracti128_si256(j, 1));
        if (_mm256_movemask_epi8(_mm256_cmpeq_epi16(x, lo8))) {
            alignas(32) int32_t ts[16], te[16];
            _mm256_store_si256(reinterpret_cast<__m256i*>(ts), s0);
            _mm256_store_si256(reinterpret_cast<__m256i*>(ts + 8), s1);
            _mm256_store_si256(reinterpret_cast<__m256i*>(te), e0);
            _mm256_store_si256(reinterpret_cast<__m256i*>(te + 8), e1);
            fix_spills(ts, te, pk, esc, i, 16);
            s0 = _mm256_load_si256(reinterpret_cast<const __m256i*>(ts));
            s1 = _mm256_load_si256(reinterpret_cast<const __m256i*>(ts + 8));
            e0 = _mm256_load_si256(reinterpret_cast<const __m256i*>(te));
            e1 = _mm256_load_si256(reinterpret_cast<const __m256i*>(te + 8));
        }
        put256(s + i, s0, s_al);
        put256(s + i + 8, s1, s_al);
        put256(e + i, e0, e_al);
        put256(e + i + 8, e1, e_al);
    }
    for (; i < hi; ++i) one(s, e, pk, esc, match, mismatch, i);
    _mm_sfence();
}

// 32 pairs per step: one full 64-byte line per non-temporal store
__attribute__((target("avx512f,avx512bw"))) inline void expand_avx512(int32_t* s, int32_t* e, const uint16_t* pk,
                                                                      const int32_t* esc, int32_t match,
                                                                      int32_t mismatch, bool nt, size_t lo,
                                                                      size_t hi) {
    size_t i = lo;
    for (; i < hi && ((uintptr_t)(s + i) & 63); ++i) one(s, e, pk, esc, match, mismatch, i);
    const bool s_al = nt, e_al = nt && ((uintptr_t)(e + i) & 63) == 0;
    const __m512i lo8 = _mm512_set1_epi16(0xFF);
    const __m512i vm = _mm512_set1_epi16((int16_t)match), vd = _mm512_set1_epi16((int16_t)(mismatch - match));
    for (; i + 32 <= hi; i += 32) {
        const __m512i v = _mm512_loadu_si512(pk + i);
        const __m512i x = _mm512_and_si512(v, lo8);
        const __m512i j = _mm512_srli_epi16(v, 8);
        const __m512i sc = _mm512_add_epi16(_mm512_mullo_epi16(j, vm), _mm512_mullo_epi16(x, vd));
        __m512i s0 = _mm512_cvtepi16_epi32(_mm512_castsi512_si256(sc));
        __m512i s1 = _mm512_cvtepi16_epi32(_mm512_extracti64x4_epi64(sc, 1));
        __m512i e0 = _mm512_cvtepu16_epi32(_mm512_castsi512_si256(j));
        __m512i e1 = _mm512_cvtepu16_epi32(_mm512_extracti64x4_epi64(j, 1));
        if (_mm512_cmpeq_epi16_mask(x, lo8)) {
            alignas(64) int32_t ts[32], te[32];
            _mm512_store_si512(ts, s0);
            _mm512_store_si512(ts + 16, s1);
            _mm512_store_si512(te, e0);
            _mm512_store_si512(te + 16, e1);
            fix_spills(ts, te, pk, esc, i, 32);
            s0 = _mm512_load_si512(ts);
            s1 = _mm512_load_si512(ts + 16);
            e0 = _mm512_load_si512(te);
            e1 = _mm512_load_si512(te + 16);
        }
        put512(s + i, s0, s_al);
        put512(s + i + 16, s1, s_al);
        put512(e + i, e0, e_al);
        put512(e + i + 16, e1, e_al);
    }
    for (; i < hi; ++i) one(s, e, pk, esc, match, mismatch, i);
    _mm_sfence();
}

// isa: "scalar", "sse2", "avx2", "avx512" or NULL / "" (the widest this CPU runs); NULL if unsupported
inline Fn pick(const char* isa) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the device pass of a HIP translation unit parses host code too)
    const bool a512 = false, a2 = false;
#else
    __builtin_cpu_init();
    const bool a512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
    const bool a2 = __builtin_cpu_supports("avx2");
#endif
    if (!isa || !*isa) return a512 ? expand_avx512 : (a2 ? expand_avx2 : expand_sse2);
    if (!strcmp(isa, "scalar")) return expand_scalar;
    if (!strcmp(isa, "sse2")) return expand_sse2;
    if (!strcmp(isa, "avx2")) return a2 ? expand_avx2 : nullptr;
    if (!strcmp(isa, "avx512")) return a512 ? expand_avx512 : nullptr;
    return nullptr;
}

}  // namespace ovl_expand
