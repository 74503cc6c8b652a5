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

// ---------------------------------------------------------------------------------------------------------------
// Tile records (ovl_kernels.hip put_tile9, sink 3): per 64-pair tile t a record at rec + 256 t --
//   bytes [0, 64) the low 8 bits of lane l's 9-bit code c, byte l;  bytes [64, 72) bit l = bit 8 of c;
//   bytes [72, ..) the uint16 OM 2 word of each lane whose code is 511 (an escape), in lane order.
// c != 511: j = lw - (c >> 4), X = ((j * rho) >> 8) + (c & 15) - 8, score = match*j + (mismatch - match)*X.
// An escape's word decodes as `one` does (0xFFFF bad, X = 0xFF: the score in esc[i]).  Ranges [lo, hi) start on
// a tile (lo % 64 == 0); the escapes seen are added to *n_esc.

struct Rec9 {
    int32_t match, mismatch, lw, rho;
};

using Fn9 = void (*)(int32_t* s, int32_t* e, const uint8_t* rec, const int32_t* esc, const Rec9& k, bool nt,
                     size_t lo, size_t hi, int64_t* n_esc);

// an escape's word v for pair i -> (score, end)
inline void rec9_esc(int32_t& s, int32_t& e, const int32_t* esc, const Rec9& k, uint32_t v, size_t i) {
    const uint32_t j = v >> 8, x = v & 0xFFu;
    if (v == 0xFFFFu) {
        s = e = -1;
        return;
    }
    s = x == 0xFFu ? esc[i] : k.match * (int32_t)(j - x) + k.mismatch * (int32_t)x;
    e = (int32_t)j;
}

// one tile's pairs [t0, t0 + cnt), scalar
inline int64_t rec9_tile_scalar(int32_t* s, int32_t* e, const uint8_t* r, const int32_t* esc, const Rec9& k,
                                size_t t0, size_t cnt) {
    uint64_t hm;
    memcpy(&hm, r + 64, 8);
    const uint8_t* ev = r + 72;
    int64_t m = 0;
    for (size_t l = 0; l < cnt; ++l) {
        const uint32_t c = r[l] | (uint32_t)((hm >> l) & 1u) << 8;
        const size_t i = t0 + l;
        if (c == 511u) {
            uint16_t v;
            memcpy(&v, ev + 2 * m++, 2);
            rec9_esc(s[i], e[i], esc, k, v, i);
            continue;
        }
        const int32_t j = k.lw - (int32_t)(c >> 4);
        const int32_t x = ((j * k.rho) >> 8) + (int32_t)(c & 15u) - 8;
        s[i] = k.match * j + (k.mismatch - k.match) * x;
        e[i] = j;
    }
    return m;
}

inline void expand9_scalar(int32_t* s, int32_t* e, const uint8_t* rec, const int32_t* esc, const Rec9& k, bool,
                           size_t lo, size_t hi, int64_t* n_esc) {
    int64_t m = 0;
    for (size_t t0 = lo; t0 < hi; t0 += 64)
        m += rec9_tile_scalar(s, e, rec + 4 * t0, esc, k, t0, hi - t0 < 64 ? hi - t0 : 64);
    if (n_esc) *n_esc += m;
}

// 64 pairs per step: the codes as two 32-lane 16-bit vectors, four 64-byte stores per array
__attribute__((target("avx512f,avx512bw"))) inline void expand9_avx512(int32_t* s, int32_t* e, const uint8_t* rec,
                                                                       const int32_t* esc, const Rec9& k, bool nt,
                                                                       size_t lo, size_t hi, int64_t* n_esc) {
    const bool al = nt && ((uintptr_t)(s + lo) & 63) == 0 && ((uintptr_t)(e + lo) & 63) == 0;
    const __m512i vlw = _mm512_set1_epi16((int16_t)k.lw), vrho = _mm512_set1_epi16((int16_t)k.rho);
    const __m512i v15 = _mm512_set1_epi16(15), v8 = _mm512_set1_epi16(8), v256 = _mm512_set1_epi16(256);
    const __m512i vm = _mm512_set1_epi16((int16_t)k.match), vd = _mm512_set1_epi16((int16_t)(k.mismatch - k.match));
    const __m512i ff = _mm512_set1_epi8((char)0xFF);
    int64_t m = 0;
    size_t t0 = lo;
    for (; t0 + 64 <= hi; t0 += 64) {
        const uint8_t* r = rec + 4 * t0;
        const __m512i bytes = _mm512_loadu_si512(r);
        uint64_t hm;
        memcpy(&hm, r + 64, 8);
        const uint64_t em = _mm512_cmpeq_epi8_mask(bytes, ff) & hm;
        __m512i out[8];  // s 0..3, e 0..3 (16 pairs each)
        for (int h = 0; h < 2; ++h) {
            __m512i c = _mm512_cvtepu8_epi16(h ? _mm512_extracti64x4_epi64(bytes, 1) : _mm512_castsi512_si256(bytes));
            c = _mm512_mask_add_epi16(c, (__mmask32)(hm >> (32 * h)), c, v256);
            const __m512i j = _mm512_sub_epi16(vlw, _mm512_srli_epi16(c, 4));
            const __m512i xc = _mm512_srli_epi16(_mm512_mullo_epi16(j, vrho), 8);
            const __m512i x = _mm512_sub_epi16(_mm512_add_epi16(xc, _mm512_and_si512(c, v15)), v8);
            const __m512i sc = _mm512_add_epi16(_mm512_mullo_epi16(j, vm), _mm512_mullo_epi16(x, vd));
            out[2 * h] = _mm512_cvtepi16_epi32(_mm512_castsi512_si256(sc));
            out[2 * h + 1] = _mm512_cvtepi16_epi32(_mm512_extracti64x4_epi64(sc, 1));
            out[4 + 2 * h] = _mm512_cvtepu16_epi32(_mm512_castsi512_si256(j));
            out[4 + 2 * h + 1] = _mm512_cvtepu16_epi32(_mm512_extracti64x4_epi64(j, 1));
        }
        if (em) {  // escapes: patched in the vectors (lane order = the order of their words)
            alignas(64) int32_t ts[64], te[64];
            for (int q = 0; q < 4; ++q) {
                _mm512_store_si512(ts + 16 * q, out[q]);
                _mm512_store_si512(te + 16 * q, out[4 + q]);
            }
            const uint8_t* ev = r + 72;
            int q = 0;
            for (uint64_t b = em; b; b &= b - 1, ++q) {
                const int l = __builtin_ctzll(b);
                uint16_t v;
                memcpy(&v, ev + 2 * q, 2);
                rec9_esc(ts[l], te[l], esc, k, v, t0 + l);
            }
            m += q;
            for (int q4 = 0; q4 < 4; ++q4) {
                out[q4] = _mm512_load_si512(ts + 16 * q4);
                out[4 + q4] = _mm512_load_si512(te + 16 * q4);
            }
        }
        for (int q = 0; q < 4; ++q) {
            put512(s + t0 + 16 * q, out[q], al);
            put512(e + t0 + 16 * q, out[4 + q], al);
        }
    }
    int64_t mt = 0;
    if (t0 < hi) mt = rec9_tile_scalar(s, e, rec + 4 * t0, esc, k, t0, hi - t0);
    if (n_esc) *n_esc += m + mt;
    _mm_sfence();
}

inline Fn9 pick9() {
#if defined(__HIP_DEVICE_COMPILE__)
    return expand9_scalar;
#else
    __builtin_cpu_init();
    const bool a512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
    return a512 ? expand9_avx512 : expand9_scalar;
#endif
}

// The record encoder (put_tile9 restated on the host), for the CPU tests of the decoders: lane l of tile t
// holds pair t0 + l's (score, end) for cnt <= 64 pairs; n is read a's length (j > n: a window pair, its score
// into esc), end -1 a bad pair.  Returns the record's bytes (72 + 2 * escapes).
inline size_t encode9_tile(uint8_t* r, int32_t* esc, const Rec9& k, const int32_t* sc, const int32_t* en,
                           const int32_t* n, size_t t0, size_t cnt) {
    uint64_t hm = 0;
    size_t m = 0;
    for (size_t l = 0; l < 64; ++l) {
        uint32_t c = 0, v = 0;
        bool is_esc = false;
        if (l < cnt) {
            const size_t i = t0 + l;
            const int32_t j = en[i];
            if (j < 0) {
                is_esc = true;
                v = 0xFFFFu;
            } else if (j > n[i]) {
                is_esc = true;
                v = (uint32_t)j << 8 | 0xFFu;
                esc[i] = sc[i];
            } else {
                const int32_t x = k.match == k.mismatch ? 0 : (k.match * j - sc[i]) / (k.match - k.mismatch);
                const int32_t dj = k.lw - j, dx = x - ((j * k.rho) >> 8) + 8;
                const uint32_t cc = (uint32_t)(16 * dj + dx);
                if ((uint32_t)dj < 32u && (uint32_t)dx < 16u && cc != 511u) {
                    c = cc;
                } else {
                    is_esc = true;
                    v = (uint32_t)j << 8 | (uint32_t)x;
                }
            }
        }
        if (is_esc) {
            c = 511u;
            const uint16_t w = (uint16_t)v;
            memcpy(r + 72 + 2 * m++, &w, 2);
        }
        r[l] = (uint8_t)c;
        hm |= (uint64_t)(c >> 8) << l;
    }
    memcpy(r + 64, &hm, 8);
    return 72 + 2 * m;
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
