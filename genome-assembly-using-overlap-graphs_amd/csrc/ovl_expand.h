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
// Tile records (ovl_kernels.hip put_ring_rec, the resident grid's ring): tile t's record is 32 dwords at r = rec + 32 t,
//   r[w] = phase << 31 | c[w + 32] << 15 | c[w]    (c[l]: the 15-bit code of the tile's pair l)
// c = j(j + 1)/2 + X (end j, X mismatches over L = j compared bases): score = match*j + (mismatch - match)*X.
// c = 0x7FFF: the pair's special word sp[l] holds it --
//   1 << 31 | j << 16 | X << 8 | n: score = match*n + (mismatch - match)*X, end j;  0xFFFFFFFF: (-1, -1).
// A record is complete when every dword's bit 31 is the lap's phase (rec_tile_ready_scalar).  The decoders take a
// tile only once all of its special words have landed (get(l) != 0): the ring's 8-byte words carry the request's
// sequence number (RingSp), so no host store ever zeroes a word a running kernel may write -- one that does was
// measured to come back with the device's value (round 5's launched record transport, ~1 in 2,000 words at cfg3).
// The side-array forms (rec_tile_scalar / rec_tile_avx512: 4-byte words, zero until they land, the words read
// reported in `taken`) serve the CPU tests (tests/c/rec_test.cpp) and tools/rec_expand_probe.cpp.  j from c: the largest j with j(j + 1)/2 <= c is floor((sqrt(8c + 1) - 1) / 2), exact in float for
// c < 2^15 (8c + 1 is a perfect square exactly when X = 0, and otherwise lies >= 1 from one, far above float's
// error at 2^18).

constexpr uint32_t kRecSpecial = 0x7FFFu;

struct RecK {
    int32_t match, mismatch;
};

inline void rec_decode_code(uint32_t c, const RecK& k, int32_t& s, int32_t& e) {
    const uint32_t j = (uint32_t)(int32_t)((__builtin_sqrtf((float)(8 * c + 1)) - 1.0f) * 0.5f);
    const int32_t x = (int32_t)(c - (j * (j + 1) >> 1));
    s = k.match * (int32_t)j + (k.mismatch - k.match) * x;
    e = (int32_t)j;
}

// a special word (non-zero) -> (score, end)
inline void rec_decode_special(uint32_t v, const RecK& k, int32_t& s, int32_t& e) {
    if (v == 0xFFFFFFFFu) {
        s = e = -1;
        return;
    }
    const int32_t j = (int32_t)(v >> 16 & 0xFFu), x = (int32_t)(v >> 8 & 0xFFu), n = (int32_t)(v & 0xFFu);
    s = k.match * n + (k.mismatch - k.match) * x;
    e = j;
}

// all 32 dwords of the record carry `phase` in bit 31
inline bool rec_tile_ready_scalar(const uint32_t* r, uint32_t phase) {
    const volatile uint32_t* v = r;
    for (int w = 0; w < 32; ++w)
        if ((v[w] >> 31) != phase) return false;
    return true;
}

// One record's pairs [0, cnt) (cnt <= 64) into s / e (scalar) once the record and all its special words have
// landed: the specials' count (the bad pairs among them added to *bad), or -2 (nothing written) while something has
// not.  get(l) is pair l's special word once it has landed, else 0 (a special word is never 0).
template <class Get>
inline int rec_tile_scalar_t(int32_t* s, int32_t* e, const uint32_t* r, const RecK& k, size_t cnt, uint32_t phase,
                             int* bad, Get&& get) {
    if (!rec_tile_ready_scalar(r, phase)) return -2;
    const volatile uint32_t* v = r;
    uint32_t wv[64];
    int m = 0;
    for (size_t l = 0; l < cnt; ++l) {  // (every special word first: a tile is taken whole or not at all)
        if (((v[l & 31] >> (l < 32 ? 0 : 15)) & 0x7FFFu) != kRecSpecial) continue;
        if ((wv[m] = get(l)) == 0u) return -2;
        ++m;
    }
    int q = 0;
    for (size_t l = 0; l < cnt; ++l) {
        const uint32_t c = (v[l & 31] >> (l < 32 ? 0 : 15)) & 0x7FFFu;
        if (c == kRecSpecial) {
            rec_decode_special(wv[q], k, s[l], e[l]);
            *bad += wv[q++] == 0xFFFFFFFFu;
        } else {
            rec_decode_code(c, k, s[l], e[l]);
        }
    }
    return m;
}

// the side-array form: special words zero until they land; the words read go to taken[0 ..)
inline int rec_tile_scalar(int32_t* s, int32_t* e, const uint32_t* r, uint32_t* sp, const RecK& k, size_t cnt,
                           uint32_t phase, int* bad, uint32_t** taken) {
    int m = 0;
    return rec_tile_scalar_t(s, e, r, k, cnt, phase, bad, [&](size_t l) -> uint32_t {
        taken[m] = sp + l;
        const uint32_t w = *(volatile uint32_t*)taken[m];
        m += w != 0u;
        return w;
    });
}

// the resident grid's ring form (ovl_kernels.h OvlResidentBody): 8-byte words {payload, seq}, current when the high
// half is the request's seq
struct RingSp {
    const uint64_t* sp;
    uint32_t seq;
    uint32_t operator()(size_t l) const {
        const uint64_t w = *(const volatile uint64_t*)(sp + l);
        return (uint32_t)(w >> 32) == seq ? (uint32_t)w : 0u;
    }
};

// AVX-512: readiness check and decode of one full record (64 pairs) from the same two loads; *ready = false (nothing
// written) while the record or one of its special words has not landed (get: as rec_tile_scalar_t).  Stores
// non-temporally when `al` (s and e 64-byte aligned).  Returns the specials' count.
template <class Get>
__attribute__((target("avx512f,avx512bw,avx512dq"))) inline int rec_tile_avx512_t(int32_t* s, int32_t* e,
                                                                                    const uint32_t* r, const RecK& k,
                                                                                    uint32_t phase, bool al,
                                                                                    bool* ready, int* bad, Get&& get) {
    const __m512i w0 = _mm512_load_si512(r), w1 = _mm512_load_si512(r + 16);
    const __m512i sign = _mm512_set1_epi32((int)0x80000000u);
    const __mmask16 want = phase ? (__mmask16)0xFFFF : (__mmask16)0;
    *ready = false;
    if (_mm512_test_epi32_mask(w0, sign) != want || _mm512_test_epi32_mask(w1, sign) != want) return 0;
    const __m512i m15 = _mm512_set1_epi32(0x7FFF), one = _mm512_set1_epi32(1);
    const __m512i vm = _mm512_set1_epi32(k.match), vd = _mm512_set1_epi32(k.mismatch - k.match);
    const __m512 f8 = _mm512_set1_ps(8.0f), f1 = _mm512_set1_ps(1.0f), fh = _mm512_set1_ps(0.5f);
    __m512i S[4], E[4];
    __mmask16 spm[4];
    const __m512i cs[4] = {_mm512_and_si512(w0, m15), _mm512_and_si512(w1, m15),
                           _mm512_and_si512(_mm512_srli_epi32(w0, 15), m15),
                           _mm512_and_si512(_mm512_srli_epi32(w1, 15), m15)};
    for (int q = 0; q < 4; ++q) {  // pairs 16q .. 16q + 15
        const __m512i c = cs[q];
        const __m512 f = _mm512_sqrt_ps(_mm512_fmadd_ps(_mm512_cvtepi32_ps(c), f8, f1));
        const __m512i j = _mm512_cvttps_epi32(_mm512_mul_ps(_mm512_sub_ps(f, f1), fh));
        const __m512i tri = _mm512_srli_epi32(_mm512_mullo_epi32(j, _mm512_add_epi32(j, one)), 1);
        const __m512i x = _mm512_sub_epi32(c, tri);
        S[q] = _mm512_add_epi32(_mm512_mullo_epi32(j, vm), _mm512_mullo_epi32(x, vd));
        E[q] = j;
        spm[q] = _mm512_cmpeq_epi32_mask(c, m15);
    }
    // each special's (score, end) into its lane of the vectors (a masked broadcast: no trip through memory); a
    // special word not landed yet leaves the tile untaken (the vectors are dropped, nothing stored)
    int m = 0, nb = 0;
    for (int q = 0; q < 4; ++q)
        for (uint32_t b = spm[q]; b; b &= b - 1, ++m) {
            const uint32_t v = get((size_t)(16 * q + __builtin_ctz(b)));
            if (v == 0u) return 0;
            int32_t sv, ev;
            rec_decode_special(v, k, sv, ev);
            nb += v == 0xFFFFFFFFu;
            const __mmask16 bit = (__mmask16)(b & (0u - b));
            S[q] = _mm512_mask_set1_epi32(S[q], bit, sv);
            E[q] = _mm512_mask_set1_epi32(E[q], bit, ev);
        }
    for (int q = 0; q < 4; ++q) {
        put512(s + 16 * q, S[q], al);
        put512(e + 16 * q, E[q], al);
    }
    *bad += nb;
    *ready = true;
    return m;
}

__attribute__((target("avx512f,avx512bw,avx512dq"))) inline int rec_tile_avx512(int32_t* s, int32_t* e,
                                                                                  const uint32_t* r, uint32_t* sp,
                                                                                  const RecK& k, uint32_t phase,
                                                                                  bool al, bool* ready, int* bad,
                                                                                  uint32_t** taken) {
    int m = 0;
    return rec_tile_avx512_t(s, e, r, k, phase, al, ready, bad, [&](size_t l) -> uint32_t {
        taken[m] = sp + l;
        const uint32_t w = *(volatile uint32_t*)taken[m];
        m += w != 0u;
        return w;
    });
}

// this CPU runs rec_tile_avx512
inline bool rec_avx512() {
#if defined(__HIP_DEVICE_COMPILE__)
    return false;
#else
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("avx512dq");
#endif
}

// The record encoder (put_ring_rec's codes restated on the host), for the CPU tests of the decoders: pairs [0, cnt) of a tile
// from (sc, en, n) -- n read a's length (j > n: a window pair), en -1 a bad pair; specials into sp.  Returns the
// specials' count.
inline int encode_rec_tile(uint32_t* r, uint32_t* sp, const RecK& k, const int32_t* sc, const int32_t* en,
                           const int32_t* n, size_t cnt, uint32_t phase) {
    uint32_t c[64] = {0};
    int m = 0;
    for (size_t l = 0; l < cnt; ++l) {
        const int32_t j = en[l];
        if (j < 0) {
            c[l] = kRecSpecial;
            sp[l] = 0xFFFFFFFFu;
            ++m;
        } else if (j > n[l]) {
            const int32_t x = k.match == k.mismatch ? 0 : (k.match * n[l] - sc[l]) / (k.match - k.mismatch);
            c[l] = kRecSpecial;
            sp[l] = 0x80000000u | (uint32_t)j << 16 | (uint32_t)x << 8 | (uint32_t)n[l];
            ++m;
        } else {
            const int32_t x = k.match == k.mismatch ? 0 : (k.match * j - sc[l]) / (k.match - k.mismatch);
            c[l] = ((uint32_t)j * (uint32_t)(j + 1) >> 1) + (uint32_t)x;
        }
    }
    for (int w = 0; w < 32; ++w) r[w] = phase << 31 | c[w + 32] << 15 | c[w];
    return m;
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
