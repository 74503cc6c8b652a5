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

#include <algorithm>
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
// Streamed tile records (ovl_kernels.hip put_tile_rec, sink 3): tile t's record is the 128-byte slot r = rec + 32 t,
//   r[0]       phase << 31 | nesc << 16 | rho << 8 | jmax
//   r[1 + w]   phase << 31 | c[w + 44] << 20 | c[w + 22] << 10 | c[w]       (w < 22: pair l's code in dword
//              1 + l % 22, field l / 22)
//   r[23 + e]  escape e (e < 9, in lane order); escapes from the tenth on in the special word sp[l]
// Code c != 1023: j = jmax - (c >> 5), X = ((j * rho) >> 8) + (c & 31) - 16, score = match*j + (mismatch - match)*X.
// c = 1023: the escape word v -- 0xFFFFFFFF a bad pair (-1, -1); else j = v >> 16 & 0xFF, X = v >> 8 & 0xFF,
// n = v & 0xFF, L = min(j, n), score = match*L + (mismatch - match)*X.  Escape words are zero until they land: the
// decoders report every escape word they read (`taken`), and the caller zeroes them once the kernel that wrote them
// has ended (ovl_api.cpp stream_chunk) -- a host store into a line of a running kernel's records was measured to
// come back with the device's value (escape slots zeroed on the box while their kernel ran were found nonzero
// again afterwards, ~1 in 2,000 escapes at cfg3).  A record's codes are complete when dwords 0..22 carry the
// launch's phase (rec_tile_ready_scalar).

struct RecK {
    int32_t match, mismatch;
};

inline void rec_decode_code(uint32_t c, uint32_t jmax, uint32_t rho, const RecK& k, int32_t& s, int32_t& e) {
    const int32_t j = (int32_t)jmax - (int32_t)(c >> 5);
    const int32_t x = (int32_t)(((uint32_t)j * rho) >> 8) + (int32_t)(c & 31u) - 16;
    s = k.match * j + (k.mismatch - k.match) * x;
    e = j;
}

// an escape word (non-zero) -> (score, end)
inline void rec_decode_escape(uint32_t v, const RecK& k, int32_t& s, int32_t& e) {
    if (v == 0xFFFFFFFFu) {
        s = e = -1;
        return;
    }
    const int32_t j = (int32_t)(v >> 16 & 0xFFu), x = (int32_t)(v >> 8 & 0xFFu), n = (int32_t)(v & 0xFFu);
    s = k.match * (j < n ? j : n) + (k.mismatch - k.match) * x;
    e = j;
}

// dwords 0..22 of the record carry `phase` in bit 31
inline bool rec_tile_ready_scalar(const uint32_t* r, uint32_t phase) {
    const volatile uint32_t* v = r;
    for (int w = 0; w < 23; ++w)
        if ((v[w] >> 31) != phase) return false;
    return true;
}

// Waits for escape word *w (spinning while `wait` says to) and decodes it; a bad pair adds 1 to *bad.  False if
// `wait` gave up first.
template <typename Wait>
inline bool rec_take_escape(uint32_t* w, const RecK& k, int32_t& s, int32_t& e, int* bad, Wait&& wait) {
    volatile uint32_t* v = w;
    uint32_t x;
    while ((x = *v) == 0u)
        if (!wait()) return false;
    rec_decode_escape(x, k, s, e);
    *bad += x == 0xFFFFFFFFu;
    return true;
}


// escape e of a tile whose lane is l: an inline slot of the record, or the lane's special word
inline uint32_t* rec_escape_slot(uint32_t* r, uint32_t* sp, int e, int l) { return e < 9 ? r + 23 + e : sp + l; }

// one complete record's pairs [0, cnt) (cnt <= 64) into s / e (scalar); the escapes' count (their words in
// taken[0 ..), the bad pairs among them added to *bad), or -1 if one never came
template <typename Wait>
inline int rec_tile_scalar(int32_t* s, int32_t* e, uint32_t* r, uint32_t* sp, const RecK& k, size_t cnt, int* bad,
                           uint32_t** taken, Wait&& wait) {
    const volatile uint32_t* v = r;
    const uint32_t hdr = v[0], jmax = hdr & 0xFFu, rho = hdr >> 8 & 0xFFu;
    int m = 0;
    for (size_t l = 0; l < cnt; ++l) {
        const uint32_t c = (v[1 + l % 22] >> (10 * (l / 22))) & 0x3FFu;
        if (c == 1023u) {
            uint32_t* w = rec_escape_slot(r, sp, m, (int)l);
            if (!rec_take_escape(w, k, s[l], e[l], bad, wait)) return -1;
            taken[m++] = w;
        } else {
            rec_decode_code(c, jmax, rho, k, s[l], e[l]);
        }
    }
    return m;
}

// pair l = 16 q + i of a record: its code in dword 1 + l % 22 (kRecIdx, an index into the two 16-dword halves), field
// l / 22 (kRecShift, the bit offset)
alignas(64) constexpr int32_t kRecIdx[4][16] = {
    {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16},
    {17, 18, 19, 20, 21, 22, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10},
    {11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 1, 2, 3, 4},
    {5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20}};
alignas(64) constexpr int32_t kRecShift[4][16] = {
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0, 0, 0, 0, 0, 0, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10},
    {10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 20, 20, 20, 20},
    {20, 20, 20, 20, 20, 20, 20, 20, 20, 20, 20, 20, 20, 20, 20, 20}};

// AVX-512: readiness check and decode of one full record (64 pairs) from the same two loads; *ready = false
// (nothing written) when the record is incomplete.  Stores non-temporally when `al` (s and e 64-byte aligned).
// Returns the escapes' count (their words in taken[0 ..)), or -1 if `wait` gave up on one.
template <typename Wait>
__attribute__((target("avx512f,avx512bw,avx512dq"))) inline int rec_tile_avx512(int32_t* s, int32_t* e, uint32_t* r,
                                                                                  uint32_t* sp, const RecK& k,
                                                                                  uint32_t phase, bool al, bool* ready,
                                                                                  int* bad, uint32_t** taken,
                                                                                  Wait&& wait) {
    const __m512i w0 = _mm512_load_si512(r), w1 = _mm512_load_si512(r + 16);
    const __m512i sign = _mm512_set1_epi32((int)0x80000000u);
    const __mmask16 m0 = _mm512_test_epi32_mask(w0, sign), m1 = _mm512_test_epi32_mask(w1, sign) & 0x7F;
    if (m0 != (phase ? (__mmask16)0xFFFF : (__mmask16)0) || m1 != (phase ? (__mmask16)0x7F : (__mmask16)0)) {
        *ready = false;
        return 0;
    }
    *ready = true;
    const uint32_t hdr = (uint32_t)_mm_cvtsi128_si32(_mm512_castsi512_si128(w0));
    const uint32_t nesc = hdr >> 16 & 0x7Fu;
    const __m512i vj = _mm512_set1_epi32((int)(hdr & 0xFFu)), vr = _mm512_set1_epi32((int)(hdr >> 8 & 0xFFu));
    const __m512i m10 = _mm512_set1_epi32(0x3FF), m5 = _mm512_set1_epi32(31), v16 = _mm512_set1_epi32(16);
    const __m512i vm = _mm512_set1_epi32(k.match), vd = _mm512_set1_epi32(k.mismatch - k.match);
    __m512i S[4], E[4];
    __mmask16 em[4];
    for (int q = 0; q < 4; ++q) {  // pairs 16q .. 16q + 15: dword 1 + l % 22, field l / 22 (kRecIdx, kRecShift)
        const __m512i d = _mm512_permutex2var_epi32(w0, _mm512_load_si512(kRecIdx[q]), w1);
        const __m512i c = _mm512_and_si512(_mm512_srlv_epi32(d, _mm512_load_si512(kRecShift[q])), m10);
        const __m512i j = _mm512_sub_epi32(vj, _mm512_srli_epi32(c, 5));
        const __m512i xc = _mm512_srli_epi32(_mm512_mullo_epi32(j, vr), 8);
        const __m512i x = _mm512_sub_epi32(_mm512_add_epi32(xc, _mm512_and_si512(c, m5)), v16);
        S[q] = _mm512_add_epi32(_mm512_mullo_epi32(j, vm), _mm512_mullo_epi32(x, vd));
        E[q] = j;
        em[q] = nesc ? _mm512_cmpeq_epi32_mask(c, m10) : (__mmask16)0;
    }
    if (nesc) {
        alignas(64) int32_t ts[64], te[64];
        for (int q = 0; q < 4; ++q) {
            _mm512_store_si512(ts + 16 * q, S[q]);
            _mm512_store_si512(te + 16 * q, E[q]);
        }
        int m = 0;
        for (int q = 0; q < 4; ++q)
            for (uint32_t b = em[q]; b; b &= b - 1, ++m) {
                const int l = 16 * q + __builtin_ctz(b);
                // (the device stores it beside the record's dwords, but nothing orders their arrival)
                uint32_t* w = rec_escape_slot(r, sp, m, l);
                if (!rec_take_escape(w, k, ts[l], te[l], bad, wait)) return -1;
                taken[m] = w;
            }
        for (int q = 0; q < 4; ++q) {
            put512(s + 16 * q, _mm512_load_si512(ts + 16 * q), al);
            put512(e + 16 * q, _mm512_load_si512(te + 16 * q), al);
        }
        return m;
    }
    for (int q = 0; q < 4; ++q) {
        put512(s + 16 * q, S[q], al);
        put512(e + 16 * q, E[q], al);
    }
    return 0;
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

// The record encoder (put_tile_rec restated on the host), for the CPU tests of the decoders: pairs [0, cnt) of a tile
// from (sc, en, n) -- n read a's length (j > n: a window pair), en -1 a bad pair; escapes beyond the record's nine
// slots into sp.  Returns the escapes' count.
inline int encode_rec_tile(uint32_t* r, uint32_t* sp, const RecK& k, const int32_t* sc, const int32_t* en,
                           const int32_t* n, size_t cnt, uint32_t phase) {
    uint32_t x[64] = {0}, c[66] = {0};
    bool normal[64] = {false};
    uint32_t jm = 0, sj = 0, sx = 0;
    for (size_t l = 0; l < cnt; ++l) {
        const int32_t L = en[l] <= n[l] ? en[l] : n[l];
        x[l] = en[l] < 0 || k.match == k.mismatch ? 0u : (uint32_t)((k.match * L - sc[l]) / (k.match - k.mismatch));
        normal[l] = en[l] >= 0 && en[l] <= n[l];
        if (normal[l]) {
            jm = jm > (uint32_t)en[l] ? jm : (uint32_t)en[l];
            sj += (uint32_t)en[l];
            sx += x[l];
        }
    }
    const uint32_t rho = sj ? std::min(255u, (256u * sx + sj / 2) / sj) : 0u;
    int m = 0;
    for (size_t l = 0; l < cnt; ++l) {
        const int32_t dj = (int32_t)jm - en[l], dx = (int32_t)x[l] - (int32_t)(((uint32_t)en[l] * rho) >> 8) + 16;
        const uint32_t cc = (uint32_t)(32 * dj + dx);
        if (normal[l] && (uint32_t)dj < 32u && (uint32_t)dx < 32u && cc != 1023u) {
            c[l] = cc;
        } else {
            c[l] = 1023u;
            const uint32_t w = en[l] < 0 ? 0xFFFFFFFFu
                                         : 0x80000000u | (uint32_t)en[l] << 16 | x[l] << 8 |
                                               (en[l] > n[l] ? (uint32_t)n[l] : 255u);
            *rec_escape_slot(r, sp, m, (int)l) = w;
            ++m;
        }
    }
    r[0] = phase << 31 | (uint32_t)m << 16 | rho << 8 | jm;
    for (int w = 0; w < 22; ++w) r[1 + w] = phase << 31 | c[w + 44] << 20 | c[w + 22] << 10 | c[w];
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
