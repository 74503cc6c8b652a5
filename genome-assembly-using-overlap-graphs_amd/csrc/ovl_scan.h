// ovl_scan.h — host pass over a read set's bytes (ovl_api.cpp stage_reads): the alphabet, and the 2-bit
// packing of ACGT-only bytes that ovl_set_reads uploads instead of the bytes (unpack2_kernel expands it on the
// device).  Host code only (tests/c/scan_test.cpp checks the vector form against the scalar one).
#pragma once

#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace ovl_scan {

// seen[v] = 1 for every byte value v in p[0 .. n) (the blocks scan_pack cannot settle with its four compares)
inline void scan_bytes(const uint8_t* p, size_t n, uint8_t* seen) {
    uint8_t t[4][256] = {};  // four tables: independent stores
    size_t q = 0;
    for (; q + 4 <= n; q += 4) {
        t[0][p[q]] = 1;
        t[1][p[q + 1]] = 1;
        t[2][p[q + 2]] = 1;
        t[3][p[q + 3]] = 1;
    }
    for (; q < n; ++q) t[0][p[q]] = 1;
    for (int v = 0; v < 256; ++v) seen[v] |= t[0][v] | t[1][v] | t[2][v] | t[3][v];
}

// One pass over p[lo, hi) (lo a multiple of 64 within the read bytes): the bytes seen (as scan_symbols) and,
// while every byte is A, C, G or T, their 2-bit packing (base i at bits 2(i % 4) of pk[i / 4], A C G T =
// 0 1 2 3; unpack2_kernel expands it on the device).  Returns false once a byte outside ACGT appears (the
// packing is abandoned there; the scan goes on).
inline bool scan_pack_scalar(const uint8_t* p, size_t lo, size_t hi, uint8_t* seen, uint8_t* pk) {
    bool ok = true;
    for (size_t q = lo; q < hi; q += 4) {
        uint8_t byte = 0;
        for (size_t i = q; i < q + 4 && i < hi; ++i) {
            const uint8_t x = p[i];
            seen[x] = 1;
            const int c = x == 'A' ? 0 : x == 'C' ? 1 : x == 'G' ? 2 : x == 'T' ? 3 : -1;
            if (c < 0) ok = false;
            byte |= (uint8_t)((c & 3) << (2 * (i - q)));
        }
        if (ok) pk[q >> 2] = byte;
    }
    return ok;
}

__attribute__((target("avx512f,avx512bw,bmi2"))) inline bool scan_pack_avx512(const uint8_t* p, size_t lo, size_t hi,
                                                                       uint8_t* seen, uint8_t* pk) {
    const __m512i A = _mm512_set1_epi8('A'), C = _mm512_set1_epi8('C'), G = _mm512_set1_epi8('G'),
                  T = _mm512_set1_epi8('T');
    constexpr uint64_t kEven = 0x5555555555555555ull, kOdd = 0xAAAAAAAAAAAAAAAAull;
    __mmask64 ma = 0, mc = 0, mg = 0, mt = 0;
    bool ok = true;
    size_t q = lo;
    for (; q + 64 <= hi; q += 64) {
        const __m512i v = _mm512_loadu_si512(reinterpret_cast<const void*>(p + q));
        const __mmask64 a = _mm512_cmpeq_epi8_mask(v, A), c = _mm512_cmpeq_epi8_mask(v, C),
                        g = _mm512_cmpeq_epi8_mask(v, G), t = _mm512_cmpeq_epi8_mask(v, T);
        if ((a | c | g | t) != ~__mmask64(0)) {
            ok = false;
            scan_bytes(p + q, 64, seen);
            continue;
        }
        ma |= a;
        mc |= c;
        mg |= g;
        mt |= t;
        if (ok) {
            // code bit 0 = C or T, bit 1 = G or T; bases 0-31 interleaved into the first 8 bytes, 32-63 the next
            const uint64_t b0 = (uint64_t)(c | t), b1 = (uint64_t)(g | t);
            const uint64_t w0 = _pdep_u64(b0 & 0xFFFFFFFFull, kEven) | _pdep_u64(b1 & 0xFFFFFFFFull, kOdd);
            const uint64_t w1 = _pdep_u64(b0 >> 32, kEven) | _pdep_u64(b1 >> 32, kOdd);
            memcpy(pk + (q >> 2), &w0, 8);
            memcpy(pk + (q >> 2) + 8, &w1, 8);
        }
    }
    seen['A'] |= ma != 0;
    seen['C'] |= mc != 0;
    seen['G'] |= mg != 0;
    seen['T'] |= mt != 0;
    if (q < hi) ok = scan_pack_scalar(p, q, hi, seen, pk) && ok;  // (pk is sized for the whole stream)
    return ok;
}

inline bool scan_pack(const uint8_t* p, size_t lo, size_t hi, uint8_t* seen, uint8_t* pk) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the device pass of a HIP translation unit parses host code too)
    const bool a512 = false;
#else
    static const bool a512 = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("bmi2");
#endif
    return a512 ? scan_pack_avx512(p, lo, hi, seen, pk) : scan_pack_scalar(p, lo, hi, seen, pk);
}

}  // namespace ovl_scan
