// ovl_digest.h -- the 128-bit digest of a read set's bytes that ovl_set_reads keeps for its resident-set check
// (ovl_api.cpp same_reads) instead of a host copy of the bytes.  Host code only.
#pragma once

#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "ovl_expand.h"
#include "ovl_pool.h"

namespace ovl_digest {

// A 128-bit digest of a read set's bytes, what same_reads compares instead of a host copy of the bytes: per 256 KiB
// part (parts on the host pool), 32 independent lanes h = rotl((h ^ w) * K, 29) over interleaved 8-byte words (one
// multiply per word; 64-bit multiplies have a long latency, so the lanes' 32 chains overlap: four zmm chains with
// AVX-512, ~7 GB/s per thread with one), the lanes folded by two independent multiply-rotate finalisers, the parts'
// pairs combined in order.  Not cryptographic: offsets are compared exactly, this catches changed bytes of the same
// layout.  (Round 6's first form, two dependent streams, cost 0.55 ms per ovl_score_pairs call at the target point.)
constexpr uint64_t kHashM = 0xC2B2AE3D27D4EB4Full;
constexpr int kHashLanes = 32;
inline uint64_t hash_rotl(uint64_t h, int r) { return (h << r) | (h >> (64 - r)); }
// the lane loop over the whole 256-byte blocks of [q, q + len) in four zmm (vpmullq: the same products as the scalar
// loop's, so either gives the same digest); returns the bytes done
__attribute__((target("avx512f,avx512dq"))) size_t hash_lanes_avx512(const uint8_t* q, size_t len, uint64_t* h) {
    __m512i v0 = _mm512_loadu_si512(h), v1 = _mm512_loadu_si512(h + 8), v2 = _mm512_loadu_si512(h + 16),
            v3 = _mm512_loadu_si512(h + 24);
    const __m512i m = _mm512_set1_epi64((long long)kHashM);
    size_t k = 0;
    for (; k + 256 <= len; k += 256) {
        v0 = _mm512_rol_epi64(_mm512_mullo_epi64(_mm512_xor_si512(v0, _mm512_loadu_si512(q + k)), m), 29);
        v1 = _mm512_rol_epi64(_mm512_mullo_epi64(_mm512_xor_si512(v1, _mm512_loadu_si512(q + k + 64)), m), 29);
        v2 = _mm512_rol_epi64(_mm512_mullo_epi64(_mm512_xor_si512(v2, _mm512_loadu_si512(q + k + 128)), m), 29);
        v3 = _mm512_rol_epi64(_mm512_mullo_epi64(_mm512_xor_si512(v3, _mm512_loadu_si512(q + k + 192)), m), 29);
    }
    _mm512_storeu_si512(h, v0);
    _mm512_storeu_si512(h + 8, v1);
    _mm512_storeu_si512(h + 16, v2);
    _mm512_storeu_si512(h + 24, v3);
    return k;
}

void reads_hash(const uint8_t* p, int64_t n, uint64_t out[2]) {
    constexpr size_t kPart = size_t(1) << 18;  // (the pool's parts: as many as round 5's byte compare had)
    static const bool a512 = ovl_expand::rec_avx512();
    const size_t parts = (size_t)((n + (int64_t)kPart - 1) / (int64_t)kPart);
    std::vector<uint64_t> ph(2 * std::max<size_t>(parts, 1), 0);
    const auto mix = [](uint64_t h, uint64_t w, uint64_t k) {
        h ^= w * k;
        h = hash_rotl(h, 31);
        return h * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    };
    CopyPool::get().parallel(parts, 1, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            const uint8_t* q = p + i * kPart;
            const size_t len = std::min<size_t>(kPart, (size_t)n - i * kPart);
            uint64_t h[kHashLanes];
            for (int l = 0; l < kHashLanes; ++l)
                h[l] = 0x9E3779B97F4A7C15ull * (uint64_t)(l + 1) ^ (len + 0x1000193ull * i);
            size_t k = a512 ? hash_lanes_avx512(q, len, h) : 0;
            for (; k + 8 * kHashLanes <= len; k += 8 * kHashLanes) {
                uint64_t w[kHashLanes];
                memcpy(w, q + k, sizeof(w));
                for (int l = 0; l < kHashLanes; ++l) h[l] = hash_rotl((h[l] ^ w[l]) * kHashM, 29);
            }
            for (int l = 0; k < len; ++l, k += 8) {  // (the tail: whole words, then the last bytes zero-padded)
                uint64_t w = 0;
                memcpy(&w, q + k, std::min<size_t>(8, len - k));
                h[l] = hash_rotl((h[l] ^ w) * kHashM, 29);
            }
            uint64_t a = 0x243F6A8885A308D3ull ^ len, b = 0x13198A2E03707344ull + i;
            for (int l = 0; l < kHashLanes; ++l) {
                a = mix(a, h[l], kHashM);
                b = mix(b, h[l] ^ 0xA0761D6478BD642Full, 0x165667B19E3779F9ull);
            }
            ph[2 * i] = a;
            ph[2 * i + 1] = b;
        }
    });
    uint64_t h0 = 0x452821E638D01377ull ^ (uint64_t)n, h1 = 0xBE5466CF34E90C6Cull;
    for (size_t i = 0; i < parts; ++i) {
        h0 = mix(h0, ph[2 * i], kHashM);
        h1 = mix(h1, ph[2 * i + 1], 0x165667B19E3779F9ull);
    }
    out[0] = h0;
    out[1] = h1;
}

}  // namespace ovl_digest
