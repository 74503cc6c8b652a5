// Streamed tile records (genome-assembly-using-overlap-graphs_amd/csrc/ovl_expand.h, ovl_kernels.hip
// put_tile_rec): (1) a one-pair tile of every (j, X), X <= j <= 254, and a tile of two pairs far apart, decode
// exactly; (2) random tiles -- pairs near the tile model and far from it, window pairs and bad pairs (escape
// words, inline and in special words past the ninth), ends of 0, partial last tiles -- encoded by the host
// restatement of put_tile_rec (encode_rec_tile) in either phase decode through the scalar form and, where this
// CPU runs it, the AVX-512 form, at aligned and misaligned destinations, to every (score, end), count their bad
// pairs, and report exactly the escape words they read (zeroed here as the caller does after the kernel's end);
// (3) a record with one phase dword still in the
// other phase is not ready, and the AVX-512 form then writes nothing; (4) an escape word that never arrives ends
// the decode when `wait` gives up.  Prints what it checked and the escape share, then "ok".
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "ovl_expand.h"

static int fails = 0;
#define CHECK(c, ...)                \
    do {                             \
        if (!(c)) {                  \
            if (fails++ < 20) {      \
                printf(__VA_ARGS__); \
                printf("\n");        \
            }                        \
        }                            \
    } while (0)

static auto never = [] { return false; };

// encodes pairs [0, cnt) and checks both decoders against them; returns the escapes' count
static int roundtrip(const ovl_expand::RecK& k, const int32_t* sc, const int32_t* en, const int32_t* na, size_t cnt,
                     uint32_t phase, int misal, bool a512, const char* what) {
    alignas(64) uint32_t rec[32] = {0};
    uint32_t sp[64] = {0};
    const int esc = ovl_expand::encode_rec_tile(rec, sp, k, sc, en, na, cnt, phase);
    int want_bad = 0;
    for (size_t l = 0; l < cnt; ++l) want_bad += en[l] < 0;
    CHECK(ovl_expand::rec_tile_ready_scalar(rec, phase), "%s: not ready", what);
    CHECK(!ovl_expand::rec_tile_ready_scalar(rec, phase ^ 1u), "%s: ready in the other phase", what);
    for (int form = 0; form < (a512 && cnt == 64 ? 2 : 1); ++form) {
        alignas(64) uint32_t r2[32];
        uint32_t sp2[64];
        memcpy(r2, rec, sizeof(rec));
        memcpy(sp2, sp, sizeof(sp));
        alignas(64) int32_t sbuf[64 + 16], ebuf[64 + 16];
        int32_t* S = sbuf + misal;
        int32_t* E = ebuf + misal;
        for (int i = 0; i < 64 + 16; ++i) sbuf[i] = ebuf[i] = 0x7777;
        int got, bad = 0;
        uint32_t* taken[64];
        if (form == 0) {
            got = ovl_expand::rec_tile_scalar(S, E, r2, sp2, k, cnt, &bad, taken, never);
        } else {
            bool ready = false;
            got = ovl_expand::rec_tile_avx512(S, E, r2, sp2, k, phase, misal == 0, &ready, &bad, taken, never);
            CHECK(ready, "%s avx512: not ready", what);
        }
        for (int i = 0; i < got; ++i) *taken[i] = 0;  // (the caller's zeroing, after the kernel's end)
        CHECK(got == esc, "%s form %d: %d escapes decoded, %d encoded", what, form, got, esc);
        CHECK(bad == want_bad, "%s form %d: %d bad pairs counted, want %d", what, form, bad, want_bad);
        for (size_t l = 0; l < cnt; ++l) {
            const int32_t ws = en[l] < 0 ? -1 : sc[l];
            CHECK(S[l] == ws && E[l] == en[l], "%s form %d scoring (%d,%d) pair %zu: (%d,%d) want (%d,%d)", what, form,
                  k.match, k.mismatch, l, S[l], E[l], ws, en[l]);
        }
        for (size_t l = cnt; l < 64 && form == 0; ++l) CHECK(S[l] == 0x7777 && E[l] == 0x7777, "scalar wrote past cnt");
        for (int w = 23; w < 32; ++w) CHECK(r2[w] == 0, "%s form %d: escape slot %d not zeroed", what, form, w - 23);
        for (int l = 0; l < 64; ++l) CHECK(sp2[l] == 0, "%s form %d: special word %d not zeroed", what, form, l);
    }
    // (3) one phase dword still in the other phase
    for (int w : {0, 1, 12, 22}) {
        alignas(64) uint32_t r3[32];
        memcpy(r3, rec, sizeof(rec));
        r3[w] ^= 0x80000000u;
        CHECK(!ovl_expand::rec_tile_ready_scalar(r3, phase), "%s: record with dword %d pending ready", what, w);
        if (a512 && cnt == 64) {
            alignas(64) int32_t S2[64], E2[64];
            for (int i = 0; i < 64; ++i) S2[i] = E2[i] = 0x5555;
            bool ready = true;
            int bad = 0;
            uint32_t sp3[64];
            uint32_t* taken[64];
            memcpy(sp3, sp, sizeof(sp));
            ovl_expand::rec_tile_avx512(S2, E2, r3, sp3, k, phase, true, &ready, &bad, taken, never);
            CHECK(!ready, "%s avx512: record with dword %d pending ready", what, w);
            for (int i = 0; i < 64; ++i) CHECK(S2[i] == 0x5555 && E2[i] == 0x5555, "avx512 wrote an incomplete record");
        }
    }
    return esc;
}

int main() {
    const bool a512 = ovl_expand::rec_avx512();
    // (1) every (j, X) alone in a tile, and beside a pair far from it
    const ovl_expand::RecK k0{10, -1};
    for (int j = 0; j <= 254; ++j)
        for (int x = 0; x <= j; ++x) {
            int32_t sc[2] = {10 * (j - x) - x, 10 * 3 - 0}, en[2] = {j, 3}, na[2] = {254, 254};
            roundtrip(k0, sc, en, na, 1, (uint32_t)(j & 1), 0, a512, "one pair");
            roundtrip(k0, sc, en, na, 2, (uint32_t)(x & 1), 1, a512, "two pairs");
        }
    printf("checked every (j, X)\n");
    std::mt19937 rng(5);
    const int scoring[][2] = {{10, -1}, {1, -1}, {2, 2}, {-1, 3}, {5, -7}, {100, -27}};
    long long escapes = 0, total = 0;
    for (const auto& scg : scoring) {
        const ovl_expand::RecK k{scg[0], scg[1]};
        for (int lw : {100, 254, 31, 1}) {
            for (int spread : {2, 12, 60}) {  // how far the pairs lie from the tile's model
                for (uint32_t phase : {0u, 1u}) {
                    for (size_t cnt : {64u, 37u, 1u}) {
                        for (int misal : {0, 3}) {
                            for (int rep = 0; rep < 12; ++rep) {
                                int32_t sc[64], en[64], na[64];
                                for (size_t l = 0; l < cnt; ++l) {
                                    const unsigned r = rng() % 100;
                                    na[l] = r < 10 ? (int32_t)(rng() % (lw + 1)) : lw;
                                    if (r < 3) {
                                        en[l] = -1;
                                        sc[l] = -1;
                                        continue;
                                    }
                                    int32_t j, L;
                                    if (r < 10 && na[l] < lw) {  // a window pair: j in (n, lw]
                                        j = na[l] + 1 + (int32_t)(rng() % (lw - na[l]));
                                        L = na[l];
                                    } else {
                                        const int32_t top = std::min(lw, na[l]);
                                        j = r < 13 ? 0 : std::max(0, top - (int32_t)(rng() % (spread + 1)));
                                        L = j;
                                    }
                                    const int32_t xc = (L * 2) / 3;
                                    int32_t x = xc + (int32_t)(rng() % (2 * spread + 1)) - spread;
                                    x = std::max(0, std::min(L, x));
                                    if (k.match == k.mismatch) x = 0;
                                    en[l] = j;
                                    sc[l] = k.match * (L - x) + k.mismatch * x;
                                }
                                escapes += roundtrip(k, sc, en, na, cnt, phase, misal, a512, "random");
                                total += (long long)cnt;
                            }
                        }
                    }
                }
            }
        }
    }
    // (4) an escape word that never comes
    {
        int32_t sc[64], en[64], na[64];
        for (int l = 0; l < 64; ++l) {
            sc[l] = 10 * l;
            en[l] = l;
            na[l] = 100;
        }
        en[9] = -1;
        alignas(64) uint32_t rec[32] = {0};
        uint32_t sp[64] = {0};
        ovl_expand::encode_rec_tile(rec, sp, k0, sc, en, na, 64, 1);
        for (int w = 23; w < 32; ++w) rec[w] = 0;  // (not arrived)
        for (int l = 0; l < 64; ++l) sp[l] = 0;
        alignas(64) int32_t S[64], E[64];
        int polls = 0, bad = 0;
        uint32_t* taken[64];
        auto three = [&] { return ++polls < 3; };
        CHECK(ovl_expand::rec_tile_scalar(S, E, rec, sp, k0, 64, &bad, taken, three) == -1,
              "scalar: missing escape not seen");
        if (a512) {
            polls = 0;
            bool ready = false;
            CHECK(ovl_expand::rec_tile_avx512(S, E, rec, sp, k0, 1u, true, &ready, &bad, taken, three) == -1,
                  "avx512: missing escape not seen");
        }
    }
    printf("checked %s, %lld pairs, %lld escapes\n", a512 ? "scalar avx512" : "scalar", total, escapes);
    if (fails) {
        printf("%d failures\n", fails);
        return 1;
    }
    printf("ok\n");
    return 0;
}
