// Read-set scan and 2-bit packing (genome-assembly-using-overlap-graphs_amd/csrc/ovl_scan.h): the AVX-512
// form against the scalar one and against a direct restatement (base i at bits 2(i % 4) of byte i / 4,
// A C G T = 0 1 2 3), on ACGT-only bytes, bytes with one other symbol anywhere, and ranges of every length
// mod 64 starting at multiples of 64.  Prints the forms checked, then "ok".
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "ovl_scan.h"

int main() {
    std::mt19937 rng(3);
    const char acgt[] = "ACGT";
    bool a512 = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("bmi2");
    for (int trial = 0; trial < 400; ++trial) {
        const size_t n = 1 + rng() % 5000;
        std::vector<uint8_t> p(n);
        for (auto& x : p) x = (uint8_t)acgt[rng() % 4];
        const int other = trial % 4 == 3 ? (int)(rng() % n) : -1;  // one byte outside ACGT
        if (other >= 0) p[(size_t)other] = (uint8_t)"NnacX"[rng() % 5];
        const size_t l0 = (rng() % 3) * 64;
        const size_t lo = l0 < n ? l0 : 0;
        const size_t hi = lo + (n - lo) - rng() % (n - lo);
        std::vector<uint8_t> want(n / 4 + 32, 0);
        for (size_t i = lo; i < hi; ++i) {
            const int c = p[i] == 'A' ? 0 : p[i] == 'C' ? 1 : p[i] == 'G' ? 2 : 3;
            want[i / 4] |= (uint8_t)(c << (2 * (i % 4)));
        }
        const bool want_ok = !(other >= 0 && (size_t)other >= lo && (size_t)other < hi);
        uint8_t s1[256] = {}, s2[256] = {}, sw[256] = {};
        for (size_t i = lo; i < hi; ++i) sw[p[i]] = 1;
        std::vector<uint8_t> k1(n / 4 + 32, 0), k2(n / 4 + 32, 0);
        const bool ok1 = ovl_scan::scan_pack_scalar(p.data(), lo, hi, s1, k1.data());
        if (ok1 != want_ok || memcmp(s1, sw, 256) || (ok1 && memcmp(k1.data() + lo / 4, want.data() + lo / 4, (hi - lo) / 4))) {
            printf("scalar mismatch trial %d n %zu lo %zu hi %zu\n", trial, n, lo, hi);
            return 1;
        }
        if (a512) {
            const bool ok2 = ovl_scan::scan_pack_avx512(p.data(), lo, hi, s2, k2.data());
            if (ok2 != want_ok || memcmp(s2, sw, 256) ||
                (ok2 && memcmp(k2.data() + lo / 4, want.data() + lo / 4, (hi - lo + 3) / 4))) {
                printf("avx512 mismatch trial %d n %zu lo %zu hi %zu ok %d/%d\n", trial, n, lo, hi, ok2, want_ok);
                return 1;
            }
        }
    }
    printf("checked scalar\n");
    if (a512) printf("checked avx512\n");
    printf("ok\n");
    return 0;
}
