/*
 * A plain C caller of libovl.so (include/ovl.h), no Python and no HIP headers: what a maintainer's
 * binding (cgo / JNI / ctypes) sees.  Reads a test case from a text file, scores it through the
 * one-shot entry point (ovl_score_pairs), through a resident read set with pinned result arrays
 * (ovl_set_reads + ovl_candidates + ovl_score_candidates), and prints the results as text.
 *
 * Input (tests/test_gpu_c_abi.py writes it):
 *   n_reads k
 *   one read per line
 *   n_pairs
 *   a b          (one pair per line)
 * Output:
 *   "pairs <score> <end>" per pair (ovl_score_pairs), "cand <a> <b> <score> <end>" per candidate
 *   (device enumeration), "err <code> <message>" for the deliberate index error, "ok".
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ovl.h"

#define CK(call)                                                                       \
    do {                                                                               \
        int rc_ = (call);                                                              \
        if (rc_ != OVL_OK) {                                                           \
            fprintf(stderr, "%s -> %d: %s\n", #call, rc_, ovl_last_error(ctx));        \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "r");
    if (!f) return 2;
    int n_reads = 0, k = 0;
    if (fscanf(f, "%d %d", &n_reads, &k) != 2) return 2;
    char** reads = calloc((size_t)n_reads, sizeof(char*));
    int64_t* off = calloc((size_t)n_reads + 1, sizeof(int64_t));
    size_t cap = 1 << 20, used = 0;
    uint8_t* seqs = malloc(cap);
    char line[4096];
    for (int i = 0; i < n_reads; ++i) {
        if (fscanf(f, "%4095s", line) != 1) return 2;
        size_t n = strcmp(line, "-") == 0 ? 0 : strlen(line);  /* "-" stands for an empty read */
        while (used + n > cap) seqs = realloc(seqs, cap *= 2);
        memcpy(seqs + used, line, n);
        used += n;
        off[i + 1] = (int64_t)used;
        reads[i] = NULL;
    }
    int64_t n_pairs = 0;
    if (fscanf(f, "%lld", (long long*)&n_pairs) != 1) return 2;
    int32_t* a = malloc(sizeof(int32_t) * (size_t)(n_pairs + 1));
    int32_t* b = malloc(sizeof(int32_t) * (size_t)(n_pairs + 1));
    for (int64_t p = 0; p < n_pairs; ++p)
        if (fscanf(f, "%d %d", &a[p], &b[p]) != 2) return 2;
    fclose(f);

    ovl_ctx* ctx = NULL;
    if (ovl_version() != OVL_ABI_VERSION) return 3;
    CK(ovl_create(1, &ctx));
    int32_t* sc = malloc(sizeof(int32_t) * (size_t)(n_pairs + 1));
    int32_t* en = malloc(sizeof(int32_t) * (size_t)(n_pairs + 1));
    /* one shot: reads uploaded, packed and scored in one call (pageable arrays) */
    CK(ovl_score_pairs(ctx, seqs, off, n_reads, a, b, n_pairs, 10, -1, -2147483648LL, -1, sc, en));
    for (int64_t p = 0; p < n_pairs; ++p) printf("pairs %d %d\n", sc[p], en[p]);
    /* resident reads, the device-enumerated candidate list, pinned result arrays */
    int64_t n_cand = 0;
    CK(ovl_candidates(ctx, k, &n_cand));
    int32_t* ca = malloc(sizeof(int32_t) * (size_t)(n_cand + 1));
    int32_t* cb = malloc(sizeof(int32_t) * (size_t)(n_cand + 1));
    CK(ovl_candidates_copy(ctx, ca, cb));
    void* ps = NULL;
    void* pe = NULL;
    CK(ovl_host_alloc(sizeof(int32_t) * (n_cand + 1), &ps));
    CK(ovl_host_alloc(sizeof(int32_t) * (n_cand + 1), &pe));
    CK(ovl_score_candidates(ctx, 10, -1, -2147483648LL, -1, (int32_t*)ps, (int32_t*)pe));
    for (int64_t p = 0; p < n_cand; ++p)
        printf("cand %d %d %d %d\n", ca[p], cb[p], ((int32_t*)ps)[p], ((int32_t*)pe)[p]);
    /* an index outside the read set: an error code and a message, no crash */
    int32_t bad_a = 0, bad_b = n_reads + 3;
    int rc = ovl_score_host(ctx, &bad_a, &bad_b, 1, 10, -1, -2147483648LL, -1, sc, en);
    printf("err %d %s\n", rc, ovl_last_error(ctx));
    CK(ovl_host_free(ps));
    CK(ovl_host_free(pe));
    CK(ovl_destroy(ctx));
    printf("ok\n");
    free(seqs); free(off); free(a); free(b); free(sc); free(en); free(ca); free(cb); free(reads);
    return 0;
}
