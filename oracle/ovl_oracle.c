/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's overlap scoring, used as the parity
 * checker by tests/, by __graft_entry__.smoke() and as bench.py's
 * cpu_baseline leg.  Nothing in the product path (ovlgraph/, csrc/) may link,
 * load or call this file.
 *
 * Follows, line by line in behaviour (not in text):
 *   aligners.py:27-30  n, m; int32 dp table and int8 traceback table, zeroed
 *                      (row 0 and column 0 stay 0: free overhangs)
 *   aligners.py:33-48  fill: diag = dp[i-1][j-1] + (match | mismatch),
 *                      up = dp[i-1][j] + indel, left = dp[i][j-1] + indel;
 *                      pick diag if diag>=up && diag>=left, elif up>=left up,
 *                      else left; store into the int32 table.
 *   aligners.py:50-57  last-row scan j = 0..m from -inf with strict '>':
 *                      best score and FIRST j attaining it.
 * Arithmetic is int64 and stores wrap to int32, as Numba compiles it
 * (integer binops are typed at >= intp width: numba/core/typing/builtins.py
 * :141-166; the omitted default indel is typed from its literal, int64).
 *
 * Parity pinning: tests/golden/ fixtures were produced by executing the
 * reference's own aligners.py/overlapGraphs.py source (see oracle/gen_golden.py
 * and DESIGN.md §Oracle for how, and for the caveat that Numba itself is absent).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_ABI_VERSION 1

int oracle_version(void) { return ORACLE_ABI_VERSION; }

/* Full DP, aligners.py:27-57.  tb (nullable) receives the (n+1)*(m+1) int8
 * traceback table, row-major.  Returns 0, or -1 on allocation failure. */
int oracle_overlap_dp(const uint8_t* s, int32_t n, const uint8_t* t, int32_t m,
                      int64_t match, int64_t mismatch, int64_t indel,
                      int32_t* out_score, int32_t* out_end, int8_t* tb)
{
    const size_t W = (size_t)m + 1;
    const size_t cells = ((size_t)n + 1) * W;
    /* the reference allocates both tables per call (aligners.py:28,30) */
    int32_t* dp = (int32_t*)calloc(cells, sizeof(int32_t));
    int8_t* tr = tb ? tb : (int8_t*)calloc(cells, 1);
    if (!dp || !tr) { free(dp); if (!tb) free(tr); return -1; }
    if (tb) memset(tb, 0, cells);
    for (int32_t i = 1; i <= n; ++i) {
        const int32_t* prev = dp + (size_t)(i - 1) * W;
        int32_t* cur = dp + (size_t)i * W;
        int8_t* trow = tr + (size_t)i * W;
        const uint8_t si = s[i - 1];
        for (int32_t j = 1; j <= m; ++j) {
            int64_t diag = (int64_t)prev[j - 1] + (si == t[j - 1] ? match : mismatch);
            int64_t up = (int64_t)prev[j] + indel;
            int64_t left = (int64_t)cur[j - 1] + indel;
            if (diag >= up && diag >= left) { cur[j] = (int32_t)diag; trow[j] = 0; }
            else if (up >= left)            { cur[j] = (int32_t)up;   trow[j] = 1; }
            else                            { cur[j] = (int32_t)left; trow[j] = 2; }
        }
    }
    double best = -INFINITY;
    int32_t end = 0;
    const int32_t* last = dp + (size_t)n * W;
    for (int32_t j = 0; j <= m; ++j) {
        if ((double)last[j] > best) { best = (double)last[j]; end = j; }
    }
    *out_score = (int32_t)best;
    *out_end = end;
    free(dp);
    if (!tb) free(tr);
    return 0;
}

/* Closed form of the DP when gaps cannot win:
 * dp[n][j] = sum over the L=min(n,j) diagonal cells ending at (n, j). */
void oracle_overlap_ungapped(const uint8_t* s, int32_t n, const uint8_t* t, int32_t m,
                             int64_t match, int64_t mismatch,
                             int32_t* out_score, int32_t* out_end)
{
    int64_t best = 0;  /* j = 0 scores 0 and is scanned first */
    int32_t end = 0;
    for (int32_t j = 1; j <= m; ++j) {
        const int32_t L = n < j ? n : j;
        const uint8_t* sp = s + (n - L);
        const uint8_t* tp = t + (j - L);
        int64_t sum = 0;
        for (int32_t q = 0; q < L; ++q) sum += (sp[q] == tp[q]) ? match : mismatch;
        if (sum > best) { best = sum; end = j; }
    }
    *out_score = (int32_t)best;
    *out_end = end;
}

/* Banded seed-and-extend variant (the build's band knob; NOT a reference mode,
 * parity with the reference only at full width).  Seed: the ungapped closed
 * form's first argmax j* (diagonal d* = n - j*).  Extend: the aligners.py:33-48
 * recurrence restricted to cells with |(i - j) - d*| <= band; predecessors
 * outside the band count as -inf (never chosen); row 0 / column 0 cells inside
 * the band are 0.  Score: last-row cells inside the band, strict '>' first argmax.
 * Requires values to fit int32 (no wrap): callers check that. */
int oracle_overlap_banded(const uint8_t* s, int32_t n, const uint8_t* t, int32_t m,
                          int64_t match, int64_t mismatch, int64_t indel, int32_t band,
                          int32_t* out_score, int32_t* out_end)
{
    int32_t seed_score, jstar;
    oracle_overlap_ungapped(s, n, t, m, match, mismatch, &seed_score, &jstar);
    const int64_t dstar = (int64_t)n - jstar;
    const size_t W = (size_t)m + 1;
    const size_t cells = ((size_t)n + 1) * W;
    int64_t* dp = (int64_t*)calloc(cells, sizeof(int64_t));
    if (!dp) return -1;
    for (int32_t i = 1; i <= n; ++i) {
        const int64_t* prev = dp + (size_t)(i - 1) * W;
        int64_t* cur = dp + (size_t)i * W;
        const int64_t jlo = (int64_t)i - dstar - band;   /* unclamped band edges of row i */
        const int64_t jhi = (int64_t)i - dstar + band;
        const uint8_t si = s[i - 1];
        for (int32_t j = 1; j <= m; ++j) {
            if (j < jlo || j > jhi) continue;
            const int64_t diag = prev[j - 1] + (si == t[j - 1] ? match : mismatch);
            const int up_ok = j != jhi;    /* (i-1, j) is inside the band */
            const int left_ok = j != jlo;  /* (i, j-1) is inside the band (or column 0) */
            const int64_t up = prev[j] + indel;
            const int64_t left = cur[j - 1] + indel;
            if ((!up_ok || diag >= up) && (!left_ok || diag >= left)) cur[j] = diag;
            else if (up_ok && (!left_ok || up >= left))               cur[j] = up;
            else                                                      cur[j] = left;
        }
    }
    int64_t best = 0;
    int32_t end = -1;
    const int64_t* last = dp + (size_t)n * W;
    for (int32_t j = 0; j <= m; ++j) {
        const int64_t k = (int64_t)n - j - dstar;
        if (k < -band || k > band) continue;
        if (end < 0 || last[j] > best) { best = last[j]; end = j; }
    }
    *out_score = (int32_t)best;
    *out_end = end;
    free(dp);
    return 0;
}

/* local_alignment, aligners.py:85-167 (Smith-Waterman with the reference's tie order):
 * cell = diag if diag>=up && diag>=left && diag>=0 (code 1), elif up>=left && up>=0 (2),
 * elif left>=0 (3), else 0 (code 0); int64 arithmetic, int32 stores.  Best cell: the
 * first strict '>' maximum in the i-major / j-minor fill order, from 0 (:128-130).
 * Walk (:133-153) from (best_i, best_j) while i > 0 && j > 0 && dp > 0, by code; ops
 * (nullable, up to cap entries) receives the codes in walk order; *start_j is the
 * column where the walk stopped (start position, :156).  Returns 0 or -1 (alloc). */
int oracle_local_align(const uint8_t* q, int32_t n, const uint8_t* r, int32_t m,
                       int64_t match, int64_t mismatch, int64_t indel,
                       int32_t* out_score, int32_t* out_bi, int32_t* out_bj, int32_t* out_start_i,
                       int32_t* out_start_j, int8_t* ops, int64_t cap, int64_t* n_ops)
{
    const size_t W = (size_t)m + 1;
    const size_t cells = ((size_t)n + 1) * W;
    int32_t* dp = (int32_t*)calloc(cells, sizeof(int32_t));
    int8_t* tb = (int8_t*)calloc(cells, 1);
    if (!dp || !tb) { free(dp); free(tb); return -1; }
    int64_t best = 0;
    int32_t bi = 0, bj = 0;
    for (int32_t i = 1; i <= n; ++i) {
        const int32_t* prev = dp + (size_t)(i - 1) * W;
        int32_t* cur = dp + (size_t)i * W;
        int8_t* trow = tb + (size_t)i * W;
        for (int32_t j = 1; j <= m; ++j) {
            const int64_t diag = (int64_t)prev[j - 1] + (q[i - 1] == r[j - 1] ? match : mismatch);
            const int64_t up = (int64_t)prev[j] + indel;
            const int64_t left = (int64_t)cur[j - 1] + indel;
            if (diag >= up && diag >= left && diag >= 0) { cur[j] = (int32_t)diag; trow[j] = 1; }
            else if (up >= left && up >= 0)              { cur[j] = (int32_t)up;   trow[j] = 2; }
            else if (left >= 0)                          { cur[j] = (int32_t)left; trow[j] = 3; }
            else                                         { cur[j] = 0; }
            if ((int64_t)cur[j] > best) { best = cur[j]; bi = i; bj = j; }
        }
    }
    int32_t i = bi, j = bj;
    int64_t k = 0;
    while (i > 0 && j > 0 && dp[(size_t)i * W + j] > 0) {
        const int8_t c = tb[(size_t)i * W + j];
        if (c == 1)      { --i; --j; }
        else if (c == 2) { --i; }
        else if (c == 3) { --j; }
        else break;
        if (ops && k < cap) ops[k] = c;
        ++k;
    }
    *out_score = (int32_t)best;
    *out_bi = bi;
    *out_bj = bj;
    *out_start_i = i;
    *out_start_j = j;
    *n_ops = k;
    free(dp);
    free(tb);
    return 0;
}

static int batch_common(int mode, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                        const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs,
                        int64_t match, int64_t mismatch, int64_t indel, int32_t band,
                        int32_t* out_score, int32_t* out_end, int32_t threads)
{
    for (int64_t p = 0; p < n_pairs; ++p) {
        if (a_idx[p] < 0 || a_idx[p] >= n_reads || b_idx[p] < 0 || b_idx[p] >= n_reads) return -2;
    }
    int err = 0;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(threads) reduction(| : err)
#endif
    for (int64_t p = 0; p < n_pairs; ++p) {
        const int32_t a = a_idx[p], b = b_idx[p];
        const uint8_t* s = seqs + offsets[a];
        const uint8_t* t = seqs + offsets[b];
        const int32_t n = (int32_t)(offsets[a + 1] - offsets[a]);
        const int32_t m = (int32_t)(offsets[b + 1] - offsets[b]);
        if (mode == 0) {
            err |= oracle_overlap_dp(s, n, t, m, match, mismatch, indel, out_score + p, out_end + p, NULL);
        } else if (mode == 2) {
            err |= oracle_overlap_banded(s, n, t, m, match, mismatch, indel, band, out_score + p, out_end + p);
        } else {
            oracle_overlap_ungapped(s, n, t, m, match, mismatch, out_score + p, out_end + p);
        }
    }
    (void)threads;
    return err ? -1 : 0;
}

/* ---------------------------------------------------------------------------
 * Optimised CPU closed form (bench.py's second CPU-baseline line, SURVEY.md §8d:
 * "the build's optimized closed-form CPU path").  Same result as
 * oracle_overlap_ungapped -- exact when gaps cannot win --
 * computed 64 bases at a time: reads are packed once into two bit planes
 * (2 bits per base, ACGT only, base i at bit i), and the mismatch count of the
 * diagonal ending at (n, j) is popcount((s0 ^ t0) | (s1 ^ t1)) over the aligned
 * windows, so dp[n][j] = match * L + (mismatch - match) * X(j).
 * ------------------------------------------------------------------------- */
#define CF_MAXW 5  /* words per plane: reads up to 256 bases (+ one spill word) */

static inline uint64_t cf_window(const uint64_t* w, int32_t start, int32_t k) {
    const int32_t q = (start >> 6) + k, r = start & 63;
    return r ? (w[q] >> r) | (w[q + 1] << (64 - r)) : w[q];
}

/* pack read bytes (ACGT -> 0..3 by byte order A<C<G<T) into planes[2][CF_MAXW] */
static int cf_pack(const uint8_t* x, int32_t n, uint64_t planes[2][CF_MAXW]) {
    memset(planes, 0, sizeof(uint64_t) * 2 * CF_MAXW);
    for (int32_t i = 0; i < n; ++i) {
        uint64_t c;
        switch (x[i]) {
            case 'A': c = 0; break;
            case 'C': c = 1; break;
            case 'G': c = 2; break;
            case 'T': c = 3; break;
            default: return -1;
        }
        planes[0][i >> 6] |= (c & 1) << (i & 63);
        planes[1][i >> 6] |= (c >> 1) << (i & 63);
    }
    return 0;
}

static void cf_pair(const uint64_t S[2][CF_MAXW], int32_t n, const uint64_t T[2][CF_MAXW], int32_t m,
                    int64_t match, int64_t mismatch, int32_t* out_score, int32_t* out_end) {
    int64_t best = 0;  /* j = 0 scores 0 and is scanned first */
    int32_t end = 0;
    const int64_t dms = mismatch - match;
    for (int32_t j = 1; j <= m; ++j) {
        const int32_t L = n < j ? n : j;
        const int32_t a = n - L, b = j - L;  /* s[a .. a+L) against t[b .. b+L) */
        int64_t x = 0;
        const int32_t words = (L + 63) >> 6;
        for (int32_t k = 0; k < words; ++k) {
            uint64_t d = (cf_window(S[0], a, k) ^ cf_window(T[0], b, k)) |
                         (cf_window(S[1], a, k) ^ cf_window(T[1], b, k));
            const int32_t rem = L - 64 * k;
            if (rem < 64) d &= (((uint64_t)1) << rem) - 1;
            x += __builtin_popcountll(d);
        }
        const int64_t sum = match * L + dms * x;
        if (sum > best) { best = sum; end = j; }
    }
    *out_score = (int32_t)best;
    *out_end = end;
}

/* Closed form over a pair list of ACGT reads up to 256 bases; -3 when a read is longer or has
 * another symbol (callers use oracle_batch_ungapped then).  threads <= 0: all OpenMP threads. */
int oracle_batch_closed_form(const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                             const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs,
                             int64_t match, int64_t mismatch,
                             int32_t* out_score, int32_t* out_end, int32_t threads)
{
    for (int64_t p = 0; p < n_pairs; ++p) {
        if (a_idx[p] < 0 || a_idx[p] >= n_reads || b_idx[p] < 0 || b_idx[p] >= n_reads) return -2;
    }
    uint64_t (*pk)[2][CF_MAXW] = (uint64_t (*)[2][CF_MAXW])malloc(sizeof(*pk) * (size_t)(n_reads > 0 ? n_reads : 1));
    if (!pk) return -1;
    int err = 0;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(threads) reduction(| : err)
#endif
    for (int32_t r = 0; r < n_reads; ++r) {
        const int64_t len = offsets[r + 1] - offsets[r];
        if (len > 64 * (CF_MAXW - 1) || cf_pack(seqs + offsets[r], (int32_t)len, pk[r])) err |= 1;
    }
    if (err) { free(pk); return -3; }
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1024) num_threads(threads)
#endif
    for (int64_t p = 0; p < n_pairs; ++p) {
        const int32_t a = a_idx[p], b = b_idx[p];
        cf_pair((const uint64_t (*)[CF_MAXW])pk[a], (int32_t)(offsets[a + 1] - offsets[a]),
                (const uint64_t (*)[CF_MAXW])pk[b], (int32_t)(offsets[b + 1] - offsets[b]),
                match, mismatch, out_score + p, out_end + p);
    }
    (void)threads;
    free(pk);
    return 0;
}

/* Batch over a pair list; threads <= 0 means all OpenMP threads. */
int oracle_batch_dp(const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                    const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs,
                    int64_t match, int64_t mismatch, int64_t indel,
                    int32_t* out_score, int32_t* out_end, int32_t threads)
{
    return batch_common(0, seqs, offsets, n_reads, a_idx, b_idx, n_pairs, match, mismatch, indel, -1,
                        out_score, out_end, threads);
}

int oracle_batch_ungapped(const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                          const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs,
                          int64_t match, int64_t mismatch,
                          int32_t* out_score, int32_t* out_end, int32_t threads)
{
    return batch_common(1, seqs, offsets, n_reads, a_idx, b_idx, n_pairs, match, mismatch, 0, -1,
                        out_score, out_end, threads);
}

int oracle_batch_banded(const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                        const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs,
                        int64_t match, int64_t mismatch, int64_t indel, int32_t band,
                        int32_t* out_score, int32_t* out_end, int32_t threads)
{
    return batch_common(2, seqs, offsets, n_reads, a_idx, b_idx, n_pairs, match, mismatch, indel, band,
                        out_score, out_end, threads);
}
