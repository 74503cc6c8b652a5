/*
 * ovl.h — C ABI of the MI355X-native overlap-scoring engine (libovl.so).
 *
 * Replaces the per-pair Python->Numba boundary of the reference:
 *   overlapGraphs.py:53   overlap_alignment(read_a, read_b) once per candidate pair
 *   aligners.py:6-82      @njit overlap_alignment(s, t, match_score=10, mismatch=-1, indel=-2**31)
 * with one batched call per candidate list.  Only (score, end) reach the
 * graph (overlapGraphs.py:53-60), so that is what the batch entry points return.
 *
 * Conventions
 *  - Plain C types only; the caller owns every pointer it passes in.
 *  - Return value 0 (OVL_OK) on success, a negative OVL_E_* code on failure;
 *    ovl_last_error() then describes it.  Nothing throws or aborts across the ABI.
 *  - One call at a time per ovl_ctx.  Contexts are independent.  A context
 *    drives one or more GPUs from the calling thread: host-array
 *    scoring calls shard the pair list over its devices (contiguous ranges
 *    balanced by sum len(a)*len(b)) and every device writes its range of the
 *    results straight into the caller's arrays.  joblib-style multi-process
 *    callers create one single-device context per process.
 *  - Host arrays may be pageable or pinned (ovl_host_alloc / ovl_host_register /
 *    hipHostMalloc).  Pinned arrays are read and written by DMA in place;
 *    pageable ones go through pinned staging.  Either way copies, kernels and
 *    result copies of consecutive chunks overlap.
 *  - Read i is the byte string seqs[offsets[i] .. offsets[i+1]).  Bytes are
 *    symbols compared for equality only (any alphabet of <= 256 symbols).
 *  - Semantics are the reference's: DP fill of aligners.py:27-48 with int64
 *    arithmetic and int32 stores, last-row strict-'>' first argmax of
 *    aligners.py:50-57.  score >= 0 and 0 <= end <= len(t) always.
 */
#ifndef OVL_H
#define OVL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OVL_ABI_VERSION 3

enum {
    OVL_OK = 0,
    OVL_E_ARG = -1,          /* bad argument (null pointer, negative size, bad offsets) */
    OVL_E_HIP = -2,          /* HIP runtime error */
    OVL_E_OOM = -3,          /* device allocation failed */
    OVL_E_UNSUPPORTED = -4,  /* read too long, >256 symbols, band at scores too large for int32 cells */
    OVL_E_RANGE = -5,        /* scoring magnitudes would overflow the int32 DP table */
    OVL_E_STATE = -6,        /* no resident reads (ovl_set_reads not called) */
    OVL_E_INDEX = -7,        /* a pair index is outside [0, n_reads) */
    OVL_E_INTERNAL = -8      /* a streamed result record never completed although its kernel had finished */
};

enum {
    OVL_KERNEL_NONE = 0,
    OVL_KERNEL_UNGAPPED = 1, /* 2-bit (or 4/8-bit) bit-plane popcount kernel; exact when gaps cannot win */
    OVL_KERNEL_DP = 2,       /* anti-diagonal wavefront DP, int64-exact, any scoring */
    OVL_KERNEL_BANDED = 3    /* ungapped seed + banded DP around its diagonal (band >= 0, gaps can win) */
};

typedef struct ovl_ctx ovl_ctx;

/* ABI version (OVL_ABI_VERSION). */
int ovl_version(void);

/* Number of visible HIP devices. */
int ovl_device_count(int32_t* out_count);

/*
 * Create a context on n_devices GPUs: 0 = every visible device;
 * otherwise the n_devices consecutive devices starting at the calling thread's
 * current device (so 1 = the current device).  The caller's current device is
 * never changed by any entry point.
 */
int ovl_create(int32_t n_devices, ovl_ctx** out_ctx);
/* Create a context on an explicit list of distinct device ordinals (device 0 of the context = devices[0]). */
int ovl_create_on_devices(const int32_t* devices, int32_t n_devices, ovl_ctx** out_ctx);
/* The context's device ordinals: *out_n = count, ids[0 .. min(cap, count)) = ordinals. */
int ovl_ctx_devices(const ovl_ctx* ctx, int32_t* ids, int32_t cap, int32_t* out_n);
int ovl_destroy(ovl_ctx* ctx);

/* Pinned host memory for result / pair arrays (DMA in place, visible to every device). */
int ovl_host_alloc(int64_t bytes, void** out_ptr);
int ovl_host_free(void* ptr);
/* Pin (register) / unpin an existing host range, e.g. a shared-memory result buffer. */
int ovl_host_register(void* ptr, int64_t bytes);
int ovl_host_unregister(void* ptr);

/* Host thread pool of the result transport (expansion of packed results, copies of pageable arrays), recounted
 * now: *cpus = this process's CPUs (affinity set, capped by the cgroup quota), *sharers = processes driving
 * libovl on the same CPU set (other libovl processes of this user with the same affinity, e.g. joblib workers,
 * or LOCAL_WORLD_SIZE when larger), *threads = threads a call uses (ovl_host_pool_rule), *packed = 1 when the
 * packed transport may be used (>= 6 threads; otherwise results cross as int32 and the pool does not poll).
 * Any output pointer may be NULL. */
int ovl_host_pool(int32_t* threads, int32_t* sharers, int32_t* cpus, int32_t* packed);
/* The sizing rule: env_threads > 0 (OVL_POOL_THREADS) wins, else min(12, cpus / sharers - 1), at least 1. */
int32_t ovl_host_pool_rule(int32_t cpus, int32_t sharers, int32_t env_threads);

/* Per-call timing of host-array scoring calls (off by default; on adds HIP timing events):
 * kernel_ms = summed kernel time of the busiest device, call_ms = wall time of the call. */
int ovl_set_timing(ovl_ctx* ctx, int32_t on);
int ovl_last_timing(const ovl_ctx* ctx, double* kernel_ms, double* call_ms);
/* The scoring launches of the last host-array call made with timing on, in issue order: *out_n = count;
 * entry i < cap gives the device ordinal, the result sink (1 int32 stored into host memory; 2 packed 2 B/pair
 * into host staging, expanded by host threads after the launch; 0, HBM, only in ovl_score_device), the pairs and
 * the launch's
 * duration in ms (HIP events recorded by the kernel's own launch for ungapped chunks, else on its stream).
 * Any output pointer may be NULL. */
int ovl_last_launches(const ovl_ctx* ctx, int32_t cap, int32_t* device, int32_t* sink, int64_t* pairs, double* ms,
                      int32_t* out_n);
/* Link traffic of the last host-array scoring call (always recorded): link_bytes = pair-list bytes the
 * devices read from host memory + result bytes they stored there (ovl_last_results: 2 per pair in packed
 * chunks, 8 per pair otherwise; the resident grid's calls 128 per 64-pair tile record plus 8 per special pair; the
 * few pairs of a 2 B/pair chunk whose score travels separately add 4 each and are not counted); packed_pairs =
 * pairs whose results crossed packed and were expanded on the host. */
int ovl_last_transfer(const ovl_ctx* ctx, int64_t* link_bytes, int64_t* packed_pairs);
/* The results' part of the last host-array call's link bytes (always recorded): result_bytes = what the kernels
 * stored into host memory for the results (8 per int32 pair, 2 per packed pair; a resident-grid call 128 per
 * tile record of 64 pairs plus 8 per special pair); record_pairs = pairs that crossed as the resident grid's tile
 * records; escapes = the special pairs among them (a shorter read a inside b's window, or a bad pair), whose word
 * travels apart. */
int ovl_last_results(const ovl_ctx* ctx, int64_t* result_bytes, int64_t* record_pairs, int64_t* escapes);
/* How the last host-array call's pair list reached the kernels (always recorded): in_place_pairs = pairs of
 * chunks the scoring kernel read in their compact encoding (b as uint16, a as tile deltas); decoded_pairs =
 * pairs of compact chunks decoded into HBM first (runs / widen kernels).  Both 0 for a call whose list crossed
 * as the caller's int32 arrays, or that had no host list. */
int ovl_last_pair_list(const ovl_ctx* ctx, int64_t* in_place_pairs, int64_t* decoded_pairs);

/* Last error message of `ctx`, or of the calling thread when ctx is NULL. */
const char* ovl_last_error(const ovl_ctx* ctx);

/*
 * One-shot batch scoring: uploads and packs the reads, scores
 * n_pairs candidates (a_idx[p], b_idx[p]) and writes out_score[p], out_end[p].
 * Replaces the loop body of overlapGraphs.py:50-53 for a whole candidate list.
 *
 * band < 0: the full DP of aligners.py:27-57 (reference semantics, bit-exact).
 * band >= 0: the build's seed-and-extend knob (not a reference mode): seed
 *   j* = the ungapped first argmax, diagonal d* = n - j*; the aligners.py:33-48
 *   recurrence on cells with |(i - j) - d*| <= band only, out-of-band
 *   predecessors = -inf; last-row strict '>' first argmax over in-band cells.
 *   Identical to band < 0 whenever gaps cannot win (e.g. the default
 *   indel = -2^31) and when band >= 2 * (longest read).
 */
int ovl_score_pairs(ovl_ctx* ctx, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads,
                    const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs,
                    int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                    int32_t* out_score, int32_t* out_end);

/* Upload + pack a read set and keep it resident in HBM (replaces any previous set). */
int ovl_set_reads(ovl_ctx* ctx, const uint8_t* seqs, const int64_t* offsets, int32_t n_reads);

/* Resident read-set facts: count, longest read, bit planes per base, device bytes held. */
int ovl_reads_info(const ovl_ctx* ctx, int32_t* n_reads, int32_t* lmax, int32_t* planes,
                   int64_t* device_bytes);

/* Which kernel a score call with these parameters would use on the resident reads. */
int ovl_plan(const ovl_ctx* ctx, int32_t match, int32_t mismatch, int64_t indel, int32_t band,
             int32_t* out_kernel);

/* Score against the resident reads; host pair/result arrays; synchronous.  Sharded over the
 * context's devices; chunked H2D / kernel / D2H pipeline per device.  A pair index outside
 * [0, n_reads) makes the call return OVL_E_INDEX (checked on the device, its results are -1). */
int ovl_score_host(ovl_ctx* ctx, const int32_t* a_idx, const int32_t* b_idx, int64_t n_pairs,
                   int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                   int32_t* out_score, int32_t* out_end);

/*
 * Score against the resident reads with DEVICE pointers (on the context's first device),
 * asynchronously on `stream` (a hipStream_t; NULL = the default stream, as in the HIP API).  Pairs with an index
 * outside [0, n_reads) get score = end = -1 and set a device error flag that
 * ovl_check_device_errors() reports.
 */
int ovl_score_device(ovl_ctx* ctx, const int32_t* d_a_idx, const int32_t* d_b_idx, int64_t n_pairs,
                     int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                     int32_t* d_score, int32_t* d_end, void* stream);

/* Synchronise the device; OVL_E_INDEX if a previous ovl_score_device saw a bad index (flag is cleared). */
int ovl_check_device_errors(ovl_ctx* ctx);

/*
 * One resident pair (a, b) through the DP kernel, optionally returning the
 * (len(a)+1) x (len(b)+1) int8 traceback table of aligners.py:30,42-48
 * (0 = diagonal, 1 = up, 2 = left) for the backtrack of aligners.py:59-78.
 */
int ovl_align_one(ovl_ctx* ctx, int32_t a, int32_t b, int32_t match, int32_t mismatch, int64_t indel,
                  int32_t* out_score, int32_t* out_end, int8_t* traceback);

/*
 * k-mer candidate enumeration on the device over the resident reads, which must
 * be the distinct reads in read_copies order (overlapGraphs.py:18-20).  Produces
 * exactly the pair list the reference scores, in its order (overlapGraphs.py:30-52):
 * for each read a in order, every read b != a whose prefix read[:k] equals a's
 * suffix read[-k:] (whole reads when shorter than k), b in read order; k == 0:
 * every b != a.  The list stays in the context (until the next ovl_candidates or
 * ovl_set_reads); *out_n_pairs receives its length.  OVL_E_UNSUPPORTED when
 * k * (bits per symbol: 2, 4 or 8) > 58.  Replaces the Python loops of
 * overlapGraphs.py:30-52 (which the host path, ovlgraph/candidates.py, restates).
 */
int ovl_candidates(ovl_ctx* ctx, int32_t k, int64_t* out_n_pairs);

/* Copy the context's candidate list to host arrays of *out_n_pairs entries each. */
int ovl_candidates_copy(ovl_ctx* ctx, int32_t* a_idx, int32_t* b_idx);

/* Device pointers (and length) of the context's candidate list, for ovl_score_device. */
int ovl_candidates_device(const ovl_ctx* ctx, const int32_t** d_a_idx, const int32_t** d_b_idx, int64_t* n_pairs);

/* Score the context's candidate list (no pair upload); host outputs; synchronous.  Every device
 * of the context enumerated the same list, each scores its shard and copies its results into its
 * slice of out_score / out_end (the "gather" of SURVEY.md §8e is these per-device D2H copies). */
int ovl_score_candidates(ovl_ctx* ctx, int32_t match, int32_t mismatch, int64_t indel, int32_t band,
                         int32_t* out_score, int32_t* out_end);

/* The same for pairs [lo, hi) of the candidate list: out_score[p - lo], out_end[p - lo].  A
 * process of a multi-process job scores its shard this way (bounds from ovl_candidates_shards). */
int ovl_score_candidates_range(ovl_ctx* ctx, int64_t lo, int64_t hi, int32_t match, int32_t mismatch,
                               int64_t indel, int32_t band, int32_t* out_score, int32_t* out_end);

/* The resident grid (one per device of a single-device context): ovl_score_candidates(_range) calls of the
 * uniform kernel's form (ungapped plan, int32 keys, <= 4 symbols, reads <= 254 bases) are served by a kernel that
 * stays on the device between calls, fed requests through pinned memory -- a call pays no launch and no completion
 * signal.  It leaves by itself after ~20 ms without a request, when another entry point of the context needs the
 * device, and at ovl_destroy.  Opt-in: OVL_RESIDENT=1 at context creation (the default, 0, routes every call
 * through the launch pipeline, which the grid did not beat on the boxes measured).  ovl_quiesce makes the
 * context's grids leave now (before a whole-device synchronisation such as torch.cuda.synchronize(), which would
 * otherwise wait for the idle deadline); the next call relaunches them.  ovl_resident_stats reports how many grids
 * are resident, their launches (relaunches: calls that found their grid gone) and whether a failed call disabled
 * the path (its calls then go through the launch pipeline). */
int ovl_quiesce(ovl_ctx* ctx);
/* How many of the context's devices (its first ones) a host-array scoring call over n_pairs uses: several only from
 * 3 devices with >= 262,144 pairs each (multi-device calls store int32 results over every device's link; below
 * that one device with packed results is faster), else 1 -- so a context over every GPU is never slower than one
 * GPU.  (A context whose slots share a GPU, OVL_SHARE_DEVICES=1, uses every slot whatever this reports.) */
int ovl_devices_for(const ovl_ctx* ctx, int64_t n_pairs, int32_t* out_devices);
int ovl_resident_stats(const ovl_ctx* ctx, int32_t* alive, int64_t* launches, int64_t* relaunches, int32_t* broken);

/* Contiguous shard bounds of the candidate list, balanced by sum len(a)*len(b) + 1:
 * bounds[0] = 0 <= bounds[1] <= ... <= bounds[n_shards] = n_pairs (the rule of
 * ovlgraph/sharded.py:shard_bounds, computed on the device). */
int ovl_candidates_shards(ovl_ctx* ctx, int32_t n_shards, int64_t* bounds);

/*
 * local_alignment (aligners.py:85-167) of query[0..n) against reference[0..m) on the whole GPU:
 * Smith-Waterman with the reference's tie order and int64-exact arithmetic; bytes are compared
 * for equality only.  Outputs: the best score and its cell (end_i, end_j) -- the first strict
 * maximum in fill order; with ops != NULL also the traceback walk of aligners.py:133-153 from
 * that cell: ops[k] in walk order (1 diag, 2 up, 3 left), *n_ops its length (OVL_E_RANGE when
 * > ops_cap; n + m always suffices) and the cell where it stopped (start_i, start_j; start_j is
 * the reference's start position, aligners.py:156).  Needs n, m < 2^20 and match*min(n,m) < 2^24.
 */
int ovl_local_align(ovl_ctx* ctx, const uint8_t* query, int32_t n, const uint8_t* reference, int32_t m,
                    int32_t match, int32_t mismatch, int64_t indel, int32_t* out_score, int32_t* out_end_i,
                    int32_t* out_end_j, int32_t* out_start_i, int32_t* out_start_j, int8_t* ops,
                    int64_t ops_cap, int64_t* out_n_ops);

/* Cycle removal of overlapGraphs.py:106-130 (remove_cycles_from_graph), host-side, no context.
 * Replaces:  while True: cycle = nx.find_cycle(G, orientation='original') ... G.remove_edge(u, v)
 * The graph is CSR: n_nodes nodes in the DiGraph's node order; node v's out-edges are
 * head[off[v] .. off[v+1]) in its adjacency (insertion) order with integer weight[] ("weight").
 * Writes to removed[] (capacity off[n_nodes]) the CSR indices of the edges the reference loop
 * removes, in its removal order, and their count to *n_removed: networkx 3.x find_cycle's
 * cycle (edge DFS from the first unexplored node in node order), its first minimum-weight edge. */
int ovl_remove_cycles(const int64_t* off, const int32_t* head, const int64_t* weight, int32_t n_nodes,
                      int64_t* removed, int64_t* n_removed);
/* ovl_remove_cycles publishing its progress to a consumer on another thread (the C builder of the surviving
 * edges' dicts, ovlgraph/_digraph build_overlap_stream, builds each node's successors as soon as they are
 * final): alive[e] (off[n_nodes] entries) is set to 1, then 0 when edge e is removed; final_nodes[0 .. *n_final)
 * lists each node once, when its out-edges are final (it can reach no cycle: settled, or explored by a start
 * whose walk found none); *n_final is stored with release order (read it with an acquire load) and reaches
 * n_nodes before a successful call returns. */
int ovl_remove_cycles_stream(const int64_t* off, const int32_t* head, const int64_t* weight, int32_t n_nodes,
                             int64_t* removed, int64_t* n_removed, uint8_t* alive, int32_t* final_nodes,
                             int64_t* n_final);

#ifdef __cplusplus
}
#endif

#endif /* OVL_H */
