// k-mer candidate-pair enumeration on the device, with the
// reference's exact output order (overlapGraphs.py:30-52):
//
//   prefix key of read i = read[:k] (the whole read when shorter, :34-37)
//   suffix key of read a = read[-k:] (the whole read when shorter, :44-47)
//   for a in read order (read_copies order, :43):
//     for b in prefix_index[suffix key of a], in read order (:38-40, :49-50):
//       if b != a (distinct reads, so index inequality is string inequality, :52): emit (a, b)
//   k == 0: every b != a in read order (:49).
//
// Device plan (all integer/byte work, HBM-light):
//   1. keys:   one thread per read packs its prefix / suffix symbol codes into a
//              64-bit key, (length << 58) | codes (2, 4 or 8 bits per symbol), so
//              equal keys <=> equal strings (lengths < k stay distinct);
//   2. sort:   stable LSD radix sort of (prefix key, read index) -> reads grouped
//              by prefix, index order kept inside a group (= prefix_index lists);
//   3. count:  per read a, binary search of its suffix key in the sorted keys ->
//              group [lo, hi); count = group size minus a itself if a is in it
//              (prefix key of a == suffix key of a);
//   4. scan:   exclusive prefix sum of the counts (int64) -> output offsets;
//   5. emit:   one wavefront per read walks its group 64 members at a time,
//              drops b == a with a ballot, writes (a, b) coalesced.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "ovl_kernels.h"

namespace ovl_cand {

__global__ __launch_bounds__(256) void key_kernel(const uint8_t* __restrict__ codes, const int64_t* __restrict__ off,
                                                  const int32_t* __restrict__ len, int32_t n_reads, int32_t k,
                                                  int32_t bits, uint64_t* __restrict__ pre_key,
                                                  uint64_t* __restrict__ suf_key, int32_t* __restrict__ iota) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_reads;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t n = len[i];
        const int32_t l = n < k ? n : k;
        const uint8_t* r = codes + off[i];
        uint64_t p = 0, s = 0;
        for (int q = 0; q < l; ++q) {
            p = (p << bits) | r[q];
            s = (s << bits) | r[n - l + q];
        }
        pre_key[i] = ((uint64_t)l << 58) | p;
        suf_key[i] = ((uint64_t)l << 58) | s;
        iota[i] = (int32_t)i;
    }
}

// first index in sorted[0, n) with sorted[idx] >= key (lower) or > key (upper)
__device__ __forceinline__ int64_t bound(const uint64_t* __restrict__ sorted, int64_t n, uint64_t key, bool upper) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const uint64_t v = sorted[mid];
        if (upper ? (v <= key) : (v < key)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void count_kernel(const uint64_t* __restrict__ sorted, const uint64_t* __restrict__ pre_key,
                                                    const uint64_t* __restrict__ suf_key, int32_t n_reads, int32_t all_pairs,
                                                    int64_t* __restrict__ lo_out, int64_t* __restrict__ hi_out,
                                                    int64_t* __restrict__ cnt) {
    for (int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; a < n_reads;
         a += (int64_t)gridDim.x * blockDim.x) {
        if (all_pairs) {  // k == 0: every other read
            lo_out[a] = 0;
            hi_out[a] = n_reads;
            cnt[a] = n_reads - 1;
            continue;
        }
        const uint64_t key = suf_key[a];
        const int64_t lo = bound(sorted, n_reads, key, false);
        const int64_t hi = bound(sorted, n_reads, key, true);
        lo_out[a] = lo;
        hi_out[a] = hi;
        // a is in its own group iff its prefix key equals its suffix key
        cnt[a] = (hi - lo) - (hi > lo && pre_key[a] == key ? 1 : 0);
    }
}

// one wavefront per read a: its group is order[lo, hi) (positions 0 .. n_reads-1
// themselves when all_pairs), members in index order; b == a is dropped
__global__ __launch_bounds__(256) void emit_kernel(const int32_t* __restrict__ order, const int64_t* __restrict__ lo_in,
                                                   const int64_t* __restrict__ hi_in, const int64_t* __restrict__ offs,
                                                   int32_t n_reads, int32_t all_pairs, int32_t* __restrict__ out_a,
                                                   int32_t* __restrict__ out_b) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t a = wave; a < n_reads; a += n_waves) {
        const int64_t lo = lo_in[a];
        const int64_t g = hi_in[a] - lo;
        const int64_t base = offs[a];
        int64_t written = 0;
        for (int64_t q0 = 0; q0 < g; q0 += 64) {
            const int64_t q = q0 + lane;
            const bool valid = q < g;
            const int32_t b = valid ? (all_pairs ? (int32_t)q : order[lo + q]) : -1;
            const bool keep = valid && b != (int32_t)a;
            const uint64_t m = __ballot(keep);
            if (keep) {
                const int64_t slot = base + written + __popcll(m & ((1ull << lane) - 1ull));
                out_a[slot] = (int32_t)a;
                out_b[slot] = b;
            }
            written += __popcll(m);
        }
    }
}

}  // namespace ovl_cand

using namespace ovl_cand;

static unsigned grid_for_threads(int64_t threads, int64_t cap) {
    int64_t b = (threads + 255) / 256;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

extern "C" hipError_t ovl_cand_keys(const uint8_t* codes, const int64_t* off, const int32_t* len, int32_t n_reads,
                                    int32_t k, int32_t bits, uint64_t* pre_key, uint64_t* suf_key, int32_t* iota,
                                    hipStream_t stream) {
    if (n_reads <= 0) return hipSuccess;
    key_kernel<<<grid_for_threads(n_reads, 8192), 256, 0, stream>>>(codes, off, len, n_reads, k, bits, pre_key,
                                                                    suf_key, iota);
    return hipGetLastError();
}

extern "C" hipError_t ovl_cand_temp_bytes(int32_t n_reads, size_t* bytes) {
    size_t s1 = 0, s2 = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, s1, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                      (const int32_t*)nullptr, (int32_t*)nullptr, n_reads, 0, 64);
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(nullptr, s2, (const int64_t*)nullptr, (int64_t*)nullptr, n_reads);
    if (e != hipSuccess) return e;
    *bytes = s1 > s2 ? s1 : s2;
    return hipSuccess;
}

extern "C" hipError_t ovl_cand_sort(void* temp, size_t temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                                    const int32_t* vals_in, int32_t* vals_out, int32_t n_reads, hipStream_t stream) {
    if (n_reads <= 0) return hipSuccess;
    return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, n_reads, 0, 64,
                                              stream);
}

extern "C" hipError_t ovl_cand_count(const uint64_t* sorted, const uint64_t* pre_key, const uint64_t* suf_key,
                                     int32_t n_reads, int32_t all_pairs, int64_t* lo, int64_t* hi, int64_t* cnt,
                                     hipStream_t stream) {
    if (n_reads <= 0) return hipSuccess;
    count_kernel<<<grid_for_threads(n_reads, 8192), 256, 0, stream>>>(sorted, pre_key, suf_key, n_reads, all_pairs,
                                                                      lo, hi, cnt);
    return hipGetLastError();
}

extern "C" hipError_t ovl_cand_scan(void* temp, size_t temp_bytes, const int64_t* cnt, int64_t* offs, int32_t n_reads,
                                    hipStream_t stream) {
    if (n_reads <= 0) return hipSuccess;
    return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, cnt, offs, n_reads, stream);
}

extern "C" hipError_t ovl_cand_emit(const int32_t* order, const int64_t* lo, const int64_t* hi, const int64_t* offs,
                                    int32_t n_reads, int32_t all_pairs, int32_t* out_a, int32_t* out_b,
                                    hipStream_t stream) {
    if (n_reads <= 0) return hipSuccess;
    emit_kernel<<<grid_for_threads((int64_t)n_reads * 64, 16384), 256, 0, stream>>>(order, lo, hi, offs, n_reads,
                                                                                    all_pairs, out_a, out_b);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------- shard bounds
// Contiguous shards of a pair list balanced by cost(p) = len[a]*len[b] + 1 (the
// DP work of a pair is n*m cells), the cut rule of ovlgraph/sharded.py:shard_bounds: inside
// [lo, hi), cut_r = the first p with (cum[p] - base) * S >= total * r, where cum is the inclusive
// prefix sum of the costs, base = cum[lo - 1] and total = cum[hi - 1] - base; cuts are made
// non-decreasing, cut_0 = lo and cut_S = hi.  cum fits int64 (<= 2^31 pairs x 2^30 + 1).
namespace ovl_cand {

struct PairCost {
    const int32_t* a;
    const int32_t* b;
    const int32_t* len;
    __host__ __device__ int64_t operator()(const int64_t& p) const {
        return (int64_t)len[a[p]] * (int64_t)len[b[p]] + 1;
    }
};

__global__ void cut_kernel(const int64_t* __restrict__ cum, int64_t lo, int64_t hi, int32_t shards,
                           int64_t* __restrict__ cuts) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int64_t base = lo > 0 ? cum[lo - 1] : 0;
    const int64_t total = hi > lo ? cum[hi - 1] - base : 0;
    int64_t prev = lo;
    cuts[0] = lo;
    for (int32_t r = 1; r < shards; ++r) {
        int64_t a = lo, b = hi;
        const int64_t want = total * r;
        while (a < b) {
            const int64_t mid = (a + b) >> 1;
            if ((cum[mid] - base) * shards >= want) b = mid;
            else a = mid + 1;
        }
        prev = a > prev ? a : prev;
        cuts[r] = prev;
    }
    cuts[shards] = hi;
}

}  // namespace ovl_cand

using ovl_cand::PairCost;
typedef hipcub::TransformInputIterator<int64_t, PairCost, hipcub::CountingInputIterator<int64_t>> CostIter;

extern "C" hipError_t ovl_shard_temp_bytes(int64_t n_pairs, size_t* bytes) {
    PairCost f{nullptr, nullptr, nullptr};
    CostIter it(hipcub::CountingInputIterator<int64_t>(0), f);
    return hipcub::DeviceScan::InclusiveSum(nullptr, *bytes, it, (int64_t*)nullptr, n_pairs);
}

extern "C" hipError_t ovl_shard_scan(void* temp, size_t temp_bytes, const int32_t* a, const int32_t* b,
                                     const int32_t* len, int64_t n_pairs, int64_t* cum, hipStream_t stream) {
    if (n_pairs <= 0) return hipSuccess;
    PairCost f{a, b, len};
    CostIter it(hipcub::CountingInputIterator<int64_t>(0), f);
    return hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, it, cum, n_pairs, stream);
}

extern "C" hipError_t ovl_shard_cut(const int64_t* cum, int64_t lo, int64_t hi, int32_t shards, int64_t* cuts,
                                    hipStream_t stream) {
    ovl_cand::cut_kernel<<<1, 64, 0, stream>>>(cum, lo, hi, shards, cuts);
    return hipGetLastError();
}
