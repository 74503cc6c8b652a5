// ovl_pairs.hip — a host pair list in compact form, decoded on the device (gfx950).
//
// A caller of the one-shot ABI (ovl_score_pairs / ovl_score_host) hands over int32 pair
// arrays in host memory: 8 bytes per pair over the link before any scoring.  The candidate list of
// overlapGraphs.py:43-52 is a-major (the outer loop walks read_copies), so `a` is runs of one value, and
// indices below 65,535 fit 16 bits.  The host encodes each pipeline chunk (ovl_api.cpp encode_chunk) as
//   b: uint16 (n_reads <= 65,535; 0xFFFF = an index outside [0, n_reads)) or int32,
//   a: runs (value int32, chunk-relative start int32, starts[R] = chunk length) when they are few, else
//      like b,
// into pinned memory, and these kernels read it through the host mapping (link reads, while the scoring
// kernels' result stores use the other direction) and write the int32 arrays into HBM for the scoring
// kernels.  HBM-bound byte work: coalesced 16-byte loads, one wavefront per run.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "ovl_kernels.h"

namespace ovl {

// dst[i] = src[i] (uint16: 0xFFFF -> -1), 8 elements per lane-iteration from one 16-byte load
template <typename T>
__global__ __launch_bounds__(256) void widen_kernel(const T* __restrict__ src, int64_t n, int32_t* __restrict__ dst) {
    constexpr int V = 16 / sizeof(T);  // elements per 16-byte load
    const int64_t groups = n / V;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + g);
        const T* e = reinterpret_cast<const T*>(&v);
        int32_t out[V];
#pragma unroll
        for (int k = 0; k < V; ++k) {
            if constexpr (sizeof(T) == 2) out[k] = e[k] == 0xFFFF ? -1 : (int32_t)e[k];
            else out[k] = (int32_t)e[k];
        }
        int4* d = reinterpret_cast<int4*>(dst + g * V);
#pragma unroll
        for (int k = 0; k < V / 4; ++k) d[k] = make_int4(out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]);
    }
    // tail (< V elements)
    const int64_t t = groups * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) {
        const T x = src[t];
        if constexpr (sizeof(T) == 2) dst[t] = x == 0xFFFF ? -1 : (int32_t)x;
        else dst[t] = (int32_t)x;
    }
}

// the same one element per lane (any alignment)
template <typename T>
__global__ __launch_bounds__(256) void widen1_kernel(const T* __restrict__ src, int64_t n, int32_t* __restrict__ dst) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
        const T x = src[t];
        if constexpr (sizeof(T) == 2) dst[t] = x == 0xFFFF ? -1 : (int32_t)x;
        else dst[t] = (int32_t)x;
    }
}

// run r of a chunk: dst[starts[r] .. starts[r + 1]) = vals[r]; one wavefront per run (grid-stride over runs)
__global__ __launch_bounds__(256) void runs_kernel(const int32_t* __restrict__ vals, const int32_t* __restrict__ starts,
                                                   int64_t n_runs, int32_t* __restrict__ dst) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n_runs; r += waves) {
        const int32_t v = vals[r];
        const int32_t s = starts[r], e = starts[r + 1];
        for (int32_t p = s + lane; p < e; p += 64) dst[p] = v;
    }
}

}  // namespace ovl

using namespace ovl;

extern "C" hipError_t ovl_launch_widen(const void* src, int32_t width, int64_t n, int32_t* dst, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15)) {
        const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
        if (width == 2)
            widen1_kernel<uint16_t><<<blocks, 256, 0, stream>>>(static_cast<const uint16_t*>(src), n, dst);
        else if (width == 4)
            widen1_kernel<int32_t><<<blocks, 256, 0, stream>>>(static_cast<const int32_t*>(src), n, dst);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
    const int64_t per = 16 / width;
    int64_t blocks = (n / per + 255) / 256 + 1;
    if (blocks > 2048) blocks = 2048;
    if (width == 2)
        widen_kernel<uint16_t><<<(unsigned)blocks, 256, 0, stream>>>(static_cast<const uint16_t*>(src), n, dst);
    else if (width == 4)
        widen_kernel<int32_t><<<(unsigned)blocks, 256, 0, stream>>>(static_cast<const int32_t*>(src), n, dst);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

extern "C" hipError_t ovl_launch_runs(const int32_t* vals, const int32_t* starts, int64_t n_runs, int32_t* dst,
                                      hipStream_t stream) {
    if (n_runs <= 0) return hipSuccess;
    int64_t blocks = (n_runs + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    runs_kernel<<<(unsigned)blocks, 256, 0, stream>>>(vals, starts, n_runs, dst);
    return hipGetLastError();
}
