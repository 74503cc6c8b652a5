// Floor measurements for the cfg2-sized scoring launch (diagnostic tool, not part of libovl):
// empty grids of various sizes, index load + store, index + packed-row gathers + store.
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o build/microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_empty(int* out) { if (threadIdx.x == 1234567) out[0] = 1; }

__global__ void k_idx(const int* a, const int* b, int n, int* os, int* oe) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) { int x = a[p], y = b[p]; os[p] = x + y; oe[p] = x - y; }
}

template <int ROW>
__global__ void k_gather(const int* a, const int* b, int n, const uint4* S, const uint4* T, int* os, int* oe) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) {
        int x = a[p], y = b[p];
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < ROW / 4; ++k) {
            uint4 s = S[(size_t)x * (ROW / 4) + k], t = T[(size_t)y * (ROW / 4) + k];
            acc += s.x ^ t.x ^ s.y ^ t.y ^ s.z ^ t.z ^ s.w ^ t.w;
        }
        os[p] = (int)acc; oe[p] = x;
    }
}

template <typename F>
static float time_it(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 10; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
}

int main() {
    const int n = 121930, nreads = 7000, ROW = 8;   // cfg2-like: ~122k pairs, W=4 x 2 planes
    std::vector<int> ha(n), hb(n);
    srand(1);
    for (int i = 0; i < n; ++i) { ha[i] = rand() % nreads; hb[i] = rand() % nreads; }
    int *a, *b, *os, *oe; uint4 *S, *T;
    CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&os, n * 4)); CK(hipMalloc(&oe, n * 4));
    CK(hipMalloc(&S, (size_t)nreads * ROW * 4)); CK(hipMalloc(&T, (size_t)nreads * ROW * 4));
    CK(hipMemset(S, 1, (size_t)nreads * ROW * 4)); CK(hipMemset(T, 2, (size_t)nreads * ROW * 4));
    CK(hipMemcpy(a, ha.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(b, hb.data(), n * 4, hipMemcpyHostToDevice));
    const int reps = 500;
    for (int blocks : {1, 64, 256, 953, 1906, 4096}) {
        float us = time_it([&] { k_empty<<<blocks, 256>>>(os); }, reps);
        printf("empty blocks=%d us_per_launch=%.2f\n", blocks, us);
    }
    for (int bs : {64, 256}) {
        int nb = (n + bs - 1) / bs;
        printf("idx bs=%d us=%.2f\n", bs, time_it([&] { k_idx<<<nb, bs>>>(a, b, n, os, oe); }, reps));
        printf("gather bs=%d us=%.2f\n", bs, time_it([&] { k_gather<ROW><<<nb, bs>>>(a, b, n, S, T, os, oe); }, reps));
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
