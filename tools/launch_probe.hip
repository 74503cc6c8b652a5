// Fixed costs of one scoring call's launch on the box (diagnostic tool, not part of libovl), host clock (us):
//   launch API time (returns), launch -> first wave running (a flag the kernel stores into pinned host memory),
//   kernel end flag -> hipEventQuery success, hipStreamSynchronize on an idle stream, and the round trip of
//   an empty launch (launch .. event seen done), for a 1-block grid and for 1000 blocks (a shard-sized grid).
// Build: hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip -o build/launch_probe
#include <hip/hip_runtime.h>
#include <x86intrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__);             \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

// block 0's first lane stores `seq` into flag[0] at the start, the last block to finish stores it into flag[1]
__global__ void k_flags(volatile uint32_t* flag, uint32_t seq, uint32_t* done, int spin) {
    if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(&flag[0], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // a little work so every block is resident for a while
    uint32_t v = threadIdx.x;
    for (int i = 0; i < spin; ++i) v = v * 1664525u + 1013904223u;
    if (v == 0x12345678u) done[1] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t c = __hip_atomic_fetch_add(&done[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (c + 1 == gridDim.x) {
            done[0] = 0;
            __hip_atomic_store(&flag[1], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// 24 pointer / scalar arguments, like uniform_kernel's
__global__ void k_args(const void* a0, const void* a1, const void* a2, int a3, const void* a4, const void* a5,
                       long a6, int a7, const void* a8, int a9, int a10, void* a11, void* a12, void* a13,
                       const void* a14, const void* a15, int a16, long a17, const void* a18, const void* a19,
                       const void* a20, unsigned a21, long a22, void* a23) {
    if (threadIdx.x == 12345) *(int*)a11 = a3 + a7 + a9 + a10 + a16 + (int)a6 + (int)a17 + (int)a21 + (int)a22;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* what, std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    printf("%-58s median %7.2f  p10 %7.2f  p90 %7.2f us\n", what, v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10]);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t* flag;
    CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent | hipHostMallocPortable));
    uint32_t* flag_dev;
    CK(hipHostGetDevicePointer((void**)&flag_dev, flag, 0));
    uint32_t* done;
    CK(hipMalloc(&done, 64));
    CK(hipMemset(done, 0, 64));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int reps = 400;
    for (int blocks : {1, 1000}) {
        for (int spin : {0, 2000}) {
            std::vector<double> api, start, endflag, evq, sync, rt;
            uint32_t seq = 1;
            for (int r = 0; r < reps + 20; ++r, ++seq) {
                flag[0] = flag[1] = 0;
                _mm_sfence();
                const double t0 = now_us();
                hipLaunchKernelGGL(k_flags, dim3(blocks), dim3(256), 0, s, (volatile uint32_t*)flag_dev, seq, done, spin);
                CK(hipEventRecord(ev, s));
                const double t1 = now_us();
                while (((volatile uint32_t*)flag)[0] != seq) _mm_pause();
                const double t2 = now_us();
                while (((volatile uint32_t*)flag)[1] != seq) _mm_pause();
                const double t3 = now_us();
                while (hipEventQuery(ev) == hipErrorNotReady) _mm_pause();
                const double t4 = now_us();
                CK(hipStreamSynchronize(s));
                const double t5 = now_us();
                if (r >= 20) {
                    api.push_back(t1 - t0);
                    start.push_back(t2 - t0);
                    endflag.push_back(t3 - t2);
                    evq.push_back(t4 - t3);
                    sync.push_back(t5 - t4);
                    rt.push_back(t4 - t0);
                }
            }
            printf("-- grid %d x 256, spin %d\n", blocks, spin);
            report("launch + event record API", api);
            report("launch -> first wave's flag seen", start);
            report("first wave -> last block's end flag seen", endflag);
            report("end flag -> hipEventQuery done", evq);
            report("hipStreamSynchronize, stream idle", sync);
            report("round trip: launch .. event done", rt);
        }
    }
    {
        std::vector<double> api;
        int* dummy;
        CK(hipMalloc(&dummy, 64));
        for (int r = 0; r < reps; ++r) {
            const double t0 = now_us();
            hipLaunchKernelGGL(k_args, dim3(1000), dim3(256), 0, s, dummy, dummy, dummy, 1, dummy, dummy, 2L, 3, dummy,
                               4, 5, dummy, dummy, dummy, dummy, dummy, 6, 7L, dummy, dummy, dummy, 8u, 9L, dummy);
            api.push_back(now_us() - t0);
            if (r % 16 == 15) CK(hipStreamSynchronize(s));
        }
        CK(hipStreamSynchronize(s));
        report("launch API, 24 arguments (queue not empty)", api);
    }
    return 0;
}
