// Round trip of one request to a resident (persistent) grid fed through pinned host memory, against the launch +
// event round trip of tools/launch_probe.hip (diagnostic tool, not part of libovl; DESIGN §9.1's lever, priced).
// The host stores request k into a pinned word; thread 0 of every block polls it (system-scope acquire load,
// s_sleep between polls), the block does `spin` rounds of work, and the last block to arrive (agent-scope
// counters: `fan` first-level counters on separate lines, then one top counter) stores k into a pinned done
// word, which the host polls.  Every wait is bounded: a block leaves at its deadline (wall clock), the host gives
// up on a request after 1 s and then releases every block by storing a request past the last one.
// Build: hipcc --offload-arch=gfx950 -O3 tools/persist_probe.hip -o build/persist_probe
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

constexpr int kLine = 32;  // uint32 words per counter (128 B apart)

// lead = 0: thread 0 of every block polls the host word; lead = 1: only block 0 polls it and passes the request on
// through a device word (cnt[kLine * (kMaxFan + 1)]) that the other blocks poll in L2.  Polls are relaxed loads (an
// acquire load at system scope invalidates the caches on every poll); one acquire fence follows the request seen.
// relaxed = 1: the fan-in counters are relaxed atomics (no per-block L2 write-back / invalidate at agent scope; the
// last block still stores the done word with a system-scope release) -- the floor for a kernel whose results go
// straight to host memory.
constexpr int kMaxFan = 64;
__global__ __launch_bounds__(256) void k_persist(const uint32_t* req, uint32_t* done, uint32_t* cnt, int iters,
                                                 int spin, int fan, int lead, int relaxed, uint64_t deadline_ticks,
                                                 uint32_t* timed_out) {
    __shared__ int s_go;
    const uint64_t t_end = wall_clock64() + deadline_ticks;
    const int g = (int)gridDim.x;
    const int f = (int)blockIdx.x % fan;
    const uint32_t in_group = (uint32_t)((g - f + fan - 1) / fan);
    const uint32_t groups = (uint32_t)(fan < g ? fan : g);
    uint32_t v = threadIdx.x;
    for (int k = 1; k <= iters; ++k) {
        if (threadIdx.x == 0) {
            int go = 1;
            uint32_t* fwd = cnt + kLine * (kMaxFan + 1);
            const bool from_host = !lead || blockIdx.x == 0;
            while ((from_host ? __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                              : __hip_atomic_load(fwd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < (uint32_t)k) {
                if (wall_clock64() > t_end) {
                    go = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            if (go && lead && blockIdx.x == 0) __hip_atomic_store(fwd, (uint32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_go = go;
        }
        __syncthreads();
        if (!s_go) {  // the same value in every thread of the block: the block leaves as a whole
            if (threadIdx.x == 0) __hip_atomic_store(timed_out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        for (int i = 0; i < spin; ++i) v = v * 1664525u + 1013904223u;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t c = relaxed ? __hip_atomic_fetch_add(&cnt[(1 + f) * kLine], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : __hip_atomic_fetch_add(&cnt[(1 + f) * kLine], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (c + 1 == (uint32_t)k * in_group) {
                const uint32_t t = relaxed ? __hip_atomic_fetch_add(&cnt[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : __hip_atomic_fetch_add(&cnt[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                if (t + 1 == (uint32_t)k * groups) __hip_atomic_store(done, (uint32_t)k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    if (v == 0x12345678u) cnt[1] = v;  // keeps the work
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
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
    uint32_t *hreq, *hdone, *hto;
    CK(hipHostMalloc((void**)&hreq, 256, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&hdone, 256, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&hto, 256, hipHostMallocCoherent | hipHostMallocMapped));
    uint32_t *dreq, *ddone, *dto;
    CK(hipHostGetDevicePointer((void**)&dreq, hreq, 0));
    CK(hipHostGetDevicePointer((void**)&ddone, hdone, 0));
    CK(hipHostGetDevicePointer((void**)&dto, hto, 0));
    uint32_t* cnt;
    const size_t cnt_bytes = sizeof(uint32_t) * kLine * (kMaxFan + 2);
    CK(hipMalloc((void**)&cnt, cnt_bytes));
    printf("wall clock %d kHz\n", clk_khz);
    const uint64_t deadline = (uint64_t)clk_khz * 3000;  // 3 s
    struct Cfg { int grid, spin, fan, lead, relaxed; };
    const Cfg cfgs[] = {{1, 0, 1, 0, 0},       {1000, 0, 32, 0, 0}, {1000, 0, 32, 1, 0}, {1000, 0, 32, 0, 1},
                        {1000, 0, 32, 1, 1},   {1000, 0, 1, 1, 1},  {1000, 2000, 32, 1, 1}, {256, 0, 16, 1, 1},
                        {256, 0, 16, 1, 0},    {1024, 0, 32, 1, 1}};
    const int warm = 50, reps = 1000, iters = warm + reps;
    int rc = 0;
    for (const Cfg& c : cfgs) {
        *(volatile uint32_t*)hreq = 0;
        *(volatile uint32_t*)hdone = 0;
        *(volatile uint32_t*)hto = 0;
        CK(hipMemsetAsync(cnt, 0, cnt_bytes, s));
        CK(hipStreamSynchronize(s));
        k_persist<<<c.grid, 256, 0, s>>>(dreq, ddone, cnt, iters, c.spin, c.fan, c.lead, c.relaxed, deadline, dto);
        CK(hipGetLastError());
        // wait until every block is running: a first request answered (not timed)
        std::vector<double> rt;
        bool ok = true;
        for (int k = 1; k <= iters && ok; ++k) {
            const double t0 = now_us();
            __atomic_store_n(hreq, (uint32_t)k, __ATOMIC_RELEASE);
            while (__atomic_load_n(hdone, __ATOMIC_ACQUIRE) != (uint32_t)k) {
                if (now_us() - t0 > 1e6) {
                    ok = false;
                    break;
                }
                _mm_pause();
            }
            if (ok && k > warm) rt.push_back(now_us() - t0);
        }
        if (!ok) __atomic_store_n(hreq, (uint32_t)(iters + 1), __ATOMIC_RELEASE);  // release every block
        CK(hipStreamSynchronize(s));
        printf("-- persistent grid %d x 256, spin %d, fan %d, %s, %s fan-in\n", c.grid, c.spin, c.fan,
               c.lead ? "block 0 polls the host" : "every block polls the host", c.relaxed ? "relaxed" : "acq_rel");
        if (!ok || *(volatile uint32_t*)hto) {
            printf("request not answered within 1 s (blocks not all resident?) timed_out=%u\n", *(volatile uint32_t*)hto);
            rc = 1;
            continue;
        }
        report("request -> done word seen (host clock)", rt);
    }
    CK(hipFree(cnt));
    CK(hipHostFree(hreq));
    CK(hipHostFree(hdone));
    CK(hipHostFree(hto));
    return rc;
}
