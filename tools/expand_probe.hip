// Probe (diagnostic tool, not part of libovl): why the host's expansion of packed results (ovl_expand.h through
// the host pool, ovl_pool.h) runs at ~27 us per M pairs alone (tools/pool_probe.cpp) but ~50 inside the step.
// Times the expansion of one 857 K-pair chunk with its packed source and int32 destinations in ordinary or pinned
// host memory (hipHostMalloc, coherent as libovl's staging, or non-coherent), the source freshly written by a
// kernel through the host mapping (as the step's staging slots are) or warm in the CPU caches, and with a kernel
// storing int32 results into other pinned memory at the same time (as the step's direct chunk does).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I genome-assembly-using-overlap-graphs_amd/csrc \
//     tools/expand_probe.hip -o genome-assembly-using-overlap-graphs_amd/build/expand_probe -lpthread
//   expand_probe [reps [numa node, -2: the GPU's own]]
#include <hip/hip_runtime.h>

#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ovl_expand.h"
#include "ovl_pool.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_packed(uint16_t* pk, int64_t n, uint32_t salt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        pk[i] = (uint16_t)((((i * 7 + salt) % 100) << 8) | (i % 5));
}

__global__ void store_int32(int32_t* a, int32_t* b, int64_t n, int32_t v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        __builtin_nontemporal_store(v, a + i);
        __builtin_nontemporal_store(v + 1, b + i);
    }
}

// the CPUs of NUMA node `node` (sysfs cpulist) as this process's affinity, before anything touches the GPU
static bool bind_node(int node) {
    char path[96], buf[4096];
    snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
    FILE* fh = fopen(path, "r");
    if (!fh) return false;
    const size_t got = fread(buf, 1, sizeof(buf) - 1, fh);
    fclose(fh);
    buf[got] = 0;
    cpu_set_t set, mine;
    CPU_ZERO(&set);
    for (char* q = buf; *q && *q != '\n';) {
        char* e;
        long lo = strtol(q, &e, 10), hi = lo;
        if (e == q) break;
        if (*e == '-') hi = strtol(e + 1, &e, 10);
        for (long c = lo; c <= hi && c < CPU_SETSIZE; ++c) CPU_SET((int)c, &set);
        q = *e == ',' ? e + 1 : e;
    }
    if (sched_getaffinity(0, sizeof(mine), &mine) == 0) CPU_AND(&set, &set, &mine);
    return CPU_COUNT(&set) > 0 && sched_setaffinity(0, sizeof(set), &set) == 0;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    int node = argc > 2 ? atoi(argv[2]) : -1;
    if (node == -2) {  // the visible GPU's node, from its PCI address
        char bus[64] = {0}, path[160];
        CK(hipDeviceGetPCIBusId(bus, sizeof(bus), 0));
        for (char* q = bus; *q; ++q) *q = (char)tolower(*q);
        snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
        FILE* fh = fopen(path, "r");
        if (!fh || fscanf(fh, "%d", &node) != 1) node = -1;
        if (fh) fclose(fh);
        printf("gpu %s node %d\n", bus, node);
    }
    if (node >= 0) printf("bind to node %d: %s\n", node, bind_node(node) ? "ok" : "failed");
    const size_t n = 857408, n_direct = 360000;
    const ovl_expand::Fn f = ovl_expand::pick(nullptr);
    CopyPool& pool = CopyPool::get();
    auto now = [] { return std::chrono::steady_clock::now(); };
    // sources
    uint16_t *src_heap = nullptr, *src_coh = nullptr, *src_nc = nullptr, *d_coh = nullptr, *d_nc = nullptr;
    if (posix_memalign((void**)&src_heap, 64, 2 * n)) return 1;
    CK(hipHostMalloc((void**)&src_coh, 2 * n, hipHostMallocPortable | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&src_nc, 2 * n, hipHostMallocPortable | hipHostMallocNonCoherent));
    CK(hipHostGetDevicePointer((void**)&d_coh, src_coh, 0));
    CK(hipHostGetDevicePointer((void**)&d_nc, src_nc, 0));
    std::vector<int32_t> esc(n, 0);
    // destinations
    int32_t *o_heap_s = nullptr, *o_heap_e = nullptr, *o_coh_s = nullptr, *o_coh_e = nullptr, *o_nc_s = nullptr,
            *o_nc_e = nullptr;
    if (posix_memalign((void**)&o_heap_s, 64, 4 * n) || posix_memalign((void**)&o_heap_e, 64, 4 * n)) return 1;
    CK(hipHostMalloc((void**)&o_coh_s, 4 * n, hipHostMallocPortable | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&o_coh_e, 4 * n, hipHostMallocPortable | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&o_nc_s, 4 * n, hipHostMallocPortable | hipHostMallocNonCoherent));
    CK(hipHostMalloc((void**)&o_nc_e, 4 * n, hipHostMallocPortable | hipHostMallocNonCoherent));
    memset(o_heap_s, 0, 4 * n);
    memset(o_heap_e, 0, 4 * n);
    // the concurrent direct chunk's destination
    int32_t *dir_a = nullptr, *dir_b = nullptr, *d_dir_a = nullptr, *d_dir_b = nullptr;
    CK(hipHostMalloc((void**)&dir_a, 4 * n_direct, hipHostMallocPortable | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&dir_b, 4 * n_direct, hipHostMallocPortable | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&d_dir_a, dir_a, 0));
    CK(hipHostGetDevicePointer((void**)&d_dir_b, dir_b, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreate(&s1));
    CK(hipStreamCreate(&s2));
    for (size_t i = 0; i < n; ++i) src_heap[i] = (uint16_t)((((i * 7) % 100) << 8) | (i % 5));

    struct Case {
        const char* name;
        uint16_t* src;
        uint16_t* dsrc;   // non-null: refilled by a kernel before every expansion
        int32_t* os;
        int32_t* oe;
        bool direct;      // a concurrent kernel stores int32 into other pinned memory
    };
    const Case cases[] = {
        {"heap src (warm) -> heap dst", src_heap, nullptr, o_heap_s, o_heap_e, false},
        {"heap src (warm) -> pinned coherent dst", src_heap, nullptr, o_coh_s, o_coh_e, false},
        {"heap src (warm) -> pinned non-coherent dst", src_heap, nullptr, o_nc_s, o_nc_e, false},
        {"pinned coherent src, kernel-written -> heap dst", src_coh, d_coh, o_heap_s, o_heap_e, false},
        {"pinned coherent src, kernel-written -> pinned coherent dst (the step)", src_coh, d_coh, o_coh_s, o_coh_e, false},
        {"  same, with a concurrent direct-chunk kernel", src_coh, d_coh, o_coh_s, o_coh_e, true},
        {"pinned non-coherent src, kernel-written -> pinned coherent dst", src_nc, d_nc, o_coh_s, o_coh_e, false},
        {"pinned coherent src (warm) -> pinned coherent dst", src_coh, nullptr, o_coh_s, o_coh_e, false},
    };
    // warm the warm pinned source once
    for (size_t i = 0; i < n; ++i) src_coh[i] = src_heap[i];
    for (const Case& c : cases) {
        double total = 0.0, best = 1e30;
        for (int r = 0; r < reps + 3; ++r) {
            if (c.dsrc) {
                fill_packed<<<1024, 256, 0, s1>>>(c.dsrc, (int64_t)n, (uint32_t)r);
                CK(hipStreamSynchronize(s1));
            }
            if (c.direct) store_int32<<<1024, 256, 0, s2>>>(d_dir_a, d_dir_b, (int64_t)n_direct, r);
            const auto t0 = now();
            pool.parallel(n, size_t(1) << 14, [&](size_t lo, size_t hi) {
                f(c.os, c.oe, c.src, esc.data(), 10, -1, true, lo, hi);
            });
            const double us = std::chrono::duration<double, std::micro>(now() - t0).count();
            if (c.direct) CK(hipStreamSynchronize(s2));
            if (r >= 3) {
                total += us;
                best = std::min(best, us);
            }
        }
        printf("%-72s mean %6.1f us  min %6.1f us  (%5.1f us per M pairs, mean)\n", c.name, total / reps, best,
               total / reps * 1e6 / (double)n);
    }
    return 0;
}
