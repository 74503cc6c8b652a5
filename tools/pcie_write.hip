// Store patterns from a kernel into pinned host memory (the step's result path): the rate of (score, end)
// for 2M pairs written as two int32 arrays, one interleaved int2 array, 16-byte stores, with and without
// non-temporal hints, next to hipMemcpyAsync D2H of the same bytes.  Build (here) and run on the box:
//   hipcc --offload-arch=gfx950 -O3 -o genome-assembly-using-overlap-graphs_amd/build/pcie_write tools/pcie_write.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__global__ void two_arrays(int32_t* a, int32_t* b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        a[i] = (int32_t)i;
        b[i] = (int32_t)(i >> 3);
    }
}

__global__ void two_arrays_nt(int32_t* a, int32_t* b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        __builtin_nontemporal_store((int32_t)i, a + i);
        __builtin_nontemporal_store((int32_t)(i >> 3), b + i);
    }
}

__global__ void interleaved(int2* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = make_int2((int32_t)i, (int32_t)(i >> 3));
}

__global__ void wide16(int4* p, int64_t n2) {  // two pairs per lane
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = make_int4((int32_t)i, (int32_t)(i >> 3), (int32_t)i + 1, (int32_t)(i >> 2));
}

__global__ void wide16_two(int4* a, int4* b, int64_t n4) {  // four pairs per lane, two arrays
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        a[i] = make_int4((int32_t)i, 1, 2, 3);
        b[i] = make_int4((int32_t)(i >> 3), 1, 2, 3);
    }
}

__global__ void packed16(uint16_t* p, int64_t n) {  // one uint16 per lane (the packed result sink)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((uint16_t)(i * 7), p + i);
}

__global__ void packed16x2(uint32_t* p, int64_t n2) {  // two uint16 per lane as one 4-byte store
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((uint32_t)(i * 7), p + i);
}

int main() {
    const int64_t n = 2000000;
    const size_t bytes = (size_t)n * 8;
    void* h = nullptr;
    void* d = nullptr;
    CHK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    CHK(hipMalloc(&d, bytes));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    int dev = 0, cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int reps = 50;
    size_t nbytes = bytes;  // bytes a timed operation moves (the GB/s column)
    auto time_it = [&](const char* name, auto fn) -> int {
        for (int w = 0; w < 3; ++w) fn();
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) fn();
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-34s %8.4f ms  %6.2f GB/s\n", name, ms, nbytes / (ms * 1e-3) / 1e9);
        return 0;
    };
    int32_t* ha = (int32_t*)h;
    int32_t* hb = ha + n;
    for (int blocks : {cus * 4, cus * 16, cus * 64}) {
        printf("-- grid %d x 256\n", blocks);
        time_it("two int32 arrays", [&] { two_arrays<<<blocks, 256>>>(ha, hb, n); });
        time_it("two int32 arrays, nontemporal", [&] { two_arrays_nt<<<blocks, 256>>>(ha, hb, n); });
        time_it("interleaved int2", [&] { interleaved<<<blocks, 256>>>((int2*)h, n); });
        time_it("int4, two pairs per lane", [&] { wide16<<<blocks, 256>>>((int4*)h, n / 2); });
        time_it("int4 x two arrays, 4 pairs/lane", [&] { wide16_two<<<blocks, 256>>>((int4*)ha, (int4*)hb, n / 4); });
    }
    // the packed sink: 2 bytes per pair, into default and into fine-grained (coherent) pinned memory
    void* hc = nullptr;
    CHK(hipHostMalloc(&hc, bytes, hipHostMallocCoherent));
    nbytes = (size_t)n * 2;
    for (int blocks : {cus * 16, cus * 64}) {
        printf("-- packed, grid %d x 256\n", blocks);
        time_it("uint16 per lane", [&] { packed16<<<blocks, 256>>>((uint16_t*)h, n); });
        time_it("uint16 per lane, coherent", [&] { packed16<<<blocks, 256>>>((uint16_t*)hc, n); });
        time_it("2 x uint16 per lane, coherent", [&] { packed16x2<<<blocks, 256>>>((uint32_t*)hc, n / 2); });
    }
    nbytes = bytes;
    CHK(hipHostFree(hc));
    time_it("hipMemcpyAsync D2H", [&] { (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0); });
    time_it("hipMemcpyAsync D2H (2 halves)", [&] {
        (void)hipMemcpyAsync(h, d, bytes / 2, hipMemcpyDeviceToHost, 0);
        (void)hipMemcpyAsync((char*)h + bytes / 2, (char*)d + bytes / 2, bytes / 2, hipMemcpyDeviceToHost, 0);
    });
    two_arrays<<<cus * 16, 256>>>((int32_t*)d, (int32_t*)d + n, n);
    time_it("device HBM, two int32 arrays", [&] { two_arrays<<<cus * 16, 256>>>((int32_t*)d, (int32_t*)d + n, n); });
    CHK(hipHostFree(h));
    CHK(hipFree(d));
    return 0;
}
