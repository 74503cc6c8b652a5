// VGPR operand banks on gfx950 (diagnostic tool, not part of libovl): throughput of three-source VALU ops
// whose VGPR sources sit in one bank (register index mod 4) against sources in distinct banks, every SIMD
// full (8 waves/SIMD).  Each step issues 8 independent instructions (destinations v40..v47) with fixed
// source registers.  Prints SIMD cycles per wave64 instruction at the measured shader clock.
// Build: hipcc --offload-arch=gfx950 -O3 tools/vgpr_banks.hip -o build/vgpr_banks
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int ITERS = 2048;

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
#define INIT asm volatile("v_mov_b32 v48, %0\n\tv_mov_b32 v49, %1\n\tv_mov_b32 v50, %0\n\tv_mov_b32 v51, %1\n\t" \
                          "v_mov_b32 v52, %0\n\tv_mov_b32 v53, %1\n\tv_mov_b32 v54, %0\n\tv_mov_b32 v55, %1\n\t" \
                          "v_mov_b32 v56, %0\n\tv_mov_b32 v57, %1\n\tv_mov_b32 v58, %0\n\tv_mov_b32 v59, %1\n\t" \
                          "v_mov_b32 v60, %0\n\tv_mov_b32 v61, %1\n\tv_mov_b32 v62, %0\n\tv_mov_b32 v63, %1" \
                          :: "v"(threadIdx.x), "v"(seed) : CLOB)
#define OUT asm volatile("v_xor_b32 %0, v40, v47" : "=v"(r) :: CLOB)

#define KERNEL(NAME, BODY)                                                            \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {      \
        INIT;                                                                         \
        for (int i = 0; i < ITERS; ++i) asm volatile(BODY ::: CLOB);                 \
        unsigned r;                                                                   \
        OUT;                                                                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                               \
    }

// sources in one bank: v48, v52, v56, v60 (bank 0); distinct banks: v48, v49, v50 (banks 0 1 2)
#define B3(OP, A, B, C, SUF) OP " v40, " A ", " B ", " C SUF "\n\t" OP " v41, " A ", " B ", " C SUF "\n\t" \
                             OP " v42, " A ", " B ", " C SUF "\n\t" OP " v43, " A ", " B ", " C SUF "\n\t" \
                             OP " v44, " A ", " B ", " C SUF "\n\t" OP " v45, " A ", " B ", " C SUF "\n\t" \
                             OP " v46, " A ", " B ", " C SUF "\n\t" OP " v47, " A ", " B ", " C SUF
#define B2(OP, A, B) OP " v40, " A ", " B "\n\t" OP " v41, " A ", " B "\n\t" OP " v42, " A ", " B "\n\t" \
                     OP " v43, " A ", " B "\n\t" OP " v44, " A ", " B "\n\t" OP " v45, " A ", " B "\n\t" \
                     OP " v46, " A ", " B "\n\t" OP " v47, " A ", " B

KERNEL(k_bitop3_same, B3("v_bitop3_b32", "v48", "v52", "v56", " bitop3:0xbe"))
KERNEL(k_bitop3_two, B3("v_bitop3_b32", "v48", "v52", "v49", " bitop3:0xbe"))
KERNEL(k_bitop3_diff, B3("v_bitop3_b32", "v48", "v49", "v50", " bitop3:0xbe"))
KERNEL(k_max3_same, B3("v_max3_i32", "v48", "v52", "v56", ""))
KERNEL(k_max3_diff, B3("v_max3_i32", "v48", "v49", "v50", ""))
KERNEL(k_alignbit_same, B3("v_alignbit_b32", "v48", "v52", "v56", ""))
KERNEL(k_alignbit_diff, B3("v_alignbit_b32", "v48", "v49", "v50", ""))
KERNEL(k_bcnt_same, B2("v_bcnt_u32_b32", "v48", "v52"))
KERNEL(k_bcnt_diff, B2("v_bcnt_u32_b32", "v48", "v49"))
KERNEL(k_xor_same, B2("v_xor_b32", "v48", "v52"))
KERNEL(k_xor_diff, B2("v_xor_b32", "v48", "v49"))
// the sweep's pattern: dependent bitop3 -> bcnt chain per word with the accumulator in one bank or another
KERNEL(k_chain, "v_xor_b32 v40, v48, v52\n\tv_bitop3_b32 v40, v49, v53, v40 bitop3:0xbe\n\tv_bcnt_u32_b32 v44, v40, v44\n\t"
                "v_xor_b32 v41, v50, v54\n\tv_bitop3_b32 v41, v51, v55, v41 bitop3:0xbe\n\tv_bcnt_u32_b32 v45, v41, v45\n\t"
                "v_xor_b32 v42, v56, v60\n\tv_bitop3_b32 v42, v57, v61, v42 bitop3:0xbe\n\tv_bcnt_u32_b32 v46, v42, v46\n\t"
                "v_xor_b32 v43, v58, v62\n\tv_bitop3_b32 v43, v59, v63, v43 bitop3:0xbe\n\tv_bcnt_u32_b32 v47, v43, v47")

__global__ void k_clock(unsigned long long* t) {
    unsigned long long a = __builtin_readcyclecounter();
    for (int i = 0; i < 1000000; ++i) asm volatile("s_nop 0");
    unsigned long long b = __builtin_readcyclecounter();
    if (threadIdx.x == 0) t[0] = b - a;
}

template <typename K>
float run(K k, unsigned* out) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k<<<2048, 256>>>(out, 1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) k<<<2048, 256>>>(out, r);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    unsigned* out;
    CK(hipMalloc(&out, 2048 * 256 * 4));
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    const double hz = clk_khz * 1e3;
    // 2048 blocks x 4 waves over 1024 SIMDs = 8 waves per SIMD; 8 instructions per step per wave
    auto cyc = [&](float ms, int per_step) {
        return ms * 1e-3 * hz / (8.0 * ITERS * per_step);
    };
#define R(K, N) printf("%-18s %6.2f SIMD cycles per wave64 instruction\n", #K, cyc(run(K, out), N))
    R(k_bitop3_same, 8); R(k_bitop3_two, 8); R(k_bitop3_diff, 8);
    R(k_max3_same, 8); R(k_max3_diff, 8);
    R(k_alignbit_same, 8); R(k_alignbit_diff, 8);
    R(k_bcnt_same, 8); R(k_bcnt_diff, 8);
    R(k_xor_same, 8); R(k_xor_diff, 8);
    R(k_chain, 12);
    printf("clock %.0f MHz (attribute)\n", hz / 1e6);
    return 0;
}
