// Per-opcode VALU throughput on gfx950 (diagnostic tool, not part of libovl):
// every SIMD full (8 waves/SIMD, 2048 blocks x 256), each lane runs 8 independent
// chains of one opcode; prints SIMD cycles per wave64 instruction at 2.4 GHz.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o build/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int ITERS = 2048;

#define BODY8(INSN)                                   \
    asm volatile(INSN : "+v"(x0) : "v"(y), "v"(z));   \
    asm volatile(INSN : "+v"(x1) : "v"(y), "v"(z));   \
    asm volatile(INSN : "+v"(x2) : "v"(y), "v"(z));   \
    asm volatile(INSN : "+v"(x3) : "v"(y), "v"(z));   \
    asm volatile(INSN : "+v"(x4) : "v"(y), "v"(z));   \
    asm volatile(INSN : "+v"(x5) : "v"(y), "v"(z));   \
    asm volatile(INSN : "+v"(x6) : "v"(y), "v"(z));   \
    asm volatile(INSN : "+v"(x7) : "v"(y), "v"(z));

#define KERNEL(NAME, INSN)                                                              \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {        \
        unsigned x0 = threadIdx.x ^ seed, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;        \
        unsigned x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                    \
        unsigned y = seed * 3 + threadIdx.x, z = seed + 7;                              \
        for (int i = 0; i < ITERS; ++i) { BODY8(INSN) }                                 \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7; \
    }

KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_and, "v_and_b32 %0, %0, %1")
KERNEL(k_max, "v_max_i32 %0, %0, %1")
KERNEL(k_lshl, "v_lshlrev_b32 %0, %1, %0")
KERNEL(k_bcnt, "v_bcnt_u32_b32 %0, %1, %0")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, %2")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xbe")
KERNEL(k_mad24, "v_mad_i32_i24 %0, %0, %1, %2")
KERNEL(k_mul24, "v_mul_i32_i24 %0, %0, %1")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_mullo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_lshlor, "v_lshl_or_b32 %0, %0, 3, %1")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, %1, %2")
KERNEL(k_max3, "v_max3_i32 %0, %0, %1, %2")
KERNEL(k_sad, "v_sad_u32 %0, %0, %1, %2")
// v_cndmask with a mask written once (loop-invariant SGPR pair) and with a fresh v_cmp per use
#define KERNEL_MASK(NAME, INSN)                                                          \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {         \
        unsigned x0 = threadIdx.x ^ seed, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;         \
        unsigned x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                     \
        unsigned y = seed * 3 + threadIdx.x, z = seed + 7;                               \
        unsigned long long m;                                                            \
        asm volatile("v_cmp_gt_u32 %0, %1, %2" : "=s"(m) : "v"(y), "v"(z));               \
        for (int i = 0; i < ITERS; ++i) {                                                \
            asm volatile(INSN : "+v"(x0) : "v"(y), "s"(m)); asm volatile(INSN : "+v"(x1) : "v"(y), "s"(m)); \
            asm volatile(INSN : "+v"(x2) : "v"(y), "s"(m)); asm volatile(INSN : "+v"(x3) : "v"(y), "s"(m)); \
            asm volatile(INSN : "+v"(x4) : "v"(y), "s"(m)); asm volatile(INSN : "+v"(x5) : "v"(y), "s"(m)); \
            asm volatile(INSN : "+v"(x6) : "v"(y), "s"(m)); asm volatile(INSN : "+v"(x7) : "v"(y), "s"(m)); \
        }                                                                                \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7; \
    }
KERNEL_MASK(k_cnd_sgpr, "v_cndmask_b32_e64 %0, %0, %1, %2")
KERNEL(k_cmp_cnd, "v_cmp_gt_i32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc")
KERNEL(k_min, "v_min_i32 %0, %0, %1")
KERNEL(k_sub, "v_sub_u32 %0, %0, %1")
KERNEL(k_or, "v_or_b32 %0, %0, %1")
KERNEL(k_mov, "v_mov_b32 %0, %1")
KERNEL(k_lshrrev, "v_lshrrev_b32 %0, %1, %0")
// mixed streams: two instructions per chain step (cost reported per instruction)
KERNEL(k_mix_xor_bcnt, "v_xor_b32 %0, %0, %1\n\tv_bcnt_u32_b32 %0, %1, %0")
KERNEL(k_mix_xor_bitop3, "v_xor_b32 %0, %0, %1\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xbe")
KERNEL(k_mix_bcnt_alignbit, "v_bcnt_u32_b32 %0, %1, %0\n\tv_alignbit_b32 %0, %0, %1, %2")
KERNEL(k_mix_add_max, "v_add_u32 %0, %0, %1\n\tv_max_i32 %0, %0, %1")
// lane-DP cell candidates: SDWA byte add (+ max3), packed 16-bit add / max / mad, 16-bit max3
#define SDWA_ADD "v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
KERNEL(k_sdwa_add, SDWA_ADD)
KERNEL(k_pk_add, "v_pk_add_i16 %0, %0, %1")
KERNEL(k_pk_max, "v_pk_max_i16 %0, %0, %1")
KERNEL(k_pk_mad, "v_pk_mad_i16 %0, %0, %1, %2")
KERNEL(k_max3_i16, "v_max3_i16 %0, %0, %1, %2")
KERNEL(k_mix_sdwa_max3, SDWA_ADD "\n\tv_max3_i32 %0, %0, %1, %2")
KERNEL(k_mix_pk_add_max, "v_pk_add_i16 %0, %0, %1\n\tv_pk_max_i16 %0, %0, %2")

// shader clock: s_memtime ticks over a fixed VALU loop, one wave per SIMD
__global__ __launch_bounds__(64) void k_clock(unsigned long long* out, unsigned seed) {
    unsigned x0 = threadIdx.x ^ seed, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    unsigned y = seed, z = seed + 1;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
    for (int i = 0; i < ITERS; ++i) { BODY8("v_xor_b32 %0, %0, %1") }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7));
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (threadIdx.x == 1 && (x0 ^ x7) == 0x12345) out[blockIdx.x] = 0;
}

typedef void (*KFn)(unsigned*, unsigned);

int main() {
    unsigned* out;
    const int blocks = 2048, threads = 256;
    CK(hipMalloc(&out, (size_t)blocks * threads * 4));
    struct { const char* name; KFn fn; } ks[] = {
        {"v_xor_b32", k_xor}, {"v_add_u32", k_add}, {"v_and_b32", k_and}, {"v_max_i32", k_max},
        {"v_lshlrev_b32", k_lshl}, {"v_bcnt_u32_b32", k_bcnt}, {"v_alignbit_b32", k_alignbit},
        {"v_bitop3_b32", k_bitop3}, {"v_mad_i32_i24", k_mad24}, {"v_mul_i32_i24", k_mul24},
        {"v_add3_u32", k_add3}, {"v_xad_u32", k_xad}, {"v_cndmask_b32", k_cndmask}, {"v_mul_lo_u32", k_mullo},
        {"v_perm_b32", k_perm}, {"v_lshl_or_b32", k_lshlor}, {"v_bfe_u32", k_bfe}, {"v_max3_i32", k_max3},
        {"v_sad_u32", k_sad},
        {"v_cndmask(sgpr)", k_cnd_sgpr}, {"mix cmp+cndmask", k_cmp_cnd}, {"v_min_i32", k_min}, {"v_sub_u32", k_sub},
        {"v_or_b32", k_or}, {"v_mov_b32", k_mov}, {"v_lshrrev_b32", k_lshrrev},
        {"mix xor+bcnt", k_mix_xor_bcnt}, {"mix xor+bitop3", k_mix_xor_bitop3},
        {"mix bcnt+alignbit", k_mix_bcnt_alignbit}, {"mix add+max", k_mix_add_max},
        {"v_add_u32_sdwa", k_sdwa_add}, {"v_pk_add_i16", k_pk_add}, {"v_pk_max_i16", k_pk_max},
        {"v_pk_mad_i16", k_pk_mad}, {"v_max3_i16", k_max3_i16}, {"mix sdwa+max3", k_mix_sdwa_max3},
        {"mix pk_add+pk_max", k_mix_pk_add_max},
    };
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const double simds = prop.multiProcessorCount * 4.0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& k : ks) {
        k.fn<<<blocks, threads>>>(out, 1);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < 5; ++r) k.fn<<<blocks, threads>>>(out, r);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double per = strncmp(k.name, "mix", 3) == 0 ? 2.0 : 1.0;
        const double wave_insts = 5.0 * blocks * (threads / 64) * (double)ITERS * 8 * per;
        const double cyc = ms * 1e-3 * 2.4e9 * simds / wave_insts;
        printf("%-16s %.2f SIMD cycles per wave64 instruction (%.3f ms)\n", k.name, cyc, ms / 5);
    }
    // clock: one wave on 1024 SIMDs-worth of blocks (one 64-thread block each), time vs ticks
    unsigned long long* ticks;
    CK(hipMalloc(&ticks, 4096 * sizeof(unsigned long long)));
    k_clock<<<1024, 64>>>(ticks, 1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    k_clock<<<1024, 64>>>(ticks, 2);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long h[1024];
    CK(hipMemcpy(h, ticks, sizeof(h), hipMemcpyDeviceToHost));
    double mx = 0, sum = 0;
    for (int i = 0; i < 1024; ++i) { sum += (double)h[i]; if (h[i] > mx) mx = (double)h[i]; }
    printf("clock probe: one wave per SIMD, %d xor per lane-chain x8: mean %.0f ticks, max %.0f ticks, kernel %.3f ms"
           " -> %.2f ticks per wave-instruction (one wave alone); ticks/ns = %.3f (max ticks / kernel time)\n",
           ITERS, sum / 1024, mx, ms, (sum / 1024) / (ITERS * 8.0), mx / (ms * 1e6));
    return 0;
}
