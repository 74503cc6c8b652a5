// local_alignment (aligners.py:85-167) for one large pair on the whole GPU.
//
// Smith-Waterman with the reference's tie order (aligners.py:116-126): a cell takes diag if
// diag >= up, diag >= left and diag >= 0 (code 1), else up if up >= left and up >= 0 (2), else
// left if left >= 0 (3), else 0 (code 0); int64-exact arithmetic.  The value is max(diag, up,
// left, 0) whatever the branch.  Best cell: the first strict maximum in the i-major / j-minor
// fill order, from 0 (aligners.py:128-130).
//
// Layout: the query's rows are cut into 64-row strips; one wavefront (one 64-thread block) owns a
// strip at a time and sweeps its anti-diagonals (lane L on row 64s+1+L, column j = tau - L + 1),
// 64 steps per chunk with the step loop unrolled and branch-free.  Strip s needs the last row of
// strip s-1, which another wavefront -- usually on another CU -- produces concurrently.  It is
// handed over through L2 as 8-byte words {value, launch epoch} written and read with 8-byte
// agent-scope atomics (MI355X_MICROARCH.md: "8-B agent atomics both sides" is a valid hand-off
// form, and 8-B words are not torn): the producer never waits, the consumer re-reads a chunk
// until all 64 words carry this launch's epoch.  Strips go round-robin to gridDim.x co-resident
// blocks, so every strip's producer is a resident wavefront that started earlier; every poll is
// bounded (err_flag bit 1) so the grid always drains.
//
// Traceback (optional): one byte per cell, code | 4 when the cell is > 0 (the walk's dp > 0 test,
// aligners.py:136), stored [strip][tau][lane] (64 contiguous bytes per step, tau padded to whole
// chunks).  A chunk's codes are collected in LDS and written out with 64-byte stores per lane
// after the next chunk's inputs have arrived, so no wait covers a store issued moments before.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ovl_kernels.h"

namespace ovl_local {

__device__ __forceinline__ int32_t shr1(int32_t v) {
    // lane L receives lane L-1's value (lane 0 gets 0): DPP wave_shr:1
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, false);
}

// vec[L] = s: v_writelane_b32 with an inline-constant lane (one SGPR read: the constant-bus limit)
template <int L>
__device__ __forceinline__ int32_t writelane(int32_t vec, int32_t s) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(vec) : "s"(s), "n"(L));
    return vec;
}

// f(integral_constant<int, U>) for U = B .. E-1: a compile-time step index inside the unrolled loop
template <int B, int E, typename F>
__device__ __forceinline__ void unroll(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        unroll<B + 1, E>(f);
    }
}

__device__ __forceinline__ uint64_t ld8(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st8(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool TB>
__device__ __forceinline__ void flush_codes(const uint8_t* tbs, int8_t* dst_chunk, int lane) {
    const uint4* src = reinterpret_cast<const uint4*>(tbs);
    uint4* dst = reinterpret_cast<uint4*>(dst_chunk);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k * 64 + lane] = src[k * 64 + lane];
}

template <typename Acc, bool TB>
__global__ __launch_bounds__(64) void sw_kernel(const uint8_t* __restrict__ q, int32_t n, const uint8_t* __restrict__ r,
                                                int32_t m, int64_t match_, int64_t mismatch_, int64_t indel_,
                                                uint64_t* __restrict__ rowbuf, int8_t* __restrict__ tb,
                                                unsigned long long* __restrict__ best, uint32_t* __restrict__ err_flag,
                                                int32_t n_strips, uint32_t epoch) {
    __shared__ __attribute__((aligned(16))) uint8_t tbs[64 * 64];  // one chunk of codes: [step][lane]
    const Acc match = (Acc)match_, mismatch = (Acc)mismatch_, indel = (Acc)indel_;
    const int lane = threadIdx.x;
    const int32_t n_chunks = (m + 62 + 64) / 64;        // steps tau = 0 .. m + 62
    const int64_t steps = (int64_t)n_chunks * 64;        // traceback row pitch
    const int64_t W = (int64_t)n_chunks * 64 + 64;       // rowbuf pitch (hand-off chunk k: columns 64k+1 .. 64k+64)
    for (int32_t s = blockIdx.x; s < n_strips; s += gridDim.x) {
        const int32_t i = 64 * s + 1 + lane;
        const bool row_ok = i <= n;
        const uint32_t sc = row_ok ? (uint32_t)q[i - 1] : 0xFFFFFFFFu;
        const bool produce = s + 1 < n_strips;  // strip s+1 reads our last row (row 64s+64 <= n)
        const uint64_t* rin = rowbuf + (int64_t)(s - 1) * W;
        uint64_t* rout = rowbuf + (int64_t)s * W;
        int32_t cur = 0;    // dp[i][j-1]
        int32_t uprev = 0;  // dp[i-1][j-1]
        int32_t tch = 0;
        int32_t bval = 0, bj = 0;       // this row's first strict maximum (from 0)
        int32_t out_a = 0, out_b = 0;   // hand-off staging: chunk c-1 (lanes 1..63) / chunk c (lane 0)
        int8_t* tbrow = TB ? tb + (int64_t)s * steps * 64 : nullptr;
        int32_t pend = -1;              // chunk whose codes sit in LDS, still to be written out
        for (int32_t c = 0; c < n_chunks; ++c) {
            // inputs of chunk c: lane u holds dp[64s][64c+1+u] (lane 0's "up" at step u) and t[64c+u]
            const int64_t tcol = (int64_t)64 * c + lane;
            const int32_t v_t = tcol < m ? (int32_t)r[tcol] : 0;
            int32_t v_rin = 0;
            if (s > 0) {
                const int64_t col = (int64_t)64 * c + 1 + lane;
                uint64_t w = 0;
                int32_t spins = 0;
                while (true) {
                    w = col <= m ? ld8(rin + (int64_t)64 * c + lane) : ((uint64_t)epoch << 32);
                    if (__all((uint32_t)(w >> 32) == epoch)) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1 << 20)) {  // never expected: keep the grid finite
                        if (lane == 0) atomicOr(err_flag, 2u);
                        break;
                    }
                }
                v_rin = (int32_t)(uint32_t)w;
            }
            unroll<0, 64>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                const int32_t tau = 64 * c + u;
                const int32_t j = tau - lane + 1;
                const int32_t lds_up = __builtin_amdgcn_readlane(v_rin, u);
                const int32_t lds_t = __builtin_amdgcn_readlane(v_t, u);
                if (TB && u == 0 && pend >= 0) {  // (u is a compile-time step index)
                    // the previous chunk's codes leave LDS once this chunk's inputs are in registers
                    flush_codes<TB>(tbs, tbrow + (int64_t)pend * 64 * 64, lane);
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
                int32_t upin = shr1(cur);
                int32_t tin = shr1(tch);
                upin = lane == 0 ? lds_up : upin;
                tin = lane == 0 ? lds_t : tin;
                const bool cell = row_ok && j >= 1 && j <= m;
                const Acc diag = (Acc)uprev + ((uint32_t)tin == sc ? match : mismatch);
                const Acc up = (Acc)upin + indel;
                const Acc left = (Acc)cur + indel;
                const Acc mx = diag > up ? diag : up;
                Acc v = mx > left ? mx : left;
                v = v > 0 ? v : 0;
                const int32_t nv = (int32_t)v;
                if constexpr (TB) {
                    int32_t code = (diag >= up && diag >= left && diag >= 0) ? 1
                                 : ((up >= left && up >= 0) ? 2 : (left >= 0 ? 3 : 0));
                    code |= nv > 0 ? 4 : 0;
                    tbs[u * 64 + lane] = (uint8_t)(cell ? code : 0);
                }
                cur = cell ? nv : cur;
                const bool better = cell && nv > bval;
                bval = better ? nv : bval;
                bj = better ? j : bj;
                if (produce) {
                    // lane 63 finished column j63 = tau - 62 of row 64s+64
                    const int32_t v63 = __builtin_amdgcn_readlane(cur, 63);
                    if constexpr (u <= 62) out_a = writelane<u + 1>(out_a, v63);  // hand-off chunk c-1, lane u+1
                    else out_b = writelane<0>(out_b, v63);                        // hand-off chunk c, lane 0
                }
                uprev = upin;
                tch = tin;
            });
            // hand-off chunk c-1 (columns 64(c-1)+1 .. 64c) is complete: publish it, no wait
            if (produce && c >= 1) {
                const int64_t col = (int64_t)64 * (c - 1) + 1 + lane;
                if (col <= m) st8(rout + (int64_t)64 * (c - 1) + lane, ((uint64_t)epoch << 32) | (uint32_t)out_a);
            }
            out_a = out_b;
            pend = c;
        }
        // the last hand-off chunk and the last chunk of codes
        if (produce) {
            const int64_t col = (int64_t)64 * (n_chunks - 1) + 1 + lane;
            if (col <= m) st8(rout + (int64_t)64 * (n_chunks - 1) + lane, ((uint64_t)epoch << 32) | (uint32_t)out_a);
        }
        if (TB && pend >= 0) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            flush_codes<TB>(tbs, tbrow + (int64_t)pend * 64 * 64, lane);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
        // strip's best: max value, then smallest row i, then smallest column j (fill order)
        unsigned long long key = 0;
        if (row_ok && bval > 0)
            key = ((unsigned long long)(uint32_t)bval << 40) | ((unsigned long long)(0xFFFFFu - (uint32_t)i) << 20) |
                  (unsigned long long)(0xFFFFFu - (uint32_t)bj);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(key, off, 64);
            key = o > key ? o : key;
        }
        if (lane == 0 && key) atomicMax(best, key);
    }
}

}  // namespace ovl_local

extern "C" hipError_t ovl_launch_local(const uint8_t* q, int32_t n, const uint8_t* r, int32_t m, int64_t match,
                                       int64_t mismatch, int64_t indel, int32_t wide, uint64_t* rowbuf, int8_t* tb,
                                       unsigned long long* best, uint32_t* err_flag, int32_t blocks, uint32_t epoch,
                                       hipStream_t stream) {
    const int32_t n_strips = (n + 63) / 64;
    if (n_strips == 0 || m == 0) return hipSuccess;
    const unsigned g = (unsigned)(blocks < n_strips ? blocks : n_strips);
    if (tb) {
        if (wide)
            ovl_local::sw_kernel<int64_t, true><<<g, 64, 0, stream>>>(q, n, r, m, match, mismatch, indel, rowbuf, tb,
                                                                       best, err_flag, n_strips, epoch);
        else
            ovl_local::sw_kernel<int32_t, true><<<g, 64, 0, stream>>>(q, n, r, m, match, mismatch, indel, rowbuf, tb,
                                                                       best, err_flag, n_strips, epoch);
    } else {
        if (wide)
            ovl_local::sw_kernel<int64_t, false><<<g, 64, 0, stream>>>(q, n, r, m, match, mismatch, indel, rowbuf,
                                                                        nullptr, best, err_flag, n_strips, epoch);
        else
            ovl_local::sw_kernel<int32_t, false><<<g, 64, 0, stream>>>(q, n, r, m, match, mismatch, indel, rowbuf,
                                                                        nullptr, best, err_flag, n_strips, epoch);
    }
    return hipGetLastError();
}
