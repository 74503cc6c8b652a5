// local_alignment (aligners.py:85-167) for one large pair on the whole GPU.
//
// Smith-Waterman with the reference's tie order (aligners.py:116-126): a cell takes diag if
// diag >= up, diag >= left and diag >= 0 (code 1), else up if up >= left and up >= 0 (2), else
// left if left >= 0 (3), else 0 (code 0); int64-exact arithmetic.  Best cell: the first strict
// maximum in the i-major / j-minor fill order, from 0 (aligners.py:128-130).
//
// Layout: the query's rows are cut into 64-row strips; one wavefront (one 64-thread block) owns a
// strip at a time and sweeps its anti-diagonals (lane L on row 64s+1+L, column j = tau - L + 1).
// Strip s needs the last row of strip s-1, which another wavefront -- usually on another CU --
// produces concurrently: it is handed over through L2 in 64-column chunks (MI355X_MICROARCH.md
// hand-off table, first row: the producer writes each chunk with sc1 stores, waits vmcnt(0), then
// one lane stores the strip's progress with an sc1 store; the consumer polls progress with sc1
// loads and reads the chunk with sc1 loads).  Strips go round-robin to gridDim.x co-resident blocks,
// so every strip's producer is always a resident wavefront that started earlier; every poll is
// bounded (err_flag bit 1) so the grid always drains.  Reference characters and the carried row
// reach lane 0 through readlane from a per-chunk register, so nothing is limited by LDS size.
//
// Traceback (optional): one byte per cell, code | 4 when the cell is > 0 (the walk's dp > 0 test,
// aligners.py:136), stored strip-major then anti-diagonal-major ([s][tau][lane]) so each step writes
// 64 contiguous bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ovl_kernels.h"

namespace ovl_local {

__device__ __forceinline__ int32_t shr1(int32_t v) {
    // lane L receives lane L-1's value (lane 0 gets 0): DPP wave_shr:1
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ int32_t ld_sc1(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename Acc>
__global__ __launch_bounds__(64) void sw_kernel(const uint8_t* __restrict__ q, int32_t n, const uint8_t* __restrict__ r,
                                                int32_t m, int64_t match_, int64_t mismatch_, int64_t indel_,
                                                int32_t* __restrict__ rowbuf, int32_t* __restrict__ progress,
                                                int8_t* __restrict__ tb, unsigned long long* __restrict__ best,
                                                uint32_t* __restrict__ err_flag, int32_t n_strips) {
    const Acc match = (Acc)match_, mismatch = (Acc)mismatch_, indel = (Acc)indel_;
    const int lane = threadIdx.x;
    const int64_t W = (int64_t)m + 1;
    const int64_t steps = (int64_t)m + 63;  // tau = 0 .. m + 62
    for (int32_t s = blockIdx.x; s < n_strips; s += gridDim.x) {
        const int32_t i = 64 * s + 1 + lane;
        const bool row_ok = i <= n;
        const uint32_t sc = row_ok ? (uint32_t)q[i - 1] : 0xFFFFFFFFu;
        const bool produce = s + 1 < n_strips;  // strip s+1 reads our last row (row 64s+64 <= n)
        const int32_t* rin = rowbuf + (int64_t)(s - 1) * W;
        int32_t* rout = rowbuf + (int64_t)s * W;
        int32_t cur = 0;    // dp[i][j-1]
        int32_t uprev = 0;  // dp[i-1][j-1]
        uint32_t tch = 0;
        int32_t v_rin = 0, v_t = 0, v_out = 0;
        int32_t bval = 0, bj = 0;  // this row's first strict maximum (from 0)
        int32_t have = 0;          // columns of strip s-1's last row known to be published
        for (int64_t tau = 0; tau < steps; ++tau) {
            const int64_t jr = tau + 1;  // column whose dp[i-1][j] lane 0 needs now
            if ((jr & 63) == 0 || tau == 0) {
                // next chunk of the carried row: columns 64c .. 64c+63
                const int64_t base = jr & ~63ll;
                if (base <= m) {
                    if (s > 0) {
                        const int32_t need = (int32_t)(base + 64 <= W ? base + 64 : W);
                        int32_t spins = 0;
                        while (have < need) {
                            have = ld_sc1(progress + (s - 1));
                            if (have >= need) break;
                            __builtin_amdgcn_s_sleep(1);
                            if (++spins > (1 << 20)) {  // never expected: keep the grid finite
                                if (lane == 0) atomicOr(err_flag, 2u);
                                have = (int32_t)W;      // stop waiting for the rest of this strip
                            }
                        }
                        v_rin = base + lane <= m ? ld_sc1(rin + base + lane) : 0;
                    } else {
                        v_rin = 0;  // row 0
                    }
                }
            }
            if ((tau & 63) == 0) {
                const int64_t c = tau + lane;
                v_t = c < m ? (int32_t)r[c] : 0;
            }
            const int32_t j = (int32_t)(tau - lane + 1);
            const int32_t lds_up = __builtin_amdgcn_readlane(v_rin, (int)(jr & 63));
            const uint32_t lds_t = (uint32_t)__builtin_amdgcn_readlane(v_t, (int)(tau & 63));
            int32_t upin = shr1(cur);
            uint32_t tin = (uint32_t)shr1((int32_t)tch);
            if (lane == 0) { upin = lds_up; tin = lds_t; }
            int8_t code = 0;
            if (row_ok && j >= 1 && j <= m) {
                const Acc diag = (Acc)uprev + (sc == tin ? match : mismatch);
                const Acc up = (Acc)upin + indel;
                const Acc left = (Acc)cur + indel;
                Acc v;
                if (diag >= up && diag >= left && diag >= 0) { v = diag; code = 1; }
                else if (up >= left && up >= 0)              { v = up;   code = 2; }
                else if (left >= 0)                          { v = left; code = 3; }
                else                                         { v = 0; }
                cur = (int32_t)v;
                if (cur > 0) code |= 4;
                if (cur > bval) { bval = cur; bj = j; }
            }
            if (tb) tb[((int64_t)s * steps + tau) * 64 + lane] = code;
            // producer: stage lane 63's value (row 64s+64, column j63) into the chunk register
            if (produce) {
                const int64_t j63 = tau - 62;
                if (j63 >= 1 && j63 <= m) {
                    const int32_t v63 = __builtin_amdgcn_readlane(cur, 63);
                    if (lane == (int)(j63 & 63)) v_out = v63;
                    if ((j63 & 63) == 63 || j63 == m) {
                        const int64_t base = j63 & ~63ll;
                        if (base + lane <= m) st_sc1(rout + base + lane, v_out);  // column 0 stays 0 (lane 0, chunk 0)
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0) st_sc1(progress + s, (int32_t)(j63 + 1 <= m ? base + 64 : W));
                    }
                }
            }
            uprev = upin;
            tch = tin;
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
                                       int64_t mismatch, int64_t indel, int32_t wide, int32_t* rowbuf,
                                       int32_t* progress, int8_t* tb, unsigned long long* best, uint32_t* err_flag,
                                       int32_t blocks, hipStream_t stream) {
    const int32_t n_strips = (n + 63) / 64;
    if (n_strips == 0 || m == 0) return hipSuccess;
    const unsigned g = (unsigned)(blocks < n_strips ? blocks : n_strips);
    if (wide)
        ovl_local::sw_kernel<int64_t><<<g, 64, 0, stream>>>(q, n, r, m, match, mismatch, indel, rowbuf, progress, tb,
                                                             best, err_flag, n_strips);
    else
        ovl_local::sw_kernel<int32_t><<<g, 64, 0, stream>>>(q, n, r, m, match, mismatch, indel, rowbuf, progress, tb,
                                                             best, err_flag, n_strips);
    return hipGetLastError();
}
