// Probe (diagnostic tool, not part of libovl): the cell cost of dp_lane_kernel's strip body (ovl_dp_lane.hip,
// CW = 32 columns, byte score profile) against the same body on two pairs per lane in packed int16
// (the int16 form was rejected on an estimate; this measures it).
//   int32 form (the kernel's): per row one 4-byte score table from the row symbol, per 4 columns a v_perm of
//     it by the strip's t codes, per cell a sign-extending SDWA byte add and a v_max3 (left chain serial);
//   int16 form: lanes hold pairs A (low halves) and B (high halves); per row two tables, per column one v_perm
//     of both tables by a per-strip selector (t codes of A and B) that yields the packed scores (zero-extended:
//     G-unit scores are >= 0 at config 5), then v_pk_add_u16 and two v_pk_max_i16.
// Both run R rows x S strips over the same number of cells per lane (int16: two pairs' worth) at 4 waves per
// SIMD (launch bounds), every SIMD full; prints ns and SIMD cycles per cell.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lane16_probe.hip -o genome-assembly-using-overlap-graphs_amd/build/lane16_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int CW = 32;
typedef short s16x2 __attribute__((ext_vector_type(2)));
constexpr int ROWS = 256;
constexpr int STRIPS = 8;

__global__ __launch_bounds__(256, 4) void cell32(const uint32_t* __restrict__ tsym, const uint32_t* __restrict__ ssym,
                                                  int32_t* __restrict__ out, int32_t s_ma, int32_t s_mm) {
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int32_t best = 0;
    const uint32_t tbl_base = ((uint32_t)s_mm & 0xFFu) * 0x01010101u;
    const uint32_t tbl_diff = ((uint32_t)(s_ma ^ s_mm)) & 0xFFu;
    for (int st = 0; st < STRIPS; ++st) {
        uint32_t TW[CW / 4];
#pragma unroll
        for (int w = 0; w < CW / 4; ++w) TW[w] = tsym[(st * (CW / 4) + w) * 64 + (gid & 63)] & 0x03030303u;
        int32_t A[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) A[c] = c;
        int32_t lb = st;
        uint32_t S = ssym[(st & 7) * 64 + (gid & 63)];
        for (int it = 0; it < ROWS; it += 2) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t x8 = ((S >> ((it + r) & 31)) & 3u) * 8u;
                const uint32_t tbl = tbl_base ^ (tbl_diff << x8);
                uint32_t P[CW / 4];
#pragma unroll
                for (int w = 0; w < CW / 4; ++w) P[w] = __builtin_amdgcn_perm(tbl, tbl, TW[w]);
                int32_t d = lb, l = lb + 1;
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const int32_t s2 = (int32_t)(int8_t)(uint8_t)(P[c >> 2] >> (8 * (c & 3)));
                    const int32_t v = max(max(d + s2, A[c]), l);
                    d = A[c];
                    A[c] = v;
                    l = v;
                }
                lb = l - 3;
            }
        }
#pragma unroll
        for (int c = 0; c < CW; ++c) best = max(best, A[c]);
    }
    out[gid] = best;
}

// two pairs per lane: G values of pair A in the low 16 bits, pair B in the high 16 bits
__global__ __launch_bounds__(256, 4) void cell16(const uint32_t* __restrict__ tsym, const uint32_t* __restrict__ ssym,
                                                  int32_t* __restrict__ out, int32_t s_ma, int32_t s_mm) {
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int32_t best = 0;
    const uint32_t tbl_base = ((uint32_t)s_mm & 0xFFu) * 0x01010101u;
    const uint32_t tbl_diff = ((uint32_t)(s_ma ^ s_mm)) & 0xFFu;
    for (int st = 0; st < STRIPS; ++st) {
        // per column the selector [tA, zero, 4 + tB, zero]: byte 0 = table A's score, byte 2 = table B's
        uint32_t SEL[CW];
#pragma unroll
        for (int w = 0; w < CW / 4; ++w) {
            const uint32_t ta = tsym[(st * (CW / 4) + w) * 64 + (gid & 63)] & 0x03030303u;
            const uint32_t tb = (tsym[(st * (CW / 4) + w) * 64 + ((gid + 17) & 63)] & 0x03030303u) | 0x04040404u;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                SEL[4 * w + k] = ((ta >> (8 * k)) & 0xFFu) | 0x0C00u | (((tb >> (8 * k)) & 0xFFu) << 16) | 0x0C000000u;
        }
        uint32_t A[CW];
#pragma unroll
        for (int c = 0; c < CW; ++c) A[c] = (uint32_t)c * 0x00010001u;
        uint32_t lb = (uint32_t)st * 0x00010001u;
        const uint32_t SA = ssym[(st & 7) * 64 + (gid & 63)], SB = ssym[(st & 7) * 64 + ((gid + 5) & 63)];
        for (int it = 0; it < ROWS; it += 2) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t xa = ((SA >> ((it + r) & 31)) & 3u) * 8u;
                const uint32_t xb = ((SB >> ((it + r) & 31)) & 3u) * 8u;
                const uint32_t tba = tbl_base ^ (tbl_diff << xa);
                const uint32_t tbb = tbl_base ^ (tbl_diff << xb);
                uint32_t d = lb, l = lb + 0x00010001u;
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const uint32_t s2 = __builtin_amdgcn_perm(tbb, tba, SEL[c]);
                    const s16x2 t = __builtin_bit_cast(s16x2, d) + __builtin_bit_cast(s16x2, s2);
                    const s16x2 m = __builtin_elementwise_max(t, __builtin_bit_cast(s16x2, A[c]));
                    const uint32_t v = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(m, __builtin_bit_cast(s16x2, l)));
                    d = A[c];
                    A[c] = v;
                    l = v;
                }
                lb = l - 0x00030003u;
            }
        }
#pragma unroll
        for (int c = 0; c < CW; ++c) best = max(best, (int32_t)(A[c] & 0xFFFFu) + (int32_t)(A[c] >> 16));
    }
    out[gid] = best;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 4 * 4;  // 4 waves per SIMD: 16 waves per CU, 4 blocks of 256
    uint32_t *tsym, *ssym;
    int32_t* out;
    CK(hipMalloc(&tsym, STRIPS * (CW / 4) * 64 * 4));
    CK(hipMalloc(&ssym, 8 * 64 * 4));
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    uint32_t h_t[STRIPS * (CW / 4) * 64], h_s[8 * 64];
    srand(7);
    for (auto& v : h_t) v = (uint32_t)rand() * 2654435761u;
    for (auto& v : h_s) v = (uint32_t)rand() * 2246822519u;
    CK(hipMemcpy(tsym, h_t, sizeof(h_t), hipMemcpyHostToDevice));
    CK(hipMemcpy(ssym, h_s, sizeof(h_s), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double lanes = (double)blocks * 256;
    for (int rep = 0; rep < 3; ++rep) {
        for (int form = 0; form < 2; ++form) {
            for (int w = 0; w < 2; ++w) {
                if (form == 0) cell32<<<blocks, 256>>>(tsym, ssym, out, 14, 3);
                else cell16<<<blocks, 256>>>(tsym, ssym, out, 14, 3);
            }
            CK(hipEventRecord(e0));
            const int n = 10;
            for (int i = 0; i < n; ++i) {
                if (form == 0) cell32<<<blocks, 256>>>(tsym, ssym, out, 14, 3);
                else cell16<<<blocks, 256>>>(tsym, ssym, out, 14, 3);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= n;
            const double cells = lanes * STRIPS * ROWS * CW * (form == 0 ? 1 : 2);
            // cells per SIMD-cycle: 1024 SIMDs (256 CUs x 4) at 2.4 GHz
            const double cyc = ms * 1e-3 * 2.4e9 * cus * 4 / (cells / 64.0);
            printf("%s: %.3f ms, %.3f ps per cell, %.2f SIMD cycles per 64 cells (one wave64 cell step)\n",
                   form == 0 ? "int32 (1 pair/lane) " : "int16 (2 pairs/lane)", ms, ms * 1e9 / cells, cyc);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
