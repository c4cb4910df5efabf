// libiddgcn_hip — MI355X (gfx950 / CDNA4) kernels for IDDGCN's multi-relational
// graph convolution, forward and backward, behind the C-ABI of include/iddgcn.h.
//
// Design notes (DESIGN.md has the full version):
//  * 64-lane wavefronts.  Row-wise memory-bound kernels map one row of D fp32 to
//    D/4 lanes (one float4 = 16 B per lane), so a wave moves 1 KiB per instruction.
//  * Dense D x D projections run on the exact-f32 MFMA v_mfma_f32_32x32x2_f32
//    (157 TFLOP/s chip peak, bitwise an fmaf chain).  The D x D weight is kept in
//    registers for the life of a persistent workgroup (one 32-column slab per
//    wave, D/2 VGPRs), the streamed rows go HBM -> LDS (padded rows, conflict-free
//    ds_read_b128 of 4 k-steps at once, k permuted identically on both operands).
//  * No float atomics anywhere: scatters are deterministic segmented gathers over
//    precomputed CSR-style permutations, and cross-block sums go through slabs
//    reduced in block order.  Results are bitwise reproducible run to run.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/iddgcn.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define MAX_R 8
#define EPS_BCE 1e-7f

namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// layer activations: v_exp_f32 + v_rcp_f32 (~2 ulp; saturates to exactly 0 / 1 like the accurate form)
__device__ __forceinline__ float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// ---- in-register cross-lane exchange for full-wave (64-lane) groups: no LDS round trip ----
// v_permlane{32,16}_swap exchange half-waves / odd-even 16-lane rows between two registers;
// DPP row_mirror (l^15), row_half_mirror (l^7) and quad_perm (l^2, l^1) pair each lane with one
// whose bit m is flipped and whose higher bits match, which is all a butterfly level needs.
// (inline asm: this hipcc returns the same register for both halves of the swap builtins;
// the two v_nop are the VALU-write -> permlane hazard.)
__device__ __forceinline__ void pl_swap32(float& a, float& b) {
    asm volatile("v_nop\n\tv_nop\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void pl_swap16(float& a, float& b) {
    asm volatile("v_nop\n\tv_nop\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_XOR2 = 0x4E, DPP_XOR1 = 0xB1;
template <int M>
__device__ __forceinline__ float xpartner_dpp(float v) {   // M in {8, 4, 2, 1}
    if constexpr (M == 8) return dpp<DPP_ROW_MIRROR>(v);
    else if constexpr (M == 4) return dpp<DPP_ROW_HALF_MIRROR>(v);
    else if constexpr (M == 2) return dpp<DPP_XOR2>(v);
    else return dpp<DPP_XOR1>(v);
}

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
    if constexpr (LPR == 64) {
        float a = v, b = v;
        pl_swap32(a, b);
        v = a + b;
        a = v, b = v;
        pl_swap16(a, b);
        v = a + b;
        v += xpartner_dpp<8>(v);
        v += xpartner_dpp<4>(v);
        v += xpartner_dpp<2>(v);
        v += xpartner_dpp<1>(v);
        return v;
    } else {
#pragma unroll
        for (int m = LPR / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        return v;
    }
}

// Reduce K values (K a power of two, K <= LPR) over an aligned group of LPR lanes with a
// butterfly that halves the value set at each level: K-1 + log2(LPR/K) ... shuffles instead of
// K*log2(LPR).  On return v[0] holds, in every lane, the full sum of value index
// sub / (LPR/K).  LPR == 64 and 32 use the permlane/DPP exchanges above (no LDS crossbar).
// The levels are a compile-time recursion (M = lane distance, KC = values still held): with the live
// count as a run-time variable the compiler indexed v[] dynamically (a v_cmp/v_cndmask/s_nop chain per
// element: ~1300 extra instructions per edge group in the R = 8 tail reduction).
template <int LPR, int K, int KC, int M>
__device__ __forceinline__ void multi_reduce_level(float (&v)[K], int sub) {
    if constexpr (M >= 1) {
        constexpr bool PERM = LPR == 64 || LPR == 32;        // permlane / DPP exchanges
        constexpr bool SWAP = (LPR == 64 && M == 32) || (PERM && M == 16);
        if constexpr (KC > 1) {
            constexpr int half = KC / 2;
            if constexpr (SWAP) {      // one register swap exchanges the kept/sent halves of a value pair
#pragma unroll
                for (int j = 0; j < half; ++j) {
                    float a = v[j], b = v[half + j];
                    if constexpr (M == 32) pl_swap32(a, b);
                    else pl_swap16(a, b);
                    v[j] = a + b;
                }
            } else {
                const bool up = (sub & M) != 0;
#pragma unroll
                for (int j = 0; j < half; ++j) {
                    const float keep = up ? v[half + j] : v[j];
                    const float send = up ? v[j] : v[half + j];
                    if constexpr (PERM) v[j] = keep + xpartner_dpp<M>(send);
                    else v[j] = keep + __shfl_xor(send, M, 64);
                }
            }
            multi_reduce_level<LPR, K, half, M / 2>(v, sub);
        } else {
            if constexpr (SWAP) {
                float a = v[0], b = v[0];
                if constexpr (M == 32) pl_swap32(a, b);
                else pl_swap16(a, b);
                v[0] = a + b;
            } else if constexpr (PERM) {
                v[0] += xpartner_dpp<M>(v[0]);
            } else {
                v[0] += __shfl_xor(v[0], M, 64);
            }
            multi_reduce_level<LPR, K, 1, M / 2>(v, sub);
        }
    }
}
template <int LPR, int K>
__device__ __forceinline__ float multi_reduce(float (&v)[K], int sub) {
    static_assert((K & (K - 1)) == 0 && K <= LPR, "K must be a power of two <= LPR");
    multi_reduce_level<LPR, K, K, LPR / 2>(v, sub);
    return v[0];
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
// bf16 edge tables (the bf16-feature mode): 4 values = 8 bytes, round-to-nearest-even on store
__device__ __forceinline__ f32x4 bf4_to_f32(bf16x4 v) {
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
__device__ __forceinline__ bf16x4 f32_to_bf4(f32x4 v) {
    return bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}
__device__ __forceinline__ f32x4 ld4bf(const __bf16* p) { return bf4_to_f32(*reinterpret_cast<const bf16x4*>(p)); }
__device__ __forceinline__ void st4bf(__bf16* p, f32x4 v) { *reinterpret_cast<bf16x4*>(p) = f32_to_bf4(v); }
// 4 consecutive elements of an edge table that is fp32 or (BF) bf16, addressed in elements
template <bool BF>
__device__ __forceinline__ f32x4 ld4e(const float* base, long long idx) {
    if constexpr (BF) return ld4bf(reinterpret_cast<const __bf16*>(base) + idx);
    else return ld4(base + idx);
}
template <bool BF>
__device__ __forceinline__ void st4e(float* base, long long idx, f32x4 v) {
    if constexpr (BF) st4bf(reinterpret_cast<__bf16*>(base) + idx, v);
    else st4(base + idx, v);
}
__device__ __forceinline__ f32x4 fma4(f32x4 a, f32x4 b, f32x4 c) {
    return f32x4{fmaf(a[0], b[0], c[0]), fmaf(a[1], b[1], c[1]), fmaf(a[2], b[2], c[2]), fmaf(a[3], b[3], c[3])};
}

inline int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
inline bool dim_ok(int d) { return d == 32 || d == 64 || d == 128 || d == 256; }

// ---------------------------------------------------------------------------
// CSR SpMM: one row per group of D/4 lanes, sequential sum in CSR order.
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void spmm_csr_kernel(int n_seg, int n_rows, const int* __restrict__ ptr,
                                                       const int* __restrict__ col, const float* __restrict__ vals,
                                                       const float* __restrict__ X, float* __restrict__ Y,
                                                       int accumulate) {
    constexpr int LPR = D / 4;
    const long long grow = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
    const int sub = threadIdx.x % LPR;
    if (grow >= (long long)n_seg * n_rows) return;
    const int s = (int)(grow / n_rows);
    const int n = (int)(grow % n_rows);
    const int* p = ptr + (long long)s * (n_rows + 1);
    const int beg = p[n], end = p[n + 1];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int k = beg;
    // two rows in flight, summed strictly in CSR order
    for (; k + 1 < end; k += 2) {
        const int c0 = col[k], c1 = col[k + 1];
        f32x4 x0 = ld4(X + (long long)c0 * D + sub * 4);
        f32x4 x1 = ld4(X + (long long)c1 * D + sub * 4);
        if (vals) {
            x0 *= vals[k];
            x1 *= vals[k + 1];
        }
        acc += x0;
        acc += x1;
    }
    if (k < end) {
        f32x4 x0 = ld4(X + (long long)col[k] * D + sub * 4);
        if (vals) x0 *= vals[k];
        acc += x0;
    }
    float* y = Y + grow * D + sub * 4;
    if (accumulate) acc += ld4(y);
    st4(y, acc);
}

// ---------------------------------------------------------------------------
// CSR SDDMM (gradient of A·X w.r.t. A's stored values): out[k] = <G[seg row], X[col[k]]>.
// One row per group of D/4 lanes; the G row stays in registers, two X rows in flight, each dot
// reduced across the group.  Output in CSR order.
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void sddmm_csr_kernel(int n_seg, int n_rows, const int* __restrict__ ptr,
                                                        const int* __restrict__ col, const float* __restrict__ G,
                                                        const float* __restrict__ X, float* __restrict__ out) {
    constexpr int LPR = D / 4;
    const long long grow = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
    const int sub = threadIdx.x % LPR;
    // groups of one wave may hold different rows: every lane runs the wave's longest row
    const bool live = grow < (long long)n_seg * n_rows;
    int beg = 0, end = 0;
    f32x4 g = {0.f, 0.f, 0.f, 0.f};
    if (live) {
        const int s = (int)(grow / n_rows);
        const int n = (int)(grow % n_rows);
        const int* p = ptr + (long long)s * (n_rows + 1);
        beg = p[n];
        end = p[n + 1];
        g = ld4(G + grow * D + sub * 4);
    }
    int len = end - beg, maxlen = len;
    if (LPR < 64) {
#pragma unroll
        for (int m = 32; m >= LPR; m >>= 1) maxlen = max(maxlen, __shfl_xor(maxlen, m, 64));
    }
    for (int k = 0; k < maxlen; k += 2) {
        const bool ok0 = k < len, ok1 = k + 1 < len;
        const f32x4 x0 = ok0 ? ld4(X + (long long)col[beg + k] * D + sub * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 x1 = ok1 ? ld4(X + (long long)col[beg + k + 1] * D + sub * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 p0 = g * x0, p1 = g * x1;
        const float d0 = group_sum<LPR>((p0[0] + p0[1]) + (p0[2] + p0[3]));
        const float d1 = group_sum<LPR>((p1[0] + p1[1]) + (p1[2] + p1[3]));
        if (sub == 0) {
            if (ok0) out[beg + k] = d0;
            if (ok1) out[beg + k + 1] = d1;
        }
    }
}

// ---------------------------------------------------------------------------
// Row GEMM with fused epilogue on v_mfma_f32_32x32x2_f32.
//   wave w: column slab cs = w % CS (32 output columns), row group rg = w / CS.
//   B slab resident in VGPRs: breg[s] = B[kk(s,h)][c0+i],  kk(s,h) = 8(s/4) + 4h + s%4,
//   A fragment for 4 consecutive k-steps = one ds_read_b128 of A_lds[row i][8q+4h..+3].
// ---------------------------------------------------------------------------
template <int D>
struct RG {
    static constexpr int CS = D / 32;
    static constexpr int NW = CS >= 4 ? CS : 4;
    static constexpr int RGS = NW / CS;
    static constexpr int TR = RGS * 32;
    static constexpr int LDA = D + 4;
};

struct RowGemmP {
    int M;
    const float* A; const int* a_idx;
    const float* B; int b_trans;
    float* C; int accumulate;
    int R;
    const float* coef; const int* coef_idx;
    const float* V; const int* v_idx;
    long long v_rel_stride, v_row_stride;
    int act; const float* aux;
    int planes;           // IDDGCN_PLANES_A | _C | _AUX (D = 256 split mode, v3 kernel only)
    int precision;        // IDDGCN_GEMM_* of this call (D = 256 v3 kernels; every other GEMM is exact f32)
    int tiles_per_block;
};

// up to ROWGEMM_BATCH independent row GEMMs of one width in one launch (blockIdx.y = entry): the
// node-level projections of a step are many tiny launches at the reference's 845 nodes.  25 = 3R + 1 at R = 8:
// config 5's whole forward projection set (three layers per AE_r, plus E S^1) in one launch, so the three
// entries reading the same AE_r run concurrently (entries r, r + R, r + 2R land on one XCD when R * per is a
// multiple of 8) and AE_r comes from HBM once instead of twice (25 x 136 B of kernel arguments)
constexpr int ROWGEMM_BATCH = 25;
struct RowGemmBatch {
    RowGemmP p[ROWGEMM_BATCH];
};

template <int D>
__global__ __launch_bounds__(RG<D>::NW * 64) void rowgemm_kernel(RowGemmBatch pb) {
    using C = RG<D>;
    const RowGemmP& p = pb.p[blockIdx.y];
    __shared__ __attribute__((aligned(16))) float As[C::TR * C::LDA];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cs = wave % C::CS;
    const int rg = wave / C::CS;
    const int i = lane & 31, h = lane >> 5;
    const int c0 = cs * 32;

    float breg[D / 2];
#pragma unroll
    for (int s = 0; s < D / 2; ++s) {
        const int kk = 8 * (s >> 2) + 4 * h + (s & 3);
        breg[s] = p.b_trans ? p.B[(c0 + i) * D + kk] : p.B[kk * D + c0 + i];
    }

    const long long ntiles = ((long long)p.M + C::TR - 1) / C::TR;
    const long long t_beg = (long long)blockIdx.x * p.tiles_per_block;
    long long t_end = t_beg + p.tiles_per_block;
    if (t_end > ntiles) t_end = ntiles;

    for (long long tile = t_beg; tile < t_end; ++tile) {
        const long long row0 = tile * C::TR;
        __syncthreads();
        constexpr int F4R = D / 4;
        constexpr int TOT = C::TR * F4R;
#pragma unroll
        for (int it = 0; it < TOT / (C::NW * 64); ++it) {
            const int idx = it * C::NW * 64 + threadIdx.x;
            const int r = idx / F4R, c4 = idx % F4R;
            const long long e = row0 + r;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (e < p.M) {
                const long long src = p.a_idx ? (long long)p.a_idx[e] : e;
                v = ld4(p.A + src * D + c4 * 4);
            }
            st4(As + r * C::LDA + c4 * 4, v);
        }
        __syncthreads();

        // IDDGCN_GEMM_F32_4CHAIN: k-step q (8 k-values) goes into chain q % 4, (c0 + c1) + (c2 + c3) at the end
        const bool c4 = p.precision == IDDGCN_GEMM_F32_4CHAIN;
        f32x16 acc, acc1, acc2, acc3;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = acc1[j] = acc2[j] = acc3[j] = 0.f;
        const float* arow = As + (rg * 32 + i) * C::LDA + 4 * h;
        if (c4) {
#pragma unroll
            for (int q = 0; q < D / 8; ++q) {
                const f32x4 a4 = ld4(arow + 8 * q);
                f32x16& ac = (q & 3) == 0 ? acc : (q & 3) == 1 ? acc1 : (q & 3) == 2 ? acc2 : acc3;
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[0], breg[4 * q + 0], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[1], breg[4 * q + 1], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[2], breg[4 * q + 2], ac, 0, 0, 0);
                ac = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[3], breg[4 * q + 3], ac, 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] = (acc[j] + acc1[j]) + (acc2[j] + acc3[j]);
        } else {
#pragma unroll
            for (int q = 0; q < D / 8; ++q) {
                const f32x4 a4 = ld4(arow + 8 * q);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[0], breg[4 * q + 0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[1], breg[4 * q + 1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[2], breg[4 * q + 2], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[3], breg[4 * q + 3], acc, 0, 0, 0);
            }
        }

        const int c = c0 + i;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const long long e = row0 + rg * 32 + row;
            if (e >= p.M) continue;
            float v = acc[reg];
            float* cp = p.C + e * D + c;
            if (p.accumulate) v += *cp;
            if (p.R > 0) {
                const long long ci = p.coef_idx ? (long long)p.coef_idx[e] : e;
                const long long vi = p.v_idx ? (long long)p.v_idx[e] : e;
                const float* vb = p.V + vi * p.v_row_stride + c;
                // every coefficient and V value of the row is loaded before the first fma (a compile-time
                // bounded, guarded loop instead of a run-time trip count that waited on each pair in turn)
                float cfv[MAX_R], vv[MAX_R];
#pragma unroll
                for (int r = 0; r < MAX_R; ++r) {
                    cfv[r] = r < p.R ? p.coef[ci * p.R + r] : 0.f;
                    vv[r] = r < p.R ? vb[r * p.v_rel_stride] : 0.f;
                }
#pragma unroll
                for (int r = 0; r < MAX_R; ++r)
                    if (r < p.R) v = fmaf(cfv[r], vv[r], v);
            }
            if (p.act == IDDGCN_ACT_SIGMOID) {
                v = sigmoid_fast(v);
            } else if (p.act == IDDGCN_ACT_DSIGMOID) {
                const float x = p.aux[e * D + c];
                v = v * (x * (1.0f - x));
            }
            *cp = v;
        }
    }
}

// LDS-DMA helpers (global_load_lds: the row lands in LDS without passing through VGPRs)
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* gbl_vptr;

__device__ __forceinline__ void dma_row_1k(const float* src_row, float* lds_row, int lane) {
    __builtin_amdgcn_global_load_lds((gbl_vptr)(src_row + lane * 4), (lds_vptr)lds_row, 16, 0, 0);
}


// ---------------------------------------------------------------------------
// Row GEMM, D = 256, v3: staggered waves, wave-private epilogue slabs.
//   * A tiles: LDS-DMA double buffer, 1040-B padded rows (one 1 KiB DMA
//     wave-instruction per row, so padding between rows is allowed): conflict-free
//     ds_read_b128 fragment reads at one base register + immediate offsets.
//   * Epilogue operands: each wave DMAs only the 32 columns it owns (gathered
//     P_r[t] rows and/or sigma' aux rows, 32 rows x 32 cols = 4 KiB per slab) plus
//     its per-row coefficients into a private LDS region.  Producer == consumer,
//     so these need no barrier, only the wave's own vmcnt.
//   * Stagger: waves 4-7 (one partner per SIMD) run the epilogue of tile t-1 at
//     the top of iteration t, while waves 0-3 run tile t's epilogue after its
//     MFMAs: each SIMD overlaps one wave's epilogue VALU with its partner's
//     MFMAs.  One barrier per tile (A buffers), raw s_barrier so the slab DMA of
//     the next tile stays in flight across it.
// ---------------------------------------------------------------------------
// ablation switches for the GEMM microbenchmark (never set in the product build)
namespace r3 {
constexpr int D = 256, NW = 8, TR = 32;
constexpr int ROWS_PER_WAVE = TR / NW;                 // A rows each wave stages
static_assert(ROWS_PER_WAVE == 4, "the early-wave s_waitcnt vmcnt(4) counts the A-row DMAs");
constexpr int LDA = D + 4;                             // padded rows: conflict-free ds_read_b128
constexpr int A_FLOATS = TR * LDA;                     // 33,280 B
constexpr int SLAB = TR * 32;                          // 32 rows x 32 cols
constexpr int COEF = 64;                               // 32 rows x R (R <= 2)
constexpr int COEF8 = 32 * MAX_R;                      // 32 rows x R (R <= 8)
constexpr int IDX = 64;                                // next tile's v_idx (32) + coef_idx (32)
constexpr int CMP = 32;                                // distinct V rows of the tile (run starts)
constexpr int CINV = 32;                               // split mode: 1/scale of the wave's 32 columns
// gathered V with more than 2 relations (NV = 4 or 8 slots, R <= NV at run time): slabs r >= 1 hold
// only the first GATHER_CAP distinct rows of a tile, so 8 relations fit the LDS; a tile with more runs
// of equal v_idx (tail-sorted edges have 1-3) reads the V rows past the cap from global memory (L2)
constexpr int GATHER_CAP = 7;
}  // namespace r3

// ---- split-fp16 operands (X3 kernels) -------------------------------------------------------
// A value x of a row (or column) whose max |x| is m is scaled by s = 2^k so that m*s lies in
// [2^14, 2^15), then split  x*s = hi + lo*2^-11  with hi = fp16_rne(x*s) and
// lo = fp16_rne((x*s - hi) * 2^11)  (x*s - hi is exact in fp32).  hi + lo*2^-11 carries 22
// significant bits: the representation error is <= 2^-22 |x*s| (<= 2^-25 absolute below 2^-3 of
// scaled range), under the sqrt(K)*2^-24 error of the K = 256 fp32 dot product itself.  That is the
// weight (column) split; the edge-row (A) side keeps lo in the units of hi (split16_same below, same
// 22 bits while lo is a normal fp16), the form the pre-split planes tables store.  A row GEMM then
// takes three f16 MFMAs per k-step (W_hi*A_hi + W_hi*A_lo into one accumulator, W_lo*A_hi into a
// second, combined as acc_hi + 2^-11 acc_lo) in place of eight f32 ones: 96 instead of 512 MFMA cycles.
__device__ __forceinline__ float pow2_scale(float amax) {     // s with amax*s in [2^14, 2^15)
    const int eb = (__float_as_int(amax) >> 23) & 0xFF;
    int se = 268 - eb;                                         // 2^(15 - (eb - 126))
    se = se < 1 ? 1 : (se > 253 ? 253 : se);                  // keep s and 1/s normal
    return __int_as_float(se << 23);
}
__device__ __forceinline__ float pow2_inv(float s) {           // exact 1/s for s = pow2_scale(.)
    return __int_as_float((254 - ((__float_as_int(s) >> 23) & 0xFF)) << 23);
}
__device__ __forceinline__ void split16(float xs, _Float16& hi, _Float16& lo) {
    hi = (_Float16)xs;
    lo = (_Float16)((xs - (float)hi) * 2048.0f);
}
// the A-side (edge row) split: lo in the units of hi, lo = fp16(xs - hi) (|lo| <= ulp(hi) / 2: 11 more
// significant bits; for xs below 2^-3 of the row's range lo goes subnormal and only bits below 2^-38 of
// the row max are lost)
__device__ __forceinline__ void split16_same(float xs, _Float16& hi, _Float16& lo) {
    hi = (_Float16)xs;
    lo = (_Float16)(xs - (float)hi);
}
// ---- pre-split edge tables ("planes", IDDGCN_PLANES_*) --------------------------------------
// A D = 256 row of values in [0, 1] (the sigmoid outputs x^1, x^2 of the tail chain) stored in 8
// column blocks of 128 B, block b = [hi f16 of columns 32b..32b+31 | lo f16 of the same columns] (1 KiB,
// the bytes of the fp32 row; block b occupies exactly the bytes of fp32 columns 32b..32b+31, so a kernel
// whose wave w owns columns 32w.. can overwrite a planes row with fp32 results in place, wave-locally),
// with the fixed scale 2^15: x*2^15 = hi + lo (split16_same).  The producer's epilogue splits once; the GEMMs that read the row
// (the next layer's forward as A, the dS TN as A, the backward's sigma' operand) skip the per-tile
// conversion.  This is the representation the per-row split gives rows whose max is in [0.5, 1)
// (22 significant bits; absolute error <= 2^-24).
constexpr float PLANE_S = 0x1p15f, PLANE_INV = 0x1p-15f;
__device__ __forceinline__ void to_planes4(const f32x4& v, f16x4& hv, f16x4& lv) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        _Float16 hi, lo;
        split16_same(v[q] * PLANE_S, hi, lo);
        hv[q] = hi;
        lv[q] = lo;
    }
}
__device__ __forceinline__ f32x4 from_planes4(const f16x4& hv, const f16x4& lv) {
    f32x4 x;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = ((float)hv[q] + (float)lv[q]) * PLANE_INV;
    return x;
}
// byte offset of the hi f16 of column c in a planes row (its lo: + 64)
__device__ __forceinline__ constexpr int plane_off(int c) { return 128 * (c >> 5) + 2 * (c & 31); }
// store 4 values of columns c..c+3 (c % 4 == 0) of a planes row (row_base = the row's first byte)
__device__ __forceinline__ void st_planes4(char* row_base, int c, const f32x4& v) {
    f16x4 hv, lv;
    to_planes4(v, hv, lv);
    *reinterpret_cast<f16x4*>(row_base + plane_off(c)) = hv;
    *reinterpret_cast<f16x4*>(row_base + plane_off(c) + 64) = lv;
}
// maxima over the 64 lanes of four values at once (halving butterfly: 2 + 1 swaps, 4 DPP steps);
// on return m[j] is wave-uniform
__device__ __forceinline__ void wave_max4(float (&m)[4]) {
    float a0 = m[0], b0 = m[2], a1 = m[1], b1 = m[3];
    pl_swap32(a0, b0);                 // lanes < 32: value 0 / 1, lanes >= 32: value 2 / 3
    pl_swap32(a1, b1);
    float v0 = fmaxf(a0, b0), v1 = fmaxf(a1, b1);
    pl_swap16(v0, v1);                 // 16-lane row k holds value k
    float v = fmaxf(v0, v1);
    v = fmaxf(v, xpartner_dpp<8>(v));
    v = fmaxf(v, xpartner_dpp<4>(v));
    v = fmaxf(v, xpartner_dpp<2>(v));
    v = fmaxf(v, xpartner_dpp<1>(v));
#pragma unroll
    for (int j = 0; j < 4; ++j)
        m[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16 * j));
}
__device__ __forceinline__ float wave_max(float v) {             // max over the 64 lanes
    float a = v, b = v;
    pl_swap32(a, b);
    v = fmaxf(a, b);
    a = v, b = v;
    pl_swap16(a, b);
    v = fmaxf(a, b);
    v = fmaxf(v, xpartner_dpp<8>(v));
    v = fmaxf(v, xpartner_dpp<4>(v));
    v = fmaxf(v, xpartner_dpp<2>(v));
    v = fmaxf(v, xpartner_dpp<1>(v));
    return v;
}

// C4 (IDDGCN_GEMM_F32_4CHAIN, f32 MFMA, plain form: the node-level projections P_r^l = AE_r K_r^l, E S^1):
// k-step q (8 k-values) accumulates into chain q % 4, the four chains summed pairwise at the end; the same
// f32 MFMA products, 64-long instead of 256-long accumulation chains (~2x less accumulation error).  The rows
// of AE_r sum ~20 entity rows, so P reaches |1e3|, and the 256-long fp32 chain was the largest error source
// of the logits at the reference's init (tools/logit_error_probe.py).  No accumulator is read mid-chain
// (a mid-chain fp64 or f32 partial-sum dump made hipcc spill the weight registers of this kernel).
// NV: gathered V tables (0 = none; 1, 2 = exactly R; 4, 8 = capacity for R <= NV, capped slabs).
// Up to ROWGEMM_BATCH independent GEMMs of the same variant run in one launch: blockIdx.y = entry.
// CW: broadcast V (NV = 0) with more than 2 coefficients per row (R <= 8); R <= 2 keeps the 2-slot
// coefficient code (the wide form is 2.4x slower on the node-level head-chain backward at R = 2).
// BF: the bf16-feature mode (perf only): A, the sigma' operand and C are bf16 edge tables (512-B rows;
// A lands in the hi-plane slot of an LDS row as it is), the weights a bf16 hi + lo pair, two
// v_mfma_f32_32x32x16_bf16 per k-step, fp32 accumulation and epilogue.  X3 must be set with it.
// PL (split mode): the planes form (IDDGCN_PLANES_*) of the variant: AUX kernels read the sigma' operand
// as planes rows, gathered-combine kernels (NV = 1, 2) write C as planes rows.
// (A planes rows are a run-time flag of every X3 kernel: convert_rows just skips.)
template <int NV, bool AUX, bool HAS_COEF, bool X3, bool CW = false, bool BF = false, bool PL = false, bool C4 = false,
          bool W1 = false>
__global__ __launch_bounds__(512) void rowgemm256_v3_kernel(RowGemmBatch pb) {
    using namespace r3;
    // A row pitch: bf16 rows (BF) need 512 B of the 1040-B fp32 row; round 4 padded them to 528 B (the fragment reads'
    // bank pattern 4i mod 64), which also let the wide R = 8 form keep three A buffers
    // (BF, round 5: 512-B slots with the 16-B chunks of row r XOR-swizzled by r & 15, two rows per full-wave DMA;
    // the swizzle keeps the fragment reads conflict-free without the pad)
    constexpr int LDA = BF ? 128 : r3::LDA;
    constexpr int A_FLOATS = TR * LDA;
    const RowGemmP p = pb.p[blockIdx.y];
    static_assert(!PL || (X3 && !BF && !CW && ((AUX && NV == 0) || (!AUX && (NV == 1 || NV == 2)))),
                  "PL: split-mode sigma' backward or R <= 2 gathered forward");
    static_assert(!BF || X3, "BF: the 16-bit A-plane pipeline");
    static_assert(!C4 || (!X3 && NV == 0 && !AUX && !HAS_COEF), "C4: the f32 plain form (node projections)");
    static_assert(!W1 || BF, "W1: bf16 weights, bf16-feature calls only");
    static_assert(NV <= 2 || NV == 4 || NV == 8, "gathered V: 1, 2 tables, or capacity 4 / 8");
    constexpr bool WIDE = NV > 2;                      // capped slabs, run-time R <= NV
    // capped V slabs r >= 1 (rows past the cap read from L2): WIDE
    constexpr bool CAPPED = WIDE;
    // the sigma' slab: after the V slabs; BF keeps it out of slab 0, whose fp32 staging of the output
    // would overwrite bf16 aux rows other lanes have not read yet (different row pitches)
    constexpr int AUXS = (BF && NV == 0) ? 1 : NV;
    constexpr int NS = AUX ? AUXS + 1 : NV;
    constexpr int NSL = NS > 1 ? NS : 1;               // slabs per wave (slab 0 also stages C)
    // Slab 0 holds 32 rows (it also stages the C tile); WIDE slabs r >= 1 hold GATHER_CAP rows.
    constexpr int CAPV = WIDE ? GATHER_CAP : 32;
    constexpr int SLABC = CAPV * 32;
    // WIDE forward, slot-major V: the tile's distinct V rows as [slot][relation][32 columns] after
    // slab 0, so ONE LDS-DMA instruction (64 lanes x 16 B, each lane its own relation row and 16-B group)
    // fetches a distinct row's 32 columns for all R <= 8 relations (two rows at R <= 4) instead of one
    // instruction per relation; CAPN slots in the bytes the capped per-relation slabs used
    constexpr bool SLOTV = WIDE && !AUX;
    constexpr int RPI = WIDE ? 64 / (NV * 8) : 1;      // distinct rows per DMA instruction (SLOTV)
    constexpr int CAPN = WIDE ? ((NSL - 1) * SLABC) / (NV * 32) / RPI * RPI : 0;
    static_assert(!SLOTV || CAPN >= 2, "slot-major V: at least two distinct rows");
    constexpr int SLABS = SLAB + (NSL - 1) * SLABC;    // floats of all slabs of one wave
    // coefficient slots: 32 rows x R; up to 8 relations for WIDE and for broadcast V (NV = 0)
    static_assert(!CW || (NV == 0 && HAS_COEF), "CW: broadcast V rows only");
    constexpr bool COEF_WIDE = WIDE || CW;
    constexpr int COEFN = COEF_WIDE ? COEF8 : COEF;
    constexpr int CFN = COEF_WIDE ? MAX_R : 2;         // coefficients each lane holds
    constexpr int WF = SLABS + COEFN + IDX + CMP + CINV;
    // A-tile pipeline depth: three buffers (A(t+2) in flight while A(t) feeds the MFMAs) when the
    // LDS budget allows, two otherwise
    // broadcast V rows (NV = 0 with coefficients: one R x D table for every row) staged in LDS once, so the
    // epilogue never issues a register-destination global load (its vmcnt wait would drain the DMAs)
    constexpr int BV = (NV == 0 && HAS_COEF) ? CFN * D : 0;
    constexpr int NBUF = (3 * A_FLOATS + NW * WF + 3 * TR + BV) * 4 <= 160 * 1024 ? 3 : 2;
    constexpr int PD = NBUF - 1;                       // prefetch distance in tiles
    constexpr int LDSF = NBUF * A_FLOATS + NW * WF + NBUF * TR + BV;
    static_assert(LDSF * 4 <= 160 * 1024, "LDS budget");
    auto soff = [](int r) { return r == 0 ? 0 : SLAB + (r - 1) * SLABC; };   // slab r of a wave
    __shared__ __attribute__((aligned(16))) float lds[LDSF];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool late = wave >= 4;         // staggered half
    const int i = lane & 31, h = lane >> 5;
    const int c0 = wave * 32;
    float* bufA = lds;
    float* slabw = lds + NBUF * A_FLOATS + wave * WF;          // slab 0 [32][32], slabs r >= 1 [CAPV][32]
    float* coefw = slabw + SLABS;                              // [32][R]
    float* cinvw = slabw + WF - CINV;                          // [32] (X3)
    float* rowinv = lds + NBUF * A_FLOATS + NW * WF;           // [NBUF][TR] (X3)
    float* bvl = rowinv + NBUF * TR;                           // [CFN][D] broadcast V rows (BV)
    const int R = p.R;

    // weights: exact f32 (breg, B[kk][c0+i] for 4 k-steps of 32x32x2 per ds_read) or, X3, the
    // hi / lo fp16 planes of the column-scaled weights, k = 16q + 8h + e for k-step q
    float breg[X3 ? 1 : D / 2];
    f16x8 bhi[X3 ? D / 16 : 1], blo[X3 ? D / 16 : 1];
    if constexpr (!X3) {
#pragma unroll
        for (int s = 0; s < D / 2; ++s) {
            const int kk = 8 * (s >> 2) + 4 * h + (s & 3);
            breg[s] = p.b_trans ? p.B[(c0 + i) * D + kk] : p.B[kk * D + c0 + i];
        }
    } else if constexpr (BF) {
        // bf16 has fp32's exponent range: no scales; W = hi + lo, hi = bf16(W), lo = bf16(W - hi)
#pragma unroll
        for (int q = 0; q < D / 16; ++q) {
            bf16x8 hv, lv;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = 16 * q + 8 * h + e;
                const float w = p.b_trans ? p.B[(c0 + i) * D + k] : p.B[k * D + c0 + i];
                hv[e] = (__bf16)w;
                lv[e] = (__bf16)(w - (float)hv[e]);
            }
            bhi[q] = __builtin_bit_cast(f16x8, hv);
            blo[q] = __builtin_bit_cast(f16x8, lv);
        }
    } else {
        auto bval = [&](int k) __attribute__((always_inline)) { return p.b_trans ? p.B[(c0 + i) * D + k] : p.B[k * D + c0 + i]; };
        float cm = 0.f;
        for (int q = 0; q < D / 16; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e) cm = fmaxf(cm, fabsf(bval(16 * q + 8 * h + e)));
        cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
        const float cs = pow2_scale(cm);
        if (h == 0) cinvw[i] = pow2_inv(cs);
#pragma unroll
        for (int q = 0; q < D / 16; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                _Float16 hi, lo;
                split16(bval(16 * q + 8 * h + e) * cs, hi, lo);
                bhi[q][e] = hi;
                blo[q][e] = lo;
            }
    }
    // X3: the wave converts its own ROWS_PER_WAVE rows of A buffer bb in place, fp32 row ->
    // [hi plane 512 B | lo plane 512 B] (k-natural order), and records 1/scale per row
    auto convert_rows = [&](int bb) __attribute__((always_inline)) {
        if constexpr (X3 && !BF) {
            if (p.planes & IDDGCN_PLANES_A) {   // rows arrive split (fixed scale)
                if (lane < ROWS_PER_WAVE) rowinv[bb * TR + wave * ROWS_PER_WAVE + lane] = PLANE_INV;
                return;
            }
            float* base = bufA + bb * A_FLOATS;
            f32x4 x[ROWS_PER_WAVE];
            float m[ROWS_PER_WAVE];
#pragma unroll
            for (int j = 0; j < ROWS_PER_WAVE; ++j) {
                x[j] = ld4(base + (wave * ROWS_PER_WAVE + j) * LDA + lane * 4);
                m[j] = fmaxf(fmaxf(fabsf(x[j][0]), fabsf(x[j][1])), fmaxf(fabsf(x[j][2]), fabsf(x[j][3])));
            }
            wave_max4(m);
#pragma unroll
            for (int j = 0; j < ROWS_PER_WAVE; ++j) {
                const int r = wave * ROWS_PER_WAVE + j;
                const float s = pow2_scale(m[j]);
                f16x4 hv, lv;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    _Float16 hi, lo;
                    split16_same(x[j][e] * s, hi, lo);
                    hv[e] = hi;
                    lv[e] = lo;
                }
                char* rowp = reinterpret_cast<char*>(base + r * LDA);
                *reinterpret_cast<f16x4*>(rowp + plane_off(lane * 4)) = hv;        // the planes layout
                *reinterpret_cast<f16x4*>(rowp + plane_off(lane * 4) + 64) = lv;
                if (lane == 0) rowinv[bb * TR + r] = pow2_inv(s);
            }
        }
    };

    const long long ntiles = ((long long)p.M + TR - 1) / TR;
    const long long t_beg = (long long)blockIdx.x * p.tiles_per_block;
    long long t_end = t_beg + p.tiles_per_block;
    if (t_end > ntiles) t_end = ntiles;
    if (t_beg >= t_end) return;
    const long long Mlast = (long long)p.M - 1;
    auto clampe = [&](long long e) __attribute__((always_inline)) { return e > Mlast ? Mlast : e; };

    // ---- row indices of the next tile: DMA'd into a wave-private LDS slot -------------
    int* idxw = reinterpret_cast<int*>(coefw + COEFN);         // [0,32) v_idx, [32,64) coef_idx
    int vslot = 0;                                               // slab row of this lane's V row
    const bool need_idx = (NV > 0 && p.v_idx) || (HAS_COEF && p.coef_idx);
    auto dma_idx = [&](long long t) __attribute__((always_inline)) {
        if (!need_idx || t >= t_end) return;
        const int* g = p.v_idx ? p.v_idx : p.coef_idx;          // valid dummy for unused lanes
        if (lane < 32) {
            if (NV > 0 && p.v_idx) g = p.v_idx + clampe(t * TR + lane);
        } else if (HAS_COEF && p.coef_idx) {
            g = p.coef_idx + clampe(t * TR + lane - 32);
        }
        __builtin_amdgcn_global_load_lds((gbl_vptr)g, (lds_vptr)idxw, 4, 0, 0);
    };
    // A rows of tile t into buffer b.  Gathered rows (a_idx, an API-only form: the training step never
    // gathers A) load their 4 indices synchronously inside this uniform branch, so no register-destination
    // load is ever left in flight across the pipelined LDS-DMA code (the compiler would otherwise guard
    // its result with a vmcnt(0) that also drains every DMA in flight).
    auto dma_A = [&](long long t, int b) __attribute__((always_inline)) {
        int sa[ROWS_PER_WAVE];
        if (p.a_idx) {
            const int v = lane < ROWS_PER_WAVE ? p.a_idx[clampe(t * TR + wave * ROWS_PER_WAVE + lane)] : 0;
#pragma unroll
            for (int j = 0; j < ROWS_PER_WAVE; ++j) sa[j] = __builtin_amdgcn_readlane(v, j);
        }
        if constexpr (BF) {
            // two 512-B bf16 rows per full-wave DMA: lane i -> row r0 + (i >> 5), LDS chunk i & 31 of its slot,
            // global chunk (i & 31) ^ (row & 15)
#pragma unroll
            for (int j = 0; j < ROWS_PER_WAVE / 2; ++j) {
                const int r0 = wave * ROWS_PER_WAVE + 2 * j;
                const int r = r0 + (lane >> 5);
                const long long src = p.a_idx ? (long long)((lane >> 5) ? sa[2 * j + 1] : sa[2 * j]) : clampe(t * TR + r);
                const char* g = reinterpret_cast<const char*>(p.A) + src * D * 2 + ((lane & 31) ^ (r & 15)) * 16;
                __builtin_amdgcn_global_load_lds((gbl_vptr)g, (lds_vptr)(bufA + b * A_FLOATS + r0 * LDA), 16, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < ROWS_PER_WAVE; ++j) {
                const int r = wave * ROWS_PER_WAVE + j;
                const long long e = clampe(t * TR + r);
                const long long src = p.a_idx ? (long long)sa[j] : e;
                const float* g = p.A + src * D + lane * 4;
                __builtin_amdgcn_global_load_lds((gbl_vptr)g, (lds_vptr)(bufA + b * A_FLOATS + r * LDA), 16, 0, 0);
            }
        }
    };
    // Slabs are [32 rows][32 cols] with the 16-B column groups of row r XOR-swizzled by
    // (r >> 1) & 7: the DMA (lane-linear destination) picks the swizzled source column, so
    // both the per-row epilogue reads and the row-major store reads are conflict-free.
    // V slabs hold only the tile's DISTINCT V rows (consecutive rows with the same v_idx form
    // a run; tail-sorted edges give 1-2 runs per tile): a ballot over the 32 row indices finds
    // the run starts, the starts' indices are compacted into a wave-private list, and
    // ceil(u / 8) DMA instructions per relation fetch the u distinct rows.  Each lane keeps the
    // slot of its row for the epilogue (vslot).
    int* cmpw = idxw + r3::IDX;
    auto dma_slabs = [&](long long t) __attribute__((always_inline)) {
        if (NV > 0) {
            int vi = 0;
            bool start = false;
            if (lane < 32) {
                const long long e = clampe(t * TR + lane);
                vi = p.v_idx ? idxw[lane] : (int)e;
                const int prev = p.v_idx ? idxw[lane > 0 ? lane - 1 : 0] : (int)e - 1;
                start = lane == 0 || vi != prev;
            }
            const unsigned long long m = __ballot(start);
            const int u = __popcll(m);
            vslot = __popcll(m & ((2ull << (lane & 31)) - 1)) - 1;
            if (start) cmpw[vslot] = vi;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (SLOTV) {
                const int un = u < CAPN ? u : CAPN;          // rows past CAPN are read from L2 in the epilogue
                const int rl = (lane >> 3) & (NV - 1);       // this lane's relation (past R: relation 0, never read)
                // element offset of this lane's relation row and 16-B group, 64-bit: (R-1)·v_rel_stride passes
                // 2^32 elements at R = 8, D = 256 from N > 2.1M
                const long long loff = (long long)(rl < R ? rl : 0) * p.v_rel_stride + c0;
                for (int kb = 0; kb < un; kb += RPI) {
                    const int slot = kb + lane / (NV * 8);
                    const int g = (lane & 7) ^ (slot & 7);
                    // RPI = 1: one row per instruction, its index wave-uniform (a scalar base)
                    const int vr = RPI == 1 ? __builtin_amdgcn_readfirstlane(cmpw[kb]) : cmpw[slot < un ? slot : un - 1];
                    const float* gp = p.V + (long long)vr * D + (loff + 4 * g);
                    __builtin_amdgcn_global_load_lds((gbl_vptr)gp, (lds_vptr)(slabw + SLAB + kb * NV * 32), 16, 0, 0);
                }
            } else
            for (int kb = 0; kb < u; kb += 8) {
                const int row = kb + (lane >> 3);
                const int g = (lane & 7) ^ ((row >> 1) & 7);
                const long long v = cmpw[row < u ? row : u - 1];
#pragma unroll
                for (int r = 0; r < NV; ++r) {
                    if constexpr (WIDE) {
                        if (r >= R) break;
                    }
                    if constexpr (CAPPED) {
                        // capped slab: rows past CAPV stay unwritten (precondition broken: stay in bounds)
                        if (r > 0 && row >= CAPV) continue;
                    }
                    const float* gp = p.V + r * p.v_rel_stride + v * D + c0 + g * 4;
                    __builtin_amdgcn_global_load_lds((gbl_vptr)gp, (lds_vptr)(slabw + soff(r) + kb * 32), 16, 0, 0);
                }
            }
        }
        if (AUX) {
            if constexpr (BF) {      // bf16 sigma' rows: [32 rows][32 bf16], 64 B per row, 16 rows per DMA
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int row = 16 * k + (lane >> 2);
                    const long long e = clampe(t * TR + row);
                    const char* gp = reinterpret_cast<const char*>(p.aux) + (e * D + c0 + (lane & 3) * 8) * 2;
                    __builtin_amdgcn_global_load_lds((gbl_vptr)gp, (lds_vptr)(slabw + soff(AUXS) + k * 256), 16, 0, 0);
                }
            } else {
                // the wave's 128 B of each row: fp32 columns c0..c0+31 (logical 16-B group g = columns
                // c0 + 4g..4g+3) or, planes rows (IDDGCN_PLANES_AUX), column block c0/32 (g < 4: hi of columns
                // c0 + 8g..8g+7, g >= 4: lo of columns c0 + 8(g-4)..)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int row = 8 * k + (lane >> 3);
                    const int g = (lane & 7) ^ ((row >> 1) & 7);
                    const long long e = clampe(t * TR + row);
                    const float* gp = p.aux + e * D + c0 + g * 4;
                    __builtin_amdgcn_global_load_lds((gbl_vptr)gp, (lds_vptr)(slabw + soff(AUXS) + k * 256), 16, 0, 0);
                }
            }
        }
        if (HAS_COEF && COEF_WIDE && (R == 4 || R == 8) && !p.coef_idx) {
            // per-edge coefficients (no coef_idx): the tile's 32 x R values are one contiguous block, one
            // 16-B DMA per lane (R = 8: 1 instruction instead of 4, and no per-lane q / R divisions); lanes
            // past the array's end re-read its last 16 B (those rows are past M and never stored)
            const long long last = (long long)(p.M - 1) * R + R - 4;
            long long off = t * TR * R + 4 * lane;
            if (off > last) off = last;
            if (lane < 8 * R)
                __builtin_amdgcn_global_load_lds((gbl_vptr)(p.coef + off), (lds_vptr)coefw, 16, 0, 0);
        } else if (HAS_COEF) {
            // 32 x R coefficients, 64 per DMA instruction (R <= 2: one instruction)
            for (int k0 = 0; k0 < TR * R; k0 += 64) {
                const float* g = p.coef;             // lanes past 32*R read a valid dummy
                const int q = k0 + lane;
                if (q < TR * R) {
                    const int row = q / R, r = q - row * R;
                    const long long ci = p.coef_idx ? (long long)idxw[32 + row] : clampe(t * TR + row);
                    g = p.coef + ci * R + r;
                }
                __builtin_amdgcn_global_load_lds((gbl_vptr)g, (lds_vptr)(coefw + k0), 4, 0, 0);
            }
        }
    };

    // Epilogue.  The MFMA computes the transposed tile (weights as operand A), so lane (i, h)
    // holds edge row i of the tile at columns c0 + 8j + 4h + {0..3}, j = 0..3: one coefficient
    // read per lane and 16-B slab reads.  Results are staged in place in slab 0 (each lane
    // rewrites exactly the slots it read), then re-read row-major for 4 buffer_store_dwordx4
    // per wave through a per-tile buffer resource whose range check drops rows past M.
    const int sw = (i >> 1) & 7;
    constexpr int EB = BF ? 2 : 4;                     // bytes per edge-table element
    auto out_rsrc = [&](long long t) __attribute__((always_inline)) {
        const long long row0 = t * TR;
        const long long left = (long long)p.M - row0;
        const unsigned nbytes = (unsigned)((left < TR ? left : TR) * D * EB);
        return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(p.C) + row0 * D * EB, (short)0, nbytes,
                                                 0x00020000);
    };
    // stage phase: combine + activation into slab 0 (LDS only, plus the C loads of `accumulate`)
    auto epi_stage = [&](long long t, const f32x16& acc) __attribute__((always_inline)) {
        const __amdgpu_buffer_rsrc_t rc = out_rsrc(t);
        float cf[CFN];
#pragma unroll
        for (int r = 0; r < CFN; ++r) cf[r] = 0.f;
        if (HAS_COEF) {
            if constexpr (COEF_WIDE) {
#pragma unroll
                for (int r = 0; r < CFN; ++r)
                    if (r < R) cf[r] = coefw[i * R + r];
            } else if (NV == 2 || (NV == 0 && R == 2)) {
                // two scalar reads (merged into one ds_read_b64): a float2-typed LDS read here made the
                // compiler guard it with a vmcnt(0) that drained the A-tile DMA in flight
                cf[0] = coefw[i * 2];
                cf[1] = coefw[i * 2 + 1];
            } else {
                cf[0] = coefw[i];
            }
        }
        // PL backward: the planes sigma' rows share slab 0 with the fp32 staging of the output, in another
        // layout (a lane's hi / lo bytes are not the 16 B it writes back): read all four column groups first
        f16x4 aux_h[PL && AUX ? 4 : 1], aux_l[PL && AUX ? 4 : 1];
        if constexpr (PL && AUX) {
            const char* rowp = reinterpret_cast<const char*>(slabw + soff(AUXS) + i * 32);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                aux_h[j] = *reinterpret_cast<const f16x4*>(rowp + 16 * (j ^ sw) + 8 * h);
                aux_l[j] = *reinterpret_cast<const f16x4*>(rowp + 16 * ((4 + j) ^ sw) + 8 * h);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int off = i * 32 + 4 * ((2 * j + h) ^ sw);
            const int col = c0 + 8 * j + 4 * h;
            f32x4 v = {acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]};
            if constexpr (!BF) {
                if (p.accumulate)
                    v += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rc, (i * D + col) * 4, 0, 0));
            }
            if (NV > 0) {
                // (SLOTV: a slot past CAPN reads slot 0's words, then takes the L2 row below)
                const int offv = SLOTV ? SLAB + (vslot < CAPN ? vslot : 0) * NV * 32 + 4 * ((2 * j + h) ^ (vslot & 7))
                                       : vslot * 32 + 4 * ((2 * j + h) ^ ((vslot >> 1) & 7));
#pragma unroll
                for (int r = 0; r < NV; ++r) {
                    if constexpr (WIDE) {
                        if (r >= R) break;
                    }
                    f32x4 s = ld4(slabw + (SLOTV ? offv + r * 32 : soff(r) + offv));
                    if constexpr (CAPPED) {
                        // a distinct row past the slots (SLOTV) or the capped slab r >= 1: from L2
                        if ((SLOTV || r > 0) && vslot >= (SLOTV ? CAPN : CAPV)) {
                            const int vrow = cmpw[vslot];
                            typedef const __attribute__((address_space(1))) f32x4* gf4p;
                            s = *(gf4p)(p.V + r * p.v_rel_stride + (long long)vrow * D + col);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = fmaf(cf[r], s[q], v[q]);
                }
            } else if (HAS_COEF) {      // broadcast V rows (v_row_stride == 0), staged in LDS (bvl)
#pragma unroll
                for (int r = 0; r < CFN; ++r) {
                    if (r >= R) break;
                    const f32x4 s = ld4(bvl + r * D + col);
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = fmaf(cf[r], s[q], v[q]);
                }
            }
            if (p.act == IDDGCN_ACT_SIGMOID) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = sigmoid_fast(v[q]);
            } else if (AUX && p.act == IDDGCN_ACT_DSIGMOID) {
                f32x4 x;
                if constexpr (BF) {
                    x = ld4bf(reinterpret_cast<const __bf16*>(slabw + soff(AUXS)) + i * 32 + 8 * j + 4 * h);
                } else if constexpr (PL) {
                    x = from_planes4(aux_h[j], aux_l[j]);
                } else {
                    x = ld4(slabw + soff(AUXS) + off);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = v[q] * (x[q] * (1.0f - x[q]));
            }
            st4(slabw + off, v);
        }
    };
    // store phase: row-major re-read of slab 0, 4 buffer_store_dwordx4 per wave
    auto epi_store = [&](long long t) __attribute__((always_inline)) {
        const __amdgpu_buffer_rsrc_t rc = out_rsrc(t);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int row = 8 * k + (lane >> 3), cg = lane & 7;
            const f32x4 o = ld4(slabw + row * 32 + 4 * (cg ^ ((row >> 1) & 7)));
            if constexpr (BF) {
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f32_to_bf4(o)), rc,
                                                      (row * D + c0 + cg * 4) * 2, 0, 0);
            } else if constexpr (PL && !AUX) {           // IDDGCN_PLANES_C: sigmoid values in [0, 1], planes row
                f16x4 hv, lv;
                to_planes4(o, hv, lv);
                const int vo = row * 1024 + plane_off(c0 + cg * 4);      // lo: soffset 64
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, hv), rc, vo, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, lv), rc, vo, 64, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(o, rc, (row * D + c0 + cg * 4) * 4, 0, 0);
            }
        }
    };
    auto epilogue = [&](long long t, const f32x16& acc) __attribute__((always_inline)) {
        epi_stage(t, acc);
        epi_store(t);
    };

    // ---- prologue: A(t_beg), indices and epilogue slabs of t_beg, indices of t_beg+1 ------
    {
        if constexpr (BV > 0) {
            for (int q = threadIdx.x; q < BV; q += 512) {
                const int r = q / D;
                bvl[q] = r < R ? p.V[r * p.v_rel_stride + (q - r * D)] : 0.f;
            }
        }
        dma_idx(t_beg);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        dma_A(t_beg, 0);
        if constexpr (PD == 2) dma_A(t_beg + 1, 1);
        dma_slabs(t_beg);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        convert_rows(0);
        dma_idx(t_beg + 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // s_waitcnt vmcnt(n): everything but the n youngest vector-memory ops of this wave has landed
    // (LDS-DMA, loads and stores count together, in issue order)
    auto wait_newest = [&](int n) __attribute__((always_inline)) {
        if (n >= 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };

    // ---- main loop, specialised per half: LATE waves run epilogue(t-1) before MFMA(t),
    // early waves epilogue(t) after it.  Branching once per wave into two compile-time copies
    // keeps one epilogue site per copy (the register allocator sees each path separately).
    // main loop, specialised per half (early / LATE); a macro keeps breg[] a plain local array
    // (capturing it in a lambda made hipcc place it in scratch).
#define V3_MAIN_LOOP(LATE) \
    { \
        f32x16 acc; \
_Pragma("unroll") \
        for (int j = 0; j < 16; ++j) acc[j] = 0.f; \
        int b = 0, b1 = 1, b2 = 2 % NBUF;     /* buffers of tiles t, t+1, t+2 */ \
        for (long long t = t_beg; t < t_end; ++t) { \
            /* A(t+PD) into the buffer of tile t-1 (its MFMAs ended before the last barrier) */ \
            const bool more = t + PD < t_end; \
            if (more) dma_A(t + PD, PD == 2 ? b2 : b1); \
            /* ops issued so far this iteration (the youngest): the A(t+PD) rows */ \
            const int n_new = more ? (BF ? ROWS_PER_WAVE / 2 : ROWS_PER_WAVE) : 0; \
            if (LATE && t > t_beg) { \
                wait_newest(n_new);          /* slabs(t-1), idx(t) and every older op */ \
                epilogue(t - 1, acc); \
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
                dma_slabs(t); \
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
                dma_idx(t + 1); \
            } \
            if constexpr (!X3) { \
_Pragma("unroll") \
                for (int j = 0; j < 16; ++j) acc[j] = 0.f; \
                /* C4: four interleaved f32 chains (k-step q into chain q % 4, 64 k-values each), summed pairwise */ \
                /* at the end: no accumulator is read mid-chain, the chains are 4x shorter */ \
                f32x16 acc1, acc2, acc3; \
_Pragma("unroll") \
                for (int j = 0; j < 16; ++j) acc1[j] = acc2[j] = acc3[j] = 0.f; \
                const float* arow = bufA + b * A_FLOATS + i * LDA + 4 * h; \
                f32x4 a_cur = ld4(arow); \
_Pragma("unroll") \
                for (int q = 0; q < D / 8; ++q) { \
                    f32x4 a_nxt = a_cur; \
                    if (q + 1 < D / 8) a_nxt = ld4(arow + 8 * (q + 1)); \
                    f32x16& ac = !C4 ? acc : ((q & 3) == 0 ? acc : (q & 3) == 1 ? acc1 : (q & 3) == 2 ? acc2 : acc3); \
                    ac = __builtin_amdgcn_mfma_f32_32x32x2f32(breg[4 * q + 0], a_cur[0], ac, 0, 0, 0); \
                    ac = __builtin_amdgcn_mfma_f32_32x32x2f32(breg[4 * q + 1], a_cur[1], ac, 0, 0, 0); \
                    ac = __builtin_amdgcn_mfma_f32_32x32x2f32(breg[4 * q + 2], a_cur[2], ac, 0, 0, 0); \
                    ac = __builtin_amdgcn_mfma_f32_32x32x2f32(breg[4 * q + 3], a_cur[3], ac, 0, 0, 0); \
                    __builtin_amdgcn_sched_barrier(0); \
                    a_cur = a_nxt; \
                } \
                if constexpr (C4) { \
_Pragma("unroll") \
                    for (int j = 0; j < 16; ++j) acc[j] = (acc[j] + acc1[j]) + (acc2[j] + acc3[j]); \
                } \
            } else if constexpr (BF) { \
                /* bf16 A fragments straight from the row; W hi and lo, one accumulator */ \
_Pragma("unroll") \
                for (int j = 0; j < 16; ++j) acc[j] = 0.f; \
                /* row i, logical chunk 2q + h at physical chunk (2q + h) ^ (i & 15) = 2q ^ (h ^ (i & 15)) */ \
                const float* arow = bufA + b * A_FLOATS + i * LDA; \
                const int su = 4 * (h ^ (i & 15)); \
                f16x8 ah[2]; \
                ah[0] = __builtin_bit_cast(f16x8, ld4(arow + su)); \
_Pragma("unroll") \
                for (int q = 0; q < D / 16; ++q) { \
                    const int cu = q & 1; \
                    if (q + 1 < D / 16) ah[cu ^ 1] = __builtin_bit_cast(f16x8, ld4(arow + ((8 * (q + 1)) ^ su))); \
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, bhi[q]), \
                                                                  __builtin_bit_cast(bf16x8, ah[cu]), acc, 0, 0, 0); \
                    if constexpr (!W1) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, blo[q]), \
                                                                  __builtin_bit_cast(bf16x8, ah[cu]), acc, 0, 0, 0); \
                    __builtin_amdgcn_sched_barrier(0); \
                } \
            } else { \
                f32x16 acc_hi, acc_lo; \
_Pragma("unroll") \
                for (int j = 0; j < 16; ++j) acc_hi[j] = acc_lo[j] = 0.f; \
                const float* arow = bufA + b * A_FLOATS + i * LDA + 4 * h; \
                /* fragments of k-steps q and q+1 in alternating registers (no copies) */ \
                f16x8 ah[2], al[2]; \
                /* planes layout: k-step q's hi at float 32(q>>1) + 8(q&1) of the row, lo 16 floats on */ \
                ah[0] = __builtin_bit_cast(f16x8, ld4(arow)); \
                al[0] = __builtin_bit_cast(f16x8, ld4(arow + 16)); \
_Pragma("unroll") \
                for (int q = 0; q < D / 16; ++q) { \
                    const int cu = q & 1; \
                    if (q + 1 < D / 16) { \
                        const int qo = 32 * ((q + 1) >> 1) + 8 * ((q + 1) & 1); \
                        ah[cu ^ 1] = __builtin_bit_cast(f16x8, ld4(arow + qo)); \
                        al[cu ^ 1] = __builtin_bit_cast(f16x8, ld4(arow + qo + 16)); \
                    } \
                    /* A lo in the units of A hi (split16_same), W lo in 2^-11 units */ \
                    acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(bhi[q], ah[cu], acc_hi, 0, 0, 0); \
                    acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(blo[q], ah[cu], acc_lo, 0, 0, 0); \
                    acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(bhi[q], al[cu], acc_hi, 0, 0, 0); \
                    __builtin_amdgcn_sched_barrier(0); \
                } \
                /* unscale: row i (1/s_row of this buffer), columns c0+8j+4h+q (1/s_col) */ \
                const float ri = rowinv[b * TR + i]; \
_Pragma("unroll") \
                for (int j = 0; j < 4; ++j) { \
                    const f32x4 cv = ld4(cinvw + 8 * j + 4 * h); \
_Pragma("unroll") \
                    for (int q = 0; q < 4; ++q) \
                        acc[4 * j + q] = (fmaf(acc_lo[4 * j + q], 0x1p-11f, acc_hi[4 * j + q]) * ri) * cv[q]; \
                } \
            } \
            if (LATE) { \
                /* A(t+1): issued this iteration (PD 1) or before slabs(t-1) (PD 2, landed) */ \
                if (PD == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
                if (t + 1 < t_end) convert_rows(b1); \
            } else { \
                wait_newest(n_new);              /* slabs(t), idx(t+1) (and A(t+1) when PD 2) */ \
                epi_stage(t, acc); \
                if (PD == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
                if (X3 && t + 1 < t_end) convert_rows(b1); \
                epi_store(t); \
                if (t + 1 < t_end) { \
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
                    dma_slabs(t + 1); \
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
                    dma_idx(t + 2); \
                } \
            } \
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
            __builtin_amdgcn_s_barrier(); \
            asm volatile("" ::: "memory"); \
            const int bt = b; b = b1; b1 = (PD == 2) ? b2 : bt; b2 = bt; \
        } \
        if (LATE) { \
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
            epilogue(t_end - 1, acc); \
        } \
    }
    if (late) V3_MAIN_LOOP(true) else V3_MAIN_LOOP(false)
#undef V3_MAIN_LOOP
}

// ---------------------------------------------------------------------------
// TN reduction GEMM  C = A^T B  over many rows, partial per workgroup.
//   wave w: output row tile ct = w % CT (32 rows of C), k-group g = w / CT.
//   A^T fragment: lane (i,h), step s -> A_tile[2s+h][32ct+i]; B: B_tile[2s+h][32cj+i].
// ---------------------------------------------------------------------------
template <int D>
struct TN {
    static constexpr int CT = D / 32;
    static constexpr int NW = CT >= 4 ? CT : 4;
    static constexpr int G = NW / CT;
    static constexpr int TK = 32;
    static constexpr int TILE = TK * D;                   // floats per operand tile
    static constexpr int RED = (G > 1) ? (NW * CT * 16 * 64) : 0;
    static constexpr int LDS = (2 * TILE > RED) ? 2 * TILE : RED;
};

template <int D>
__global__ __launch_bounds__(TN<D>::NW * 64) void gemm_tn_kernel(long long M, long long rows_per_block,
                                                                  const float* __restrict__ A,
                                                                  const float* __restrict__ B,
                                                                  float* __restrict__ slab) {
    using C = TN<D>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS];
    float* As = lds;
    float* Bs = lds + C::TILE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ct = wave % C::CT, g = wave / C::CT;
    const int i = lane & 31, h = lane >> 5;

    f32x16 acc[C::CT];
#pragma unroll
    for (int cj = 0; cj < C::CT; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[cj][j] = 0.f;

    const long long r_beg = (long long)blockIdx.x * rows_per_block;
    long long r_end = r_beg + rows_per_block;
    if (r_end > M) r_end = M;

    for (long long row0 = r_beg; row0 < r_end; row0 += C::TK) {
        __syncthreads();
        constexpr int F4R = D / 4;
        constexpr int TOT = C::TK * F4R;
#pragma unroll
        for (int it = 0; it < TOT / (C::NW * 64); ++it) {
            const int idx = it * C::NW * 64 + threadIdx.x;
            const int r = idx / F4R, c4 = idx % F4R;
            const long long e = row0 + r;
            f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
            if (e < r_end) {
                a = ld4(A + e * D + c4 * 4);
                b = ld4(B + e * D + c4 * 4);
            }
            st4(As + r * D + c4 * 4, a);
            st4(Bs + r * D + c4 * 4, b);
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < C::TK / 2; ++s) {
            if ((s % C::G) != g) continue;
            const float a = As[(2 * s + h) * D + 32 * ct + i];
#pragma unroll
            for (int cj = 0; cj < C::CT; ++cj) {
                const float b = Bs[(2 * s + h) * D + 32 * cj + i];
                acc[cj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[cj], 0, 0, 0);
            }
        }
    }

    if (C::G > 1) {
        __syncthreads();
        // groups 1..G-1 park their accumulators in LDS, group 0 adds them in group order
        if (g > 0) {
#pragma unroll
            for (int cj = 0; cj < C::CT; ++cj)
#pragma unroll
                for (int j = 0; j < 16; ++j) lds[((wave * C::CT + cj) * 16 + j) * 64 + lane] = acc[cj][j];
        }
        __syncthreads();
        if (g == 0) {
            for (int gg = 1; gg < C::G; ++gg) {
                const int w2 = gg * C::CT + ct;
#pragma unroll
                for (int cj = 0; cj < C::CT; ++cj)
#pragma unroll
                    for (int j = 0; j < 16; ++j) acc[cj][j] += lds[((w2 * C::CT + cj) * 16 + j) * 64 + lane];
            }
        }
    }
    if (g == 0) {
        float* out = slab + (long long)blockIdx.x * D * D;
#pragma unroll
        for (int cj = 0; cj < C::CT; ++cj)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int row = 32 * ct + (j & 3) + 8 * (j >> 2) + 4 * h;
                out[row * D + 32 * cj + i] = acc[cj][j];
            }
    }
}

// ---------------------------------------------------------------------------
// TN reduction GEMM, D = 256, LDS-DMA double-buffered: the next 32-row tile of A
// and B (64 one-KiB rows) is DMA'd while the 8 waves run the current tile's
// 16 x 8 MFMAs; rows past the block's range are zero-filled with plain LDS stores.
// ---------------------------------------------------------------------------
namespace tn256 {
constexpr int D = 256, TK = 32, TILE = TK * D;          // floats per operand tile
}

__global__ __launch_bounds__(512) void gemm_tn256_dma_kernel(long long M, long long rows_per_block,
                                                             const float* __restrict__ A,
                                                             const float* __restrict__ B,
                                                             float* __restrict__ slab) {
    using namespace tn256;
    __shared__ __attribute__((aligned(16))) float lds[2 * 2 * TILE];    // [buf][A|B][TK][D]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int i = lane & 31, h = lane >> 5;

    f32x16 acc[8];
#pragma unroll
    for (int cj = 0; cj < 8; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[cj][j] = 0.f;

    const long long r_beg = (long long)blockIdx.x * rows_per_block;
    long long r_end = r_beg + rows_per_block;
    if (r_end > M) r_end = M;
    const long long nt = r_end > r_beg ? (r_end - r_beg + TK - 1) / TK : 0;

    // wave w stages rows 4w..4w+3 of both operands
    auto stage = [&](long long t, int b) {
        float* As = lds + (b * 2 + 0) * TILE;
        float* Bs = lds + (b * 2 + 1) * TILE;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = wave * 4 + j;
            const long long e = r_beg + t * TK + r;
            if (e < r_end) {
                dma_row_1k(A + e * D, As + r * D, lane);
                dma_row_1k(B + e * D, Bs + r * D, lane);
            } else {
                st4(As + r * D + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
                st4(Bs + r * D + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
            }
        }
    };

    if (nt > 0) {
        stage(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    int b = 0;
    for (long long t = 0; t < nt; ++t, b ^= 1) {
        if (t + 1 < nt) stage(t + 1, b ^ 1);
        const float* As = lds + (b * 2 + 0) * TILE;
        const float* Bs = lds + (b * 2 + 1) * TILE;
        float a_cur = As[h * D + 32 * wave + i];
        float b_cur[8];
#pragma unroll
        for (int cj = 0; cj < 8; ++cj) b_cur[cj] = Bs[h * D + 32 * cj + i];
#pragma unroll
        for (int s = 0; s < TK / 2; ++s) {
            float a_nxt = a_cur, b_nxt[8];
#pragma unroll
            for (int cj = 0; cj < 8; ++cj) b_nxt[cj] = b_cur[cj];
            if (s + 1 < TK / 2) {
                a_nxt = As[(2 * (s + 1) + h) * D + 32 * wave + i];
#pragma unroll
                for (int cj = 0; cj < 8; ++cj) b_nxt[cj] = Bs[(2 * (s + 1) + h) * D + 32 * cj + i];
            }
#pragma unroll
            for (int cj = 0; cj < 8; ++cj)
                acc[cj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur, b_cur[cj], acc[cj], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            a_cur = a_nxt;
#pragma unroll
            for (int cj = 0; cj < 8; ++cj) b_cur[cj] = b_nxt[cj];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    float* out = slab + (long long)blockIdx.x * D * D;
#pragma unroll
    for (int cj = 0; cj < 8; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int row = 32 * wave + (j & 3) + 8 * (j >> 2) + 4 * h;
            out[row * D + 32 * cj + i] = acc[cj][j];
        }
}

// ---------------------------------------------------------------------------
// TN reduction GEMM, D = 256, split-fp16 operands.  Same partial-slab contract as
// gemm_tn256_dma_kernel.  Per 32-row tile, wave w converts column block w (32 columns x 32 rows)
// of A and of B IN PLACE from the DMA'd fp32 rows (1040-B padded) into k-contiguous planes:
// segment i of block w (row i's bytes [128w, 128w+128)) becomes column 32w+i as
// [hi: 32 rows fp16 | lo: 32 rows fp16], so an MFMA fragment (8 consecutive rows of one column)
// is one ds_read_b128.  The reduction runs over rows, so scales cannot be per row: each block has
// a running power-of-two scale that only decreases (first tile: max*s in [2^14, 2^15); a later
// tile whose max would overflow lowers it and the accumulators that used it are rescaled
// exactly).  A block w is private to wave w; B block cj's scale is published in LDS with its
// planes and every wave rescales acc[cj] when it changes.  One accumulator per tile:
// hi*hi + hi*lo + lo*hi with lo = fp16(x*s - hi) (same units; a lo below the fp16 normal range
// only loses bits below 2^-38 of the block max).
// ---------------------------------------------------------------------------
namespace tn3 {
constexpr int D = 256, TK = 32, LDR = D + 4, TILE = TK * LDR;
constexpr float S_INIT = 0x1p126f;                       // pow2_scale(0): "no data yet"
}


// PA: A arrives as planes rows (IDDGCN_PLANES_A, fixed scale 2^15): no A conversion; the A fragments
// (8 consecutive rows of one column) are read straight from the row-major hi / lo planes with two
// ds_read_b64_tr_b16 each.  A rows then use a 272-float pitch (row stride = 16 banks mod 64: the four rows
// of a transposed read land on disjoint banks).
typedef short v4s16 __attribute__((vector_size(8)));
__device__ __forceinline__ f16x8 tr_frag16(const char* p0, const char* p1) {
    typedef __attribute__((address_space(3))) v4s16* l4p;
    const v4s16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)p0);
    const v4s16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)p1);
    return __builtin_shufflevector(__builtin_bit_cast(f16x4, a), __builtin_bit_cast(f16x4, b), 0, 1, 2, 3, 4, 5, 6, 7);
}
// Batched launches (TnBatch.n > 0): up to TN_BATCH independent TN GEMMs of the same form in one launch,
// blockIdx.y = entry, each with its own row range split, operands and slab region (the node-level dK_r
// and dS partials of a layer: one launch of ~256 workgroups instead of three of 256 each).
constexpr int TN_BATCH = 4;
struct TnBatch {
    int n;                                    // 0: the kernel's scalar arguments
    int nb[TN_BATCH];                         // workgroups (slabs) of each entry; the launch has max(nb)
    long long M[TN_BATCH], rpb[TN_BATCH];
    const float* A[TN_BATCH];
    const float* B[TN_BATCH];
    float* slab[TN_BATCH];
};
template <bool PA = false>
__global__ __launch_bounds__(512) void gemm_tn256_x3_kernel(long long M_, long long rpb_, const float* __restrict__ A_,
                                                            const float* __restrict__ B_, float* __restrict__ slab_,
                                                            TnBatch tb) {
    using namespace tn3;
    const bool bat = tb.n > 0;
    const int ent = bat ? (int)blockIdx.y : 0;
    if (bat && (int)blockIdx.x >= tb.nb[ent]) return;     // past this entry's slabs (whole workgroup)
    const long long M = bat ? tb.M[ent] : M_;
    const long long rows_per_block = bat ? tb.rpb[ent] : rpb_;
    const float* __restrict__ A = bat ? tb.A[ent] : A_;
    const float* __restrict__ B = bat ? tb.B[ent] : B_;
    float* __restrict__ slab = bat ? tb.slab[ent] : slab_;
    constexpr int LDRA = PA ? 272 : LDR;                 // A row pitch (floats)
    constexpr int TILE_A = TK * LDRA;
    constexpr int BUF = TILE_A + TILE;                   // one [A | B] buffer
    __shared__ __attribute__((aligned(16))) float lds[2 * BUF + 2 * 8];   // [buf][A|B][TK][pitch], sB[buf][8]
    static_assert((2 * BUF + 2 * 8) * 4 <= 160 * 1024, "LDS budget");
    float* sBpub = lds + 2 * BUF;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int i = lane & 31, h = lane >> 5;

    f32x16 acc[8];
#pragma unroll
    for (int cj = 0; cj < 8; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[cj][j] = 0.f;
    float sA = S_INIT, sBrun = S_INIT;       // running scales of the blocks this wave converts
    float curB[8];                           // scale acc[cj] is currently expressed in (B side)
#pragma unroll
    for (int cj = 0; cj < 8; ++cj) curB[cj] = S_INIT;

    const long long r_beg = (long long)blockIdx.x * rows_per_block;
    long long r_end = r_beg + rows_per_block;
    if (r_end > M) r_end = M;
    const long long nt = r_end > r_beg ? (r_end - r_beg + TK - 1) / TK : 0;

    auto stage = [&](long long t, int b) {
        float* As = lds + b * BUF;
        float* Bs = As + TILE_A;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = wave * 4 + j;
            const long long e = r_beg + t * TK + r;
            if (e < r_end) {
                dma_row_1k(A + e * D, As + r * LDRA, lane);
                dma_row_1k(B + e * D, Bs + r * LDR, lane);
            } else {                                     // zero rows (zero planes for PA)
                st4(As + r * LDRA + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
                st4(Bs + r * LDR + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
            }
        }
    };
    // convert column block `wave` of one operand tile in place; returns the block scale used
    auto convert_block = [&](float* T, float& srun, bool is_a) {
        float v[16];
        float m = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            v[r] = T[(16 * h + r) * LDR + 32 * wave + i];
            m = fmaxf(m, fabsf(v[r]));
        }
        m = wave_max(m);
        if (m * srun >= 32768.0f) {                      // lower the running scale (exact rescale)
            const float s_new = pow2_scale(m);
            if (is_a) {
                const float f = s_new * pow2_inv(srun);
#pragma unroll
                for (int cj = 0; cj < 8; ++cj) acc[cj] *= f;
            }
            srun = s_new;
        }
        f16x8 hv[2], lv[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            _Float16 hi, lo;
            split16_same(v[r] * srun, hi, lo);
            hv[r >> 3][r & 7] = hi;
            lv[r >> 3][r & 7] = lo;
        }
        char* seg = reinterpret_cast<char*>(T + i * LDR + 32 * wave);
        *reinterpret_cast<f16x8*>(seg + 32 * h) = hv[0];
        *reinterpret_cast<f16x8*>(seg + 32 * h + 16) = hv[1];
        *reinterpret_cast<f16x8*>(seg + 64 + 32 * h) = lv[0];
        *reinterpret_cast<f16x8*>(seg + 64 + 32 * h + 16) = lv[1];
    };
    auto convert = [&](int b) {
        if constexpr (!PA) convert_block(lds + b * BUF, sA, true);
        convert_block(lds + b * BUF + TILE_A, sBrun, false);
        if (lane == 0) sBpub[b * 8 + wave] = sBrun;
    };
    if constexpr (PA) sA = PLANE_S;

    if (nt > 0) {
        stage(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        convert(0);
        if (nt > 1) stage(1, 1);                     // tile 1 in flight while tile 0's MFMAs run
        __syncthreads();
    }
    // Tile t+2's DMA is issued as soon as every wave's MFMAs of tile t are done (the barrier after them
    // frees buffer b), so it is in flight during tile t+1's conversion AND its MFMAs; issued at the top of
    // the iteration instead (round 2 until here), nothing was in flight during the conversions and
    // barriers and the TN ran at the sum of its DMA time and its compute time (ablations,
    // profiles/r02/ablations/tn_abl.txt).
    int b = 0;
    for (long long t = 0; t < nt; ++t, b ^= 1) {
        // B-side scales of this tile: rescale the accumulators whose block scale dropped
#pragma unroll
        for (int cj = 0; cj < 8; ++cj) {
            const float s = sBpub[b * 8 + cj];
            if (s != curB[cj]) {
                acc[cj] *= s * pow2_inv(curB[cj]);
                curB[cj] = s;
            }
        }
        const char* Aseg = reinterpret_cast<const char*>(lds + b * BUF + i * LDRA + 32 * wave);
        const char* Bseg = reinterpret_cast<const char*>(lds + b * BUF + TILE_A + i * LDR);
        // PA: lane 4q+p of its 16-lane group addresses row 8h + q, columns 32w + 16((lane>>4)&1) + 4p (planes
        // column block w: hi at 128w + 2(column - 32w), lo 64 B on)
        const char* Atr = reinterpret_cast<const char*>(lds + b * BUF) + ((8 * h + ((lane >> 2) & 3)) * LDRA) * 4 +
                          128 * wave + 32 * ((lane >> 4) & 1) + 8 * (lane & 3);
#pragma unroll
        for (int s = 0; s < TK / 16; ++s) {
            f16x8 ah, al;
            if constexpr (PA) {
                const char* r0 = Atr + (16 * s) * LDRA * 4;
                ah = tr_frag16(r0, r0 + 4 * LDRA * 4);
                al = tr_frag16(r0 + 64, r0 + 4 * LDRA * 4 + 64);
            } else {
                ah = *reinterpret_cast<const f16x8*>(Aseg + 32 * s + 16 * h);
                al = *reinterpret_cast<const f16x8*>(Aseg + 64 + 32 * s + 16 * h);
            }
#pragma unroll
            for (int cj = 0; cj < 8; ++cj) {
                const f16x8 bh = *reinterpret_cast<const f16x8*>(Bseg + 128 * cj + 32 * s + 16 * h);
                const f16x8 bl = *reinterpret_cast<const f16x8*>(Bseg + 128 * cj + 64 + 32 * s + 16 * h);
                acc[cj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[cj], 0, 0, 0);
                acc[cj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[cj], 0, 0, 0);
                acc[cj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[cj], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // tile t+1 landed (issued one tile ago)
        __syncthreads();                                         // buffer b free
        if (t + 2 < nt) stage(t + 2, b);
        if (t + 1 < nt) {
            convert(b ^ 1);
            // the converted tile visible to every wave: LDS only (a __syncthreads here also waited for tile t+2's DMA
            // just issued, so it never overlapped tile t+1's MFMAs)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    }
    float* out = slab + (long long)blockIdx.x * D * D;
    const float ia = pow2_inv(sA);
#pragma unroll
    for (int cj = 0; cj < 8; ++cj) {
        const float ib = pow2_inv(curB[cj]);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int row = 32 * wave + (j & 3) + 8 * (j >> 2) + 4 * h;
            out[row * D + 32 * cj + i] = (acc[cj][j] * ia) * ib;
        }
    }
}

// s_waitcnt vmcnt(min(n, 15)) for a run-time, wave-uniform n: every vector-memory op of this wave but the n
// youngest has completed (LDS-DMA, loads and stores count together, in issue order)
__device__ __forceinline__ void wait_vm(int n) {
#define WVM(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    switch (n < 15 ? n : 15) {
        WVM(0) WVM(1) WVM(2) WVM(3) WVM(4) WVM(5) WVM(6) WVM(7)
        WVM(8) WVM(9) WVM(10) WVM(11) WVM(12) WVM(13) WVM(14)
        default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    }
#undef WVM
}
// TN reduction GEMM over bf16 edge tables, transposed reads (round 4; replaces gemm_tn256_bf16_kernel's in-LDS
// software transpose).  The 512-B rows of A and B land in LDS by LDS-DMA, three 32-row buffers deep; the MFMA
// fragments (8 consecutive rows of one column) come straight from the row-major rows through ds_read_b64_tr_b16.
// Round 5: the rows sit in 512-B slots with their 16-B chunks XOR-swizzled (chunk c of row r at chunk c ^ 4(r & 3)),
// so one full-wave DMA (64 lanes x 16 B) fills TWO row slots — each lane picks the global chunk that belongs at its
// LDS position — where the round-4 layout (576-B slots, the pad making the transposed reads conflict-free) needed a
// half-wave DMA per row: 4 instead of 8 DMA issues per wave per tile.  The transposed reads stay conflict-free: a
// 32-lane half reads 4 rows x 64 B, and the swizzle puts the 4 rows' 64-B pieces on the 4 different quarters of the
// 256-B bank row.  Wave w owns output rows 32w..32w+31 (columns of A) x all 256 columns (8 accumulator tiles); one
// v_mfma_f32_32x32x16_bf16 per (k-step, column tile), rows 16s..16s+15 of the tile in k-step s with the same lane
// k-order as before, so the partials are bitwise the round-4 kernel's.  One barrier per tile.
// ds_read_b64_tr_b16 issued in asm (the caller waits for it with an explicit lgkmcnt tied to the result)
__device__ __forceinline__ void tr_read_asm(v4s16& d, const char* p) {
    const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(d) : "v"(a) : "memory");
}
namespace tbf {
constexpr int D = 256, TK = 32, PT = 512, OPB = TK * PT, BUF = 2 * OPB, NBUF = 3, PD = NBUF - 1;   // 4 buffers: 10.1 vs 9.8 ms
}  // namespace tbf
__device__ __forceinline__ bf16x8 tr_frag_bf(const char* p0) {
    typedef __attribute__((address_space(3))) v4s16* l4p;
    const v4s16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)p0);
    const v4s16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)(p0 + 4 * tbf::PT));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
__global__ __launch_bounds__(512) void gemm_tn256_bf16t_kernel(long long M, long long rows_per_block,
                                                               const __bf16* __restrict__ A,
                                                               const __bf16* __restrict__ B,
                                                               float* __restrict__ slab) {
    using namespace tbf;
    static_assert(NBUF * BUF <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char lds[NBUF * BUF];     // [buf][A | B][TK][PT], chunks swizzled
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    f32x16 acc[8];
#pragma unroll
    for (int cj = 0; cj < 8; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[cj][j] = 0.f;
    const long long r_beg = (long long)blockIdx.x * rows_per_block;
    long long r_end = r_beg + rows_per_block;
    if (r_end > M) r_end = M;
    const long long nt = r_end > r_beg ? (r_end - r_beg + TK - 1) / TK : 0;
    // rows 4w .. 4w+3 of both operands of tile t into buffer bb; returns the LDS-DMA count (wave-uniform).  A full
    // tile: two DMAs per operand, each filling the slots of rows (r, r+1): lane i -> row r + (i >> 5), LDS chunk
    // i & 31, global chunk (i & 31) ^ 4((r + (i >> 5)) & 3).  The range's last, partial tile: one half-wave DMA per
    // row in range (lane i < 32 -> LDS chunk i, global chunk i ^ 4(r & 3)), fp32 zeros for the rows past it.
    auto stage = [&](long long t, int bb) __attribute__((always_inline)) {
        const long long t0 = r_beg + t * TK;
        int n = 0;
        if (t0 + TK <= r_end) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = 4 * wave + 2 * j + (lane >> 5);
                const int c = (lane & 31) ^ (4 * (r & 3));
                const long long e = t0 + r;
                char* ra = lds + bb * BUF + (4 * wave + 2 * j) * PT;
                __builtin_amdgcn_global_load_lds((gbl_vptr)(A + e * D + c * 8), (lds_vptr)ra, 16, 0, 0);
                __builtin_amdgcn_global_load_lds((gbl_vptr)(B + e * D + c * 8), (lds_vptr)(ra + OPB), 16, 0, 0);
            }
            n = 4;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = 4 * wave + j;
                const long long e = t0 + r;
                char* ra = lds + bb * BUF + r * PT;
                if (e < r_end) {
                    if (lane < 32) {
                        const int c = lane ^ (4 * (r & 3));
                        __builtin_amdgcn_global_load_lds((gbl_vptr)(A + e * D + c * 8), (lds_vptr)ra, 16, 0, 0);
                        __builtin_amdgcn_global_load_lds((gbl_vptr)(B + e * D + c * 8), (lds_vptr)(ra + OPB), 16, 0, 0);
                    }
                    n += 2;
                } else if (lane < 32) {
                    st4(reinterpret_cast<float*>(ra) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
                    st4(reinterpret_cast<float*>(ra + OPB) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
                }
            }
        }
        return n;
    };
    auto wait_newest = [&](int n) __attribute__((always_inline)) { wait_vm(n); };
    // this lane's transposed-read address: rows 8(l>>5) + x (+4: second read), x = (l>>2)&3, logical columns
    // 16((l>>4)&1) + 4(l&3) of the 32-column block blk, i.e. logical chunk 4 blk + 2((l>>4)&1) + ((l&3)>>1), at
    // physical chunk 4(blk ^ x) + 2((l>>4)&1) + ((l&3)>>1) (the +4 row has the same r & 3)
    const int xs = (lane >> 2) & 3;
    const int roff = (8 * (lane >> 5) + xs) * PT + 2 * (16 * ((lane >> 4) & 1) + 4 * (lane & 3));
    // per 16-row k-step: the A fragment and all eight B fragments read (in asm) before one tied wait, then the eight
    // MFMAs; hipcc guards the builtin transposed read (no alias information) with a vmcnt(0), which drained the DMAs
    // of the tiles in flight every k-step (round 5; same MFMA order, bitwise the same partials)
    auto mfma_tile = [&](int bb) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < TK / 16; ++s) {
            const char* base = lds + bb * BUF + 16 * s * PT + roff;
            v4s16 ta[2], tb[8][2];
            tr_read_asm(ta[0], base + 64 * (wave ^ xs));
            tr_read_asm(ta[1], base + 64 * (wave ^ xs) + 4 * PT);
#pragma unroll
            for (int cj = 0; cj < 8; ++cj) {
                tr_read_asm(tb[cj][0], base + OPB + 64 * (cj ^ xs));
                tr_read_asm(tb[cj][1], base + OPB + 64 * (cj ^ xs) + 4 * PT);
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(ta[0]), "+v"(ta[1]), "+v"(tb[0][0]), "+v"(tb[0][1]), "+v"(tb[1][0]), "+v"(tb[1][1]),
                           "+v"(tb[2][0]), "+v"(tb[2][1]), "+v"(tb[3][0]), "+v"(tb[3][1]), "+v"(tb[4][0]),
                           "+v"(tb[4][1]), "+v"(tb[5][0]), "+v"(tb[5][1]), "+v"(tb[6][0]), "+v"(tb[6][1]),
                           "+v"(tb[7][0]), "+v"(tb[7][1])::"memory");
            const bf16x8 a = __builtin_bit_cast(bf16x8, __builtin_shufflevector(ta[0], ta[1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
            for (int cj = 0; cj < 8; ++cj)
                acc[cj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    a, __builtin_bit_cast(bf16x8, __builtin_shufflevector(tb[cj][0], tb[cj][1], 0, 1, 2, 3, 4, 5, 6, 7)),
                    acc[cj], 0, 0, 0);
        }
    };
    // cnt[k]: the LDS-DMA count of the tile in buffer k (the waits below let the younger tiles' DMAs fly)
    int cnt[NBUF] = {};
    if (nt > 0) {
#pragma unroll
        for (int k = 0; k < PD; ++k) cnt[k] = k < nt ? stage(k, k) : 0;
        int younger = 0;                            // tile 0 landed: tiles 1 .. PD-1 may still fly
#pragma unroll
        for (int k = 1; k < PD; ++k) younger += cnt[k];
        wait_newest(younger);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    }
    int b = 0;
    for (long long t = 0; t < nt; ++t) {
        const int bn = (b + PD) % NBUF;             // the buffer tile t+PD goes to (read last in iteration t-1)
        cnt[bn] = t + PD < nt ? stage(t + PD, bn) : 0;
        mfma_tile(b);
        // tile t+1 landed: only tiles t+2 .. t+PD may still fly
        int younger = 0;
#pragma unroll
        for (int k = 2; k <= PD; ++k) younger += cnt[(b + k) % NBUF];
        wait_newest(younger);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        b = (b + 1) % NBUF;
    }
    float* out = slab + (long long)blockIdx.x * D * D;
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int cj = 0; cj < 8; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int row = 32 * wave + (j & 3) + 8 * (j >> 2) + 4 * h;
            out[row * D + 32 * cj + i] = acc[cj][j];
        }
}

// ---- sigma' backward + dS TN in one pass over the bf16 edge tables (round 5, config 5) --------------------------
// A layer's edge backward reads do^l and x^{l-1} twice: dS^l = x^{l-1,T} do^l (gemm_tn256_bf16t_kernel, 51.2 GB per
// config-5 launch) and dx^{l-1} = (do^l S^{l,T}) x^{l-1}(1 - x^{l-1}) written over x^{l-1} (the v3 sigma' kernel,
// 76.8 GB); both run at the box's HBM ceiling.  This kernel reads each tile once: 76.8 GB for both.
// Workgroup pair per row range (column half h = 0, 1; blockIdx 8 apart: the same XCD, so the pair's second read of a
// do tile is an L2 hit).  Workgroup h reads do (all columns) and x[:, half h] only, and writes dx[:, half h] only (the
// same bytes of x), so the in-place write never meets the other workgroup's reads:
//   * dx[:, half h]: wave w owns columns c0 = 128h + 16w .. +15; the weights S[c][k] (S^T) as a bf16 hi + lo pair are
//     operand A of v_mfma_f32_16x16x32_bf16 (64 VGPRs), the do rows operand B (ds_read_b128); lane l ends with row
//     l & 15 (+16) at columns c0 + 4(l >> 4) .. +3; epilogue x(1 - x) from the x tile, bf16 8-B stores.  Per 32 k:
//     hi then lo into one accumulator, as the v3 kernel's per-16-k pair.
//   * dS[half h rows, :]: wave w owns dS rows 128h + 32(w & 3) .. +31 (x columns) x columns 128(w >> 2) .. +127 (four
//     32 x 32 tiles, 64 VGPRs), v_mfma_f32_32x32x16_bf16 on ds_read_b64_tr_b16 fragments (8 rows of one column), as
//     gemm_tn256_bf16t_kernel; per-range partials in slab[range] (rows of half h), summed by reduce_slabs.
// Tiles of 32 rows, three buffers [do: 32 x 512 B | x half: 32 x 256 B], filled by full-wave LDS-DMAs (two do rows or
// four x half rows per instruction, 3 per wave per tile).  16-B chunk c of row r sits at c ^ stn_sw(r): the sixteen
// lanes of each ds_read_b128 group (rows l & 15, chunk 4q + (l >> 4)) hit 16 distinct chunks mod 16 (stn_sw maps rows
// {0-3, 12-15} onto pairs {2m, 2m + 1}), and the four rows of a transposed read's 32-lane half land on the four
// 64-B quarters of the bank row (stn_sw(r) >> 2 = r & 3).
namespace stn {
constexpr int D = 256, TR = 32, DPT = 512, XPT = 256, DOB = TR * DPT, XB = TR * XPT, BUF = DOB + XB,
              PD = 2, NBUF = PD + 1;     // 3 / 4 tiles ahead: 21.2 / 21.5 vs 20.8 ms
}  // namespace stn
__device__ __forceinline__ int stn_sw(int r) { return (4 * (r & 3)) ^ ((0x1320 >> (4 * ((r >> 2) & 3))) & 15); }
template <bool W1>
__global__ __launch_bounds__(512) void sigma_tn_bf16_kernel(long long M, int tiles_per_block, int n_ranges,
                                                            const __bf16* __restrict__ dO, __bf16* __restrict__ X,
                                                            const float* __restrict__ S, float* __restrict__ slab) {
    using namespace stn;
    static_assert(NBUF * BUF <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char lds[NBUF * BUF];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bx = blockIdx.x;
    const int half = (bx >> 3) & 1;
    const int range = ((bx >> 4) << 3) | (bx & 7);
    if (range >= n_ranges) return;
    const long long ntiles = (M + TR - 1) / TR;
    const long long t_beg = (long long)range * tiles_per_block;
    long long t_end = t_beg + tiles_per_block;
    if (t_end > ntiles) t_end = ntiles;            // a range past the table still writes its (zero) partial
    const int i16 = lane & 15, g = lane >> 4;
    const int c0 = 128 * half + 16 * wave;
    const int swi = stn_sw(i16);

    // S^T as operand A: column c0 + i16, k = 32q + 8g + e; W = hi + lo, hi = bf16(W), lo = bf16(W - hi)
    bf16x8 whi[8], wlo[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float w = S[(c0 + i16) * D + 32 * q + 8 * g + e];
            whi[q][e] = (__bf16)w;
            wlo[q][e] = W1 ? (__bf16)0.f : (__bf16)(w - (float)whi[q][e]);
        }
    f32x16 tacc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) tacc[j][k] = 0.f;

    // rows of tile t into buffer bb; returns the LDS-DMA count (wave-uniform).  Rows past M (the table's last tile)
    // are zeros in both operands (0 x whatever-bits could be NaN in the TN).
    auto stage = [&](long long t, int bb) __attribute__((always_inline)) -> int {
        char* base = lds + bb * BUF;
        const long long t0 = t * TR;
        if (t0 + TR <= M) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = 4 * wave + 2 * j + (lane >> 5);
                const int c = (lane & 31) ^ stn_sw(r);
                __builtin_amdgcn_global_load_lds((gbl_vptr)(dO + (t0 + r) * D + c * 8),
                                                 (lds_vptr)(base + (4 * wave + 2 * j) * DPT), 16, 0, 0);
            }
            const int r = 4 * wave + (lane >> 4);
            const int c = (lane & 15) ^ stn_sw(r);
            __builtin_amdgcn_global_load_lds((gbl_vptr)(X + (t0 + r) * D + 128 * half + c * 8),
                                             (lds_vptr)(base + DOB + 4 * wave * XPT), 16, 0, 0);
            return 3;
        }
        int n = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = 4 * wave + j;
            const long long e = t0 + r;
            if (e < M) {
                if (lane < 32)
                    __builtin_amdgcn_global_load_lds((gbl_vptr)(dO + e * D + (lane ^ stn_sw(r)) * 8),
                                                     (lds_vptr)(base + r * DPT), 16, 0, 0);
                if (lane < 16)
                    __builtin_amdgcn_global_load_lds((gbl_vptr)(X + e * D + 128 * half + (lane ^ stn_sw(r)) * 8),
                                                     (lds_vptr)(base + DOB + r * XPT), 16, 0, 0);
                n += 2;
            } else {
                if (lane < 32) st4(reinterpret_cast<float*>(base + r * DPT) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
                if (lane < 16) st4(reinterpret_cast<float*>(base + DOB + r * XPT) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
            }
        }
        return n;
    };
    // transposed-read lane geometry (gemm_tn256_bf16t_kernel's): rows 8(l >> 5) + xs (+4: second read), logical chunk
    // 4 blk + colq of the 32-column block blk, byte 8(l & 1) in it
    const int xs = (lane >> 2) & 3;
    const int colq = 2 * ((lane >> 4) & 1) + ((lane & 3) >> 1);
    const int cb = 8 * (lane & 1);
    const int wb = wave & 3, cbase = 4 * (wave >> 2);
    auto mfma_tile = [&](int bb, f32x4 (&sacc)[2]) __attribute__((always_inline)) {
        const char* dob = lds + bb * BUF;
        const char* xb = dob + DOB;
        // sigma': do rows x S^T, k-step q's fragments of both row blocks loaded one step ahead
        sacc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
        sacc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
        bf16x8 bv[2][2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
            bv[0][rb] = *reinterpret_cast<const bf16x8*>(dob + (16 * rb + i16) * DPT + 16 * (g ^ swi));
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int cu = q & 1;
            if (q + 1 < 8) {
#pragma unroll
                for (int rb = 0; rb < 2; ++rb)
                    bv[cu ^ 1][rb] = *reinterpret_cast<const bf16x8*>(dob + (16 * rb + i16) * DPT +
                                                                      16 * ((4 * (q + 1) + g) ^ swi));
            }
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                sacc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi[q], bv[cu][rb], sacc[rb], 0, 0, 0);
                if constexpr (!W1)
                    sacc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo[q], bv[cu][rb], sacc[rb], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // dS: x[:, half]^T do, both 16-row k-steps' fragments read before one wait (-1.5% against a wait per k-step),
        // then four column tiles each.  The transposed reads are issued in asm with an explicit tied wait: hipcc guards
        // the builtin form (no alias information) with a vmcnt(0), i.e. it drained the tile t + 2 DMAs issued at the top
        // of the iteration
        __builtin_amdgcn_sched_barrier(0);
        {
            v4s16 ta[2][2], tb[2][4][2];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int ra = 16 * s + 8 * (lane >> 5) + xs, rq = ra + 4;
                tr_read_asm(ta[s][0], xb + ra * XPT + 16 * ((4 * wb + colq) ^ stn_sw(ra)) + cb);
                tr_read_asm(ta[s][1], xb + rq * XPT + 16 * ((4 * wb + colq) ^ stn_sw(rq)) + cb);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int blk = cbase + j;
                    tr_read_asm(tb[s][j][0], dob + ra * DPT + 16 * ((4 * blk + colq) ^ stn_sw(ra)) + cb);
                    tr_read_asm(tb[s][j][1], dob + rq * DPT + 16 * ((4 * blk + colq) ^ stn_sw(rq)) + cb);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(ta[0][0]), "+v"(ta[0][1]), "+v"(ta[1][0]), "+v"(ta[1][1]), "+v"(tb[0][0][0]),
                           "+v"(tb[0][0][1]), "+v"(tb[0][1][0]), "+v"(tb[0][1][1]), "+v"(tb[0][2][0]),
                           "+v"(tb[0][2][1]), "+v"(tb[0][3][0]), "+v"(tb[0][3][1]), "+v"(tb[1][0][0]),
                           "+v"(tb[1][0][1]), "+v"(tb[1][1][0]), "+v"(tb[1][1][1]), "+v"(tb[1][2][0]),
                           "+v"(tb[1][2][1]), "+v"(tb[1][3][0]), "+v"(tb[1][3][1])::"memory");
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const bf16x8 a = __builtin_bit_cast(bf16x8, __builtin_shufflevector(ta[s][0], ta[s][1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        a, __builtin_bit_cast(bf16x8, __builtin_shufflevector(tb[s][j][0], tb[s][j][1], 0, 1, 2, 3, 4, 5, 6, 7)),
                        tacc[j], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    // epilogue: dx = acc x(1 - x) (the v3 kernel's order), bf16 over the x rows of this half; rows past M dropped by the
    // buffer range.  Returns its store count.
    auto epilogue = [&](long long t, int bb, const f32x4 (&sacc)[2]) __attribute__((always_inline)) -> int {
        const char* xb = lds + bb * BUF + DOB;
        const long long row0 = t * TR;
        const long long left = M - row0;
        const unsigned nbytes = (unsigned)((left < TR ? left : TR) * D * 2);
        const __amdgpu_buffer_rsrc_t rc =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(X) + row0 * D * 2, (short)0, nbytes, 0x00020000);
        const int xc = (2 * wave + (g >> 1)) ^ swi;          // x half chunk of columns 16w + 4g .. +3 (row & 15 = i16)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int r = 16 * rb + i16;
            const f32x4 x = bf4_to_f32(*reinterpret_cast<const bf16x4*>(xb + r * XPT + 16 * xc + 8 * (g & 1)));
            f32x4 v = sacc[rb];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = v[q] * (x[q] * (1.0f - x[q]));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f32_to_bf4(v)), rc, (r * D + c0 + 4 * g) * 2,
                                                  0, 0);
        }
        return 2;
    };

    // PD tiles in flight ahead of the one computed; per iteration it = t - t_beg the wave issues the DMAs of tile t + PD
    // and then the stores of tile t (the prologue counts as iterations -PD .. -1, DMAs only), so the ops younger than
    // tile t + 1's DMAs are the stores of their iteration and everything of the PD - 1 iterations after it
    if (t_beg < t_end) {
        int dc[PD], sc[PD];
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            dc[k] = t_beg + k < t_end ? stage(t_beg + k, k) : 0;
            sc[k] = 0;
        }
        int younger = 0;
#pragma unroll
        for (int k = 1; k < PD; ++k) younger += dc[k];
        wait_vm(younger);                          // tile t_beg landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
        f32x4 sacc[2];
        int b = 0;
        for (long long t = t_beg; t < t_end; ++t) {
            const int it = (int)(t - t_beg);
            const int slot = it % PD;               // iteration it - PD's entries, no longer needed
            dc[slot] = t + PD < t_end ? stage(t + PD, (b + PD) % NBUF) : 0;
            mfma_tile(b, sacc);
            sc[slot] = epilogue(t, b, sacc);
            int y = sc[(it + 1) % PD];              // iteration it + 1 - PD: issued tile t + 1's DMAs, then stores
#pragma unroll
            for (int j = 2; j <= PD; ++j) {
                const int s2 = (it + j) % PD;       // iterations it + 2 - PD .. it
                y += dc[s2] + sc[s2];
            }
            wait_vm(y);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            b = (b + 1) % NBUF;
        }
    }
    float* out = slab + (long long)range * D * D;
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int row = 128 * half + 32 * wb + (k & 3) + 8 * (k >> 2) + 4 * h;
            out[row * D + 32 * (cbase + j) + i] = tacc[j][k];
        }
}

// ---------------------------------------------------------------------------
// bf16x3 operands (IDDGCN_GEMM_BF16X3), D = 256.  Every fp32 operand value x is the EXACT sum of three
// bf16 values:  b0 = bf16_rne(x), b1 = bf16_rne(x - b0), b2 = (x - b0) - b1.  Each difference is exact in
// fp32 and an fp32 significand has 24 bits = 3 x 8, so b2 is exact (while x is above ~2^-110, where b2 would
// go subnormal).  A product a*w takes the six piece products of order >= 2^-16:
//   a0 w0 | a0 w1 + a1 w0 | a1 w1 + a0 w2 + a2 w0
// on bf16 MFMAs (bf16 x bf16 products are exact, accumulation fp32); the dropped a1 w2 + a2 w1 + a2 w2 are at
// most 2^-23 |a w| (|a1| <= 2^-8 |a|, |a2| <= 2^-16 |a|), the size of fp32's own rounding of one product.
// MFMA cost: 6 x v_mfma_f32_16x16x32_bf16 (16 cycles) per 32 k-values against 16 x v_mfma_f32_32x32x2_f32
// (64 cycles) per 32 k-values x 2 column halves in the exact mode: 2.7x the exact mode's rate per flop.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void split3(float x, __bf16& b0, __bf16& b1, __bf16& b2) {
    b0 = (__bf16)x;
    const float r1 = x - (float)b0;
    b1 = (__bf16)r1;
    b2 = (__bf16)(r1 - (float)b1);
}
// Two values at a time: one v_cvt_pk_bf16_f32 rounds both, the pair's dword is unpacked back to fp32 by a
// shift (low) and a mask (high), then the two exact subtractions; 5.5 VALU per value instead of the 7.5 of
// per-value conversions followed by a packing conversion.  Same values as split3 (RNE both ways).
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned cvt_pk_bf16(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}
__device__ __forceinline__ void split3x2(float x0, float x1, unsigned& p0, unsigned& p1, unsigned& p2) {
    p0 = cvt_pk_bf16(x0, x1);
    const float r0 = x0 - __builtin_bit_cast(float, p0 << 16);
    const float r1 = x1 - __builtin_bit_cast(float, p0 & 0xffff0000u);
    p1 = cvt_pk_bf16(r0, r1);
    const float s0 = r0 - __builtin_bit_cast(float, p1 << 16);
    const float s1 = r1 - __builtin_bit_cast(float, p1 & 0xffff0000u);
    p2 = cvt_pk_bf16(s0, s1);
}
__device__ __forceinline__ void split3x4(const f32x4& v, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
    unsigned a0, b0, c0, a1, b1, c1;
    split3x2(v[0], v[1], a0, b0, c0);
    split3x2(v[2], v[3], a1, b1, c1);
    const u32x2 a = {a0, a1}, b = {b0, b1}, c = {c0, c1};
    p0 = __builtin_bit_cast(bf16x4, a);
    p1 = __builtin_bit_cast(bf16x4, b);
    p2 = __builtin_bit_cast(bf16x4, c);
}
// a staged fp32 row of 256 values (bytes [0, 1024) of `row`) -> its three bf16 planes in place: plane j at
// bytes [512 j, 512 j + 512), column k at byte 2k of its plane.  The wave's one ds_read_b128 of the whole row
// precedes (data dependence) the stores that overwrite it.
__device__ __forceinline__ void planes_from3(const f32x4& x, char* row, int lane) {
    bf16x4 p0, p1, p2;
    split3x4(x, p0, p1, p2);
    *reinterpret_cast<bf16x4*>(row + lane * 8) = p0;
    *reinterpret_cast<bf16x4*>(row + 512 + lane * 8) = p1;
    *reinterpret_cast<bf16x4*>(row + 1024 + lane * 8) = p2;
}
__device__ __forceinline__ void row_to_planes3(char* row, int lane) {
    planes_from3(ld4(reinterpret_cast<const float*>(row) + lane * 4), row, lane);
}

// ---- row GEMM, bf16x3 operands: C = epilogue(A B) over T rows --------------------------------------------
// The 256 x 256 weight as three bf16 planes is 384 KiB: it cannot live in one CU's registers beside
// anything else, so each workgroup owns ONE column half (128 columns, 192 KiB of planes = 96 VGPRs per lane
// in each of 8 waves, 16 columns per wave).  The two halves of a row range run on workgroups 8 apart, i.e.
// on the same XCD (workgroup b -> XCD b mod 8), so the second workgroup's read of an A tile hits L2.
//   * MFMA v_mfma_f32_16x16x32_bf16 with the weight planes as operand A (16 columns x 32 k) and the A tile
//     as operand B: lane l ends with edge rows l&15 and 16 + (l&15), columns c0 + 4(l>>4) .. +3.
//   * A tiles (32 rows) arrive by LDS-DMA into 1568-B row slots and each wave converts its 4 rows in place
//     to the three planes; fragment reads are ds_read_b128 (row l&15 at k-chunk l>>4: the 1568-B pitch,
//     8 banks mod 64, makes every 16-lane group of the read conflict-free).
//   * accumulators: a0 w0 in one, the five smaller products in a second (fp32), summed at the end.
//   * epilogue as the v3 kernel: gathered P_r[t] rows (the tile's distinct tails), per-edge coefficients
//     and sigma' rows (or, accumulating, the old C rows) DMA'd into wave-private slabs ([32][16] fp32, XOR-swizzled 16-B groups); waves 4-7 run
//     the epilogue of tile t-1 while waves 0-3 run tile t's MFMAs on the same SIMDs; one barrier per tile.
__device__ __forceinline__ unsigned lds_u32(const void* p) {
    return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}
namespace rb3 {
constexpr int D = 256, NW = 8, TR = 32, CWG = 128, CWV = 16;
constexpr int PITCH = 1568;                 // A row slot: three 512-B planes + 32 B
constexpr int ABYTES = TR * PITCH;          // 50,176 B per A buffer (two buffers)
constexpr int RPW = TR / NW;                // A rows each wave stages and converts
constexpr int SLAB = TR * CWV;              // floats of a [32 rows][16 columns] slab
}  // namespace rb3
// float offset of (slot, 16-B column group g) in a [32][16] slab: groups XOR (-(slot / 4)) & 3, so the
// epilogue's ds_read_b128 (slot l&15 [+16], group l>>4) is conflict-free in each of its four lane groups
__device__ __forceinline__ int slab16_off(int slot, int g) { return slot * 16 + 4 * (g ^ ((-(slot >> 2)) & 3)); }

template <int NV, bool AUX, bool BC = false>
__global__ __launch_bounds__(512) void rowgemm256_b3_kernel(RowGemmP p, int n_ranges) {
    using namespace rb3;
    static_assert(NV >= 0 && NV <= 2 && !(NV > 0 && AUX), "b3: gathered forward (NV = R = 1, 2), sigma' backward, plain");
    static_assert(!BC || NV == 0, "BC: one broadcast V row per relation (R <= 2), e.g. dz W_a^T");
    constexpr int NSL = NV + (AUX ? 1 : 0);
    constexpr int WF = NSL * SLAB + 64 + 64 + 32;               // slabs, coef [32][R], idx [64], cmp [32]
    constexpr int LDSB = 2 * ABYTES + NW * WF * 4;
    static_assert(LDSB <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char lds[LDSB];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int i = lane & 15, g = lane >> 4;
    const int bx = blockIdx.x;
    const int half = (bx >> 3) & 1;
    const int range = ((bx >> 4) << 3) | (bx & 7);
    if (range >= n_ranges) return;
    const int c0 = half * CWG + wave * CWV;
    float* slabw = reinterpret_cast<float*>(lds + 2 * ABYTES) + wave * WF;
    float* coefw = slabw + NSL * SLAB;
    int* idxw = reinterpret_cast<int*>(coefw + 64);
    int* cmpw = idxw + 64;

    const long long ntiles = ((long long)p.M + TR - 1) / TR;
    const long long t_beg = (long long)range * p.tiles_per_block;
    long long t_end = t_beg + p.tiles_per_block;
    if (t_end > ntiles) t_end = ntiles;
    if (t_beg >= t_end) return;
    const long long Mlast = (long long)p.M - 1;
    auto clampe = [&](long long e) __attribute__((always_inline)) { return e > Mlast ? Mlast : e; };

    // weight planes: k-step q (32 k), lane l: column c0 + (l&15), k = 32q + 8(l>>4) + e
    bf16x8 w0[8], w1[8], w2[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = 32 * q + 8 * g + e;
            const float wv = p.b_trans ? p.B[(c0 + i) * D + k] : p.B[k * D + c0 + i];
            __bf16 a, b, c;
            split3(wv, a, b, c);
            w0[q][e] = a;
            w1[q][e] = b;
            w2[q][e] = c;
        }

    // BC: the broadcast V rows (v_row_stride 0: the same R <= 2 rows for every output row), this lane's columns
    f32x4 vb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if constexpr (BC) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
            if (r < p.R) vb[r] = ld4(p.V + r * p.v_rel_stride + c0 + 4 * g);
    }
    // Every issue site returns its count of vector-memory ops (wave-uniform), so each wait below is the exact
    // vmcnt for what it needs, never a drain of the prefetches behind it.
    auto dma_idx = [&](long long t) __attribute__((always_inline)) -> int {
        if (NV == 0 || !p.v_idx || t >= t_end) return 0;
        const int* src = p.v_idx + (lane < 32 ? clampe(t * TR + lane) : 0);
        __builtin_amdgcn_global_load_lds((gbl_vptr)src, (lds_vptr)idxw, 4, 0, 0);
        return 1;
    };
    // Measured and not kept (round 6, profiles/r06/ab_gemm_rega_r06j.txt): the A rows through registers
    // (global_load_dwordx4, converted from there, no fp32 copy in LDS) instead of LDS-DMA: forward 3.216 vs 3.145 ms,
    // sigma' 3.212 vs 3.136, only the plain form faster (2.770 vs 2.843).  And the L2 prefetch of the A tile two tiles
    // ahead that this loop had through round 6 is gone: forward 3.277 -> 3.119 ms, sigma' 3.289 -> 3.120, plain 2.933
    // -> 2.834 (profiles/r06/ab_gemm_nopf_r06i.txt): its DMA cost the issuing waves more than the L2 hits saved.
    auto dma_A = [&](long long t, int bb) __attribute__((always_inline)) -> int {
        if (t >= t_end) return 0;
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int r = wave * RPW + j;
            const float* src = p.A + clampe(t * TR + r) * D + lane * 4;
            __builtin_amdgcn_global_load_lds((gbl_vptr)src, (lds_vptr)(lds + bb * ABYTES + r * PITCH), 16, 0, 0);
        }
        return RPW;
    };
    auto convert = [&](int bb) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < RPW; ++j) row_to_planes3(lds + bb * ABYTES + (wave * RPW + j) * PITCH, lane);
    };
    // the tile's distinct V rows (runs of equal v_idx; tail-sorted edges give 1-3 per tile) into slots 0..u-1,
    // each lane's two rows' slots (vs0: row l&15, vs1: row 16 + (l&15)); sigma' rows; coefficients
    int vs0 = 0, vs1 = 0;
    auto dma_slabs = [&](long long t) __attribute__((always_inline)) -> int {
        int n = 0;
        if constexpr (NV > 0) {
            int vi = 0;
            bool start = false;
            if (lane < 32) {
                const long long e = clampe(t * TR + lane);
                vi = p.v_idx ? idxw[lane] : (int)e;
                const int prev = p.v_idx ? idxw[lane > 0 ? lane - 1 : 0] : (int)e - 1;
                start = lane == 0 || vi != prev;
            }
            const unsigned long long m = __ballot(start);
            const int u = __popcll(m);
            vs0 = __popcll(m & ((2ull << i) - 1)) - 1;
            vs1 = __popcll(m & ((2ull << (16 + i)) - 1)) - 1;
            if (start) cmpw[__popcll(m & ((2ull << lane) - 1)) - 1] = vi;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            for (int kb = 0; kb < u; kb += 16) {
                const int slot = kb + (lane >> 2);
                const int gg = (lane & 3) ^ ((-(slot >> 2)) & 3);
                const long long v = cmpw[slot < u ? slot : u - 1];
#pragma unroll
                for (int r = 0; r < NV; ++r) {
                    const float* src = p.V + r * p.v_rel_stride + v * D + c0 + gg * 4;
                    __builtin_amdgcn_global_load_lds((gbl_vptr)src, (lds_vptr)(slabw + r * SLAB + kb * 16), 16, 0, 0);
                }
                n += NV;
            }
            // 32 x R per-edge coefficients, one 4-B DMA per lane (lanes past 32 R re-read the last value)
            const long long last = (long long)p.M * NV - 1;
            long long ci = t * TR * NV + lane;
            if (ci > last) ci = last;
            __builtin_amdgcn_global_load_lds((gbl_vptr)(p.coef + ci), (lds_vptr)coefw, 4, 0, 0);
            n += 1;
        }
        if constexpr (BC) {      // the tile's 32 x R row coefficients, one 4-B DMA per lane
            const long long last = (long long)p.M * p.R - 1;
            long long ci = t * TR * p.R + lane;
            if (ci > last) ci = last;
            __builtin_amdgcn_global_load_lds((gbl_vptr)(p.coef + ci), (lds_vptr)coefw, 4, 0, 0);
            n += 1;
        }
        if constexpr (AUX) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int slot = 16 * k + (lane >> 2);
                const int gg = (lane & 3) ^ ((-(slot >> 2)) & 3);
                const float* src = p.aux + clampe(t * TR + slot) * D + c0 + gg * 4;
                __builtin_amdgcn_global_load_lds((gbl_vptr)src, (lds_vptr)(slabw + NV * SLAB + k * 256), 16, 0, 0);
            }
            n += 2;
        }
        return n;
    };
    auto epilogue = [&](long long t, const f32x4 (&acc)[2]) __attribute__((always_inline)) -> int {
        const long long row0 = t * TR;
        const long long left = (long long)p.M - row0;
        const unsigned nbytes = (unsigned)((left < TR ? left : TR) * D * 4);
        const __amdgpu_buffer_rsrc_t rc =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(p.C) + row0 * D * 4, (short)0, nbytes, 0x00020000);
#pragma unroll
        for (int rh = 0; rh < 2; ++rh) {
            const int row = 16 * rh + i;
            f32x4 v = acc[rh];
            if constexpr (NV > 0) {
                const int vs = rh ? vs1 : vs0;
#pragma unroll
                for (int r = 0; r < NV; ++r) {
                    const float cf = coefw[row * NV + r];
                    const f32x4 s = ld4(slabw + r * SLAB + slab16_off(vs, g));
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = fmaf(cf, s[q], v[q]);
                }
            }
            if constexpr (BC) {
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if (r >= p.R) break;
                    const float cf = coefw[row * p.R + r];
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = fmaf(cf, vb[r][q], v[q]);
                }
            }
            if (AUX && p.accumulate) {
                v += ld4(slabw + NV * SLAB + slab16_off(row, g));
            } else if (p.act == IDDGCN_ACT_SIGMOID) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = sigmoid_fast(v[q]);
            } else if (AUX && p.act == IDDGCN_ACT_DSIGMOID) {
                const f32x4 x = ld4(slabw + NV * SLAB + slab16_off(row, g));
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = v[q] * (x[q] * (1.0f - x[q]));
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, rc, (row * D + c0 + 4 * g) * 4, 0, 0);
        }
        return 2;
    };
    // Measured and not kept (round 6, profiles/r06/ab_gemm_fwd_interleave_r06c.txt): the next tile's four rows converted
    // inside this tile's MFMA phase (each row's read issued with a k-step's fragment reads, its split and stores behind
    // that k-step's MFMAs): bitwise the same, forward 3.333 vs 3.278 ms, sigma' 3.334 vs 3.274, plain 2.925 vs 2.930
    auto mfma_tile = [&](int bb, f32x4 (&acc)[2]) __attribute__((always_inline)) {
        f32x4 hi0 = {0.f, 0.f, 0.f, 0.f}, lo0 = hi0, hi1 = hi0, lo1 = hi0;
        // Fragment reads in inline asm, one k-step ahead of the MFMAs that use them, each k-step's MFMAs behind an
        // s_waitcnt lgkmcnt(6) that "defines" its six fragments (so the MFMAs cannot be scheduled above it): the
        // compiler's own waits were lgkmcnt(0) right after the next k-step's loads, exposing the LDS latency once
        // per k-step (8 per tile) in a phase no partner wave covers (tools/bench_gemm.py: ~2x the MFMA time)
        const unsigned ab = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(lds + bb * ABYTES) +
                            i * PITCH + 16 * g;
        u32x4 fx[2][3], fy[2][3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#define B3_LOADQ(Q, S)                                                                                    \
        asm volatile("ds_read_b128 %0, %6 offset:%7\n\tds_read_b128 %1, %6 offset:%8\n\t"                 \
                     "ds_read_b128 %2, %6 offset:%9\n\tds_read_b128 %3, %6 offset:%10\n\t"                \
                     "ds_read_b128 %4, %6 offset:%11\n\tds_read_b128 %5, %6 offset:%12"                   \
                     : "=&v"(fx[S][0]), "=&v"(fx[S][1]), "=&v"(fx[S][2]), "=&v"(fy[S][0]), "=&v"(fy[S][1]),     \
                       "=&v"(fy[S][2])                                                                   \
                     : "v"(ab), "i"(64 * (Q)), "i"(64 * (Q) + 512), "i"(64 * (Q) + 1024),                \
                       "i"(64 * (Q) + 16 * PITCH), "i"(64 * (Q) + 16 * PITCH + 512),                      \
                       "i"(64 * (Q) + 16 * PITCH + 1024)                                                 \
                     : "memory")
        B3_LOADQ(0, 0);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int S = q & 1;
            if (q + 1 < 8) {
                switch (q) {      // the offsets are immediates: one asm per k-step
                    case 0: B3_LOADQ(1, 1); break;
                    case 1: B3_LOADQ(2, 0); break;
                    case 2: B3_LOADQ(3, 1); break;
                    case 3: B3_LOADQ(4, 0); break;
                    case 4: B3_LOADQ(5, 1); break;
                    case 5: B3_LOADQ(6, 0); break;
                    default: B3_LOADQ(7, 1); break;
                }
                asm volatile("s_waitcnt lgkmcnt(6)"
                             : "+v"(fx[S][0]), "+v"(fx[S][1]), "+v"(fx[S][2]), "+v"(fy[S][0]), "+v"(fy[S][1]),
                               "+v"(fy[S][2])::"memory");
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(fx[S][0]), "+v"(fx[S][1]), "+v"(fx[S][2]), "+v"(fy[S][0]), "+v"(fy[S][1]),
                               "+v"(fy[S][2])::"memory");
            }
            const bf16x8 x0 = __builtin_bit_cast(bf16x8, fx[S][0]), x1 = __builtin_bit_cast(bf16x8, fx[S][1]),
                         x2 = __builtin_bit_cast(bf16x8, fx[S][2]);
            const bf16x8 y0 = __builtin_bit_cast(bf16x8, fy[S][0]), y1 = __builtin_bit_cast(bf16x8, fy[S][1]),
                         y2 = __builtin_bit_cast(bf16x8, fy[S][2]);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], x2, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], y2, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[q], x0, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[q], y0, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], x1, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], y1, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], x1, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], y1, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], x0, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], y0, lo1, 0, 0, 0);
            hi0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], x0, hi0, 0, 0, 0);
            hi1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], y0, hi1, 0, 0, 0);
        }
#undef B3_LOADQ
        acc[0] = hi0 + lo0;
        acc[1] = hi1 + lo1;
    };

    // prologue: indices, A and slabs of t_beg; A converted; indices of t_beg + 1
    dma_idx(t_beg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    dma_A(t_beg, 0);
    dma_slabs(t_beg);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    convert(0);
    dma_idx(t_beg + 1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // per iteration t: A(t+1) loads; waves 4-7 run epilogue(t-1) and the slab /
    // index DMAs of t, t+1 before MFMA(t), waves 0-3 epilogue(t) and those of t+1, t+2 after it
#define B3_MAIN_LOOP(LATE)                                                                           \
    {                                                                                                \
        f32x4 acc[2];                                                                                \
        int b = 0;                                                                                   \
        for (long long t = t_beg; t < t_end; ++t) {                                                  \
            const bool more = t + 1 < t_end;                                                         \
            const int nA = dma_A(t + 1, b ^ 1);                                                      \
            int after_A = 0;                        /* ops issued after A(t+1) */                    \
            if (LATE && t > t_beg) {                                                                 \
                wait_vm(nA);                        /* slabs(t-1), idx(t) */                         \
                after_A += epilogue(t - 1, acc);                                                     \
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                   \
                after_A += dma_slabs(t);                                                             \
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                   \
                after_A += dma_idx(t + 1);                                                           \
            }                                                                                        \
            mfma_tile(b, acc);                                                                       \
            if (LATE) {                                                                              \
                if (more) {                                                                          \
                    wait_vm(after_A);                                                                \
                    convert(b ^ 1);                                                                  \
                }                                                                                    \
            } else {                                                                                 \
                wait_vm(nA);                        /* slabs(t), idx(t+1) */                         \
                after_A += epilogue(t, acc);                                                         \
                if (more) {                                                                          \
                    wait_vm(after_A);               /* A(t+1) */                                     \
                    convert(b ^ 1);                                                                  \
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                               \
                    dma_slabs(t + 1);                                                                \
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                               \
                    dma_idx(t + 2);                                                                  \
                }                                                                                    \
            }                                                                                        \
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                       \
            __builtin_amdgcn_s_barrier();                                                            \
            asm volatile("" ::: "memory");                                                           \
            b ^= 1;                                                                                  \
        }                                                                                            \
        if (LATE) {                                                                                  \
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                         \
            epilogue(t_end - 1, acc);                                                                \
        }                                                                                            \
    }
    if (wave >= 4) B3_MAIN_LOOP(true) else B3_MAIN_LOOP(false)
#undef B3_MAIN_LOOP
}

// ---- TN reduction GEMM, bf16x3 operands: C = A^T B over M rows, partial per workgroup --------------------
// Wave w owns output rows 32w..32w+31 (columns of A) x all 256 columns (8 accumulator tiles, 128 VGPRs).
// 16-row tiles of A and B (one v_mfma_f32_32x32x16_bf16 k-step) arrive by LDS-DMA into 1600-B row slots,
// three buffers deep; each wave converts its 2 rows of each operand in place to the three bf16 planes, and
// the MFMA fragments (8 consecutive rows of one column) are read with ds_read_b64_tr_b16 from the row-major
// planes (1600-B pitch = 16 banks mod 64: each 32-lane half's four rows x 64 B are conflict-free).  Six
// MFMAs per (k-step, column tile) into one fp32 accumulator, the smaller products first.  Waves 4-7 convert
// tile t+1 before their MFMAs of tile t, waves 0-3 after theirs: a SIMD's two waves overlap conversion and
// MFMA.  One barrier per tile.
namespace tb3 {
constexpr int D = 256, TK = 16, PT = 1600, OPB = TK * PT, BUF = 2 * OPB, NBUF = 3;
}  // namespace tb3
__device__ __forceinline__ bf16x8 tr_frag_b3(const char* p0) {
    typedef __attribute__((address_space(3))) v4s16* l4p;
    const v4s16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)p0);
    const v4s16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)(p0 + 4 * tb3::PT));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
// Batched (TnBatch.n > 0, as gemm_tn256_x3_kernel): blockIdx.y = entry, each entry its own operands, row split and
// slab region — a layer's node-level TNs (dS head part, dK_r) in one launch of ~256 workgroups instead of one launch
// of 256 per entry, each with its prologue, its drain and 256 partial slabs to sum.
__global__ __launch_bounds__(512) void gemm_tn256_b3_kernel(long long M_, long long rpb_, const float* __restrict__ A_,
                                                            const float* __restrict__ B_, float* __restrict__ slab_,
                                                            TnBatch tb) {
    using namespace tb3;
    const bool bat = tb.n > 0;
    const int ent = bat ? (int)blockIdx.y : 0;
    if (bat && (int)blockIdx.x >= tb.nb[ent]) return;     // past this entry's slabs (whole workgroup)
    const long long M = bat ? tb.M[ent] : M_;
    const long long rows_per_block = bat ? tb.rpb[ent] : rpb_;
    const float* __restrict__ A = bat ? tb.A[ent] : A_;
    const float* __restrict__ B = bat ? tb.B[ent] : B_;
    float* __restrict__ slab = bat ? tb.slab[ent] : slab_;
    static_assert(NBUF * BUF <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char lds[NBUF * BUF];     // [buf][A | B][TK][PT]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool late = wave >= 4;
    f32x16 acc[8];
#pragma unroll
    for (int cj = 0; cj < 8; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[cj][j] = 0.f;
    const long long r_beg = (long long)blockIdx.x * rows_per_block;
    long long r_end = r_beg + rows_per_block;
    if (r_end > M) r_end = M;
    const long long nt = r_end > r_beg ? (r_end - r_beg + TK - 1) / TK : 0;

    // rows 2w, 2w+1 of both operands of tile t into buffer bb (rows past the range as fp32 zeros); returns the
    // LDS-DMA count (wave-uniform)
    auto stage = [&](long long t, int bb) __attribute__((always_inline)) {
        int n = 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = 2 * wave + j;
            const long long e = r_beg + t * TK + r;
            char* ra = lds + bb * BUF + r * PT;
            if (e < r_end) {
                __builtin_amdgcn_global_load_lds((gbl_vptr)(A + e * D + lane * 4), (lds_vptr)ra, 16, 0, 0);
                __builtin_amdgcn_global_load_lds((gbl_vptr)(B + e * D + lane * 4), (lds_vptr)(ra + OPB), 16, 0, 0);
                n += 2;
            } else {
                st4(reinterpret_cast<float*>(ra) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
                st4(reinterpret_cast<float*>(ra + OPB) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
            }
        }
        return n;
    };
    auto convert = [&](int bb) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            char* ra = lds + bb * BUF + (2 * wave + j) * PT;
            row_to_planes3(ra, lane);
            row_to_planes3(ra + OPB, lane);
        }
    };
    auto wait_newest = [&](int n) __attribute__((always_inline)) {
        if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    // this lane's transposed-read address: rows 8(l>>5) + ((l>>2)&3) (+4: second read), columns
    // 16((l>>4)&1) + 4(l&3) of a 32-column block
    const int roff = (8 * (lane >> 5) + ((lane >> 2) & 3)) * PT + 2 * (16 * ((lane >> 4) & 1) + 4 * (lane & 3));
    // fragments by transposed reads issued in asm with tied lgkmcnt waits (round 5): hipcc guards the builtin form (no
    // alias information) with a vmcnt(0) before the first one, a drain of the tile t+2 DMAs every tile
    auto tie6 = [&](v4s16 (&f)[3][2]) __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(f[0][0]), "+v"(f[0][1]), "+v"(f[1][0]), "+v"(f[1][1]), "+v"(f[2][0]), "+v"(f[2][1])::"memory");
    };
    auto frag = [&](const v4s16 (&f)[2]) __attribute__((always_inline)) {
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(f[0], f[1], 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto mfma_tile = [&](int bb) __attribute__((always_inline)) {
        const char* pa = lds + bb * BUF + roff + 64 * wave;
        const char* pb0 = lds + bb * BUF + OPB + roff;
        v4s16 fa[3][2], fb[3][2], fn[3][2];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            tr_read_asm(fa[k][0], pa + 512 * k);
            tr_read_asm(fa[k][1], pa + 512 * k + 4 * PT);
            tr_read_asm(fb[k][0], pb0 + 512 * k);
            tr_read_asm(fb[k][1], pb0 + 512 * k + 4 * PT);
        }
        tie6(fa);
        tie6(fb);
        const bf16x8 a0 = frag(fa[0]), a1 = frag(fa[1]), a2 = frag(fa[2]);
        // B fragments of column tile cj+1 in flight during tile cj's MFMAs (two register sets: the 128
        // accumulator VGPRs leave no room for all eight tiles' fragments)
        // per tile the five smaller products start from zero and join the running sum with one fp32 add
        // (v_add_f32, round-to-nearest-even) in front of the a0 b0 MFMA: all six MFMAs chained on the running sum
        // over a block's 16k rows gave 1.46x the exact mode's fmaf-chain error (tools/bench_gemm.py)
#pragma unroll
        for (int cj = 0; cj < 8; ++cj) {
            if (cj + 1 < 8) {
                const char* pb = pb0 + 64 * (cj + 1);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    tr_read_asm(fn[k][0], pb + 512 * k);
                    tr_read_asm(fn[k][1], pb + 512 * k + 4 * PT);
                }
            }
            const bf16x8 b0 = frag(fb[0]), b1 = frag(fb[1]), b2 = frag(fb[2]);
            f32x16 c;
#pragma unroll
            for (int j = 0; j < 16; ++j) c[j] = 0.f;
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c, 0, 0, 0);
            acc[cj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[cj] + c, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (cj + 1 < 8) {
                tie6(fn);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    fb[k][0] = fn[k][0];
                    fb[k][1] = fn[k][1];
                }
            }
        }
    };

    if (nt > 0) {
        stage(0, 0);
        const int n1 = nt > 1 ? stage(1, 1) : 0;
        wait_newest(n1);
        convert(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // one compile-time copy of the loop per half (one MFMA site each: the register allocator sees each path alone)
#define TB3_LOOP(LATE)                                                               \
    {                                                                                \
        int b = 0;                                                                   \
        for (long long t = 0; t < nt; ++t) {                                         \
            const int b1 = b == 2 ? 0 : b + 1, b2 = b1 == 2 ? 0 : b1 + 1;            \
            const int n2 = t + 2 < nt ? stage(t + 2, b2) : 0;                        \
            if (LATE && t + 1 < nt) {                                                \
                wait_newest(n2);                                                     \
                convert(b1);                                                         \
            }                                                                        \
            mfma_tile(b);                                                            \
            if (!LATE && t + 1 < nt) {                                               \
                wait_newest(n2);                                                     \
                convert(b1);                                                         \
            }                                                                        \
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                       \
            __builtin_amdgcn_s_barrier();                                            \
            asm volatile("" ::: "memory");                                           \
            b = b1;                                                                  \
        }                                                                            \
    }
    if (late) TB3_LOOP(true) else TB3_LOOP(false)
#undef TB3_LOOP
    float* out = slab + (long long)blockIdx.x * D * D;
    const int i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int cj = 0; cj < 8; ++cj)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int row = 32 * wave + (j & 3) + 8 * (j >> 2) + 4 * h;
            out[row * D + 32 * cj + i] = acc[cj][j];
        }
}

// ---- sigma' backward + dS TN in one pass over the fp32 edge tables, bf16x3 operands (round 6, configs 3 / 4) ------
// The headline mode's layer-2/3 edge backward (the autodiff of IDDGCN.py:62-63,79 for x_t^{l-1} S^l):
//   dS = X^T dO (per-range partials, summed by reduce_slabs)  and  X = (dO S^T) X (1 - X) in place.
// rowgemm256_b3_kernel<0, true> (sigma') and gemm_tn256_b3_kernel (TN) ran it as two passes: both read dO and X
// (20.5 GB per config-3 layer) and each converted its operands to bf16 planes on its own.  One pass here reads each
// tile once (12.3 GB) and converts each row once per workgroup.
// Workgroup pair per row range (column half h = 0, 1; blockIdx 8 apart: the same XCD, so the pair's second read of a
// dO tile is an L2 hit), as sigma_tn_bf16_kernel: workgroup h reads dO (all columns) and X[:, half h], and writes
// dX[:, half h] over the same bytes, so the in-place write never meets the other workgroup's reads.
//   * sigma': wave w owns output columns c0 = 128h + 16w .. +15; S^T as three bf16 planes is operand A of
//     v_mfma_f32_16x16x32_bf16 (96 VGPRs), the dO planes operand B (ds_read_b128): rowgemm256_b3_kernel's six
//     products in its order, so dX is bitwise that kernel's.  Epilogue x(1 - x) with x = p0 + p1 + p2 rebuilt (exactly:
//     the pieces are an exact split) from the X planes in LDS.
//   * dS[half h rows, :]: wave w owns X columns 128h + 32(w & 3) .. +31 x dO columns 128(w >> 2) .. +127 as 2 x 8
//     16x16 tiles (64 VGPRs); v_mfma_f32_16x16x32_bf16 over the tile's 32 rows (one k-step) on ds_read_b64_tr_b16
//     fragments (T10 geometry: lane l supplies row 8(l >> 4) + ((l >> 2) & 3) (+4), columns 4(l & 3) .. +3 of a
//     16-column block); per 16x16 tile the five smaller products start from zero and join the running sum by one fp32
//     add in front of the a0 b0 MFMA (gemm_tn256_b3_kernel's accuracy form, 32 rows per join).
// LDS: two buffers of [dO: 32 x 1536 B | X half: 32 x 768 B] (147,456 B).  An fp32 dO row arrives by one full-wave
// LDS-DMA at the start of its 1536-B slot, a pair of X-half rows by one full-wave DMA across their two 768-B slots; the
// wave that DMA'd them converts them in place (all six reads before any write) to three bf16 planes (plane j at byte
// 512 j / 256 j of the slot) with 16-B chunk c of row r at c ^ stn_sw(r).  Every slot starts at bank 0, so the
// conflict analysis of sigma_tn_bf16_kernel's 512 / 256-B slots holds for the ds_read_b128 row fragments and the
// transposed reads alike.  Tile t + 1 is DMA'd while tile t computes and converted after its MFMAs, both by waves 0-3
// for their SIMD's two waves (waves 4-7: MFMAs and epilogue only); one barrier per tile.  Every LDS read of the loop
// is issued in asm with a tied lgkmcnt wait (no compiler vmcnt drain of the DMAs).
namespace st3 {
constexpr int D = 256, TR = 32, DP = 1536, XP = 768, DOB = TR * DP, XB = TR * XP, BUF = DOB + XB, NBUF = 2;
}  // namespace st3
// three transposed reads at a, a + PS, a + 2 PS (the three planes of one 4-row block).  Every multi-instruction asm
// read here marks its outputs early-clobber ("=&v"): without it the compiler may give an output the input address
// register, which the first read then overwrites (asynchronously) while the later reads still use it as address
// (tests/test_host.py::test_asm_transposed_reads_are_waited_for caught exactly that in this kernel's first build)
template <int PS>
__device__ __forceinline__ void tr_read3(v4s16 (&d)[3], unsigned a) {
    asm volatile("ds_read_b64_tr_b16 %0, %3\n\tds_read_b64_tr_b16 %1, %3 offset:%4\n\tds_read_b64_tr_b16 %2, %3 offset:%5"
                 : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2])
                 : "v"(a), "i"(PS), "i"(2 * PS)
                 : "memory");
}
__device__ __forceinline__ bf16x8 cat_tr(const v4s16& a, const v4s16& b) {
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
// bf16 element q of a packed 4-element u32x2, as fp32
__device__ __forceinline__ float bf_at(const u32x2& v, int q) {
    const unsigned w = v[q >> 1];
    return __builtin_bit_cast(float, (q & 1) ? (w & 0xffff0000u) : (w << 16));
}
__global__ __launch_bounds__(512) void sigma_tn_b3_kernel(long long M, int tiles_per_block, int n_ranges,
                                                          const float* __restrict__ dO, float* __restrict__ X,
                                                          const float* __restrict__ S, float* __restrict__ slab) {
    using namespace st3;
    static_assert(NBUF * BUF <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char lds[NBUF * BUF];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bx = blockIdx.x;
    const int half = (bx >> 3) & 1;
    const int range = ((bx >> 4) << 3) | (bx & 7);
    if (range >= n_ranges) return;
    const long long ntiles = (M + TR - 1) / TR;
    const long long t_beg = (long long)range * tiles_per_block;
    long long t_end = t_beg + tiles_per_block;
    if (t_end > ntiles) t_end = ntiles;            // a range past the table still writes its (zero) partial
    const int i16 = lane & 15, g = lane >> 4;
    const int c0 = 128 * half + 16 * wave;
    const unsigned lds0 = lds_u32(lds);
    // a lane index the compiler cannot hoist out of the loop: the per-lane LDS offsets of every phase are recomputed
    // from it there (a few VALU each) instead of being kept live across the loop, where they spilled (23 VGPRs)
    auto fresh_lane = [&]() __attribute__((always_inline)) {
        int l = lane;
        asm volatile("" : "+v"(l));
        return l;
    };

    // S^T as operand A: column c0 + i16, k = 32q + 8g + e, split exactly into three bf16 pieces
    bf16x8 w0[8], w1[8], w2[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            __bf16 a, b, c;
            split3(S[(c0 + i16) * D + 32 * q + 8 * g + e], a, b, c);
            w0[q][e] = a;
            w1[q][e] = b;
            w2[q][e] = c;
        }
    f32x4 tacc[2][8];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) tacc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

    // fp32 rows of tile t into buffer bb: dO rows 4w .. 4w+3 (one full-wave DMA each), X-half rows 4w .. 4w+3 (a pair
    // per full-wave DMA); rows past M as fp32 zeros (0 x whatever-bits could be NaN in the TN).  Returns the DMA count.
    auto stage = [&](long long t, int bb, int wave) __attribute__((always_inline)) -> int {
        const int lane = fresh_lane();
        char* base = lds + bb * BUF;
        const long long t0 = t * TR;
        if (t0 + TR <= M) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = 4 * wave + j;
                __builtin_amdgcn_global_load_lds((gbl_vptr)(dO + (t0 + r) * D + lane * 4), (lds_vptr)(base + r * DP), 16,
                                                 0, 0);
            }
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int r = 4 * wave + 2 * p;
                __builtin_amdgcn_global_load_lds(
                    (gbl_vptr)(X + (t0 + r + (lane >> 5)) * D + 128 * half + (lane & 31) * 4),
                    (lds_vptr)(base + DOB + r * XP), 16, 0, 0);
            }
            return 6;
        }
        int n = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = 4 * wave + j;
            const long long e = t0 + r;
            char* xr = base + DOB + (r & ~1) * XP + 512 * (r & 1);     // where the pair DMA would put row r
            if (e < M) {
                __builtin_amdgcn_global_load_lds((gbl_vptr)(dO + e * D + lane * 4), (lds_vptr)(base + r * DP), 16, 0, 0);
                if (lane < 32)
                    __builtin_amdgcn_global_load_lds((gbl_vptr)(X + e * D + 128 * half + lane * 4), (lds_vptr)xr, 16, 0,
                                                     0);
                n += 2;
            } else {
                st4(reinterpret_cast<float*>(base + r * DP) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
                if (lane < 32) st4(reinterpret_cast<float*>(xr) + lane * 4, f32x4{0.f, 0.f, 0.f, 0.f});
            }
        }
        return n;
    };
    // this wave's rows of buffer bb, fp32 -> three bf16 planes in place: the six 1-KiB reads first (one wait), then the
    // writes (a row's planes overwrite its own fp32 bytes and, for an X pair, the second row's)
    auto convert = [&](int bb, int wave) __attribute__((always_inline)) {
        char* base = lds + bb * BUF;
        const int lane = fresh_lane();
        u32x4 v[6];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            asm volatile("ds_read_b128 %0, %1" : "=v"(v[j]) : "v"(lds_u32(base + (4 * wave + j) * DP) + 16 * lane) : "memory");
#pragma unroll
        for (int p = 0; p < 2; ++p)
            asm volatile("ds_read_b128 %0, %1"
                         : "=v"(v[4 + p])
                         : "v"(lds_u32(base + DOB + (4 * wave + 2 * p) * XP) + 16 * lane)
                         : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5])::"memory");
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = 4 * wave + j;
            char* row = base + r * DP + 16 * ((lane >> 1) ^ stn_sw(r)) + 8 * (lane & 1);
            bf16x4 p0, p1, p2;
            split3x4(__builtin_bit_cast(f32x4, v[j]), p0, p1, p2);
            *reinterpret_cast<bf16x4*>(row) = p0;
            *reinterpret_cast<bf16x4*>(row + 512) = p1;
            *reinterpret_cast<bf16x4*>(row + 1024) = p2;
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int r = 4 * wave + 2 * p + (lane >> 5);
            char* row = base + DOB + r * XP + 16 * (((lane & 31) >> 1) ^ stn_sw(r)) + 8 * (lane & 1);
            bf16x4 p0, p1, p2;
            split3x4(__builtin_bit_cast(f32x4, v[4 + p]), p0, p1, p2);
            *reinterpret_cast<bf16x4*>(row) = p0;
            *reinterpret_cast<bf16x4*>(row + 256) = p1;
            *reinterpret_cast<bf16x4*>(row + 512) = p2;
        }
    };
    // sigma': row fragment of row i16 (+16 rb) at k-step q, plane j: chunk (4q + g) ^ swi = 4(q ^ sa) + (g ^ sl)
    auto mfma_sigma = [&](int bb, f32x4 (&acc)[2]) __attribute__((always_inline)) {
        const int lane = fresh_lane();
        const int i16 = lane & 15, g = lane >> 4, swi = stn_sw(i16), sa = swi >> 2, sl = swi & 3;
        const unsigned rb0 = lds0 + bb * BUF + i16 * DP + 16 * (g ^ sl);
        const unsigned ad0 = rb0 + 64 * (0 ^ sa), ad1 = rb0 + 64 * (1 ^ sa), ad2 = rb0 + 64 * (2 ^ sa),
                       ad3 = rb0 + 64 * (3 ^ sa);
        f32x4 hi0 = {0.f, 0.f, 0.f, 0.f}, lo0 = hi0, hi1 = hi0, lo1 = hi0;
        u32x4 fx[2][3], fy[2][3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#define ST3_LOADQ(Q, S_, AD)                                                                              \
        asm volatile("ds_read_b128 %0, %6 offset:%7\n\tds_read_b128 %1, %6 offset:%8\n\t"                 \
                     "ds_read_b128 %2, %6 offset:%9\n\tds_read_b128 %3, %6 offset:%10\n\t"                \
                     "ds_read_b128 %4, %6 offset:%11\n\tds_read_b128 %5, %6 offset:%12"                   \
                     : "=&v"(fx[S_][0]), "=&v"(fx[S_][1]), "=&v"(fx[S_][2]), "=&v"(fy[S_][0]), "=&v"(fy[S_][1]),  \
                       "=&v"(fy[S_][2])                                                                  \
                     : "v"(AD), "i"(256 * ((Q) >> 2)), "i"(256 * ((Q) >> 2) + 512),                       \
                       "i"(256 * ((Q) >> 2) + 1024), "i"(256 * ((Q) >> 2) + 16 * DP),                     \
                       "i"(256 * ((Q) >> 2) + 16 * DP + 512), "i"(256 * ((Q) >> 2) + 16 * DP + 1024)      \
                     : "memory")
        ST3_LOADQ(0, 0, ad0);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int S_ = q & 1;
            if (q + 1 < 8) {
                switch (q) {      // the offsets are immediates: one asm per k-step
                    case 0: ST3_LOADQ(1, 1, ad1); break;
                    case 1: ST3_LOADQ(2, 0, ad2); break;
                    case 2: ST3_LOADQ(3, 1, ad3); break;
                    case 3: ST3_LOADQ(4, 0, ad0); break;
                    case 4: ST3_LOADQ(5, 1, ad1); break;
                    case 5: ST3_LOADQ(6, 0, ad2); break;
                    default: ST3_LOADQ(7, 1, ad3); break;
                }
                asm volatile("s_waitcnt lgkmcnt(6)"
                             : "+v"(fx[S_][0]), "+v"(fx[S_][1]), "+v"(fx[S_][2]), "+v"(fy[S_][0]), "+v"(fy[S_][1]),
                               "+v"(fy[S_][2])::"memory");
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(fx[S_][0]), "+v"(fx[S_][1]), "+v"(fx[S_][2]), "+v"(fy[S_][0]), "+v"(fy[S_][1]),
                               "+v"(fy[S_][2])::"memory");
            }
            const bf16x8 x0 = __builtin_bit_cast(bf16x8, fx[S_][0]), x1 = __builtin_bit_cast(bf16x8, fx[S_][1]),
                         x2 = __builtin_bit_cast(bf16x8, fx[S_][2]);
            const bf16x8 y0 = __builtin_bit_cast(bf16x8, fy[S_][0]), y1 = __builtin_bit_cast(bf16x8, fy[S_][1]),
                         y2 = __builtin_bit_cast(bf16x8, fy[S_][2]);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], x2, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], y2, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[q], x0, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[q], y0, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], x1, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], y1, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], x1, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], y1, lo1, 0, 0, 0);
            lo0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], x0, lo0, 0, 0, 0);
            lo1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[q], y0, lo1, 0, 0, 0);
            hi0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], x0, hi0, 0, 0, 0);
            hi1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[q], y0, hi1, 0, 0, 0);
        }
#undef ST3_LOADQ
        acc[0] = hi0 + lo0;
        acc[1] = hi1 + lo1;
    };
    auto mfma_tn = [&](int bb) __attribute__((always_inline)) {
        // transposed-read rows of this lane (first / second read of a fragment) and their swizzles; the byte of the
        // lane's 4 columns in a row of 16-column block blk is 16 ((2 blk) ^ (sw & 14)) + 16 (tb ^ (sw & 1)) + 8 (l & 1)
        const int lane = fresh_lane();
        const int tra = 8 * (lane >> 4) + ((lane >> 2) & 3), trq = tra + 4;
        const int swa = stn_sw(tra), swq = stn_sw(trq);
        const int tb = (lane & 3) >> 1;
        const unsigned xoa = tra * XP + 16 * (tb ^ (swa & 1)) + 8 * (lane & 1),
                       xoq = trq * XP + 16 * (tb ^ (swq & 1)) + 8 * (lane & 1);
        const unsigned doa = tra * DP + 16 * (tb ^ (swa & 1)) + 8 * (lane & 1) + 256 * (wave >> 2),
                       doq = trq * DP + 16 * (tb ^ (swq & 1)) + 8 * (lane & 1) + 256 * (wave >> 2);
        const int swa_e = swa & 14, swq_e = swq & 14;
        const unsigned db = lds0 + bb * BUF, xb = db + DOB;
        v4s16 xa[2][2][3], fb[2][2][3];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const int cx = 4 * (wave & 3) + 2 * mb;
            tr_read3<256>(xa[mb][0], xb + xoa + 16 * (cx ^ swa_e));
            tr_read3<256>(xa[mb][1], xb + xoq + 16 * (cx ^ swq_e));
        }
        tr_read3<512>(fb[0][0], db + doa + 16 * (0 ^ swa_e));
        tr_read3<512>(fb[0][1], db + doq + 16 * (0 ^ swq_e));
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(xa[0][0][0]), "+v"(xa[0][0][1]), "+v"(xa[0][0][2]), "+v"(xa[0][1][0]), "+v"(xa[0][1][1]),
                       "+v"(xa[0][1][2]), "+v"(xa[1][0][0]), "+v"(xa[1][0][1]), "+v"(xa[1][0][2]), "+v"(xa[1][1][0]),
                       "+v"(xa[1][1][1]), "+v"(xa[1][1][2]), "+v"(fb[0][0][0]), "+v"(fb[0][0][1]), "+v"(fb[0][0][2]),
                       "+v"(fb[0][1][0]), "+v"(fb[0][1][1]), "+v"(fb[0][1][2])::"memory");
        bf16x8 a[2][3];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int j = 0; j < 3; ++j) a[mb][j] = cat_tr(xa[mb][0][j], xa[mb][1][j]);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) {
            const int s = nb & 1;
            if (nb + 1 < 8) {
                tr_read3<512>(fb[s ^ 1][0], db + doa + 16 * ((2 * (nb + 1)) ^ swa_e));
                tr_read3<512>(fb[s ^ 1][1], db + doq + 16 * ((2 * (nb + 1)) ^ swq_e));
            }
            const bf16x8 b0 = cat_tr(fb[s][0][0], fb[s][1][0]), b1 = cat_tr(fb[s][0][1], fb[s][1][1]),
                         b2 = cat_tr(fb[s][0][2], fb[s][1][2]);
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            f32x4 e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][0], b2, z, 0, 0, 0);
            f32x4 e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][0], b2, z, 0, 0, 0);
            e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][2], b0, e0, 0, 0, 0);
            e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][2], b0, e1, 0, 0, 0);
            e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][1], b1, e0, 0, 0, 0);
            e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][1], b1, e1, 0, 0, 0);
            e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][0], b1, e0, 0, 0, 0);
            e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][0], b1, e1, 0, 0, 0);
            e0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][1], b0, e0, 0, 0, 0);
            e1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][1], b0, e1, 0, 0, 0);
            tacc[0][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][0], b0, tacc[0][nb] + e0, 0, 0, 0);
            tacc[1][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][0], b0, tacc[1][nb] + e1, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (nb + 1 < 8)
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(fb[s ^ 1][0][0]), "+v"(fb[s ^ 1][0][1]), "+v"(fb[s ^ 1][0][2]), "+v"(fb[s ^ 1][1][0]),
                               "+v"(fb[s ^ 1][1][1]), "+v"(fb[s ^ 1][1][2])::"memory");
        }
    };
    // epilogue: dX = acc x(1 - x) (rowgemm256_b3_kernel's order), x rebuilt from the planes of columns 16w + 4g .. +3;
    // fp32 16-B stores over the X rows of this half, rows past M dropped by the buffer range.  Returns its store count.
    auto epilogue = [&](long long t, int bb, const f32x4 (&acc)[2]) __attribute__((always_inline)) -> int {
        const int lane = fresh_lane();
        const int i16 = lane & 15, g = lane >> 4, swi = stn_sw(i16);
        const unsigned xb = lds0 + bb * BUF + DOB + 16 * ((2 * wave + (g >> 1)) ^ swi) + 8 * (g & 1);
        u32x2 xr[2][3];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
            asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %3 offset:256\n\tds_read_b64 %2, %3 offset:512"
                         : "=&v"(xr[rb][0]), "=&v"(xr[rb][1]), "=&v"(xr[rb][2])
                         : "v"(xb + (16 * rb + i16) * XP)
                         : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(xr[0][0]), "+v"(xr[0][1]), "+v"(xr[0][2]), "+v"(xr[1][0]), "+v"(xr[1][1]), "+v"(xr[1][2])::"memory");
        const long long row0 = t * TR;
        const long long left = M - row0;
        const unsigned nbytes = (unsigned)((left < TR ? left : TR) * D * 4);
        const __amdgpu_buffer_rsrc_t rc =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(X) + row0 * D * 4, (short)0, nbytes, 0x00020000);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int r = 16 * rb + i16;
            f32x4 v = acc[rb];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float x = (bf_at(xr[rb][0], q) + bf_at(xr[rb][1], q)) + bf_at(xr[rb][2], q);
                v[q] = v[q] * (x * (1.0f - x));
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, rc, (r * D + 128 * half + 16 * wave + 4 * g) * 4, 0, 0);
        }
        return 2;
    };

    if (t_beg < t_end) {
        stage(t_beg, 0, wave);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        convert(0, wave);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
        // per iteration: the DMA of tile t + 1, the sigma' MFMAs of tile t, its epilogue, its TN MFMAs, then tile t + 1's
        // conversion once its DMA has landed (only the epilogue's stores younger); one barrier.  Measured and not kept
        // (round 6, profiles/r06/ab_sigma_tn_b3_r06b.txt): the epilogue and the conversion issued behind the TN MFMAs,
        // one piece per column block (5.24 vs 4.99 ms per config-3 launch), and s_setprio 1 for waves 4-7 of that form
        // (5.25-5.32); waves 4-7 running TN before sigma' (profiles/r06/ab_sigma_tn_b3_r06a.txt: 4.99-5.02 vs 4.78-4.89)
        {
            int b = 0;
            // Split roles: waves 0-3 stage and convert the rows of their SIMD's partner wave (w + 4) too, so waves 4-7
            // run only MFMAs and their epilogue: they start the tile's MFMAs at once and end it with no conversion.
            // 4.83 vs 4.98-5.04 ms per config-3 launch for every wave staging and converting its own rows; the
            // conversions between the epilogue and the TN MFMAs instead of after them 4.89-4.90
            // (profiles/r06/ab_sigma_tn_roles_r06l.txt, phase stamps in profiles/r06/stamps)
            const bool stager = wave < 4;
            for (long long t = t_beg; t < t_end; ++t) {
                const bool more = t + 1 < t_end;
                if (more && stager) {
                    stage(t + 1, b ^ 1, wave);
                    stage(t + 1, b ^ 1, wave + 4);
                }
                f32x4 acc[2];
                mfma_sigma(b, acc);
                const int ns = epilogue(t, b, acc);
                mfma_tn(b);
                if (more && stager) {
                    wait_vm(ns);
                    convert(b ^ 1, wave);
                    convert(b ^ 1, wave + 4);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                b ^= 1;
            }
        }
    }
    float* out = slab + (long long)range * D * D;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = 128 * half + 32 * (wave & 3) + 16 * mb + 4 * g + j;
                out[row * D + 128 * (wave >> 2) + 16 * nb + i16] = tacc[mb][nb][j];
            }
}

// out[D][R] partial of A^T dz and colsum(dz) per block; slab row layout [(D+1)][R]
template <int D>
__global__ __launch_bounds__(D) void gemm_tn_narrow_kernel(long long M, long long rows_per_block, int R,
                                                           const float* __restrict__ A,
                                                           const float* __restrict__ dz,
                                                           float* __restrict__ slab) {
    const int d = threadIdx.x;
    float acc[MAX_R], accb[MAX_R];
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) acc[r] = accb[r] = 0.f;
    const long long r_beg = (long long)blockIdx.x * rows_per_block;
    long long r_end = r_beg + rows_per_block;
    if (r_end > M) r_end = M;
    for (long long e = r_beg; e < r_end; ++e) {
        const float a = A[e * D + d];
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
            if (r < R) {
                const float z = dz[e * R + r];
                acc[r] += a * z;
                accb[r] += z;
            }
    }
    float* out = slab + (long long)blockIdx.x * (D + 1) * R;
#pragma unroll
    for (int r = 0; r < MAX_R; ++r)
        if (r < R) {
            out[d * R + r] = acc[r];
            if (d == 0) out[D * R + r] = accb[r];
        }
}

// ---------------------------------------------------------------------------
// alpha: z = x·Wa + ba ; s = softmax(z) ; w = sigmoid(s)
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void alpha_kernel(int M, int R, const float* __restrict__ X,
                                                    const int* __restrict__ x_idx, const float* __restrict__ Wa,
                                                    const float* __restrict__ ba, float* __restrict__ S_out,
                                                    float* __restrict__ W_out) {
    // persistent over rows: lane sub keeps its 4 rows of W_alpha (4 x R) in registers; the R dot
    // products of a row are reduced together (multi_reduce: one butterfly for all relations)
    constexpr int LPR = D / 4;
    constexpr int K = LPR < MAX_R ? LPR : MAX_R;         // relations reduced per butterfly
    const int sub = threadIdx.x % LPR;
    float wa[4][MAX_R];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < MAX_R; ++r) wa[j][r] = r < R ? Wa[(sub * 4 + j) * R + r] : 0.f;
    float bav[MAX_R];
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) bav[r] = r < R ? ba[r] : 0.f;
    const long long gstride = (long long)gridDim.x * (blockDim.x / LPR);
    // the loop condition is uniform over a row's LPR lanes (the butterflies stay inside a group)
    for (long long row = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / LPR; row < M; row += gstride) {
        const long long src = x_idx ? (long long)x_idx[row] : row;
        const f32x4 x = ld4(X + src * D + sub * 4);
        float z[MAX_R];
#pragma unroll
        for (int r0 = 0; r0 < MAX_R; r0 += K) {
            float part[K];
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const int r = r0 + q;
                part[q] = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) part[q] = fmaf(x[j], wa[j][r], part[q]);
            }
            const float tot = multi_reduce<LPR, K>(part, sub);     // lane sub: relation r0 + sub / (LPR / K)
#pragma unroll
            for (int q = 0; q < K; ++q) z[r0 + q] = __shfl(tot, (threadIdx.x & ~(LPR - 1) & 63) + q * (LPR / K), 64);
        }
        if (sub != 0) continue;
        float mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
            if (r < R) {
                z[r] += bav[r];
                mx = fmaxf(mx, z[r]);
            }
        float sum = 0.f;
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
            if (r < R) {
                z[r] = expf(z[r] - mx);
                sum += z[r];
            }
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
            if (r < R) {
                const float sm = z[r] / sum;
                S_out[row * R + r] = sm;
                W_out[row * R + r] = sigmoidf_(sm);
            }
    }
}

// ---------------------------------------------------------------------------
// combine (no GEMM): out = sigmoid(Y[yi] + sum_r coef[ci][r] * V_r[vi])
// ---------------------------------------------------------------------------
// Persistent, software-pipelined: each lane group walks batches of CU_ROWS rows (stride GROUPS
// inside a block-batch).  vmcnt counts loads and stores together in issue order, so the rows of
// batch b+1 (and the indices of batch b+2) are issued BEFORE batch b's stores: no load ever
// waits behind a store acknowledgement.
constexpr int CU_ROWS = 4;
constexpr int CU_BLOCKS = 2048;
template <int D, int R>
__global__ __launch_bounds__(256) void combine_kernel(int M, const float* __restrict__ Y,
                                                      const int* __restrict__ y_idx, const float* __restrict__ coef,
                                                      const int* __restrict__ coef_idx, const float* __restrict__ V,
                                                      const int* __restrict__ v_idx, long long v_rel_stride,
                                                      float* __restrict__ out) {
    constexpr int LPR = D / 4;
    constexpr int GROUPS = 256 / LPR;
    constexpr int BATCH = GROUPS * CU_ROWS;          // rows per block-batch
    constexpr int RR = R > 0 ? R : 1;
    const int grp = threadIdx.x / LPR;
    const int sub = threadIdx.x % LPR;
    const long long nbatch = ((long long)M + BATCH - 1) / BATCH;
    const long long gstride = gridDim.x;
    // indices of one batch (rows past M / batches past the end read row 0: harmless, never stored)
    int yi[CU_ROWS], ci[CU_ROWS], vi[CU_ROWS];
#define CB_LOAD_IDX(BT)                                                           \
    _Pragma("unroll") for (int u = 0; u < CU_ROWS; ++u) {                          \
        const long long e = (BT) * BATCH + grp + (long long)u * GROUPS;            \
        const bool ok = (BT) < nbatch && e < M;                                    \
        yi[u] = ok ? (y_idx ? y_idx[e] : (int)e) : 0;                              \
        ci[u] = ok ? (coef_idx ? coef_idx[e] : (int)e) : 0;                        \
        vi[u] = ok ? (v_idx ? v_idx[e] : (int)e) : 0;                              \
    }
#define CB_LOAD_ROWS(YV, PV, WV)                                                   \
    _Pragma("unroll") for (int u = 0; u < CU_ROWS; ++u) {                          \
        YV[u] = ld4(Y + (long long)yi[u] * D + sub * 4);                           \
        _Pragma("unroll") for (int r = 0; r < R; ++r) {                            \
            WV[r][u] = coef[(long long)ci[u] * R + r];                             \
            PV[r][u] = ld4(V + r * v_rel_stride + (long long)vi[u] * D + sub * 4); \
        }                                                                          \
    }
    f32x4 yc[CU_ROWS], pc[RR][CU_ROWS];
    float wc[RR][CU_ROWS];
    long long bt = blockIdx.x;
    CB_LOAD_IDX(bt)
    CB_LOAD_ROWS(yc, pc, wc)
    CB_LOAD_IDX(bt + gstride)
    for (; bt < nbatch; bt += gstride) {
        f32x4 yn[CU_ROWS], pn[RR][CU_ROWS];
        float wn[RR][CU_ROWS];
        CB_LOAD_ROWS(yn, pn, wn)
        CB_LOAD_IDX(bt + 2 * gstride)
#pragma unroll
        for (int u = 0; u < CU_ROWS; ++u) {
            f32x4 v = yc[u];
#pragma unroll
            for (int r = 0; r < R; ++r) v += wc[r][u] * pc[r][u];
            const long long e = bt * BATCH + grp + (long long)u * GROUPS;
            if (e < M) {
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = sigmoid_fast(v[j]);
                st4(out + e * D + sub * 4, v);
            }
        }
#pragma unroll
        for (int u = 0; u < CU_ROWS; ++u) {
            yc[u] = yn[u];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                pc[r][u] = pn[r][u];
                wc[r][u] = wn[r][u];
            }
        }
    }
#undef CB_LOAD_IDX
#undef CB_LOAD_ROWS
}

// Run combine, D = 256, shared row index (y_idx == v_idx, typically tail-sorted edges):
// out[e] = sigmoid(Y[t_e] + sum_r coef[e][r] * V_r[t_e]).  One wave per 64-edge chunk, one
// row per wave instruction.  Consecutive edges with the same t form a run; the node rows
// (Y, V_r) are loaded once per run, and the NEXT run's rows (or the next chunk's first run)
// are issued before the current run's stores, so the only loads a store ever sits in front
// of are the ones already needed.  Per-edge indices/coefficients: one per lane, broadcast
// with readlane.
constexpr int RC_CH = 64;
template <int R, bool BF = false, bool PL = false>
__global__ __launch_bounds__(256) void run_combine256_kernel(int M, const float* __restrict__ Y,
                                                             const int* __restrict__ idx,
                                                             const float* __restrict__ coef,
                                                             const float* __restrict__ V, long long v_rel_stride,
                                                             float* __restrict__ out) {
    constexpr int D = 256;
    constexpr int RR = R > 0 ? R : 1;
    const int lane = threadIdx.x & 63;
    const long long nchunk = ((long long)M + RC_CH - 1) / RC_CH;
    const long long wstride = (long long)gridDim.x * 4;
    long long c = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nchunk) return;
    // per-lane edge state of a chunk
    auto load_chunk = [&](long long ch, int& tv, float (&cf)[RR]) {
        const long long e = ch * RC_CH + lane;
        const bool ok = ch < nchunk && e < M;
        tv = ok ? idx[e] : -1;
#pragma unroll
        for (int r = 0; r < R; ++r) cf[r] = ok ? coef[e * R + r] : 0.f;
    };
    int tv;
    float cf[RR];
    load_chunk(c, tv, cf);
    f32x4 yc, pc[RR], yn, pn[RR];
    auto load_rows = [&](int t, f32x4& yv, f32x4 (&pv)[RR]) {
        yv = ld4(Y + (long long)t * D + lane * 4);
#pragma unroll
        for (int r = 0; r < R; ++r) pv[r] = ld4(V + r * v_rel_stride + (long long)t * D + lane * 4);
    };
    load_rows(__builtin_amdgcn_readfirstlane(tv), yc, pc);
    for (; c < nchunk; c += wstride) {
        const long long e0 = c * RC_CH;
        const int nvalid = (int)((long long)M - e0 < RC_CH ? (long long)M - e0 : RC_CH);
        const int tprev = __shfl_up(tv, 1, 64);
        unsigned long long starts = __ballot(lane < nvalid && (lane == 0 || tv != tprev));
        starts &= starts - 1;                          // run 0 is already loaded
        // next chunk's per-lane state, issued now (tiny loads, long before they are needed)
        int tv_n;
        float cf_n[RR];
        load_chunk(c + wstride, tv_n, cf_n);
        int cur = 0;
        while (true) {
            int next;
            if (starts) {
                next = __builtin_ctzll(starts);
                starts &= starts - 1;
                load_rows(__builtin_amdgcn_readlane(tv, next), yn, pn);
            } else {
                next = nvalid;
                if (c + wstride < nchunk) load_rows(__builtin_amdgcn_readfirstlane(tv_n), yn, pn);
            }
            for (int j = cur; j < next; ++j) {
                f32x4 v = yc;
#pragma unroll
                for (int r = 0; r < R; ++r) v += __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cf[r]), j)) * pc[r];
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = sigmoid_fast(v[q]);
                if constexpr (PL)
                    st_planes4(reinterpret_cast<char*>(out) + (e0 + j) * 1024, lane * 4, v);
                else
                    if constexpr (BF) st4e<BF>(out, (e0 + j) * D + lane * 4, v);
                    else   // written once, read by a later kernel: nontemporal (0.883-0.886 vs 0.901-0.912 ms, r06ag)
                        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out + (e0 + j) * D + lane * 4));
            }
            yc = yn;
#pragma unroll
            for (int r = 0; r < R; ++r) pc[r] = pn[r];
            if (next >= nvalid) break;
            cur = next;
        }
        tv = tv_n;
#pragma unroll
        for (int r = 0; r < R; ++r) cf[r] = cf_n[r];
    }
}

// ---------------------------------------------------------------------------
// DistMult + Keras BCE + backward seed.  256-thread blocks, grid-stride over rows;
// per-lane-group register partials for drel and loss, block-ordered reduction.
// ---------------------------------------------------------------------------
template <int D, bool BF = false>
__global__ __launch_bounds__(256) void distmult_kernel(long long T, int R, const float* __restrict__ Xh,
                                                       const int* __restrict__ h_idx, const float* __restrict__ Xt,
                                                       const int* __restrict__ t_idx, const int* __restrict__ r_idx,
                                                       const float* __restrict__ rel, const float* __restrict__ y,
                                                       float scale, float* __restrict__ p_out,
                                                       float* __restrict__ s_out,
                                                       float* __restrict__ ds_out, float* __restrict__ do_out,
                                                       float* __restrict__ drel_slab, float* __restrict__ loss_slab) {
    constexpr int LPR = D / 4;
    constexpr int GROUPS = 256 / LPR;  // row groups per block
    __shared__ __attribute__((aligned(16))) float red[GROUPS * MAX_R * D];
    __shared__ float lred[GROUPS];
    const int grp = threadIdx.x / LPR;
    const int sub = threadIdx.x % LPR;
    const bool train = (y != nullptr);
    f32x4 dr[MAX_R];
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) dr[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    float lacc = 0.f;

    // U rows per group per iteration (same visit order as a plain grid-stride loop, so the
    // drel / loss partial sums are order-identical).  Software-pipelined: the rows of the next
    // iteration and the indices of the one after are issued before this iteration's stores
    // (vmcnt counts loads and stores together, in order).
    constexpr int U = 2;
    const long long stride = (long long)gridDim.x * GROUPS;
    int hr[U], rr[U];
    long long ti[U];
    float yv[U];
#define DM_LOAD_IDX(E0)                                                        \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                             \
        const long long ee = (E0) + u * stride;                                 \
        const bool ok = ee < T;                                                 \
        hr[u] = ok ? h_idx[ee] : 0;                                             \
        rr[u] = ok ? r_idx[ee] : 0;                                             \
        ti[u] = ok ? (t_idx ? (long long)t_idx[ee] : ee) : 0;                   \
        yv[u] = (train && ok) ? y[ee] : 0.f;                                    \
    }
#define DM_LOAD_ROWS(A, B, RHO, YY, RI)                                        \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                             \
        A[u] = ld4(Xh + (long long)hr[u] * D + sub * 4);                        \
        B[u] = ld4e<BF>(Xt, ti[u] * D + sub * 4);                               \
        RHO[u] = ld4(rel + (long long)rr[u] * D + sub * 4);                     \
        YY[u] = yv[u];                                                          \
        RI[u] = rr[u];                                                          \
    }
    long long e0 = (long long)blockIdx.x * GROUPS + grp;
    f32x4 a[U], b[U], rho[U];
    float yy[U];
    int rc[U];
    DM_LOAD_IDX(e0)
    DM_LOAD_ROWS(a, b, rho, yy, rc)
    DM_LOAD_IDX(e0 + U * stride)
    for (; e0 < T; e0 += U * stride) {
        f32x4 an[U], bn[U], rhon[U];
        float yn[U];
        int rn[U];
        DM_LOAD_ROWS(an, bn, rhon, yn, rn)
        DM_LOAD_IDX(e0 + 2 * U * stride)
        float sc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const f32x4 prod = a[u] * rho[u] * b[u];
            sc[u] = group_sum<LPR>(prod[0] + prod[1] + prod[2] + prod[3]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long e = e0 + u * stride;
            if (e >= T) continue;
            const float p = sigmoidf_(sc[u]);
            if (sub == 0) {
                if (p_out) p_out[e] = p;
                if (s_out) s_out[e] = sc[u];
            }
            if (!train) continue;
            const float pc = fminf(fmaxf(p, EPS_BCE), 1.0f - EPS_BCE);
            const bool pass = (p >= EPS_BCE) && (p <= 1.0f - EPS_BCE);
            const float g =
                pass ? scale * (-(yy[u] / (pc + EPS_BCE)) + (1.0f - yy[u]) / (1.0f - pc + EPS_BCE)) : 0.f;
            const float ds = g * p * (1.0f - p);
            if (sub == 0) {
                ds_out[e] = ds;
                lacc += -(yy[u] * logf(pc + EPS_BCE) + (1.0f - yy[u]) * logf(1.0f - pc + EPS_BCE));
            }
            f32x4 dx = (ds * rho[u]) * a[u];
            dx = dx * (b[u] * (1.0f - b[u]));
            st4e<BF>(do_out, e * D + sub * 4, dx);
            const f32x4 dre = ds * (a[u] * b[u]);
#pragma unroll
            for (int r = 0; r < MAX_R; ++r)
                if (r == rc[u]) dr[r] += dre;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = an[u];
            b[u] = bn[u];
            rho[u] = rhon[u];
            yy[u] = yn[u];
            rc[u] = rn[u];
        }
    }
#undef DM_LOAD_IDX
#undef DM_LOAD_ROWS
    if (!train) return;
#pragma unroll
    for (int r = 0; r < MAX_R; ++r)
        if (r < R) st4(red + (grp * MAX_R + r) * D + sub * 4, dr[r]);
    if (sub == 0) lred[grp] = lacc;
    __syncthreads();
    for (int x = threadIdx.x; x < R * D; x += 256) {
        const int r = x / D, c = x % D;
        float s = 0.f;
        for (int gq = 0; gq < GROUPS; ++gq) s += red[(gq * MAX_R + r) * D + c];
        drel_slab[(long long)blockIdx.x * R * D + x] = s;
    }
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int gq = 0; gq < GROUPS; ++gq) s += lred[gq];
        loss_slab[blockIdx.x] = s;
    }
}

// ---------------------------------------------------------------------------
// DistMult + Keras BCE + both backward seeds, one pass over edges grouped by HEAD.
// A lane group owns one head node at a time (persistent loop): Xh[n] is read once, each edge's
// tail row Xt[e] once (the tail-seed do_out[e] is written from it), and the head seed
// dXh[n] = Xh(1-Xh) * sum ds_e rel[r_e] Xt[e] accumulates in registers in perm order.  Per-edge
// arithmetic is that of distmult_kernel + seg_gather_reduce_kernel, so p / ds / do / dXh are
// bitwise the same; only the drel / loss partial sums visit edges in another order.
// do_out may alias Xt (the engine writes do^3 over x^3): each element is read, then written, by
// the same lane, and every edge is visited once.
// ---------------------------------------------------------------------------
template <int D, int RT, bool BF = false>
__global__ __launch_bounds__(256) void distmult_heads_kernel(int n_nodes, int R, const int* __restrict__ seg_ptr,
                                                             const int* __restrict__ perm,
                                                             const float* __restrict__ Xh,
                                                             const float* Xt,    // may alias do_out
                                                             const int* __restrict__ r_idx,
                                                             const float* __restrict__ rel,
                                                             const float* __restrict__ y, float scale,
                                                             float* __restrict__ p_out, float* __restrict__ s_out,
                                                             float* __restrict__ ds_out,
                                                             float* do_out, float* __restrict__ dXh,
                                                             float* __restrict__ drel_slab,
                                                             float* __restrict__ loss_slab) {
    constexpr int LPR = D / 4;
    constexpr int GROUPS = 256 / LPR;
    constexpr int DM_UW = 4;
    constexpr int DM_SC_MINR = 2;     // R = 2 too: 1.96 -> 1.84 ms at config 3 (tools/bench_tailseg.py), bitwise equal
    // edges per group; the R >= DM_SC_MINR loop (one head per wave, next group prefetched) takes DM_UW
    constexpr int U = (64 / LPR == 1 && RT >= DM_SC_MINR) ? DM_UW : 4;
    __shared__ __attribute__((aligned(16))) float red[GROUPS * RT * D];
    __shared__ float lred[GROUPS];
    constexpr int SLOTS = 64 / LPR;      // edge slots per head node (one wave per node)
    constexpr int NPB = 256 / 64;
    const int grp = threadIdx.x / LPR;
    const int sub = threadIdx.x % LPR;
    const int slot = (threadIdx.x % 64) / LPR;
    f32x4 dr[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) dr[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    // R >= 4 with one head per wave: the per-relation partials of drel live in the block's LDS slab instead of dr[]
    // (the relation of an edge is wave-uniform, and selecting one of 8 register quads per edge cost ~45 instructions
    // of branches and moves per edge: config-5 launch 18.3 -> 15.9 ms); same values added in the same order per lane
    // (the register form's add was contracted into an fma: drel partials within 2e-7)
    constexpr bool LDS_DR = SLOTS == 1 && RT >= 4 && RT >= DM_SC_MINR;
    if constexpr (LDS_DR) {
#pragma unroll
        for (int r = 0; r < RT; ++r) st4(red + (grp * RT + r) * D + sub * 4, f32x4{0.f, 0.f, 0.f, 0.f});
    }
    float lacc = 0.f;
    const long long nstride = (long long)gridDim.x * NPB;
    for (long long n0 = (long long)blockIdx.x * NPB; n0 < n_nodes; n0 += nstride) {
        const long long n = n0 + threadIdx.x / 64;
        const bool live = n < n_nodes;
        int beg = live ? seg_ptr[n] : 0, end = live ? seg_ptr[n + 1] : 0;
        // D = 256 and R >= 2: the whole wave is one head, so its edges' indices are wave-uniform and the
        // software-pipelined loop below applies (R = 8: -13%, R = 2: -6%)
        constexpr bool SCALAR = SLOTS == 1 && RT >= DM_SC_MINR;
        if constexpr (SCALAR) {
            beg = __builtin_amdgcn_readfirstlane(beg);
            end = __builtin_amdgcn_readfirstlane(end);
        }
        const int len = end - beg;
        const f32x4 a = live ? ld4(Xh + n * D + sub * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        // one group of U edges: e[u] (-1 past the segment), their relations, labels and tail rows
        auto body = [&](const long long (&e)[U], const int (&rr)[U], const float (&yy)[U],
                        const f32x4 (&b)[U]) __attribute__((always_inline)) {
            f32x4 rho[U];
#pragma unroll
            for (int u = 0; u < U; ++u) rho[u] = ld4(rel + (long long)rr[u] * D + sub * 4);
            float sc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const f32x4 prod = a * rho[u] * b[u];
                sc[u] = group_sum<LPR>(prod[0] + prod[1] + prod[2] + prod[3]);
            }
            // the per-edge scalar chain (sigmoid, Keras BCE seed and loss term: two logf, two IEEE divisions, expf)
            auto scalar_chain = [&](float sv, float yv, float& p, float& ds, float& lterm) __attribute__((always_inline)) {
                p = sigmoidf_(sv);
                float g;
                if (y) {        // Keras BCE seed
                    const float pc = fminf(fmaxf(p, EPS_BCE), 1.0f - EPS_BCE);
                    const bool pass = (p >= EPS_BCE) && (p <= 1.0f - EPS_BCE);
                    g = pass ? scale * (-(yv / (pc + EPS_BCE)) + (1.0f - yv) / (1.0f - pc + EPS_BCE)) : 0.f;
                    lterm = -(yv * logf(pc + EPS_BCE) + (1.0f - yv) * logf(1.0f - pc + EPS_BCE));
                } else {        // prediction seed: gradient of scale * sum_e p_e
                    g = scale;
                    lterm = p;
                }
                ds = g * p * (1.0f - p);
            };
            // one head per wave (LPR = 64): the group's U scores are wave-uniform, so lane u runs edge u's scalar chain
            // and the results are broadcast (readlane) — one chain per group instead of U redundant ones; the same
            // function of the same inputs, so p, s, ds and the loss terms are bitwise those of the redundant form
            float ds_l = 0.f, lt_l = 0.f;
            if constexpr (LPR == 64) {
                float sv = sc[0], yv = yy[0];
                long long el = e[0];
#pragma unroll
                for (int u = 1; u < U; ++u) {
                    sv = sub == u ? sc[u] : sv;
                    yv = sub == u ? yy[u] : yv;
                    el = sub == u ? e[u] : el;
                }
                float p_l;
                scalar_chain(sv, yv, p_l, ds_l, lt_l);
                if (sub < U && el >= 0) {
                    if (p_out) p_out[el] = p_l;
                    if (s_out) s_out[el] = sv;
                    if (ds_out) ds_out[el] = ds_l;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (e[u] < 0) continue;
                float ds, lterm;
                if constexpr (LPR == 64) {
                    ds = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ds_l), u));
                    lterm = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lt_l), u));
                    if (sub == 0) lacc += lterm;
                } else {
                    float p;
                    scalar_chain(sc[u], yy[u], p, ds, lterm);
                    if (sub == 0) {
                        if (p_out) p_out[e[u]] = p;
                        if (s_out) s_out[e[u]] = sc[u];
                        if (ds_out) ds_out[e[u]] = ds;
                        lacc += lterm;
                    }
                }
                f32x4 dx = (ds * rho[u]) * a;
                dx = dx * (b[u] * (1.0f - b[u]));
                if constexpr (BF) st4e<BF>(do_out, e[u] * D + sub * 4, dx);
                else     // written once, read by later kernels: nontemporal (1.767-1.776 vs 1.823-1.833 ms, r06aj)
                    __builtin_nontemporal_store(dx, reinterpret_cast<f32x4*>(do_out + e[u] * D + sub * 4));
                const f32x4 dre = ds * (a * b[u]);
                if constexpr (LDS_DR) {
                    float* dst = red + (grp * RT + rr[u]) * D + sub * 4;     // this lane's own 16 B
                    st4(dst, ld4(dst) + dre);
                } else {
#pragma unroll
                    for (int r = 0; r < RT; ++r)
                        if (r == rr[u]) dr[r] += dre;
                }
                acc = fma4(b[u] * ds, rho[u], acc);     // same explicit fma as seg_gather_reduce
            }
        };
        if constexpr (SCALAR) {
            // many relations (one head per wave): a software pipeline over edge groups — the perm entries of
            // group i+2 and the relations, labels and rows of group i+1 load while group i is computed.  Every
            // index goes through a VECTOR load (lane u < U: edge u of the group) and is broadcast with readlane:
            // the scalar loads of the previous form return out of order, so each wait for one of them was an
            // lgkmcnt(0) on everything in flight (a full memory latency, twice per group: perm, then r_idx).
            // Rows stay in their storage type until used.
            using RawT = typename std::conditional<BF, bf16x4, f32x4>::type;
            auto load_perm = [&](int k) __attribute__((always_inline)) {
                return (sub < U && k + sub < len) ? perm[beg + k + sub] : -1;
            };
            // two groups in flight at R >= 4: config-5 shape 7.22 -> 6.91 ms; R = 2: +3%, not taken
            // one group's indices (lane u: edge u), relations, labels and raw tail rows
            struct Grp {
                int ev, rv;
                float yv;
                RawT bn[U];
            };
            auto load_group = [&](int ev, Grp& G) __attribute__((always_inline)) {
                G.rv = ev >= 0 ? r_idx[ev] : 0;
                G.yv = (ev >= 0 && y) ? y[ev] : 0.f;
                G.ev = ev;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int eu = __builtin_amdgcn_readlane(ev, u);
                    const RawT* src = reinterpret_cast<const RawT*>(reinterpret_cast<const char*>(Xt) +
                                                                   ((long long)eu * D + sub * 4) * (BF ? 2 : 4));
                    if (eu >= 0) G.bn[u] = *src;
                    else G.bn[u] = RawT{};
                }
            };
            auto unpack = [&](const Grp& G, long long (&e)[U], int (&rr)[U], float (&yy)[U], f32x4 (&b)[U])
                __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    e[u] = __builtin_amdgcn_readlane(G.ev, u);
                    rr[u] = __builtin_amdgcn_readlane(G.rv, u);
                    yy[u] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, G.yv), u));
                    if constexpr (BF) b[u] = bf4_to_f32(G.bn[u]);
                    else b[u] = G.bn[u];
                }
            };
            if constexpr (RT >= 4) {
                // two groups in flight: while group i is computed, the rows of groups i+1 and i+2
                // and the perm entries of group i+3 load; the group registers alternate between two sets
                // (the loop is unrolled by two, so every index into them is static)
                Grp GA, GB;
                int evp = -1;
                if (len > 0) {
                    const int ev0 = load_perm(0), ev1 = load_perm(U);
                    evp = load_perm(2 * U);
                    load_group(ev0, GA);
                    if (U < len) load_group(ev1, GB);
                }
                for (int k0 = 0; k0 < len; k0 += 2 * U) {
                    {
                        long long e[U];
                        int rr[U];
                        float yy[U];
                        f32x4 b[U];
                        unpack(GA, e, rr, yy, b);
                        const int evq = load_perm(k0 + 3 * U);
                        if (k0 + 2 * U < len) load_group(evp, GA);
                        evp = evq;
                        body(e, rr, yy, b);
                    }
                    if (k0 + U >= len) break;
                    {
                        long long e[U];
                        int rr[U];
                        float yy[U];
                        f32x4 b[U];
                        unpack(GB, e, rr, yy, b);
                        const int evq = load_perm(k0 + 4 * U);
                        if (k0 + 3 * U < len) load_group(evp, GB);
                        evp = evq;
                        body(e, rr, yy, b);
                    }
                }
            } else {
                Grp G;
                int ev2 = -1;
                if (len > 0) {
                    const int ev1 = load_perm(0);
                    ev2 = load_perm(U);
                    load_group(ev1, G);
                }
                for (int k0 = 0; k0 < len; k0 += U) {
                    long long e[U];
                    int rr[U];
                    float yy[U];
                    f32x4 b[U];
                    unpack(G, e, rr, yy, b);
                    const int ev3 = load_perm(k0 + 2 * U);
                    if (k0 + U < len) load_group(ev2, G);
                    ev2 = ev3;
                    body(e, rr, yy, b);
                }
            }
        } else {
            // slot s takes edge groups k = (it*SLOTS + s)*U: same trip count for the whole wave
            const int iters = (len + SLOTS * U - 1) / (SLOTS * U);
            for (int it = 0; it < iters; ++it) {
                const int k = (it * SLOTS + slot) * U;
                long long e[U];
#pragma unroll
                for (int u = 0; u < U; ++u) e[u] = (k + u < len) ? (long long)perm[beg + k + u] : -1;
                int rr[U];
                float yy[U];
                f32x4 b[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool ok = e[u] >= 0;
                    rr[u] = ok ? r_idx[e[u]] : 0;
                    yy[u] = (ok && y) ? y[e[u]] : 0.f;
                    b[u] = ok ? ld4e<BF>(Xt, e[u] * D + sub * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
                }
                body(e, rr, yy, b);
            }
        }
#pragma unroll
        for (int m = 1; m < SLOTS; m <<= 1)          // slot partials, fixed order
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] += __shfl_xor(acc[q], LPR * m, 64);
        if (live && slot == 0) st4(dXh + n * D + sub * 4, acc * (a * (1.0f - a)));
    }
    if constexpr (!LDS_DR) {
#pragma unroll
        for (int r = 0; r < RT; ++r) st4(red + (grp * RT + r) * D + sub * 4, dr[r]);
    }
    if (sub == 0) lred[grp] = lacc;
    __syncthreads();
    for (int x = threadIdx.x; x < R * D; x += 256) {
        const int r = x / D, c = x % D;
        float s = 0.f;
        for (int gq = 0; gq < GROUPS; ++gq) s += red[(gq * RT + r) * D + c];
        drel_slab[(long long)blockIdx.x * R * D + x] = s;
    }
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int gq = 0; gq < GROUPS; ++gq) s += lred[gq];
        loss_slab[blockIdx.x] = s;
    }
}

// ---------------------------------------------------------------------------
// segmented gather-reduce (head side): out[n] = dsig * sum coef[e] rel[r_e] rows[e]
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void seg_gather_reduce_kernel(int n_nodes, const int* __restrict__ seg_ptr,
                                                                const int* __restrict__ perm,
                                                                const float* __restrict__ coef,
                                                                const int* __restrict__ r_idx,
                                                                const float* __restrict__ rel,
                                                                const float* __restrict__ rows,
                                                                const float* __restrict__ X, float* __restrict__ out) {
    constexpr int LPR = D / 4;
    const long long n = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
    const int sub = threadIdx.x % LPR;
    if (n >= n_nodes) return;
    const int beg = seg_ptr[n], end = seg_ptr[n + 1];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    constexpr int U = 4;
    for (int k0 = beg; k0 < end; k0 += U) {
        long long e[U];
        f32x4 v[U], q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = (k0 + u < end) ? (perm ? (long long)perm[k0 + u] : (long long)(k0 + u)) : -1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (e[u] < 0) continue;
            v[u] = ld4(rows + e[u] * D + sub * 4);
            if (coef) v[u] *= coef[e[u]];
            if (rel) q[u] = ld4(rel + (long long)r_idx[e[u]] * D + sub * 4);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (e[u] < 0) continue;
            acc = rel ? fma4(v[u], q[u], acc) : acc + v[u];   // explicit fma: no contraction ambiguity
        }
    }
    if (X) {
        const f32x4 x = ld4(X + n * D + sub * 4);
        acc = acc * (x * (1.0f - x));
    }
    st4(out + n * D + sub * 4, acc);
}

// ---------------------------------------------------------------------------
// tail-side layer backward over tail-sorted contiguous segments.
// One node per group of D/4 lanes; the node's edges are contiguous rows of dO,
// walked 4 at a time with all 4 row loads (and their W[h] loads) issued before
// any use, so each wave keeps 4 KiB in flight.  R is a template parameter so
// the per-relation state stays in a handful of registers (R = 2: 76 VGPRs, 6 waves per SIMD;
// forcing 7 or 8 waves is slower, profiles/r02/ablations/tail_seg_depth_ab.txt).
// D < 256: a node gets the whole wave, 64 / (D/4) edge SLOTS of D/4 lanes each walking every
// SLOTS-th group of U edges (graphs with few nodes, e.g. the reference's 845, would otherwise
// leave most of the chip idle behind a few long serial segments); the slot partials are summed
// in fixed order (xor-shuffles) at the end, so results stay deterministic.
// ---------------------------------------------------------------------------
template <int D, int R, bool BF = false>
__global__ __launch_bounds__(256) void tail_seg_reduce_kernel(int n_nodes, const int* __restrict__ seg_ptr,
                                                              const int* __restrict__ h_idx,
                                                              const float* __restrict__ W,
                                                              const float* __restrict__ dO,
                                                              const float* __restrict__ P, long long p_rel_stride,
                                                              float* __restrict__ dP, long long dp_rel_stride,
                                                              float* __restrict__ dsum, float* __restrict__ dWedge) {
    constexpr int LPR = D / 4;
    constexpr int SLOTS = 64 / LPR;                     // edge slots per node (one wave per node)
    constexpr int TS_U = 4;
// R >= 4 (one node per wave, next group prefetched): 8 edge rows per group, i.e. U x R = 64 coefficients, one
// per lane.  Rows in flight per wave are what this loop is bound by: at the config-5 shape (R = 8, bf16 rows,
// degree 50) 4 -> 8 rows per group took a launch from 4.86 to 3.03 ms (tools/bench_tailseg.py)
    constexpr int TS_UW = 8;
// fp32 rows at R <= 2: nontemporal loads (the rows are read once; -2% at config 3, the probe's read-only
// streams gain 10% from it); the R >= 4 loop with 8 rows in flight is slower with them (3.41 vs 3.03 ms)
    const long long n = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const int sub = threadIdx.x % LPR;
    const int slot = (threadIdx.x % 64) / LPR;
    const bool live = n < n_nodes;
    int beg = live ? seg_ptr[n] : 0, end = live ? seg_ptr[n + 1] : 0;
    // D = 256 with many relations: one node per wave, its edge rows (and W rows) wave-uniform, the R
    // coefficients of an edge through scalar loads (R = 8: -39%; at R <= 2 the vector loads are faster)
    constexpr int TS_PF_MINR = 4;
    constexpr bool SCALAR = SLOTS == 1 && R >= TS_PF_MINR;
    constexpr int U = SCALAR ? TS_UW : TS_U;         // edge rows per group
    if constexpr (SCALAR) {
        beg = __builtin_amdgcn_readfirstlane(beg);
        end = __builtin_amdgcn_readfirstlane(end);
    }
    f32x4 pr[R], acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        pr[r] = live ? ld4(P + r * p_rel_stride + n * D + sub * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
    const int len = end - beg;
    // One edge group: its rows d[U] and coefficients w[U][R] (zeros past the segment), then the sums.
    auto load_group = [&](int k, f32x4 (&d)[U], float (&w)[U][R]) __attribute__((always_inline)) {
        int hh[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool a = k + u < len;
            // h_idx == NULL: W is already per edge (W[e][r], gathered once per layer)
            hh[u] = a ? (h_idx ? h_idx[beg + k + u] : beg + k + u) : 0;
            if constexpr (SCALAR) hh[u] = __builtin_amdgcn_readfirstlane(hh[u]);     // scalar W loads
            if constexpr (!BF)
                d[u] = a ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(dO + (long long)(beg + k + u) * D + sub * 4))
                         : f32x4{0.f, 0.f, 0.f, 0.f};
            else
                d[u] = a ? ld4e<BF>(dO, (long long)(beg + k + u) * D + sub * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < R; ++r) w[u][r] = (k + u < len) ? W[(long long)hh[u] * R + r] : 0.f;
    };
    auto group = [&](int k, const f32x4 (&d)[U], const float (&w)[U][R]) __attribute__((always_inline)) {
        constexpr int KV = U * R;
        // reduced in chunks of at most 32 values (a power of two); every value is summed over the 64 lanes in
        // the same butterfly order whatever the chunk size, so an 8-row group gives bitwise the 4-row sums
        constexpr int KP = KV <= 4 ? 4 : KV <= 8 ? 8 : KV <= 16 ? 16 : 32;
        constexpr int NCH = (KV + KP - 1) / KP;
        float dw[NCH * KP];
#pragma unroll
        for (int j = 0; j < NCH * KP; ++j) dw[j] = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            s4 += d[u];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                acc[r] += w[u][r] * d[u];
                const f32x4 q = d[u] * pr[r];
                dw[u * R + r] = q[0] + q[1] + q[2] + q[3];
            }
        }
        if constexpr (KP <= LPR) {
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                float part[KP];
#pragma unroll
                for (int j = 0; j < KP; ++j) part[j] = dw[ch * KP + j];
                const float tot = multi_reduce<LPR, KP>(part, sub);
                constexpr int SPAN = LPR / KP;             // lanes sharing one value
                const int j = ch * KP + sub / SPAN;
                if (sub % SPAN == 0 && j < KV) {
                    const int u = j / R, r = j % R;
                    if (k + u < len) dWedge[(long long)(beg + k + u) * R + r] = tot;
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < KV; ++j) dw[j] = group_sum<LPR>(dw[j]);
            if (sub == 0) {
#pragma unroll
                for (int j = 0; j < KV; ++j)
                    if (k + j / R < len) dWedge[(long long)(beg + k + j / R) * R + j % R] = dw[j];
            }
        }
    };
    if constexpr (SCALAR) {
        // many relations (R >= 4, one node per wave): ~150 VGPRs leave 3 waves per SIMD, and one group
        // of U rows in flight per wave did not cover the memory latency (R = 8 bf16: 1.4 TB/s).  The next
        // group's rows and coefficients are loaded while this group is summed (same sums, same order).
        // Rows stay in their storage type (bf16 or fp32) until used: a conversion next to the load would
        // make the compiler wait for it there.  The group's U x R coefficients arrive by ONE vector load
        // (lane j: coefficient j, contiguous for per-edge W) and are broadcast with readlane: scalar loads
        // (the previous form) return out of order, so waiting for this group's coefficients meant
        // lgkmcnt(0), i.e. also for the next group's, a full memory latency per group.
        static_assert(U * R <= 64, "one coefficient per lane");
        using RawT = typename std::conditional<BF, bf16x4, f32x4>::type;
        RawT dn[U];
        float wvn;
        auto load_raw = [&](int k) __attribute__((always_inline)) {
            const int u = sub / R, r = sub - u * R;          // this lane's coefficient (sub < U * R)
            const bool wa = sub < U * R && k + u < len;
            const long long we = h_idx ? (wa ? (long long)h_idx[beg + k + u] : 0) : (long long)(beg + k + u);
            wvn = wa ? W[we * R + r] : 0.f;
#pragma unroll
            for (int uu = 0; uu < U; ++uu) {
                const RawT* src = reinterpret_cast<const RawT*>(reinterpret_cast<const char*>(dO) +
                                                               ((long long)(beg + k + uu) * D + sub * 4) * (BF ? 2 : 4));
                if (k + uu < len) dn[uu] = *src;
                else dn[uu] = RawT{};
            }
        };
        if (len > 0) load_raw(0);
        for (int k0 = 0; k0 < len; k0 += U) {
            f32x4 dc[U];
            float wc[U][R];
            const float wv = wvn;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (BF) dc[u] = bf4_to_f32(dn[u]);
                else dc[u] = dn[u];
#pragma unroll
                for (int r = 0; r < R; ++r)
                    wc[u][r] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, wv), u * R + r));
            }
            if (k0 + U < len) load_raw(k0 + U);
            group(k0, dc, wc);
        }
    } else {
        // slot s takes edge groups k = k0 + s*U, k0 = 0, SLOTS*U, ...: the whole wave is one node and every
        // slot runs the same trip count (wave-uniform).  The k0 < len form (not an iteration count) keeps
        // the D = 256 loop (SLOTS = 1) as fast as the pre-slot kernel: 0.92 vs 1.01 ms per config-3 launch.
        for (int k0 = 0; k0 < len; k0 += SLOTS * U) {
            const int k = k0 + slot * U;
            f32x4 d[U];
            float w[U][R];
            load_group(k, d, w);
            group(k, d, w);
        }
    }
    // slot partials, fixed order: pairs (s, s ^ 1), then (s, s ^ 2), ... (lane distance LPR * m)
#pragma unroll
    for (int m = 1; m < SLOTS; m <<= 1) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] += __shfl_xor(acc[r][q], LPR * m, 64);
#pragma unroll
        for (int q = 0; q < 4; ++q) s4[q] += __shfl_xor(s4[q], LPR * m, 64);
    }
    if (!live || slot != 0) return;
#pragma unroll
    for (int r = 0; r < R; ++r) st4(dP + r * dp_rel_stride + n * D + sub * 4, acc[r]);
    if (dsum) st4(dsum + n * D + sub * 4, s4);
}

// ---------------------------------------------------------------------------
// tail-side layer backward on MFMAs: R = 8 relations, bf16 edge rows, D = 256 (config 5; round 4).
// Per tail node t (one wave) and per chunk of 32 of its edges (rows e of do, coefficients W[e][0..7]):
//   dWedge[e][r] = do[e] . P_r[t]        the chunk (32 x 256, bf16) times P[t]^T (256 x 8, split hi + lo bf16)
//   dP_r[t]     += sum_e W[e][r] do[e]   W^T (8 x 32, hi + lo) times the chunk (32 x 256)
//   dsum[t]     += sum_e do[e]           (DSUM, layer 1: a ones row beside W^T)
// on v_mfma_f32_16x16x32_bf16: the products are exact (bf16 x bf16), accumulation fp32; the fp32 operands P and W
// enter EXACTLY as three bf16 pieces each (hi + mid + lo = 24 significant bits, as in the bf16x3 GEMMs; the bf16 rows
// are exact as they are), so the only difference from fp32 arithmetic is the order of the fp32 sums.  The VALU form (tail_seg_reduce_kernel<256, 8, true>) spends ~1100 instructions per 8
// edges here (two FMA chains per relation and a 64-value butterfly per edge group) and is VALU-bound (11.6 ms per
// config-5 launch); this one issues ~250 per 32 edges (80 of them MFMAs) and is bound by the rows' bytes.
//   dWedge product: A = the chunk's rows (lane l: row l&15 of a 16-row block, columns 32 s + 8 (l>>4) .. +7: one
//     16-B load), B = P[t]'s pieces (lane l: column n = l&15 -> relation n&7; first MFMA: lo for n < 8, none for
//     n >= 8; second: hi for n < 8, mid for n >= 8, into the same accumulator), so C[e][n] + C[e][n ^ 8] (one DPP row
//     rotate) is the dot product.
//   dP product: A = W^T rows (m < 8: relation m; m = 8: ones when DSUM), with the lo, mid and hi pieces in turn into
//     the same accumulators; B = the chunk transposed (8 consecutive edges of one column per lane),
//     read with ds_read_b64_tr_b16 from the row-major copy each wave keeps of its chunk in LDS (544-B row pitch, rows
//     8-15 of every 16 shifted 128 B (tsm_row): the 32 lanes of a transposed read hit distinct banks, the 8 of a row
//     write up to 2-way).
// Edges past the segment enter as zero rows with zero coefficients; every node (also an empty one) stores its dP rows.
// HEAD (ABI 9, iddgcn_tail_seg_reduce_head_bf16): the head chain's node terms of the same layer are added before the
// store, dP[r][n] = tail sum + Wn[n][r] head_dO[n] and dsum[n] = tail sum + head_dO[n], and the node's own part of the
// dynamic-weight gradient, dwh[n][r] = <head_dO[n], P_r[n]>, is formed from the P pieces already in registers (one
// 16x16x32 MFMA pair per k-step: rows 0-2 of A = the three bf16 pieces of head_dO[n], so all nine piece products
// enter), so the rest of the head backward (iddgcn_head_dz_f32) reads neither P nor head_dO again.
namespace tsm {
constexpr int D = 256, R = 8, CH = 32, PITCH = 544, CHB = CH * PITCH + 256;
}  // namespace tsm
// row r's slot: rows 8-15 of every 16 shifted 128 B (bank spread of the transposed reads), and each later 16-row half
// a further 128 B so that the shifted rows never reach into the next half's first row
__device__ __forceinline__ int tsm_row(int r) { return r * tsm::PITCH + ((r >> 3) & 1) * 128 + (r >> 4) * 128; }

template <bool DSUM, bool HEAD>
__global__ __launch_bounds__(256) void tail_seg_mfma8_kernel(int n_nodes, const int* __restrict__ seg_ptr,
                                                             const float* __restrict__ W, const __bf16* __restrict__ dO,
                                                             const float* __restrict__ P, long long p_rel_stride,
                                                             float* __restrict__ dP, long long dp_rel_stride,
                                                             float* __restrict__ dsum, float* __restrict__ dWedge,
                                                             const float* __restrict__ head_dO,
                                                             const float* __restrict__ Wn, float* __restrict__ dwh) {
    using namespace tsm;
    __shared__ __attribute__((aligned(16))) char lds[4 * CHB + (HEAD ? 4 * 1024 : 0)];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long n = (long long)blockIdx.x * 4 + wave;
    if (n >= n_nodes) return;                       // whole waves; the kernel has no barrier
    char* buf = lds + wave * CHB;
    const int beg = __builtin_amdgcn_readfirstlane(seg_ptr[n]);
    const int end = __builtin_amdgcn_readfirstlane(seg_ptr[n + 1]);
    const int i16 = lane & 15, g = lane >> 4;
    // HEAD: the node's head-seed row by one LDS-DMA (1 KiB, kept for dwh below and the store phase; loaded in the store
    // phase it doubled the launch, held in 16 more VGPRs it took the kernel past 256 registers) and this lane's 4
    // dynamic weights, issued before the P loads: the wait for those covers them
    float wn[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (HEAD) {
        __builtin_amdgcn_global_load_lds((gbl_vptr)(head_dO + n * D + lane * 4), (lds_vptr)(lds + 4 * CHB + wave * 1024),
                                         16, 0, 0);
        if (g < 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i) wn[i] = Wn[n * R + 4 * g + i];
        }
    }
    const __attribute__((address_space(3))) float* hrow =
        (const __attribute__((address_space(3))) float*)(lds + 4 * CHB + wave * 1024);
    // B pieces of the dWedge product: k-step s, lane l: P_{(l&15)&7}[t][32 s + 8 g + j] split3; pl: lo (l&15 < 8)
    // or 0, ph: hi (l&15 < 8) or mid
    bf16x8 pl[8], ph[8];
    {
        const float* pr = P + (long long)(i16 & 7) * p_rel_stride + n * D + 8 * g;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const f32x4 a = ld4(pr + 32 * s), b = ld4(pr + 32 * s + 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 hi, mid, lo;
                split3(j < 4 ? a[j] : b[j - 4], hi, mid, lo);
                ph[s][j] = i16 < 8 ? hi : mid;
                pl[s][j] = i16 < 8 ? lo : (__bf16)0.0f;
            }
        }
    }
    if constexpr (HEAD) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the head-seed row's DMA
        // dwh[n][r] = <head_dO[n], P_r[n]>: A row m < 3 = piece m of head_dO[n] (columns 32 s + 8 g + j), B = the P
        // pieces (pl: lo | 0, ph: hi | mid), so C[m][r] + C[m][r + 8] summed over m holds all nine piece products
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const f32x4 x0 = *(const __attribute__((address_space(3))) f32x4*)(hrow + 32 * s + 8 * g);
            const f32x4 x1 = *(const __attribute__((address_space(3))) f32x4*)(hrow + 32 * s + 8 * g + 4);
            bf16x8 a;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 hi, mid, lo;
                split3(j < 4 ? x0[j] : x1[j - 4], hi, mid, lo);
                a[j] = i16 == 0 ? hi : i16 == 1 ? mid : i16 == 2 ? lo : (__bf16)0.0f;
            }
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pl[s], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ph[s], c, 0, 0, 0);
        }
        // lanes 0-15 hold C[0..3][l&15]: rows 0-2 are the pieces
        const float v = (c[0] + c[1]) + c[2];
        const float tot = v + dpp<0x128>(v);
        if (lane < 8) dwh[n * R + lane] = tot;
    }
    f32x4 acc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    typedef __attribute__((address_space(3))) u32x4* lu4;
    typedef __attribute__((address_space(3))) v4s16* l4p;
    // transposed-read address of this lane: rows 8 g + ((l>>2)&3) (+4: second read), columns 4 (l&3) of a block
    const int tr0 = tsm_row(8 * g + ((lane >> 2) & 3)) + 8 * (lane & 3);
    const int tr1 = tsm_row(8 * g + 4 + ((lane >> 2) & 3)) + 8 * (lane & 3);
    for (int c0 = beg; c0 < end; c0 += CH) {
        const int cnt = end - c0 < CH ? end - c0 : CH;
        // the chunk's row fragments (block b: rows 16 b + (l&15); zero past the segment)
        u32x4 fr[2][8];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const bool ok = 16 * b + i16 < cnt;
            const __bf16* row = dO + (long long)(ok ? c0 + 16 * b + i16 : c0) * D + 8 * g;
#pragma unroll
            for (int s = 0; s < 8; ++s)
                fr[b][s] = ok ? *reinterpret_cast<const u32x4*>(row + 32 * s) : u32x4{0u, 0u, 0u, 0u};
        }
        // W^T rows of the dP product: lane l: row m = l&15, edges 8 g + j of the chunk, split3
        bf16x8 wh, wm, wl;
        {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int e = 8 * g + j;
                float w = 0.f;
                if (i16 < 8 && e < cnt) w = W[(long long)(c0 + e) * R + i16];
                __bf16 hi, mid, lo;
                split3(w, hi, mid, lo);
                wh[j] = (DSUM && i16 == 8 && e < cnt) ? (__bf16)1.0f : hi;
                wm[j] = mid;
                wl[j] = lo;
            }
        }
        // row-major copy of the chunk for the transposed reads
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int s = 0; s < 8; ++s) *(lu4)(buf + tsm_row(16 * b + i16) + 64 * s + 16 * g) = fr[b][s];
        // dWedge: two 16-edge blocks x 8 k-steps
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const bf16x8 a = __builtin_bit_cast(bf16x8, fr[b][s]);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pl[s], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ph[s], c, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v = c[i] + dpp<0x128>(c[i]);      // (hi + lo) + the mid column (lane (l&15) ^ 8)
                const int e = 16 * b + 4 * g + i;
                if (i16 < 8 && e < cnt) dWedge[(long long)(c0 + e) * R + i16] = v;
            }
        }
        // dP (+ dsum): 16 column blocks, lo, mid and hi pieces of W
#pragma unroll
        for (int cb = 0; cb < 16; ++cb) {
            const v4s16 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)(buf + tr0 + 32 * cb));
            const v4s16 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((l4p)(buf + tr1 + 32 * cb));
            const bf16x8 bx = __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, bx, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, bx, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, bx, acc[cb], 0, 0, 0);
        }
    }
    // lane l holds rows 4 g + i (relations 0-3: g = 0, 4-7: g = 1, dsum: g = 2, i = 0) of columns 16 cb + (l&15)
#pragma unroll
    for (int cb = 0; cb < 16; ++cb) {
        const long long col = n * D + 16 * cb + i16;
        const float hd = HEAD ? hrow[16 * cb + i16] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = 4 * g + i;
            if (m < 8) dP[m * dp_rel_stride + col] = HEAD ? fmaf(wn[i], hd, acc[cb][i]) : acc[cb][i];
            else if (DSUM && m == 8) dsum[col] = HEAD ? acc[cb][i] + hd : acc[cb][i];
        }
    }
}

// ---------------------------------------------------------------------------
// head-chain node backward (one layer)
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void head_bwd_node_kernel(int n_nodes, int R, const float* __restrict__ dO,
                                                            const float* __restrict__ P, long long p_rel_stride,
                                                            const float* __restrict__ Ssm,
                                                            const float* __restrict__ W,
                                                            const int* __restrict__ hseg_ptr,
                                                            const int* __restrict__ hperm,
                                                            const float* __restrict__ dWedge,
                                                            const float* __restrict__ ep_in,
                                                            float* __restrict__ dP, long long dp_rel_stride,
                                                            float* __restrict__ dsum, float* __restrict__ dz) {
    constexpr int LPR = D / 4;
    const long long n = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
    const int sub = threadIdx.x % LPR;
    const bool live = n < n_nodes;
    f32x4 d = {0.f, 0.f, 0.f, 0.f};
    if (live) d = ld4(dO + n * D + sub * 4);
    if (live && dsum) {
        float* sp = dsum + n * D + sub * 4;
        st4(sp, ld4(sp) + d);
    }
    const int beg = (live && hseg_ptr) ? hseg_ptr[n] : 0;
    const int end = (live && hseg_ptr) ? hseg_ptr[n + 1] : 0;
    // edge contributions, one pass over the head segment for every relation: lane sub takes
    // k = beg+sub, beg+sub+LPR, ... and reads the edge's R contiguous dWedge values
    float ep[MAX_R];
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) ep[r] = 0.f;
    for (int k = beg + sub; k < end; k += LPR) {
        const float* dwe = dWedge + (long long)hperm[k] * R;
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
            if (r < R) ep[r] += dwe[r];
    }
    // node-partitioned steps: the head sums arrive complete from the ranks (iddgcn_head_wsum_f32 + reduce-scatter)
    if (ep_in && live && sub == 0) {
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
            if (r < R) ep[r] += ep_in[n * R + r];
    }
    float dw[MAX_R];
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) {
        float part = 0.f;
        if (r < R) {
            if (live) {
                const f32x4 q = d * ld4(P + r * p_rel_stride + n * D + sub * 4);
                part = q[0] + q[1] + q[2] + q[3];
            }
            part += ep[r];
        }
        dw[r] = r < R ? group_sum<LPR>(part) : 0.f;
    }
    if (!live) return;
    float s[MAX_R], w[MAX_R], dsv[MAX_R];
    float dot = 0.f;
#pragma unroll
    for (int r = 0; r < MAX_R; ++r)
        if (r < R) {
            s[r] = Ssm[n * R + r];
            w[r] = W[n * R + r];
            dsv[r] = dw[r] * w[r] * (1.0f - w[r]);
            dot += dsv[r] * s[r];
        }
    if (sub == 0) {
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
            if (r < R) dz[n * R + r] = (dsv[r] - dot) * s[r];
    }
    if (!dP) return;                 // (ABI 9) the dP term was added by iddgcn_tail_seg_reduce_head_bf16
#pragma unroll
    for (int r = 0; r < MAX_R; ++r)
        if (r < R) {
            float* pp = dP + r * dp_rel_stride + n * D + sub * 4;
            st4(pp, ld4(pp) + w[r] * d);
        }
}

// dst[e][:] = src[idx[e]][:] for a row width of 4 or 8 floats: one thread per edge, 16-B loads and stores (the
// per-element form below spent one index load and a 4-B access per float: 1.14 ms per config-5 launch)
template <int W>
__global__ __launch_bounds__(256) void gather_rows_vec_kernel(long long M, const float* __restrict__ src,
                                                              const int* __restrict__ idx, float* __restrict__ dst) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= M) return;
    const float* s = src + (long long)idx[e] * W;
#pragma unroll
    for (int q = 0; q < W; q += 4) st4(dst + e * W + q, ld4(s + q));
}
// dst[e][j] = src[idx[e]][j] for a narrow row width (per-edge copies of node tables)
__global__ __launch_bounds__(256) void gather_rows_kernel(long long M, int width, const float* __restrict__ src,
                                                          const int* __restrict__ idx, float* __restrict__ dst) {
    const long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= M * width) return;
    const long long e = x / width;
    const int j = (int)(x % width);
    dst[x] = src[(long long)idx[e] * width + j];
}

// out[n][r] = sum_{k in [hptr[n], hptr[n+1])} w[hperm[k]][r]: the per-head sums of per-edge narrow rows (the
// dWedge head sums of a node-partitioned step), one thread per (node, relation), the segment in order
__global__ __launch_bounds__(256) void head_wsum_kernel(int n_nodes, int R, const int* __restrict__ hptr,
                                                        const int* __restrict__ hperm, const float* __restrict__ w,
                                                        float* __restrict__ out) {
    const long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= (long long)n_nodes * R) return;
    const long long n = x / R;
    const int r = (int)(x % R);
    float s = 0.f;
    for (int k = hptr[n]; k < hptr[n + 1]; ++k) s += w[(long long)hperm[k] * R + r];
    out[x] = s;
}

// The rest of the head backward after iddgcn_tail_seg_reduce_head_bf16: 8 lanes per node, lane r < R owning
// relation r: dW_r = dwh[n][r] + the head segment's dWedge rows (in segment order; the 8 lanes of a node read one
// row's R contiguous floats together), then the softmax-sigmoid backward of head_bwd_node_kernel -> dz (the 8-lane
// dot product by three xor shuffles).  One thread per node with the whole row per thread ran 1.83 ms per config-5
// launch, latency-bound on its serial row loads.
__global__ __launch_bounds__(256) void head_dz_kernel(int n_nodes, int R, const float* __restrict__ Ssm,
                                                      const float* __restrict__ W, const int* __restrict__ hptr,
                                                      const int* __restrict__ hperm, const float* __restrict__ dWedge,
                                                      const float* __restrict__ dwh, float* __restrict__ dz) {
    const long long x = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long n = x >> 3;
    const int r = (int)(x & 7);
    const bool live = n < n_nodes;
    const bool on = live && r < R;
    float dw = on ? dwh[n * R + r] : 0.f;
    const int beg = live ? hptr[n] : 0, end = live ? hptr[n + 1] : 0;
    for (int k = beg; k < end; ++k)
        if (on) dw += dWedge[(long long)hperm[k] * R + r];
    const float sv = on ? Ssm[n * R + r] : 0.f;
    const float w = on ? W[n * R + r] : 0.f;
    const float dsv = dw * w * (1.0f - w);
    float dot = dsv * sv;
    dot += __shfl_xor(dot, 1, 8);
    dot += __shfl_xor(dot, 2, 8);
    dot += __shfl_xor(dot, 4, 8);
    if (on) dz[n * R + r] = (dsv - dot) * sv;
}

__global__ __launch_bounds__(256) void reduce_slabs_kernel(int n_slabs, long long n, const float* __restrict__ slab,
                                                           float* __restrict__ out, int accumulate, float scale) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
#pragma unroll 8
    for (int b = 0; b < n_slabs; ++b) s += slab[(long long)b * n + i];
    s *= scale;
    out[i] = accumulate ? out[i] + s : s;
}
// The same sums for n % 4 == 0 and a 16-B aligned slab: lane = one float4 column group (1 KB per wave load
// instead of 256 B), the 4 waves of a block take fixed quarters of the slab range, combined in wave order
// through LDS (deterministic; the association differs from reduce_slabs_kernel's single chain).  `out` may
// be only 4-B aligned (weights inside the flat gradient buffer): scalar stores.
__global__ __launch_bounds__(256) void reduce_slabs4_kernel(int n_slabs, long long n4, const f32x4* __restrict__ slab,
                                                            float* __restrict__ out, int accumulate, float scale) {
    __shared__ f32x4 part[3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long i = (long long)blockIdx.x * 64 + lane;
    const int b0 = (int)((long long)n_slabs * w / 4), b1 = (int)((long long)n_slabs * (w + 1) / 4);
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
#pragma unroll 8
        for (int b = b0; b < b1; ++b) s += slab[(long long)b * n4 + i];
    }
    if (w > 0) part[w - 1][lane] = s;
    __syncthreads();
    if (w == 0 && i < n4) {
        s += part[0][lane];
        s += part[1][lane];
        s += part[2][lane];
        s *= scale;
        float* o = out + 4 * i;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = accumulate ? o[q] + s[q] : s[q];
    }
}
// Any n, many slabs (the W_alpha TN's 1024 partials of (D + 1) R floats, the DistMult loss / drel partials):
// 64 outputs per 1024-thread block, the 16 waves take fixed sixteenths of the slab range (one chain each),
// combined in wave order through LDS.
__global__ __launch_bounds__(1024) void reduce_slabs_split_kernel(int n_slabs, long long n, const float* __restrict__ slab,
                                                                  float* __restrict__ out, int accumulate, float scale) {
    __shared__ float part[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long i = (long long)blockIdx.x * 64 + lane;
    const int b0 = (int)((long long)n_slabs * w / 16), b1 = (int)((long long)n_slabs * (w + 1) / 16);
    float s = 0.f;
    if (i < n) {
#pragma unroll 8
        for (int b = b0; b < b1; ++b) s += slab[(long long)b * n + i];
    }
    part[w][lane] = s;
    __syncthreads();
    if (w == 0 && i < n) {
        float t = part[0][lane];
#pragma unroll
        for (int q = 1; q < 16; ++q) t += part[q][lane];
        t *= scale;
        out[i] = accumulate ? out[i] + t : t;
    }
}
void launch_reduce_slabs(hipStream_t st, int n_slabs, long long n, const float* slab, float* out, int accumulate,
                         float scale) {
    // the float4 form gives one 64-output block per 256 threads: below ~64 blocks (e.g. DistMult's R x D drel
    // partials, 2 blocks summing 2048 slabs in 43 us) the 16-wave split form spreads the slabs wider
    const bool few_blocks = n / 4 < 64 * 64 && n_slabs >= 64;
    if (n % 4 == 0 && n_slabs >= 8 && !few_blocks && (reinterpret_cast<uintptr_t>(slab) & 15) == 0) {
        const long long n4 = n / 4;
        hipLaunchKernelGGL(reduce_slabs4_kernel, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st, n_slabs, n4,
                           reinterpret_cast<const f32x4*>(slab), out, accumulate, scale);
    } else if (n_slabs >= 64) {
        hipLaunchKernelGGL(reduce_slabs_split_kernel, dim3((unsigned)((n + 63) / 64)), dim3(1024), 0, st, n_slabs, n,
                           slab, out, accumulate, scale);
    } else {
        hipLaunchKernelGGL(reduce_slabs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n_slabs, n, slab,
                           out, accumulate, scale);
    }
}

__global__ __launch_bounds__(256) void adam_kernel(long long n, float* __restrict__ var, float* __restrict__ m,
                                                   float* __restrict__ v, const float* __restrict__ g, float alpha,
                                                   float b1, float b2, float eps, int sparse_form,
                                                   const float* __restrict__ alpha_table,
                                                   const int* __restrict__ step) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (alpha_table) alpha = alpha_table[*step];    // graph-replayable form: alpha of this iteration
    const float gi = g[i];
    float mi = m[i], vi = v[i];
    if (sparse_form) {
        mi = mi * b1 + gi * (1.0f - b1);
        vi = vi * b2 + (gi * gi) * (1.0f - b2);
    } else {
        mi = mi + (gi - mi) * (1.0f - b1);
        vi = vi + (gi * gi - vi) * (1.0f - b2);
    }
    m[i] = mi;
    v[i] = vi;
    var[i] = var[i] - (mi * alpha) / (sqrtf(vi) + eps);
}

// end of a graph-replayed training step: record the step's loss, advance the iteration counter
__global__ void step_advance_kernel(int* __restrict__ step, float* __restrict__ loss_history,
                                    const float* __restrict__ loss) {
    if (threadIdx.x != 0) return;
    const int s = *step;
    if (loss_history && loss) loss_history[s] = *loss;
    *step = s + 1;
}

// ---- D = 256 row-GEMM variant selection (rowgemm256_v3_kernel) ----
struct V3Sel {
    int nv;                 // gathered V tables (template NV)
    bool aux, hc;
    bool cw = false;        // broadcast V with R > 2 coefficients
    bool pl = false;        // planes C (gathered forward) / planes sigma' operand (backward)
    bool split = false;     // IDDGCN_GEMM_SPLIT_F16 operands (template X3), else exact f32
    bool c4 = false;        // IDDGCN_GEMM_F32_4CHAIN (template C4)
    bool same(const V3Sel& o) const {
        return nv == o.nv && aux == o.aux && hc == o.hc && cw == o.cw && pl == o.pl && split == o.split &&
               c4 == o.c4;
    }
};
// Which v3 instantiation computes this call, or false (the register-staged rowgemm_kernel<256> then runs:
// a gathered V with the sigma' epilogue, or V rows that are not dense D-float rows).
bool v3_select(const RowGemmP& p, V3Sel& sel) {
    const bool gatherV = p.R > 0 && p.v_row_stride != 0;
    const bool dsig = p.act == IDDGCN_ACT_DSIGMOID;
    if (gatherV) {
        if (dsig || p.v_row_stride != 256) return false;
        // R <= 2: exactly R slabs; more relations: capped slabs (rows past the cap of a tile come from L2)
        sel = {p.R <= 2 ? p.R : (p.R <= 4 ? 4 : 8), false, true};
    } else {
        sel = {0, dsig, p.R > 0, p.R > 2};
    }
    sel.split = p.precision == IDDGCN_GEMM_SPLIT_F16;
    sel.c4 = p.precision == IDDGCN_GEMM_F32_4CHAIN;
    if (sel.c4 && (sel.nv || sel.aux || sel.hc)) return false;      // C4 at D = 256: plain form only
    sel.pl = (p.planes & (IDDGCN_PLANES_C | IDDGCN_PLANES_AUX)) != 0;
    if (!sel.pl) return true;
    // the planes forms: C planes on the R <= 2 gathered forward, sigma' planes on the plain backward
    if ((p.planes & IDDGCN_PLANES_C) && !(sel.nv >= 1 && sel.nv <= 2 && !sel.aux)) return false;
    if ((p.planes & IDDGCN_PLANES_AUX) && !(sel.aux && sel.nv == 0 && !sel.hc)) return false;
    return true;
}

// The device-side copy of one iddgcn_rowgemm_t (tiles_per_block is set at launch).
RowGemmP to_p(const iddgcn_rowgemm_t& a) {
    RowGemmP p;
    p.M = a.M; p.A = a.A; p.a_idx = a.a_idx; p.B = a.B; p.b_trans = a.b_trans;
    p.C = a.C; p.accumulate = a.accumulate; p.R = a.R; p.coef = a.coef; p.coef_idx = a.coef_idx;
    p.V = a.V; p.v_idx = a.v_idx; p.v_rel_stride = a.v_rel_stride; p.v_row_stride = a.v_row_stride;
    p.act = a.act; p.aux = a.aux; p.planes = a.planes; p.precision = a.precision;
    p.tiles_per_block = 1;
    return p;
}
// Argument check shared by the f32 row-GEMM entries (0 = fine).  Planes operands (IDDGCN_PLANES_*) need
// D = 256, the split-fp16 mode and the v3 kernel; a planes C holds sigmoid outputs only.
int check_rowgemm(const iddgcn_rowgemm_t& a) {
    if (!dim_ok(a.D)) return IDDGCN_E_BAD_DIM;
    if (a.R < 0 || a.R > MAX_R) return IDDGCN_E_BAD_REL;
    if (a.precision != IDDGCN_GEMM_EXACT_F32 && a.precision != IDDGCN_GEMM_SPLIT_F16 &&
        a.precision != IDDGCN_GEMM_F32_4CHAIN && a.precision != IDDGCN_GEMM_BF16X3)
        return IDDGCN_E_BAD_ARG;
    // F32_4CHAIN at D = 256: the plain form (no coefficients, no sigma' operand, no planes)
    if (a.precision == IDDGCN_GEMM_F32_4CHAIN && a.D == 256 && (a.R > 0 || a.act == IDDGCN_ACT_DSIGMOID || a.planes))
        return IDDGCN_E_BAD_ARG;
    if (a.M == 0) return 0;
    if (a.M < 0 || !a.A || !a.B || !a.C) return IDDGCN_E_BAD_ARG;
    if (a.R > 0 && (!a.coef || !a.V)) return IDDGCN_E_BAD_ARG;
    if (a.act == IDDGCN_ACT_DSIGMOID && !a.aux) return IDDGCN_E_BAD_ARG;
    if (a.act < IDDGCN_ACT_NONE || a.act > IDDGCN_ACT_DSIGMOID) return IDDGCN_E_BAD_ARG;
    if (a.planes) {
        if (a.planes & ~(IDDGCN_PLANES_A | IDDGCN_PLANES_C | IDDGCN_PLANES_AUX)) return IDDGCN_E_BAD_ARG;
        if (a.D != 256 || a.precision != IDDGCN_GEMM_SPLIT_F16 || a.a_idx) return IDDGCN_E_BAD_ARG;
        if ((a.planes & IDDGCN_PLANES_C) && (a.act != IDDGCN_ACT_SIGMOID || a.accumulate)) return IDDGCN_E_BAD_ARG;
        if ((a.planes & IDDGCN_PLANES_AUX) && a.act != IDDGCN_ACT_DSIGMOID) return IDDGCN_E_BAD_ARG;
        V3Sel sel;
        if (!v3_select(to_p(a), sel)) return IDDGCN_E_BAD_ARG;
    }
    return 0;
}

// The bf16x3 row GEMM's forms (rowgemm256_b3_kernel<NV, AUX, BC>): plain, C += A B, sigma' backward (AUX),
// gathered-combine forward with exactly R = NV in {1, 2} per-edge coefficients, broadcast V with R <= 2 row
// coefficients (BC, plain or sigma'); no a_idx, coef_idx or planes.
bool b3_select(const RowGemmP& p, int& nv, bool& aux, bool& bc) {
    bc = false;
    if (p.precision != IDDGCN_GEMM_BF16X3 || p.a_idx || p.planes) return false;
    if (p.R > 0 && p.v_row_stride == 0 && !p.v_idx) {
        // broadcast V (one row per relation for every output row: dz W_a^T), plain or with the sigma' factor
        if (p.R > 2 || p.coef_idx || p.accumulate || p.act == IDDGCN_ACT_SIGMOID) return false;
        nv = 0;
        aux = p.act == IDDGCN_ACT_DSIGMOID;
        bc = true;
        return true;
    }
    if (p.R > 0) {
        if (p.R > 2 || p.v_row_stride != 256 || p.coef_idx || p.act == IDDGCN_ACT_DSIGMOID || p.accumulate) return false;
        nv = p.R;
        aux = false;
        return true;
    }
    // C += A B (act none): the sigma' kernel's aux slab carries the old C rows (read before the tile is stored)
    if (p.accumulate && p.act != IDDGCN_ACT_NONE) return false;
    nv = 0;
    aux = p.act == IDDGCN_ACT_DSIGMOID || p.accumulate;
    return true;
}
// ~128 row ranges (a multiple of 8) x 2 column halves: one workgroup per CU, every one resident
void launch_b3(hipStream_t st, RowGemmP p, int nv, bool aux, bool bc) {
    const long long nt = ((long long)p.M + rb3::TR - 1) / rb3::TR;
    long long nr = nt < 128 ? nt : 128;
    p.tiles_per_block = (int)((nt + nr - 1) / nr);
    nr = (nt + p.tiles_per_block - 1) / p.tiles_per_block;
    nr = (nr + 7) / 8 * 8;
    const int n_ranges = (int)nr;
    if (p.accumulate) p.aux = p.C;
    const dim3 g((unsigned)(2 * nr)), blk(512);
    if (bc && aux) hipLaunchKernelGGL((rowgemm256_b3_kernel<0, true, true>), g, blk, 0, st, p, n_ranges);
    else if (bc) hipLaunchKernelGGL((rowgemm256_b3_kernel<0, false, true>), g, blk, 0, st, p, n_ranges);
    else if (nv == 1) hipLaunchKernelGGL((rowgemm256_b3_kernel<1, false>), g, blk, 0, st, p, n_ranges);
    else if (nv == 2) hipLaunchKernelGGL((rowgemm256_b3_kernel<2, false>), g, blk, 0, st, p, n_ranges);
    else if (aux) hipLaunchKernelGGL((rowgemm256_b3_kernel<0, true>), g, blk, 0, st, p, n_ranges);
    else hipLaunchKernelGGL((rowgemm256_b3_kernel<0, false>), g, blk, 0, st, p, n_ranges);
}

// One launch of up to ROWGEMM_BATCH v3 GEMMs of the same variant (blockIdx.y = entry).  The persistent
// grid is ~256 workgroups in all (one per CU: 131-155 KB of LDS each), shared out over the entries.
void launch_v3(hipStream_t st, RowGemmBatch& pb, int n, const V3Sel& sel, bool bf = false) {
    // floor: every workgroup of the launch resident at once (ceil gave 7 entries 37 x 7 = 259 > 256 CUs, so three
    // workgroups ran in a second wave and the launch took ~2x)
    const long long per = n > 0 ? (256 / n > 0 ? 256 / n : 1) : 256;
    long long nbmax = 0;
    for (int k = 0; k < n; ++k) {
        RowGemmP& p = pb.p[k];
        const long long nt = ((long long)p.M + r3::TR - 1) / r3::TR;
        long long nb = nt < per ? nt : per;
        if (nb < 1) nb = 1;
        p.tiles_per_block = (int)((nt + nb - 1) / nb);
        if (p.tiles_per_block < 1) p.tiles_per_block = 1;
        nb = (nt + p.tiles_per_block - 1) / p.tiles_per_block;
        if (nb > nbmax) nbmax = nb;
    }
    if (nbmax == 0) return;
    const dim3 g((unsigned)nbmax, (unsigned)n), blk(512);
    if (bf) {      // bf16 edge tables: gathered-combine forward, sigma' backward, plain
#define V3B(NV, AUX, HC)                                                                                         \
    do {                                                                                                          \
        if (pb.p[0].precision == IDDGCN_GEMM_BF16)                                                                \
            hipLaunchKernelGGL((rowgemm256_v3_kernel<NV, AUX, HC, true, false, true, false, false, true>), g, blk, 0, st, pb); \
        else hipLaunchKernelGGL((rowgemm256_v3_kernel<NV, AUX, HC, true, false, true>), g, blk, 0, st, pb);        \
    } while (0)
        if (sel.nv == 1) V3B(1, false, true);
        else if (sel.nv == 2) V3B(2, false, true);
        else if (sel.nv == 4) V3B(4, false, true);
        else if (sel.nv == 8) V3B(8, false, true);
        else if (sel.aux) V3B(0, true, false);
        else V3B(0, false, false);
#undef V3B
        return;
    }
    const bool x3 = sel.split;
#define V3L(NV, AUX, HC)                                                                        \
    {                                                                                           \
        if (x3) hipLaunchKernelGGL((rowgemm256_v3_kernel<NV, AUX, HC, true>), g, blk, 0, st, pb); \
        else hipLaunchKernelGGL((rowgemm256_v3_kernel<NV, AUX, HC, false>), g, blk, 0, st, pb);   \
    }
#define V3W(AUX)                                                                                     \
    {                                                                                                \
        if (x3) hipLaunchKernelGGL((rowgemm256_v3_kernel<0, AUX, true, true, true>), g, blk, 0, st, pb); \
        else hipLaunchKernelGGL((rowgemm256_v3_kernel<0, AUX, true, false, true>), g, blk, 0, st, pb);   \
    }
    if (sel.c4) {           // check_rowgemm / v3_select: the plain f32 form
        hipLaunchKernelGGL((rowgemm256_v3_kernel<0, false, false, false, false, false, false, true>), g, blk, 0, st, pb);
    } else if (sel.pl) {    // check_rowgemm: split mode
        if (sel.nv == 1) hipLaunchKernelGGL((rowgemm256_v3_kernel<1, false, true, true, false, false, true>), g, blk, 0, st, pb);
        else if (sel.nv == 2) hipLaunchKernelGGL((rowgemm256_v3_kernel<2, false, true, true, false, false, true>), g, blk, 0, st, pb);
        else hipLaunchKernelGGL((rowgemm256_v3_kernel<0, true, false, true, false, false, true>), g, blk, 0, st, pb);
    } else if (sel.nv == 1) V3L(1, false, true)
    else if (sel.nv == 2) V3L(2, false, true)
    else if (sel.nv == 4) V3L(4, false, true)
    else if (sel.nv == 8) V3L(8, false, true)
    else if (sel.hc && sel.cw) {
        if (sel.aux) V3W(true)
        else V3W(false)
    } else if (sel.hc && sel.aux) V3L(0, true, true)
    else if (sel.hc) V3L(0, false, true)
    else if (sel.aux) V3L(0, true, false)
    else V3L(0, false, false)
#undef V3L
#undef V3W
}

// the run combine (D = 256) writing bf16 rows (BF) or planes rows (PL)
template <bool BF, bool PL>
int run_combine_out(void* stream, int M, int d, int R, const float* Y, const int* idx, const float* coef,
                    const float* V, long long v_rel_stride, void* out) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (R < 0 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (M < 0 || !Y || !idx || !out || (R > 0 && (!coef || !V))) return IDDGCN_E_BAD_ARG;
    if (M == 0) return 0;
    const long long nchunk = ((long long)M + RC_CH - 1) / RC_CH;
    long long nb = (nchunk + 3) / 4;
    if (nb > 2048) nb = 2048;
    hipStream_t st = (hipStream_t)stream;
    float* o = (float*)out;
#define RCB(RR) hipLaunchKernelGGL((run_combine256_kernel<RR, BF, PL>), dim3((unsigned)nb), dim3(256), 0, st, M, Y, idx, coef, V, v_rel_stride, o)
    switch (R) {
        case 0: RCB(0); break;
        case 1: RCB(1); break;
        case 2: RCB(2); break;
        case 3: RCB(3); break;
        case 4: RCB(4); break;
        case 5: RCB(5); break;
        case 6: RCB(6); break;
        case 7: RCB(7); break;
        default: RCB(8); break;
    }
#undef RCB
    return launch_status();
}

inline unsigned grid_for(long long rows, int lpr) {
    const long long threads = rows * lpr;
    return (unsigned)((threads + 255) / 256);
}

// ---------------------------------------------------------------------------
// Forward edge GEMM of the bf16-feature mode at R = 8 (config 5; round 4, replaces rowgemm256_v3_kernel<8, ..., BF>
// for this form): x^l[e] = act(x^{l-1}[e] S + sum_r coef[e][r] V_r[v_idx[e]])  (IDDGCN.py:76-77 with the node-level
// P_r^l = AE_r K_r^l as V), A and C bf16 edge tables, S fp32 as bf16 hi + lo pieces, coef [M][8] fp32 per edge,
// V = 8 fp32 node tables v_rel_stride apart.  64-row tiles; wave w owns output columns 32w..32w+31.  Both terms run
// on v_mfma_f32_16x16x32_bf16 with the weight / node-row side as operand A, so lane l ends with edge row l&15 of each
// 16-row block at 4 consecutive columns: one 8-B bf16 store per 16 x 16 block, no LDS staging of the output.
//   x S:     k-step q: A = S^T pieces (registers, 128 VGPRs: the wave's 32 columns x 256 k x hi / lo), B = 8
//            consecutive k of an edge row straight from the LDS-DMA'd A tile (512-B row slots, 16-B chunks XOR-
//            swizzled by row, two rows per full-wave DMA; round 4: 528-B slots, one half-wave DMA per row; either
//            way the b128 fragment reads are conflict-free).
//   combine: the tile's distinct V rows ("slots": runs of equal v_idx; tail-sorted config-5 edges give 1-3 per
//            64-row tile) are the k axis, k = 8 s + r for slot s < 4 of a block of four: A = V_r[slot s] at the lane's
//            column (hi / lo), B = coef[e][r] where slot(e) = s, else 0 (hi / lo); three products (hi hi, hi lo,
//            lo hi) per 16 x 16 block.  Slots 0-3 come by LDS-DMA (one instruction per slot: 8 relations x the wave's
//            32 columns) a whole MFMA phase ahead; later slots of a tile (short runs, unsorted v_idx) are DMA'd when
//            their block comes up.  The combine products carry 16 significant bits, as the weights' hi + lo do, 2^8
//            below the bf16 rounding of the stored output.
// The v3 epilogue this replaces read 8 KiB of fp32 V slab per edge row from LDS and ran 2048 FMAs per row on the
// VALU; here the combine is 24 MFMAs per 64 x 32 wave tile plus 16 LDS reads and 48 two-piece splits per lane.
// Schedule (every wave alike): A(t+2) DMA; wait for tile t-1's slots and A(t+1); combine of t-1 (into a second
// accumulator set); prepare t (slots, coefficients, the next v_idx: wave-private, producer = consumer, the wave's own
// vmcnt); MFMAs of t with t-1's activation, conversion and stores issued one 16 x 16 block per k-step between them
// (18.5-18.6 vs 18.7-18.8 ms, bitwise the same; profiles/r04/fg8/probe_overlap_ab.log); one barrier per tile
// (A buffers, three deep).  Measured per config-5 launch (tools/fg8_probe.py, one box): v3
// kernel 24.7 ms; this design at 32-row tiles 20.6 ms with the v3 stagger (waves 4-7 one epilogue behind), 19.7 ms
// all waves alike; 64-row tiles 18.1 ms; the stagger at 64 rows 20.3 ms (profiles/r04/fg8/).
namespace fg8 {
constexpr int D = 256, R = 8, TR = 64, NW = 8, NBUF = 3;
constexpr int RPW = TR / NW;                             // A rows each wave DMAs per tile
constexpr int PITCH = 512;                               // bytes per bf16 A row slot, 16-B chunks XOR-swizzled
constexpr int ABUF = TR * PITCH;                         // 32,768 B per A buffer
constexpr int CAPS = 4;                                  // slots staged in LDS per tile (one block of the k axis)
constexpr int SLOTB = 1088;                              // bytes per slot: [8 relations][32 columns] fp32 + 64 pad
// per wave: v_idx [64], slot -> V row [64], coefficients [64][8], slots
constexpr int WIDX = 0, WTAIL = 256, WCOEF = 512, WV = WCOEF + TR * R * 4;
constexpr int WREG = WV + CAPS * SLOTB;                  // 6,912 B per wave
constexpr int LDSB = NBUF * ABUF + NW * WREG;            // 153,600 B
static_assert(LDSB <= 160 * 1024, "LDS budget");
}  // namespace fg8

template <bool HL>
__global__ __launch_bounds__(512) void fwd_gather8_bf16_kernel(RowGemmP p) {
    using namespace fg8;
    __shared__ __attribute__((aligned(16))) char lds[LDSB];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // per-lane index math inside the tile loop starts from an opaque copy of the lane id, so the compiler recomputes
    // it (a few VALU ops) instead of hoisting every loop-invariant address and mask out of the loop (hoisted, they
    // took the kernel past 256 VGPRs and into scratch, whose loads' vmcnt waits drain the DMAs in flight)
    auto fresh_lane = [&]() __attribute__((always_inline)) {
        int l = lane;
        asm volatile("" : "+v"(l));
        return l;
    };
    const int i16 = lane & 15, g = lane >> 4;
    const int c0 = wave * 32;
    char* wreg = lds + NBUF * ABUF + wave * WREG;
    int* idxw = reinterpret_cast<int*>(wreg + WIDX);
    int* tailw = reinterpret_cast<int*>(wreg + WTAIL);
    float* coefw = reinterpret_cast<float*>(wreg + WCOEF);
    char* vsl = wreg + WV;
    const long long vrs = p.v_rel_stride;

    const long long ntiles = ((long long)p.M + TR - 1) / TR;
    const long long t_beg = (long long)blockIdx.x * p.tiles_per_block;
    long long t_end = t_beg + p.tiles_per_block;
    if (t_end > ntiles) t_end = ntiles;
    if (t_beg >= t_end) return;                          // whole workgroup: before any barrier
    const long long Mlast = (long long)p.M - 1;
    auto clampe = [&](long long e) __attribute__((always_inline)) { return e > Mlast ? Mlast : e; };

    // weights: lane (g, i16), column block cb, k-step q: S[32q + 8g + j][c0 + 16cb + i16], j < 8, as bf16 hi + lo
    bf16x8 wh[2][8], wl[2][HL ? 8 : 1];
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float w = p.B[(32 * q + 8 * g + j) * D + c0 + 16 * cb + i16];
                const __bf16 hi = (__bf16)w;
                wh[cb][q][j] = hi;
                if constexpr (HL) wl[cb][q][j] = (__bf16)(w - (float)hi);
            }

    // vector-memory ops this wave has issued (wave-uniform): a wait for "op k and everything older" is
    // s_waitcnt vmcnt(nops - k) (ops complete in issue order; LDS-DMA, loads and stores count alike)
    int nops = 0;
    // A(t): the wave's 8 rows, two per full-wave DMA: lane i -> row r0 + (i >> 5), LDS chunk i & 31 of that row's slot,
    // global chunk (i & 31) ^ (row & 15) (the swizzle that makes the fragment reads below conflict-free without a pad)
    auto dma_A = [&](long long t, int b) __attribute__((always_inline)) {
        const int lane = fresh_lane();
#pragma unroll
        for (int j = 0; j < RPW / 2; ++j) {
            const int r0 = wave * RPW + 2 * j;
            const int r = r0 + (lane >> 5);
            const char* gp = reinterpret_cast<const char*>(p.A) + clampe(t * TR + r) * (D * 2) +
                             ((lane & 31) ^ (r & 15)) * 16;
            __builtin_amdgcn_global_load_lds((gbl_vptr)gp, (lds_vptr)(lds + b * ABUF + r0 * PITCH), 16, 0, 0);
        }
        nops += RPW / 2;
    };
    auto dma_idx = [&](long long t) __attribute__((always_inline)) {
        const int lane = fresh_lane();
        __builtin_amdgcn_global_load_lds((gbl_vptr)(p.v_idx + clampe(t * TR + lane)), (lds_vptr)idxw, 4, 0, 0);
        nops += 1;
    };
    // prep(t): idx(t) has landed; find the slots of tile t (runs of equal v_idx; lane = row), DMA its slots < CAPS and
    // its coefficients, then idx(t + 1) into the idx slot just read
    unsigned long long msk = 0;                          // run starts of the prepared tile
    auto prep = [&](long long t) __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int lane = fresh_lane();
        const int vi = idxw[lane];
        const int pv = idxw[lane > 0 ? lane - 1 : 0];
        const bool start = lane == 0 || vi != pv;
        msk = __ballot(start);
        const int u = __popcll(msk);
        if (start) tailw[__popcll(msk & (~0ull >> (63 - lane))) - 1] = vi;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        unsigned long long mm = msk;
        const int un = u < CAPS ? u : CAPS;
        const long long loff = (long long)(lane >> 3) * vrs + c0 + 4 * (lane & 7);
        for (int s = 0; s < un; ++s) {
            const int ls = __builtin_ctzll(mm);
            mm &= mm - 1;
            const int tail = __builtin_amdgcn_readlane(vi, ls);
            __builtin_amdgcn_global_load_lds((gbl_vptr)(p.V + (long long)tail * D + loff), (lds_vptr)(vsl + s * SLOTB),
                                             16, 0, 0);
        }
        nops += un;
        const long long clast = (long long)p.M * R - 4;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            long long co = t * TR * R + 256 * k + 4 * lane;
            if (co > clast) co = clast;
            __builtin_amdgcn_global_load_lds((gbl_vptr)(p.coef + co), (lds_vptr)(coefw + 256 * k), 16, 0, 0);
        }
        nops += 2;
        if (t + 1 < t_end) dma_idx(t + 1);
    };

    f32x4 acc[4][2];                                     // the tile in the x S MFMAs
    f32x4 accP[4][2];                                    // the previous tile: combine, activation, stores
    // combine(): the prepared tile's V term (slots and coefficients in the wave's LDS) into accP
    auto combine = [&]() __attribute__((always_inline)) {
        const int lane = fresh_lane();
        const int i16 = lane & 15, g = lane >> 4;
        const int u = __popcll(msk);
        int slot[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) slot[rb] = __popcll(msk & (~0ull >> (63 - i16 - 16 * rb))) - 1;
        for (int b0 = 0; b0 < u; b0 += CAPS) {
            const int s = b0 + g;
            if (b0 > 0) {
                // slots past the staged block (short runs / unsorted v_idx): this block's V rows into the slot
                // buffers, synchronously (tail-sorted config-5 tiles rarely have more than 4 distinct rows)
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const long long loff = (long long)(lane >> 3) * vrs + c0 + 4 * (lane & 7);
                for (int k = 0; k < CAPS && b0 + k < u; ++k) {
                    const int tail = __builtin_amdgcn_readfirstlane(tailw[b0 + k]);
                    __builtin_amdgcn_global_load_lds((gbl_vptr)(p.V + (long long)tail * D + loff),
                                                     (lds_vptr)(vsl + k * SLOTB), 16, 0, 0);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // A: V_r[slot s] at the lane's column, r = 0..7, for both column blocks (hi / lo)
            bf16x8 vh[2], vl[2];
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                const float* vp = reinterpret_cast<const float*>(vsl + g * SLOTB) + 16 * cb + i16;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float x = s < u ? vp[32 * j] : 0.f;
                    const __bf16 hi = (__bf16)x;
                    vh[cb][j] = hi;
                    if constexpr (HL) vl[cb][j] = (__bf16)(x - (float)hi);
                }
            }
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) {
                // B: the coefficients of the lane's row where its slot is s (hi / lo)
                const float* cp = coefw + (16 * rb + i16) * 8;
                const f32x4 lo4 = ld4(cp), hi4 = ld4(cp + 4);
                bf16x8 ch, cl;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float x = slot[rb] == s ? (j < 4 ? lo4[j] : hi4[j - 4]) : 0.f;
                    const __bf16 hi = (__bf16)x;
                    ch[j] = hi;
                    if constexpr (HL) cl[j] = (__bf16)(x - (float)hi);
                }
#pragma unroll
                for (int cb = 0; cb < 2; ++cb) {
                    accP[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh[cb], ch, accP[rb][cb], 0, 0, 0);
                    if constexpr (HL) {
                        accP[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vh[cb], cl, accP[rb][cb], 0, 0, 0);
                        accP[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vl[cb], ch, accP[rb][cb], 0, 0, 0);
                    }
                }
            }
        }
    };
    // finish(t, q): block q = (rb, cb) of the previous tile t: activation, bf16, one 8-B store per lane
    auto finish = [&](long long t, int q) __attribute__((always_inline)) {
        const int lane = fresh_lane();
        const int i16 = lane & 15, g = lane >> 4;
        const int rb = q >> 1, cb = q & 1;
        const long long row0 = t * TR;
        const long long left = (long long)p.M - row0;
        const unsigned nbytes = (unsigned)((left < TR ? left : TR) * D * 2);
        const __amdgpu_buffer_rsrc_t rc =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(p.C) + row0 * D * 2, (short)0, nbytes, 0x00020000);
        f32x4 v = accP[rb][cb];
        if (p.act == IDDGCN_ACT_SIGMOID) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = sigmoid_fast(v[e]);
        }
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f32_to_bf4(v)), rc,
                                              ((16 * rb + i16) * D + c0 + 16 * cb + 4 * g) * 2, 0, 0);
        nops += 1;
    };
    auto mfma_main = [&](int b, long long tprev) __attribute__((always_inline)) {
        const int lane = fresh_lane();
        const int i16 = lane & 15, g = lane >> 4;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
        // row 16 rb + i16, logical chunk 4q + g at physical chunk (4q + g) ^ i16 = 4q ^ (g ^ i16): the 16 lanes of each
        // ds_read_b128 group on 16 different 16-B bank groups
        const char* ab = lds + b * ABUF + i16 * PITCH;
        const int sv = 16 * (g ^ i16);
        // fragments of k-steps q and q+1 in alternating registers; one k-step per scheduling region (the fully
        // unrolled loop otherwise hoists all the fragment loads and takes the kernel past 256 VGPRs)
        bf16x8 x[2][4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) x[0][rb] = *reinterpret_cast<const bf16x8*>(ab + 16 * rb * PITCH + sv);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int cu = q & 1;
            if (q + 1 < 8) {
#pragma unroll
                for (int rb = 0; rb < 4; ++rb)
                    x[cu ^ 1][rb] = *reinterpret_cast<const bf16x8*>(ab + 16 * rb * PITCH + ((64 * (q + 1)) ^ sv));
            }
#pragma unroll
            for (int cb = 0; cb < 2; ++cb)
#pragma unroll
                for (int rb = 0; rb < 4; ++rb) {
                    acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[cb][q], x[cu][rb], acc[rb][cb], 0, 0, 0);
                    if constexpr (HL) acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[cb][q], x[cu][rb], acc[rb][cb], 0, 0, 0);
                }
            // the previous tile's block q: its VALU and store issue in the shadow of this k-step's MFMAs
            if (tprev >= 0) finish(tprev, q);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // prologue: idx(t_beg), A(t_beg), A(t_beg + 1) landed, then prepare t_beg
    dma_idx(t_beg);
    dma_A(t_beg, 0);
    if (t_beg + 1 < t_end) dma_A(t_beg + 1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    prep(t_beg);
    int mark = nops;                                     // the next epilogue's inputs: every op up to mark
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    int b = 0;
    // every wave: combine of t-1, prepare t, MFMAs of t with t-1's activation and stores interleaved (a tile's V rows
    // and coefficients are requested a whole MFMA phase before its combine; staggering half the waves, as the v3
    // kernel does, measured slower here: 20.6 vs 19.7 ms per config-5 launch at 32-row tiles, 20.3 vs 18.1 at 64)
    for (long long t = t_beg; t < t_end; ++t) {
        // A(t+2) into the buffer of tile t-1 (every wave's MFMAs on it ended before the last barrier)
        if (t + 2 < t_end) dma_A(t + 2, b == 0 ? 2 : b - 1);
        if (t > t_beg) {
            wait_vm(nops - mark);            // prep(t-1) and A(t+1), with everything older
            combine();
            prep(t);
            mark = nops;
        } else {
            mark = nops;                     // (t_beg: the next wait must also cover A(t_beg + 2))
        }
        mfma_main(b, t > t_beg ? t - 1 : -1);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) accP[rb][cb] = acc[rb][cb];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        b = b == 2 ? 0 : b + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    combine();
#pragma unroll
    for (int q = 0; q < 8; ++q) finish(t_end - 1, q);
}

// config-5 forward form (R = 8, per-edge coefficients, gathered V rows, bf16 A / C): one persistent workgroup per CU
void launch_fwd_gather8(hipStream_t st, RowGemmP p) {
    const long long ntiles = ((long long)p.M + fg8::TR - 1) / fg8::TR;
    long long nb = ntiles < 256 ? ntiles : 256;
    p.tiles_per_block = (int)((ntiles + nb - 1) / nb);
    nb = (ntiles + p.tiles_per_block - 1) / p.tiles_per_block;
    if (p.precision == IDDGCN_GEMM_BF16) hipLaunchKernelGGL(fwd_gather8_bf16_kernel<false>, dim3((unsigned)nb), dim3(512), 0, st, p);
    else hipLaunchKernelGGL(fwd_gather8_bf16_kernel<true>, dim3((unsigned)nb), dim3(512), 0, st, p);
}

// the config-5 tail reduction on MFMAs (tail_seg_mfma8_kernel), with or without the head chain's node terms
void launch_tail_mfma8(hipStream_t st, int n_nodes, const int* seg_ptr, const float* W, const void* dO,
                       const float* P, long long p_rel_stride, float* dP, long long dp_rel_stride, float* dsum,
                       float* dWedge, const float* head_dO, const float* Wn, float* dwh) {
    const unsigned g4 = (unsigned)((n_nodes + 3) / 4);
#define TM8(DS, HD) hipLaunchKernelGGL((tail_seg_mfma8_kernel<DS, HD>), dim3(g4), dim3(256), 0, st, n_nodes, seg_ptr, W, (const __bf16*)dO, P, p_rel_stride, dP, dp_rel_stride, dsum, dWedge, head_dO, Wn, dwh)
    if (head_dO) {
        if (dsum) TM8(true, true);
        else TM8(false, true);
    } else {
        if (dsum) TM8(true, false);
        else TM8(false, false);
    }
#undef TM8
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int iddgcn_abi_version(void) { return IDDGCN_ABI_VERSION; }

int iddgcn_spmm_csr_f32(void* stream, int n_seg, int n_rows, int d, const int* row_ptr, const int* col,
                        const float* vals, const float* X, float* Y, int accumulate) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (n_seg < 0 || n_rows < 0 || !row_ptr || !X || !Y) return IDDGCN_E_BAD_ARG;
    const long long rows = (long long)n_seg * n_rows;
    if (rows == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = grid_for(rows, d / 4);
#define SPMM(DD) hipLaunchKernelGGL(spmm_csr_kernel<DD>, dim3(grid), dim3(256), 0, st, n_seg, n_rows, row_ptr, col, vals, X, Y, accumulate)
    switch (d) {
        case 32: SPMM(32); break;
        case 64: SPMM(64); break;
        case 128: SPMM(128); break;
        default: SPMM(256); break;
    }
#undef SPMM
    return launch_status();
}

int iddgcn_sddmm_csr_f32(void* stream, int n_seg, int n_rows, int d, const int* row_ptr, const int* col,
                         const float* G, const float* X, float* out) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (n_seg < 0 || n_rows < 0 || !row_ptr || !col || !G || !X || !out) return IDDGCN_E_BAD_ARG;
    const long long rows = (long long)n_seg * n_rows;
    if (rows == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = grid_for(rows, d / 4);
#define SDK(DD) hipLaunchKernelGGL(sddmm_csr_kernel<DD>, dim3(grid), dim3(256), 0, st, n_seg, n_rows, row_ptr, col, G, X, out)
    switch (d) {
        case 32: SDK(32); break;
        case 64: SDK(64); break;
        case 128: SDK(128); break;
        default: SDK(256); break;
    }
#undef SDK
    return launch_status();
}

int iddgcn_rowgemm_f32(void* stream, const iddgcn_rowgemm_t* a) {
    if (!a) return IDDGCN_E_BAD_ARG;
    if (const int rc = check_rowgemm(*a)) return rc;
    if (a->M == 0) return 0;                 // nothing to do (an empty C may have a null pointer)
    RowGemmP p = to_p(*a);
    hipStream_t st = (hipStream_t)stream;
    if (p.precision == IDDGCN_GEMM_BF16X3) {
        int nv;
        bool aux, bc;
        if (a->D == 256 && b3_select(p, nv, aux, bc)) {
            launch_b3(st, p, nv, aux, bc);
            return launch_status();
        }
        p.precision = IDDGCN_GEMM_EXACT_F32;      // the forms the bf16x3 kernel does not take: exact f32
    }
    V3Sel sel;
    if (a->D == 256 && v3_select(p, sel)) {
        RowGemmBatch pb;
        pb.p[0] = p;
        launch_v3(st, pb, 1, sel);
        return launch_status();
    }
    // D < 256, and the D = 256 forms the v3 kernel does not take: the register-staged kernel (exact f32)
#define RGEMM(DD, MAXB)                                                                         \
    {                                                                                           \
        const long long nt = ((long long)p.M + RG<DD>::TR - 1) / RG<DD>::TR;                    \
        long long nb = nt < (MAXB) ? nt : (MAXB);                                               \
        p.tiles_per_block = (int)((nt + nb - 1) / nb);                                          \
        nb = (nt + p.tiles_per_block - 1) / p.tiles_per_block;                                  \
        RowGemmBatch pb;                                                                        \
        pb.p[0] = p;                                                                            \
        hipLaunchKernelGGL(rowgemm_kernel<DD>, dim3((unsigned)nb), dim3(RG<DD>::NW * 64), 0, st, pb); \
    }
    switch (a->D) {
        case 32: RGEMM(32, 2048); break;
        case 64: RGEMM(64, 2048); break;
        case 128: RGEMM(128, 1024); break;
        default: RGEMM(256, 256); break;
    }
#undef RGEMM
    return launch_status();
}

int iddgcn_rowgemm_kernel_id(const iddgcn_rowgemm_t* a) {
    if (!a || !dim_ok(a->D)) return -1;
    RowGemmP p = to_p(*a);
    if (p.precision == IDDGCN_GEMM_BF16X3) {
        int nv;
        bool aux, bc;
        if (a->D == 256 && b3_select(p, nv, aux, bc)) return 500 + 10 * nv + (aux ? 1 : 0) + (bc ? 2 : 0);
        p.precision = IDDGCN_GEMM_EXACT_F32;
    }
    V3Sel sel;
    if (a->D == 256 && v3_select(p, sel))
        return 300 + 10 * sel.nv + (sel.aux ? 1 : 0) + (sel.hc ? 2 : 0) + (sel.cw ? 8 : 0) + (sel.split ? 2000 : 0) +
               (sel.c4 ? 4000 : 0) + (sel.pl ? 1000 : 0);
    return 100;
}

int iddgcn_rowgemm_batched_f32(void* stream, const iddgcn_rowgemm_t* a, int n) {
    if (!a || n < 0 || n > ROWGEMM_BATCH) return IDDGCN_E_BAD_ARG;
    if (n == 0) return 0;
    bool one_launch = a[0].D != 256;
    for (int k = 0; k < n; ++k) {
        if (!dim_ok(a[k].D) || a[k].D != a[0].D) return IDDGCN_E_BAD_DIM;
        if (const int rc = check_rowgemm(a[k])) return rc;
    }
    for (int k = 0; k < n && !one_launch; ++k)
        if (a[k].precision == IDDGCN_GEMM_BF16X3) {      // D = 256 bf16x3: one call per entry
            for (int j = 0; j < n; ++j) {
                const int rc = iddgcn_rowgemm_f32(stream, a + j);
                if (rc) return rc;
            }
            return 0;
        }
    if (!one_launch) {          // D = 256: one v3 launch when every entry maps to the same variant
        RowGemmBatch pb;
        V3Sel sel0{}, sel{};
        bool same = true;
        int m = 0;
        for (int k = 0; k < n && same; ++k) {
            if (a[k].M == 0) continue;
            RowGemmP& p = pb.p[m];
            p = to_p(a[k]);
            if (!v3_select(p, sel)) same = false;
            else if (m == 0) sel0 = sel;
            else same = sel.same(sel0);
            ++m;
        }
        if (same) {
            if (m > 0) launch_v3((hipStream_t)stream, pb, m, sel0);
            return launch_status();
        }
        for (int k = 0; k < n; ++k) {
            const int rc = iddgcn_rowgemm_f32(stream, a + k);
            if (rc) return rc;
        }
        return 0;
    }
    RowGemmBatch pb;
    long long nbmax = 0;
    const int d = a[0].D;
    const int tr = d == 32 ? RG<32>::TR : d == 64 ? RG<64>::TR : RG<128>::TR;
    const long long maxb = d == 128 ? 1024 : 2048;
    for (int k = 0; k < n; ++k) {
        RowGemmP& p = pb.p[k];
        p = to_p(a[k]);
        const long long nt = ((long long)p.M + tr - 1) / tr;
        long long nb = nt < maxb ? nt : maxb;
        p.tiles_per_block = nb > 0 ? (int)((nt + nb - 1) / nb) : 1;
        nb = nb > 0 ? (nt + p.tiles_per_block - 1) / p.tiles_per_block : 0;
        if (nb > nbmax) nbmax = nb;
    }
    if (nbmax == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const dim3 g((unsigned)nbmax, (unsigned)n);
    switch (d) {
        case 32: hipLaunchKernelGGL(rowgemm_kernel<32>, g, dim3(RG<32>::NW * 64), 0, st, pb); break;
        case 64: hipLaunchKernelGGL(rowgemm_kernel<64>, g, dim3(RG<64>::NW * 64), 0, st, pb); break;
        default: hipLaunchKernelGGL(rowgemm_kernel<128>, g, dim3(RG<128>::NW * 64), 0, st, pb); break;
    }
    return launch_status();
}

int iddgcn_gemm_tn_blocks(long long M, int d) {
    const long long tiles = (M + 31) / 32;
    const long long cap = (d >= 256) ? 256 : 1024;
    long long nb = tiles < cap ? tiles : cap;
    return (int)(nb < 1 ? 1 : nb);
}

int iddgcn_gemm_tn_f32(void* stream, long long M, int d, const float* A, const float* B, float* slab, int n_blocks,
                       float* C, int accumulate, int precision) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (M < 0 || n_blocks < 1 || !A || !B || !slab || !C) return IDDGCN_E_BAD_ARG;
    if (precision != IDDGCN_GEMM_EXACT_F32 && precision != IDDGCN_GEMM_SPLIT_F16 && precision != IDDGCN_GEMM_BF16X3)
        return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    long long rpb = (M + n_blocks - 1) / n_blocks;
    rpb = ((rpb + 31) / 32) * 32;
    if (rpb < 32) rpb = 32;
#define TNK(DD) hipLaunchKernelGGL(gemm_tn_kernel<DD>, dim3(n_blocks), dim3(TN<DD>::NW * 64), 0, st, M, rpb, A, B, slab)
    if (d == 256 && precision == IDDGCN_GEMM_BF16X3) {
        hipLaunchKernelGGL(gemm_tn256_b3_kernel, dim3(n_blocks), dim3(512), 0, st, M, rpb, A, B, slab, TnBatch{});
    } else if (d == 256 && precision == IDDGCN_GEMM_SPLIT_F16) {
        hipLaunchKernelGGL(gemm_tn256_x3_kernel<>, dim3(n_blocks), dim3(512), 0, st, M, rpb, A, B, slab, TnBatch{});
    } else if (d == 256) {
        hipLaunchKernelGGL(gemm_tn256_dma_kernel, dim3(n_blocks), dim3(512), 0, st, M, rpb, A, B, slab);
    } else switch (d) {
        case 32: TNK(32); break;
        case 64: TNK(64); break;
        default: TNK(128); break;
    }
#undef TNK
    int rc = launch_status();
    if (rc) return rc;
    const long long n = (long long)d * d;
    launch_reduce_slabs(st, n_blocks, n, slab, C, accumulate, 1.0f);
    return launch_status();
}

int iddgcn_gemm_tn_batched_f32(void* stream, int d, const iddgcn_tn_t* e, int n, float* slab, long long slab_floats,
                               int precision) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (n < 0 || n > IDDGCN_TN_BATCH || (n > 0 && (!e || !slab))) return IDDGCN_E_BAD_ARG;
    if (precision != IDDGCN_GEMM_EXACT_F32 && precision != IDDGCN_GEMM_SPLIT_F16 && precision != IDDGCN_GEMM_BF16X3)
        return IDDGCN_E_BAD_ARG;
    for (int k = 0; k < n; ++k)
        if (e[k].M < 0 || (e[k].M > 0 && (!e[k].A || !e[k].B)) || !e[k].C) return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long long dd = (long long)d * d;
    const bool b3 = d == 256 && precision == IDDGCN_GEMM_BF16X3;
    if (!(d == 256 && (precision == IDDGCN_GEMM_SPLIT_F16 || b3))) {
        // other widths and the exact mode: the single-call kernels one after another (slab reused in order)
        for (int k = 0; k < n; ++k) {
            if (e[k].M == 0) {                     // no rows: C = 0, or C unchanged when accumulating
                if (!e[k].accumulate && hipMemsetAsync(e[k].C, 0, dd * sizeof(float), st) != hipSuccess)
                    return launch_status();
                continue;
            }
            long long nb = iddgcn_gemm_tn_blocks(e[k].M, d);
            if (nb * dd > slab_floats) nb = slab_floats / dd;           // fewer partials, longer row ranges
            if (nb < 1) return IDDGCN_E_BAD_ARG;
            const int rc = iddgcn_gemm_tn_f32(stream, e[k].M, d, e[k].A, e[k].B, slab, (int)nb, e[k].C, e[k].accumulate,
                                              precision);
            if (rc) return rc;
        }
        return 0;
    }
    TnBatch tb{};
    tb.n = n;
    long long off = 0;
    int nbk[IDDGCN_TN_BATCH] = {0};
    unsigned nbmax = 1;
    for (int k = 0; k < n; ++k) {
        const long long tiles = (e[k].M + 31) / 32;
        long long nb = 256 / n;                    // every workgroup of the launch resident at once
        if (nb > tiles) nb = tiles;
        if (nb < 1) nb = 1;
        long long rpb = (e[k].M + nb - 1) / nb;
        rpb = ((rpb + 31) / 32) * 32;
        if (rpb < 32) rpb = 32;
        nbk[k] = (int)nb;
        tb.nb[k] = (int)nb;
        if ((unsigned)nb > nbmax) nbmax = (unsigned)nb;
        tb.M[k] = e[k].M;
        tb.rpb[k] = rpb;
        tb.A[k] = e[k].A;
        tb.B[k] = e[k].B;
        tb.slab[k] = slab + off;
        off += nb * dd;
    }
    if (off > slab_floats) return IDDGCN_E_BAD_ARG;
    if (n == 0) return 0;
    if (b3)
        hipLaunchKernelGGL(gemm_tn256_b3_kernel, dim3(nbmax, (unsigned)n), dim3(512), 0, st, 0LL, 0LL, nullptr, nullptr,
                           nullptr, tb);
    else
        hipLaunchKernelGGL(gemm_tn256_x3_kernel<>, dim3(nbmax, (unsigned)n), dim3(512), 0, st, 0LL, 0LL, nullptr,
                           nullptr, nullptr, tb);
    int rc = launch_status();
    if (rc) return rc;
    for (int k = 0; k < n; ++k) launch_reduce_slabs(st, nbk[k], dd, tb.slab[k], e[k].C, e[k].accumulate, 1.0f);
    return launch_status();
}

int iddgcn_gemm_tn_planes_f32(void* stream, long long M, int d, const void* A, const float* B, float* slab,
                              int n_blocks, float* C, int accumulate) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (M < 0 || n_blocks < 1 || !A || !B || !slab || !C) return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    long long rpb = (M + n_blocks - 1) / n_blocks;
    rpb = ((rpb + 31) / 32) * 32;
    if (rpb < 32) rpb = 32;
    hipLaunchKernelGGL((gemm_tn256_x3_kernel<true>), dim3(n_blocks), dim3(512), 0, st, M, rpb, (const float*)A, B, slab,
                       TnBatch{});
    int rc = launch_status();
    if (rc) return rc;
    const long long n = (long long)d * d;
    launch_reduce_slabs(st, n_blocks, n, slab, C, accumulate, 1.0f);
    return launch_status();
}

int iddgcn_gemm_tn_narrow_blocks(long long M) {
    long long nb = (M + 15) / 16;          // <= 16 rows per block: short serial chains at small M
    if (nb > 1024) nb = 1024;
    return (int)(nb < 1 ? 1 : nb);
}

int iddgcn_gemm_tn_narrow_f32(void* stream, long long M, int d, int R, const float* A, const float* dz, float* slab,
                              int n_blocks, float* dWa, float* dba, int accumulate) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (M < 0 || n_blocks < 1 || !A || !dz || !slab || !dWa || !dba) return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long long rpb = (M + n_blocks - 1) / n_blocks;
#define NK(DD) hipLaunchKernelGGL(gemm_tn_narrow_kernel<DD>, dim3(n_blocks), dim3(DD), 0, st, M, rpb, R, A, dz, slab)
    switch (d) {
        case 32: NK(32); break;
        case 64: NK(64); break;
        case 128: NK(128); break;
        default: NK(256); break;
    }
#undef NK
    int rc = launch_status();
    if (rc) return rc;
    // slab rows are [(D+1)*R]; reduce the weight part and the bias part separately
    const long long nw = (long long)d * R;
    const long long stride = (long long)(d + 1) * R;
    // reduce with stride: reuse reduce_slabs on a strided view by reducing the whole row then copying
    // (n_blocks x (D+1)R is tiny), writing into dWa / dba through two launches.
    launch_reduce_slabs(st, n_blocks, stride, slab, slab + (long long)n_blocks * stride, 0, 1.0f);
    rc = launch_status();
    if (rc) return rc;
    const float* red = slab + (long long)n_blocks * stride;
    hipLaunchKernelGGL(reduce_slabs_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, 1, nw, red, dWa,
                       accumulate, 1.0f);
    hipLaunchKernelGGL(reduce_slabs_kernel, dim3(1), dim3(256), 0, st, 1, (long long)R, red + nw, dba, accumulate,
                       1.0f);
    return launch_status();
}

int iddgcn_alpha_fwd_f32(void* stream, int M, int d, int R, const float* X, const int* x_idx, const float* Wa,
                         const float* ba, float* S_out, float* W_out) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (M < 0 || !X || !Wa || !ba || !S_out || !W_out) return IDDGCN_E_BAD_ARG;
    if (M == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    unsigned grid = grid_for(M, d / 4);
    if (grid > 2048) grid = 2048;            // persistent: W_alpha loaded once per lane group
#define AK(DD) hipLaunchKernelGGL(alpha_kernel<DD>, dim3(grid), dim3(256), 0, st, M, R, X, x_idx, Wa, ba, S_out, W_out)
    switch (d) {
        case 32: AK(32); break;
        case 64: AK(64); break;
        case 128: AK(128); break;
        default: AK(256); break;
    }
#undef AK
    return launch_status();
}

int iddgcn_combine_f32(void* stream, int M, int d, int R, const float* Y, const int* y_idx, const float* coef,
                       const int* coef_idx, const float* V, const int* v_idx, long long v_rel_stride, float* out) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (R < 0 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (M < 0 || !Y || !out || (R > 0 && (!coef || !V))) return IDDGCN_E_BAD_ARG;
    if (M == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (d == 256 && y_idx && y_idx == v_idx && !coef_idx) {
        const long long nchunk = ((long long)M + RC_CH - 1) / RC_CH;
        long long nb = (nchunk + 3) / 4;
        if (nb > 2048) nb = 2048;
#define RCK(RR) hipLaunchKernelGGL((run_combine256_kernel<RR>), dim3((unsigned)nb), dim3(256), 0, st, M, Y, y_idx, coef, V, v_rel_stride, out)
        switch (R) {
            case 0: RCK(0); break;
            case 1: RCK(1); break;
            case 2: RCK(2); break;
            case 3: RCK(3); break;
            case 4: RCK(4); break;
            case 5: RCK(5); break;
            case 6: RCK(6); break;
            case 7: RCK(7); break;
            default: RCK(8); break;
        }
#undef RCK
        return launch_status();
    }
    const long long nbatch = ((long long)M + (256 / (d / 4)) * CU_ROWS - 1) / ((256 / (d / 4)) * CU_ROWS);
    const unsigned grid = (unsigned)(nbatch < CU_BLOCKS ? nbatch : CU_BLOCKS);
#define CK(DD, RR) hipLaunchKernelGGL((combine_kernel<DD, RR>), dim3(grid), dim3(256), 0, st, M, Y, y_idx, coef, coef_idx, V, v_idx, v_rel_stride, out)
#define CKR(DD)                    \
    switch (R) {                   \
        case 0: CK(DD, 0); break;  \
        case 1: CK(DD, 1); break;  \
        case 2: CK(DD, 2); break;  \
        case 3: CK(DD, 3); break;  \
        case 4: CK(DD, 4); break;  \
        case 5: CK(DD, 5); break;  \
        case 6: CK(DD, 6); break;  \
        case 7: CK(DD, 7); break;  \
        default: CK(DD, 8); break; \
    }
    switch (d) {
        case 32: CKR(32); break;
        case 64: CKR(64); break;
        case 128: CKR(128); break;
        default: CKR(256); break;
    }
#undef CKR
#undef CK
    return launch_status();
}

int iddgcn_distmult_blocks(long long T) {
    long long nb = (T + 255) / 256;
    if (nb > 2048) nb = 2048;
    return (int)(nb < 1 ? 1 : nb);
}

int iddgcn_distmult_bce_f32(void* stream, long long T, int d, int R, const float* Xh, const int* h_idx,
                            const float* Xt, const int* t_idx, const int* r_idx, const float* rel, const float* y,
                            float scale, float* p_out, float* s_out, float* ds_out, float* do_out,
                            float* drel_slab, float* loss_slab, int n_blocks) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (T < 0 || n_blocks < 1 || !Xh || !h_idx || !Xt || !r_idx || !rel) return IDDGCN_E_BAD_ARG;
    if (y && (!ds_out || !do_out || !drel_slab || !loss_slab)) return IDDGCN_E_BAD_ARG;
    if (T == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
#define DK(DD) hipLaunchKernelGGL(distmult_kernel<DD>, dim3(n_blocks), dim3(256), 0, st, T, R, Xh, h_idx, Xt, t_idx, r_idx, rel, y, scale, p_out, s_out, ds_out, do_out, drel_slab, loss_slab)
    switch (d) {
        case 32: DK(32); break;
        case 64: DK(64); break;
        case 128: DK(128); break;
        default: DK(256); break;
    }
#undef DK
    return launch_status();
}

int iddgcn_distmult_bce_heads_f32(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const int* perm,
                                  const float* Xh, const float* Xt, const int* r_idx, const float* rel,
                                  const float* y, float scale, float* p_out, float* s_out, float* ds_out,
                                  float* do_out, float* dXh, float* drel_slab, float* loss_slab, int n_blocks) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || n_blocks < 1 || !seg_ptr || !perm || !Xh || !Xt || !r_idx || !rel || !do_out ||
        !dXh || !drel_slab || !loss_slab)
        return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
#define HK(DD, RT) hipLaunchKernelGGL((distmult_heads_kernel<DD, RT>), dim3(n_blocks), dim3(256), 0, st, n_nodes, R, seg_ptr, perm, Xh, Xt, r_idx, rel, y, scale, p_out, s_out, ds_out, do_out, dXh, drel_slab, loss_slab)
#define HKR(DD)                                            \
    {                                                      \
        if (R <= 1) HK(DD, 1);                             \
        else if (R <= 2) HK(DD, 2);                        \
        else if (R <= 4) HK(DD, 4);                        \
        else HK(DD, 8);                                    \
    }
    switch (d) {
        case 32: HKR(32); break;
        case 64: HKR(64); break;
        case 128: HKR(128); break;
        default: HKR(256); break;
    }
#undef HKR
#undef HK
    return launch_status();
}

int iddgcn_seg_gather_reduce_f32(void* stream, int n_nodes, int d, const int* seg_ptr, const int* perm,
                                 const float* coef, const int* r_idx, const float* rel, const float* rows,
                                 const float* X, float* out) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (n_nodes < 0 || !seg_ptr || !rows || !out || (rel && !r_idx)) return IDDGCN_E_BAD_ARG;
    if (n_nodes == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = grid_for(n_nodes, d / 4);
#define GK(DD) hipLaunchKernelGGL(seg_gather_reduce_kernel<DD>, dim3(grid), dim3(256), 0, st, n_nodes, seg_ptr, perm, coef, r_idx, rel, rows, X, out)
    switch (d) {
        case 32: GK(32); break;
        case 64: GK(64); break;
        case 128: GK(128); break;
        default: GK(256); break;
    }
#undef GK
    return launch_status();
}

int iddgcn_tail_seg_reduce_f32(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const int* h_idx,
                               const float* W, const float* dO, const float* P, long long p_rel_stride, float* dP,
                               long long dp_rel_stride, float* dsum, float* dWedge) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || !seg_ptr || !W || !dO || !P || !dP || !dWedge) return IDDGCN_E_BAD_ARG;
    if (n_nodes == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = grid_for(n_nodes, 64);       // one wave per node
#define TK(DD, RR) hipLaunchKernelGGL((tail_seg_reduce_kernel<DD, RR>), dim3(grid), dim3(256), 0, st, n_nodes, seg_ptr, h_idx, W, dO, P, p_rel_stride, dP, dp_rel_stride, dsum, dWedge)
#define TKR(DD)                \
    switch (R) {               \
        case 1: TK(DD, 1); break; \
        case 2: TK(DD, 2); break; \
        case 3: TK(DD, 3); break; \
        case 4: TK(DD, 4); break; \
        case 5: TK(DD, 5); break; \
        case 6: TK(DD, 6); break; \
        case 7: TK(DD, 7); break; \
        default: TK(DD, 8); break; \
    }
    switch (d) {
        case 32: TKR(32); break;
        case 64: TKR(64); break;
        case 128: TKR(128); break;
        default: TKR(256); break;
    }
#undef TKR
#undef TK
    return launch_status();
}

int iddgcn_head_bwd_node_f32(void* stream, int n_nodes, int d, int R, const float* dO, const float* P,
                             long long p_rel_stride, const float* Ssm, const float* W, const int* hseg_ptr,
                             const int* hperm, const float* dWedge, const float* ep_in, float* dP,
                             long long dp_rel_stride, float* dsum, float* dz) {
    if (!dim_ok(d)) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || !dO || !P || !Ssm || !W || !dz) return IDDGCN_E_BAD_ARG;
    if (hseg_ptr && (!hperm || !dWedge)) return IDDGCN_E_BAD_ARG;
    if (n_nodes == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = grid_for(n_nodes, d / 4);
#define HK(DD) hipLaunchKernelGGL(head_bwd_node_kernel<DD>, dim3(grid), dim3(256), 0, st, n_nodes, R, dO, P, p_rel_stride, Ssm, W, hseg_ptr, hperm, dWedge, ep_in, dP, dp_rel_stride, dsum, dz)
    switch (d) {
        case 32: HK(32); break;
        case 64: HK(64); break;
        case 128: HK(128); break;
        default: HK(256); break;
    }
#undef HK
    return launch_status();
}

int iddgcn_head_wsum_f32(void* stream, int n_nodes, int R, const int* hptr, const int* hperm, const float* w,
                         float* out) {
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || !hptr || !hperm || !w || !out) return IDDGCN_E_BAD_ARG;
    if (n_nodes == 0) return 0;
    const long long total = (long long)n_nodes * R;
    hipLaunchKernelGGL(head_wsum_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       n_nodes, R, hptr, hperm, w, out);
    return launch_status();
}

int iddgcn_gather_rows_f32(void* stream, long long M, int width, const float* src, const int* idx, float* dst) {
    if (M < 0 || width < 1 || !src || !idx || !dst) return IDDGCN_E_BAD_ARG;
    if (M == 0) return 0;
    const bool al16 = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
    if (al16 && (width == 4 || width == 8)) {
        const unsigned g = (unsigned)((M + 255) / 256);
        if (width == 8) hipLaunchKernelGGL((gather_rows_vec_kernel<8>), dim3(g), dim3(256), 0, (hipStream_t)stream, M, src, idx, dst);
        else hipLaunchKernelGGL((gather_rows_vec_kernel<4>), dim3(g), dim3(256), 0, (hipStream_t)stream, M, src, idx, dst);
        return launch_status();
    }
    const long long n = M * width;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, M,
                       width, src, idx, dst);
    return launch_status();
}

int iddgcn_reduce_slabs_f32(void* stream, int n_slabs, long long n, const float* slab, float* out, int accumulate,
                            float scale) {
    if (n_slabs < 1 || n < 0 || !slab || !out) return IDDGCN_E_BAD_ARG;
    if (n == 0) return 0;
    launch_reduce_slabs((hipStream_t)stream, n_slabs, n, slab, out, accumulate, scale);
    return launch_status();
}

int iddgcn_adam_f32(void* stream, long long n, float* var, float* m, float* v, const float* g, float alpha, float b1,
                    float b2, float eps, int sparse_form) {
    if (n < 0 || !var || !m || !v || !g) return IDDGCN_E_BAD_ARG;
    if (n == 0) return 0;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, var, m, v,
                       g, alpha, b1, b2, eps, sparse_form, nullptr, nullptr);
    return launch_status();
}

int iddgcn_adam_table_f32(void* stream, long long n, float* var, float* m, float* v, const float* g,
                          const float* alpha_table, const int* step, float b1, float b2, float eps, int sparse_form) {
    if (n < 0 || !var || !m || !v || !g || !alpha_table || !step) return IDDGCN_E_BAD_ARG;
    if (n == 0) return 0;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, var, m, v,
                       g, 0.0f, b1, b2, eps, sparse_form, alpha_table, step);
    return launch_status();
}

int iddgcn_rowgemm_bf16(void* stream, const iddgcn_rowgemm_t* a) {
    if (!a) return IDDGCN_E_BAD_ARG;
    if (a->D != 256) return IDDGCN_E_BAD_DIM;
    if (a->R < 0 || a->R > MAX_R) return IDDGCN_E_BAD_REL;
    if (a->M == 0) return 0;
    if (a->M < 0 || !a->A || !a->B || !a->C || a->accumulate) return IDDGCN_E_BAD_ARG;
    const bool gatherV = a->R > 0 && a->v_row_stride != 0;
    const bool dsig = a->act == IDDGCN_ACT_DSIGMOID;
    if (a->act != IDDGCN_ACT_NONE && a->act != IDDGCN_ACT_SIGMOID && !dsig) return IDDGCN_E_BAD_ARG;
    if (dsig && (!a->aux || a->R > 0)) return IDDGCN_E_BAD_ARG;
    if (a->R > 0 && (!gatherV || a->v_row_stride != 256 || !a->coef || !a->V)) return IDDGCN_E_BAD_ARG;
    if (a->planes) return IDDGCN_E_BAD_ARG;
    RowGemmP p = to_p(*a);
    p.accumulate = 0;
    auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    if (a->R == 8 && a->v_idx && !a->coef_idx && !a->a_idx && !a->b_trans && !dsig && al16(a->A) && al16(a->C) &&
        al16(a->coef) && al16(a->V) && (a->v_rel_stride & 3) == 0) {
        launch_fwd_gather8((hipStream_t)stream, p);
        return launch_status();
    }
    V3Sel sel;
    sel.nv = a->R == 0 ? 0 : a->R == 1 ? 1 : a->R == 2 ? 2 : a->R <= 4 ? 4 : 8;
    sel.aux = dsig;
    sel.hc = a->R > 0;
    RowGemmBatch pb;
    pb.p[0] = p;
    launch_v3((hipStream_t)stream, pb, 1, sel, true);
    return launch_status();
}

int iddgcn_gemm_tn_bf16(void* stream, long long M, int d, const void* A, const void* B, float* slab, int n_blocks,
                        float* C, int accumulate) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (M < 0 || n_blocks < 1 || !A || !B || !slab || !C) return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    long long rpb = (M + n_blocks - 1) / n_blocks;
    rpb = ((rpb + 31) / 32) * 32;
    if (rpb < 32) rpb = 32;
    hipLaunchKernelGGL(gemm_tn256_bf16t_kernel, dim3(n_blocks), dim3(512), 0, st, M, rpb,
                       (const __bf16*)A, (const __bf16*)B, slab);
    int rc = launch_status();
    if (rc) return rc;
    const long long n = (long long)d * d;
    launch_reduce_slabs(st, n_blocks, n, slab, C, accumulate, 1.0f);
    return launch_status();
}

int iddgcn_sigma_tn_ranges(long long M) {
    const long long nt = (M + stn::TR - 1) / stn::TR;
    long long nr = nt < 128 ? nt : 128;
    if (nr < 1) nr = 1;
    const long long tpb = (nt + nr - 1) / nr > 0 ? (nt + nr - 1) / nr : 1;
    nr = (nt + tpb - 1) / tpb;
    return (int)((nr + 7) / 8 * 8 > 0 ? (nr + 7) / 8 * 8 : 8);
}

int iddgcn_sigma_tn_bf16(void* stream, long long M, int d, const void* dO, void* X, const float* S, float* slab,
                         long long slab_floats, float* dS, int precision) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    // the weights as a bf16 hi + lo pair for the fp32-operand modes, rounded to bf16 for IDDGCN_GEMM_BF16; nothing else
    if (precision != IDDGCN_GEMM_EXACT_F32 && precision != IDDGCN_GEMM_SPLIT_F16 && precision != IDDGCN_GEMM_BF16X3 &&
        precision != IDDGCN_GEMM_BF16)
        return IDDGCN_E_BAD_ARG;
    if (M < 0 || !S || !slab || !dS || (M > 0 && (!dO || !X))) return IDDGCN_E_BAD_ARG;
    if (((uintptr_t)dO & 15) || ((uintptr_t)X & 15)) return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long long nt = (M + stn::TR - 1) / stn::TR;
    const int nr = iddgcn_sigma_tn_ranges(M);
    const long long tpb = nt > 0 ? (nt + nr - 1) / nr : 1;
    const long long n = (long long)d * d;
    if (slab_floats < nr * n) return IDDGCN_E_BAD_ARG;
    if (precision == IDDGCN_GEMM_BF16)
        hipLaunchKernelGGL(sigma_tn_bf16_kernel<true>, dim3((unsigned)(2 * nr)), dim3(512), 0, st, M, (int)tpb, nr,
                           (const __bf16*)dO, (__bf16*)X, S, slab);
    else
        hipLaunchKernelGGL(sigma_tn_bf16_kernel<false>, dim3((unsigned)(2 * nr)), dim3(512), 0, st, M, (int)tpb, nr,
                           (const __bf16*)dO, (__bf16*)X, S, slab);
    int rc = launch_status();
    if (rc) return rc;
    launch_reduce_slabs(st, nr, n, slab, dS, 0, 1.0f);
    return launch_status();
}

int iddgcn_sigma_tn_f32(void* stream, long long M, int d, const float* dO, float* X, const float* S, float* slab,
                        long long slab_floats, float* dS, int precision) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (precision != IDDGCN_GEMM_BF16X3) return IDDGCN_E_BAD_ARG;
    if (M < 0 || !S || !slab || !dS || (M > 0 && (!dO || !X))) return IDDGCN_E_BAD_ARG;
    if (((uintptr_t)dO & 15) || ((uintptr_t)X & 15)) return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
    const long long nt = (M + st3::TR - 1) / st3::TR;
    const int nr = iddgcn_sigma_tn_ranges(M);
    const long long tpb = nt > 0 ? (nt + nr - 1) / nr : 1;
    const long long n = (long long)d * d;
    if (slab_floats < nr * n) return IDDGCN_E_BAD_ARG;
    hipLaunchKernelGGL(sigma_tn_b3_kernel, dim3((unsigned)(2 * nr)), dim3(512), 0, st, M, (int)tpb, nr, dO, X, S, slab);
    int rc = launch_status();
    if (rc) return rc;
    launch_reduce_slabs(st, nr, n, slab, dS, 0, 1.0f);
    return launch_status();
}

int iddgcn_combine_bf16(void* stream, int M, int d, int R, const float* Y, const int* idx, const float* coef,
                        const float* V, long long v_rel_stride, void* out) {
    return run_combine_out<true, false>(stream, M, d, R, Y, idx, coef, V, v_rel_stride, out);
}

int iddgcn_combine_planes_f32(void* stream, int M, int d, int R, const float* Y, const int* idx, const float* coef,
                              const float* V, long long v_rel_stride, void* out) {
    return run_combine_out<false, true>(stream, M, d, R, Y, idx, coef, V, v_rel_stride, out);
}

int iddgcn_distmult_bce_bf16(void* stream, long long T, int d, int R, const float* Xh, const int* h_idx,
                             const void* Xt, const int* t_idx, const int* r_idx, const float* rel, const float* y,
                             float scale, float* p_out, float* s_out, float* ds_out, void* do_out,
                             float* drel_slab, float* loss_slab, int n_blocks) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (T < 0 || n_blocks < 1 || !Xh || !h_idx || !Xt || !r_idx || !rel) return IDDGCN_E_BAD_ARG;
    if (y && (!ds_out || !do_out || !drel_slab || !loss_slab)) return IDDGCN_E_BAD_ARG;
    if (T == 0) return 0;
    hipLaunchKernelGGL((distmult_kernel<256, true>), dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, T, R, Xh, h_idx,
                       (const float*)Xt, t_idx, r_idx, rel, y, scale, p_out, s_out, ds_out, (float*)do_out, drel_slab,
                       loss_slab);
    return launch_status();
}

int iddgcn_distmult_bce_heads_bf16(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const int* perm,
                                   const float* Xh, const void* Xt, const int* r_idx, const float* rel,
                                   const float* y, float scale, float* p_out, float* s_out, float* ds_out,
                                   void* do_out, float* dXh, float* drel_slab, float* loss_slab, int n_blocks) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || n_blocks < 1 || !seg_ptr || !perm || !Xh || !Xt || !r_idx || !rel || !do_out || !dXh ||
        !drel_slab || !loss_slab)
        return IDDGCN_E_BAD_ARG;
    hipStream_t st = (hipStream_t)stream;
#define HKB(RT) hipLaunchKernelGGL((distmult_heads_kernel<256, RT, true>), dim3(n_blocks), dim3(256), 0, st, n_nodes, R, seg_ptr, perm, Xh, (const float*)Xt, r_idx, rel, y, scale, p_out, s_out, ds_out, (float*)do_out, dXh, drel_slab, loss_slab)
    if (R <= 1) HKB(1);
    else if (R <= 2) HKB(2);
    else if (R <= 4) HKB(4);
    else HKB(8);
#undef HKB
    return launch_status();
}

int iddgcn_tail_seg_reduce_head_bf16(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const float* W,
                                     const void* dO, const float* P, long long p_rel_stride, float* dP,
                                     long long dp_rel_stride, float* dsum, float* dWedge, const float* head_dO,
                                     const float* Wn, float* dwh) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (R != 8) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || !seg_ptr || !W || !dO || !P || !dP || !dWedge || !head_dO || !Wn || !dwh)
        return IDDGCN_E_BAD_ARG;
    if (n_nodes == 0) return 0;
    launch_tail_mfma8((hipStream_t)stream, n_nodes, seg_ptr, W, dO, P, p_rel_stride, dP, dp_rel_stride, dsum, dWedge,
                      head_dO, Wn, dwh);
    return launch_status();
}

int iddgcn_head_dz_f32(void* stream, int n_nodes, int R, const float* Ssm, const float* W, const int* hseg_ptr,
                       const int* hperm, const float* dWedge, const float* dwh, float* dz) {
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || !Ssm || !W || !hseg_ptr || !hperm || !dWedge || !dwh || !dz) return IDDGCN_E_BAD_ARG;
    if (n_nodes == 0) return 0;
    hipLaunchKernelGGL(head_dz_kernel, dim3((unsigned)(((long long)n_nodes * 8 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, n_nodes, R, Ssm, W, hseg_ptr, hperm, dWedge, dwh, dz);
    return launch_status();
}

int iddgcn_tail_seg_reduce_bf16(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const int* h_idx,
                                const float* W, const void* dO, const float* P, long long p_rel_stride, float* dP,
                                long long dp_rel_stride, float* dsum, float* dWedge) {
    if (d != 256) return IDDGCN_E_BAD_DIM;
    if (R < 1 || R > MAX_R) return IDDGCN_E_BAD_REL;
    if (n_nodes < 0 || !seg_ptr || !W || !dO || !P || !dP || !dWedge) return IDDGCN_E_BAD_ARG;
    if (n_nodes == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const unsigned grid = grid_for(n_nodes, 64);
    const float* d_o = (const float*)dO;
    if (R == 8 && !h_idx) {          // per-edge W, 8 relations (config 5): the MFMA form
        launch_tail_mfma8(st, n_nodes, seg_ptr, W, dO, P, p_rel_stride, dP, dp_rel_stride, dsum, dWedge, nullptr,
                          nullptr, nullptr);
        return launch_status();
    }
#define TKB(RR) hipLaunchKernelGGL((tail_seg_reduce_kernel<256, RR, true>), dim3(grid), dim3(256), 0, st, n_nodes, seg_ptr, h_idx, W, d_o, P, p_rel_stride, dP, dp_rel_stride, dsum, dWedge)
    switch (R) {
        case 1: TKB(1); break;
        case 2: TKB(2); break;
        case 3: TKB(3); break;
        case 4: TKB(4); break;
        case 5: TKB(5); break;
        case 6: TKB(6); break;
        case 7: TKB(7); break;
        default: TKB(8); break;
    }
#undef TKB
    return launch_status();
}

int iddgcn_step_advance(void* stream, int* step, float* loss_history, const float* loss) {
    if (!step) return IDDGCN_E_BAD_ARG;
    hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step, loss_history, loss);
    return launch_status();
}

}  // extern "C"
