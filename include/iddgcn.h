/*
 * iddgcn.h — C-ABI of libiddgcn_hip.so, the MI355X (gfx950) hot path of
 * IDDGCN's directed multi-relational graph convolution (forward + backward).
 *
 * The reference (AhauBioinformatics/IDDGCN) is pure Python on TensorFlow 2.7;
 * it has no FFI.  Each entry point below replaces the TF ops that one Keras
 * call site lowers to (file:line in /root/reference/prediction/IDDGCN.py or
 * utils1.py); the Python host layer (iddgcn_amd/) binds them with ctypes and
 * keeps the Keras-shaped surface (IDDGCN_Layer, DistMult, get_IDDGCN_Model,
 * fit/predict) — see INTEGRATION.md.
 *
 * Conventions (all entry points):
 *   - pointers are DEVICE pointers to contiguous row-major fp32 (indices int32);
 *   - the caller allocates every output and workspace; the library never
 *     allocates or frees device memory and never synchronises the stream;
 *   - `stream` is a hipStream_t passed as void*; NULL = default stream;
 *   - return 0 on success, a positive hipError_t on a launch error, or a
 *     negative IDDGCN_E* code on invalid arguments (nothing is launched then);
 *   - feature width D must be one of 32, 64, 128, 256; relations R <= 8;
 *   - re-entrant: no process-global state.  Every option (the GEMM operand
 *     precision included) travels with its call, so calls on different streams,
 *     devices or host threads do not interact (ABI 6).
 */
#ifndef IDDGCN_H_
#define IDDGCN_H_

#ifdef __cplusplus
extern "C" {
#endif

#define IDDGCN_ABI_VERSION 12

#define IDDGCN_E_BAD_DIM   (-1)   /* D not in {32,64,128,256} */
#define IDDGCN_E_BAD_REL   (-2)   /* R < 0 or R > 8 */
#define IDDGCN_E_BAD_ARG   (-3)   /* null required pointer / negative size */

/* activation applied by the row-GEMM epilogue */
#define IDDGCN_ACT_NONE     0
#define IDDGCN_ACT_SIGMOID  1
#define IDDGCN_ACT_DSIGMOID 2     /* v *= aux * (1 - aux)   (sigmoid backward) */

/* Operand precision of the D = 256 MFMA GEMMs (iddgcn_rowgemm_t.precision, the TN entries' `precision`):
 *   IDDGCN_GEMM_EXACT_F32 (0, the default of a zero-initialised struct): v_mfma_f32_32x32x2_f32, bitwise an
 *     fmaf chain (the reference's fp32 arithmetic);
 *   IDDGCN_GEMM_SPLIT_F16: each operand row (A) / column (B) is scaled by a power of two so its max lies in
 *     [2^14, 2^15), every value is split as hi + lo (two fp16, 22-23 significant bits: within one fp32 ulp
 *     of the value), and hi*hi + hi*lo + lo*hi runs on v_mfma_f32_32x32x16_f16 with fp32 accumulation; the
 *     power-of-two scales are undone exactly in the epilogue.  An opt-in faster mode: results are
 *     deterministic but not bitwise equal to the exact mode.
 *   IDDGCN_GEMM_F32_4CHAIN (row GEMMs: any D; at D = 256 the plain form only — no coefficients, no sigma'
 *     operand, no planes): the exact mode's f32 MFMA arithmetic with the accumulation over k split into
 *     four interleaved fp32 chains (k-block q of 8 values into chain q mod 4), summed pairwise at the end:
 *     4x shorter rounding chains, ~2x less accumulation error at K = 256; deterministic.  The node-level
 *     projections P_r^l = AE_r K_r^l (|P| up to ~1e3: AE_r sums ~20 entity rows) use it in the exact mode.
 *   IDDGCN_GEMM_BF16X3 (ABI 7): every fp32 operand value is split EXACTLY into three bf16 pieces
 *     x = b0 + b1 + b2 (b0 = bf16(x), b1 = bf16(x - b0), b2 = x - b0 - b1: 3 x 8 = 24 significant bits, the
 *     whole fp32 significand, while |x| > ~2^-110), and a product takes the six piece products of order
 *     >= 2^-16 on bf16 MFMAs (exact products, fp32 accumulation): a0w0 + a0w1 + a1w0 + a1w1 + a0w2 + a2w0.
 *     The dropped terms are <= 2^-23 |a w| per product (fp32's own product rounding is <= 2^-24 |a w|).
 *     Row GEMMs: the plain form, C += A B (accumulate with act none), the gathered-combine forward with
 *     R = 1 or 2 per-edge coefficients (no coef_idx), broadcast V rows (v_row_stride 0, R <= 2, plain or
 *     sigma') and the sigma' backward, without a_idx / planes; every other form takes the exact f32 kernel.  TN GEMMs: D = 256.  Deterministic; not bitwise equal to the exact mode.
 *   IDDGCN_GEMM_BF16 (ABI 10; iddgcn_rowgemm_bf16 only, i.e. bf16 edge tables): every MFMA operand rounded to
 *     bf16 once (RNE) — the weights, and in the R = 8 gathered forward also the node rows and per-edge
 *     coefficients of the combine — one bf16 x bf16 product per term, fp32 accumulation and epilogue
 *     (an opt-in form of BASELINE config 5's "bf16 features with MFMA XW", as autocast would run it): fewer
 *     MFMAs, but the weights' own rounding (2^-9 relative per product) reaches the logits — at config 5, 8x the
 *     99%-quantile logit error of the hi + lo form.  Any other precision on a bf16 call keeps the
 *     weights (and combine operands) as a bf16 hi + lo pair (16 significant bits).  iddgcn_rowgemm_f32 rejects
 *     it (IDDGCN_E_BAD_ARG).
 * Row GEMMs for D < 256 and every other kernel compute in exact f32 (or F32_4CHAIN where asked). */
#define IDDGCN_GEMM_EXACT_F32 0
#define IDDGCN_GEMM_SPLIT_F16 1
#define IDDGCN_GEMM_F32_4CHAIN 2
#define IDDGCN_GEMM_BF16X3 3
#define IDDGCN_GEMM_BF16 4

/* Pre-split edge tables ("planes", ABI 4; D = 256, split-fp16 GEMM mode only).  A row of values in
 * [0, 1] (sigmoid outputs) stored as 8 column blocks of 128 B, block b = [hi f16 of columns 32b..32b+31 |
 * lo f16 of the same columns] (1 KiB, the bytes of an fp32 row; block b lies where fp32 columns
 * 32b..32b+31 lie, so the backward may write fp32 results over its planes sigma' operand), with
 * x * 2^15 = hi + lo, hi = fp16(x * 2^15), lo = fp16(x * 2^15 - hi): 22 significant bits, absolute error
 * <= 2^-24.  The producer splits once; GEMMs reading the table skip their per-tile conversion.
 * Flags of iddgcn_rowgemm_t.planes: */
#define IDDGCN_PLANES_A    1      /* A rows are planes rows */
#define IDDGCN_PLANES_C    2      /* C is written as planes rows (act SIGMOID, no accumulate) */
#define IDDGCN_PLANES_AUX  4      /* the sigma' operand aux is planes rows (act DSIGMOID) */

int iddgcn_abi_version(void);
/* ABI 12: sha256 (hex) of the sources the library was built from (the .hip sources and device_flags.txt of
 * iddgcn_amd/csrc, the headers in include/; iddgcn_amd/_srchash.py), written into the library by the build; the
 * Python loader refuses a library whose digest is not the tree's. */
const char* iddgcn_source_sha256(void);

/* Y[s][n][:] = (accumulate ? Y[s][n][:] : 0) + sum_{k=ptr[s*(n_rows+1)+n]}^{..+1} (vals ? vals[k] : 1) * X[col[k]][:]
 * for s in [0, n_seg).  One CSR per relation, row_ptr holds absolute offsets into col/vals.
 * Replaces tf.sparse.sparse_dense_matmul (IDDGCN.py:69-70) and, fed the CSC (= CSR of A^T),
 * its gradient w.r.t. the dense operand (TF SparseTensorDenseMatMul adjoint_a).  Per-row sums
 * are sequential in CSR order, the order TF's CPU kernel walks the sorted COO. */
int iddgcn_spmm_csr_f32(void* stream, int n_seg, int n_rows, int d,
                        const int* row_ptr, const int* col, const float* vals,
                        const float* X, float* Y, int accumulate);

/* out[k] = sum_c G[s*n_rows + n][c] * X[col[k]][c]   for every stored entry k of row n of
 * segment s (same batched CSR as iddgcn_spmm_csr_f32; out in CSR order).  With G = dAE_r (the
 * gradient w.r.t. A_r·E) and X = E this is the gradient w.r.t. the adjacency VALUES that the
 * explainers take: tape.gradient(pred, adj_mat.values) (explanation/explaiNE.py:17) and the
 * mask gradients of adj*sigmoid(mask) (explanation/GnnExplainer.py:33,51,
 * explanation/IDDGCN_explain.py:52,80). */
int iddgcn_sddmm_csr_f32(void* stream, int n_seg, int n_rows, int d,
                         const int* row_ptr, const int* col,
                         const float* G, const float* X, float* out);

/* Row GEMM on f32 MFMA with a fused epilogue.  For e in [0, M), c in [0, D):
 *   v  = sum_k A[a_idx ? a_idx[e] : e][k] * (b_trans ? B[c][k] : B[k][c])
 *   v += accumulate ? C[e][c] : 0
 *   v += sum_{r<R} coef[(coef_idx ? coef_idx[e] : e)*R + r]
 *                  * V[r*v_rel_stride + (v_idx ? v_idx[e] : e)*v_row_stride + c]
 *   C[e][c] = act(v)   (NONE | SIGMOID | DSIGMOID with aux[e][c]; C may alias aux: the backward
 *                       writes do^{l-1} over its sigma' operand x^{l-1})
 * at the operand precision `precision` (IDDGCN_GEMM_*; D = 256 only, other widths are exact f32)
 * Replaces IDDGCN.py:62-63 + 71-79 (x·S, + sigmoid(alpha_r)·(AE_r[idx]·K_r), sigmoid)
 * with P_r = AE_r·K_r precomputed at node level, and the matching backward GEMMs. */
typedef struct {
    int M, D;
    const float* A; const int* a_idx;
    const float* B; int b_trans;
    float* C; int accumulate;
    int R;
    const float* coef; const int* coef_idx;
    const float* V; const int* v_idx;
    long long v_rel_stride, v_row_stride;
    int act; const float* aux;
    int planes;           /* IDDGCN_PLANES_* flags (ABI 4; 0 = every table fp32).  Nonzero needs D = 256,
                             the split-fp16 mode and no a_idx; invalid combinations return IDDGCN_E_BAD_ARG */
    int precision;        /* IDDGCN_GEMM_EXACT_F32 (0), _SPLIT_F16, _F32_4CHAIN or _BF16X3 (per call) */
} iddgcn_rowgemm_t;
int iddgcn_rowgemm_f32(void* stream, const iddgcn_rowgemm_t* args);

/* Which kernel iddgcn_rowgemm_f32 would run for these arguments (a test / benchmark hook; nothing is
 * launched): 300 + 10*NV + aux + 2*coef + 8*(broadcast V with R > 2 coefficients) + 1000 for the planes
 * form (C or aux planes) + 2000 for split-fp16 operands + 4000 for F32_4CHAIN, for the D = 256 v3 pipeline (NV = gathered V
 * tables: 1, 2, or capacity 4 / 8 for R <= 8, whose LDS slabs keep 7 distinct V rows per 32-row tile
 * and read further ones from L2); 100 for the register-staged kernel (D < 256, and D = 256 forms the v3
 * kernel does not take: a gathered V with the sigma' epilogue, V rows that are not dense); 500 + 10*NV + aux
 * (+ 2 for broadcast V rows) for the bf16x3 row GEMM (IDDGCN_GEMM_BF16X3 forms it takes); -1 for an invalid D. */
int iddgcn_rowgemm_kernel_id(const iddgcn_rowgemm_t* args);

/* C[D][D] (+)= A^T · B over M rows (A, B are M x D).  Two stages: each of n_blocks
 * workgroups writes a D x D partial into `slab` (n_blocks*D*D floats), then the
 * partials are summed in block order (deterministic).  n_blocks from
 * iddgcn_gemm_tn_blocks().  precision: IDDGCN_GEMM_* (D = 256; other widths exact f32).
 * Weight gradients dS, dK_r (tape.gradient, IDDGCN.py:172). */
int iddgcn_gemm_tn_blocks(long long M, int d);
int iddgcn_gemm_tn_f32(void* stream, long long M, int d, const float* A, const float* B,
                       float* slab, int n_blocks, float* C, int accumulate, int precision);
/* Up to IDDGCN_TN_BATCH independent C_k (+)= A_k^T B_k (fp32, same D) in one launch (ABI 5): at D = 256 in the
 * split-fp16 and (round 6) bf16x3 modes one launch of ~256 workgroups shared out over the entries (blockIdx.y = entry), then each
 * entry's partials summed in block order; otherwise the single-call kernels in turn.  slab: slab_floats floats,
 * at least sum_k min(256 / n, ceil(M_k / 32)) * D * D (the single-call fallback uses up to
 * iddgcn_gemm_tn_blocks(M_k, D) partials, fewer when the slab is smaller, at least one D * D).  The node-level weight gradients of one layer: dK_r = AE_r^T dP_r
 * and the head-chain part of dS (tape.gradient, IDDGCN.py:172, of :62-63 and :71-77). */
#define IDDGCN_TN_BATCH 4
typedef struct {
    long long M;
    const float* A;
    const float* B;
    float* C;
    int accumulate;
} iddgcn_tn_t;
int iddgcn_gemm_tn_batched_f32(void* stream, int d, const iddgcn_tn_t* e, int n, float* slab, long long slab_floats,
                               int precision);
/* iddgcn_gemm_tn_f32 with A a planes table (IDDGCN_PLANES_A; D = 256, split-fp16 mode): dS = x^T do
 * with x^{l} pre-split by its producer (IDDGCN.py:62-63 autodiff). */
int iddgcn_gemm_tn_planes_f32(void* stream, long long M, int d, const void* A, const float* B, float* slab,
                              int n_blocks, float* C, int accumulate);

/* out[D][R] (+)= A^T·dz and out_b[R] (+)= colsum(dz) over M rows (dW_alpha, db_alpha).
 * slab holds (n_blocks+1)*(D+1)*R floats; n_blocks from iddgcn_gemm_tn_narrow_blocks(). */
int iddgcn_gemm_tn_narrow_blocks(long long M);
int iddgcn_gemm_tn_narrow_f32(void* stream, long long M, int d, int R, const float* A,
                              const float* dz, float* slab, int n_blocks,
                              float* dWa, float* dba, int accumulate);

/* Dynamic relation weights (IDDGCN.py:66,75): z = X[x_idx? x_idx[n]:n]·Wa + ba,
 * s = softmax(z), w = sigmoid(s).  Writes S_out[M][R] (softmax, kept for backward)
 * and W_out[M][R]. */
int iddgcn_alpha_fwd_f32(void* stream, int M, int d, int R, const float* X, const int* x_idx,
                         const float* Wa, const float* ba, float* S_out, float* W_out);

/* Gather-combine without GEMM (layer 1, x·S pre-projected at node level):
 *   out[e][c] = sigmoid(Y[y_idx? y_idx[e]:e][c]
 *                       + sum_r coef[(coef_idx? coef_idx[e]:e)*R+r] * V[r*v_rel_stride + (v_idx? v_idx[e]:e)*D + c]) */
int iddgcn_combine_f32(void* stream, int M, int d, int R,
                       const float* Y, const int* y_idx,
                       const float* coef, const int* coef_idx,
                       const float* V, const int* v_idx, long long v_rel_stride, float* out);
/* The run form (y_idx == v_idx = idx, coefficients per row, D = 256) writing a planes table (the layer-1
 * tail output x^1, IDDGCN.py:62-79, pre-split for the layer-2 GEMMs). */
int iddgcn_combine_planes_f32(void* stream, int M, int d, int R, const float* Y, const int* idx, const float* coef,
                              const float* V, long long v_rel_stride, void* out);

/* DistMult decoder (IDDGCN.py:103-109) fused with Keras BCE (IDDGCN.py:161-168)
 * and the seed of the backward.  For each scored edge e:
 *   a = Xh[h_idx[e]], b = Xt[t_idx ? t_idx[e] : e], rho = rel[r_idx[e]]
 *   s = sum a*rho*b                             -> s_out[e] (if s_out; the pre-sigmoid logit, IDDGCN.py:108)
 *   p = sigmoid(s)                              -> p_out[e] (if p_out)
 * If y != NULL (training):
 *   loss_e = -(y log(clip(p)+eps) + (1-y) log(1-clip(p)+eps)), eps = 1e-7
 *   g = scale * dloss_e/dp (0 where p is clipped), ds = g p (1-p)
 *   ds_out[e] = ds;  do_out[e] = ds*rho*a * b*(1-b)
 *   drel_slab[blk][r][:] += ds*a*b ; loss_slab[blk] += loss_e
 * n_blocks from iddgcn_distmult_blocks(); slabs hold n_blocks*R*D and n_blocks floats. */
int iddgcn_distmult_blocks(long long T);
int iddgcn_distmult_bce_f32(void* stream, long long T, int d, int R,
                            const float* Xh, const int* h_idx, const float* Xt, const int* t_idx,
                            const int* r_idx, const float* rel, const float* y, float scale,
                            float* p_out, float* s_out, float* ds_out, float* do_out,
                            float* drel_slab, float* loss_slab, int n_blocks);

/* Training form of the above that also produces the head-side seed, in ONE pass over the
 * scored edges grouped by head (seg_ptr/perm: head segments, perm in edge order within a head):
 * for head node n and e = perm[k], k in [seg_ptr[n], seg_ptr[n+1]), with a = Xh[n], b = Xt[e]:
 * p_out / s_out / ds_out (all optional), do_out, drel_slab and loss_slab exactly as
 * iddgcn_distmult_bce_f32 (t_idx = NULL), and
 *   dXh[n][c] = a(1-a) * sum_k (b[c]*ds_e)*rel[r_idx[e]][c]     (summed in perm order)
 * which is iddgcn_seg_gather_reduce_f32(seg_ptr, perm, ds, r_idx, rel, Xt, Xh).  Rows of nodes with
 * no edge get zeros.  n_blocks from iddgcn_distmult_blocks(); the drel / loss partials are
 * per block, as for iddgcn_distmult_bce_f32.
 * do_out may alias Xt (do^3 written over x^3 in place).
 * y == NULL selects the PREDICTION seed: g = scale for every edge (the gradient of
 * scale * sum_e p_e, no clipping) and loss_slab accumulates sum_e p_e — the seed of the
 * explainers' tape.gradient(pred, ...) (explanation/explaiNE.py:85-94).
 * Replaces IDDGCN.py:103-109 + the loss of 161-168 and the head-side gradient of
 * DistMult's embedding lookup, one launch. */
int iddgcn_distmult_bce_heads_f32(void* stream, int n_nodes, int d, int R, const int* seg_ptr,
                                  const int* perm, const float* Xh, const float* Xt, const int* r_idx,
                                  const float* rel, const float* y, float scale, float* p_out,
                                  float* s_out, float* ds_out, float* do_out, float* dXh,
                                  float* drel_slab, float* loss_slab, int n_blocks);

/* Deterministic segmented gather-reduce (replaces the UnsortedSegmentSum of
 * embedding_lookup's gradient): for node n,
 *   out[n][c] = (dsig ? X[n][c](1-X[n][c]) : 1)
 *               * sum_{k=seg_ptr[n]}^{seg_ptr[n+1]-1} coef[e] * (rel ? rel[r_idx[e]][c] : 1) * rows[e][c],
 *   e = perm[k] (perm NULL -> e = k).  Sums run in perm order. */
int iddgcn_seg_gather_reduce_f32(void* stream, int n_nodes, int d, const int* seg_ptr, const int* perm,
                                 const float* coef, const int* r_idx, const float* rel,
                                 const float* rows, const float* X, float* out);

/* Tail-side backward of one layer over edges sorted by tail (contiguous segments):
 *   dP[r][n][:]   = sum_{e in seg(n)} W[h_idx[e]][r] * dO[e][:]        (gradient of P_r[t])
 *                   (h_idx == NULL: W is per edge, W[e][r] — see iddgcn_gather_rows_f32)
 *   dsum[n][:]    = sum_{e in seg(n)} dO[e][:]                          (if dsum; layer-1 x·S input)
 *   dWedge[e][r]  = <dO[e], P[r][n]>                                    (gradient of sigmoid(alpha_r)) */
int iddgcn_tail_seg_reduce_f32(void* stream, int n_nodes, int d, int R, const int* seg_ptr,
                               const int* h_idx, const float* W, const float* dO, const float* P,
                               long long p_rel_stride, float* dP, long long dp_rel_stride,
                               float* dsum, float* dWedge);

/* Node-level (head chain) backward of one layer, node n:
 *   dsum[n] += dO[n]                                   (if dsum)
 *   dW_r     = <dO[n], P[r][n]> + sum_{k in hseg(n)} dWedge[hperm[k]][r] (+ ep_in[n][r] if ep_in)
 *   ds_r     = dW_r w_r (1-w_r);  dz[n][j] = s_j (ds_j - sum_r ds_r s_r)   (softmax-sigmoid backward)
 *   dP[r][n] += w_r * dO[n]                             (skipped when dP is NULL, ABI 9: added by
 *                                                        iddgcn_tail_seg_reduce_head_bf16)
 * ep_in (ABI 8): per-node head sums of dWedge computed elsewhere (a node-partitioned step: each rank's
 * iddgcn_head_wsum_f32 over its edges, summed across the ranks), hseg_ptr NULL then.          */
int iddgcn_head_bwd_node_f32(void* stream, int n_nodes, int d, int R, const float* dO,
                             const float* P, long long p_rel_stride, const float* Ssm, const float* W,
                             const int* hseg_ptr, const int* hperm, const float* dWedge, const float* ep_in,
                             float* dP, long long dp_rel_stride, float* dsum, float* dz);

/* out[n][r] = sum_{k in [hptr[n], hptr[n+1])} w[hperm[k]][r], in segment order (ABI 8): the head sums of the
 * per-edge dynamic-weight gradients dWedge (IDDGCN.py:66,75), for a node-partitioned step's reduce-scatter. */
int iddgcn_head_wsum_f32(void* stream, int n_nodes, int R, const int* hptr, const int* hperm, const float* w,
                         float* out);

/* dst[e][j] = src[idx[e]][j], j < width: per-edge copies of narrow node tables
 * (the dynamic weights W[h_e] of each layer, IDDGCN.py:66,75, reused by forward and backward). */
int iddgcn_gather_rows_f32(void* stream, long long M, int width, const float* src, const int* idx, float* dst);

/* out[i] = (accumulate ? out[i] : 0) + scale * sum_{b<n_slabs} slab[b*n + i]  (block order) */
int iddgcn_reduce_slabs_f32(void* stream, int n_slabs, long long n, const float* slab,
                            float* out, int accumulate, float scale);

/* Up to 25 (IDDGCN_ROWGEMM_BATCH) independent iddgcn_rowgemm_f32 calls of one width D (e.g. the per-relation, per-layer
 * node projections A_r·E·K_r of IDDGCN.py:71-77) in ONE launch (blockIdx.y = entry); at D = 256 when
 * every entry maps to the same v3 variant (iddgcn_rowgemm_kernel_id), else one launch per entry. */
#define IDDGCN_ROWGEMM_BATCH 25
int iddgcn_rowgemm_batched_f32(void* stream, const iddgcn_rowgemm_t* args, int n);

/* Keras-2.7 Adam, one tensor (IDDGCN.py:174,392).  sparse_form=0: TF ApplyAdam
 *   m += (g-m)(1-b1); v += (g^2-v)(1-b2); var -= alpha m/(sqrt(v)+eps)
 * sparse_form=1 (_resource_apply_sparse, embeddings): m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2.
 * alpha = lr sqrt(1-b2^t)/(1-b1^t) is computed by the caller. */
int iddgcn_adam_f32(void* stream, long long n, float* var, float* m, float* v, const float* g,
                    float alpha, float b1, float b2, float eps, int sparse_form);

/* The same update with alpha = alpha_table[*step] read on the device, so a captured training step
 * (HIP graph) can be replayed for successive iterations; iddgcn_step_advance (one thread) then
 * stores *loss into loss_history[*step] (either may be NULL) and increments *step.  The table
 * holds the host-computed alphas of the iterations to run (IDDGCN.py:399 fit epochs). */
int iddgcn_adam_table_f32(void* stream, long long n, float* var, float* m, float* v, const float* g,
                          const float* alpha_table, const int* step, float b1, float b2, float eps,
                          int sparse_form);
int iddgcn_step_advance(void* stream, int* step, float* loss_history, const float* loss);

/* ---- bf16-feature mode (BASELINE config 5: "bf16 features with MFMA XW"; perf only) -----------------
 * The edge tables x^1..x^3 and the edge-level gradients do^l are stored as bf16 (512-B rows at D = 256,
 * passed as void*); node tables, weights, coefficients, accumulation and every epilogue stay fp32.
 * GEMMs multiply bf16 edge rows by the weights as a bf16 hi + lo pair (two v_mfma_f32_32x32x16_bf16 per
 * k-step), so the only rounding beyond fp32 is the bf16 storage of the edge tables; with precision
 * IDDGCN_GEMM_BF16 (ABI 10) the weights are bf16 too (one product per k-step).  D = 256 only. */

/* iddgcn_rowgemm_f32 with A, aux and C bf16: the edge forward (gathered V, R <= 8, coefficients per row),
 * the sigma' backward (act DSIGMOID with aux) and plain forms; no accumulate, no broadcast V. */
int iddgcn_rowgemm_bf16(void* stream, const iddgcn_rowgemm_t* args);

/* iddgcn_gemm_tn_f32 with bf16 A and B (slab / blocks / C as there). */
int iddgcn_gemm_tn_bf16(void* stream, long long M, int d, const void* A, const void* B, float* slab, int n_blocks,
                        float* C, int accumulate);

/* ABI 11: a layer's whole edge backward GEMM pair in one pass over the bf16 tables (replaces iddgcn_gemm_tn_bf16 +
 * iddgcn_rowgemm_bf16 with act DSIGMOID, the autodiff of IDDGCN.py:62-63,79 for x_t^{l-1} S^l):
 *   dS = X^T dO  (dS[k][c] = sum_e X[e][k] dO[e][c]; overwritten)
 *   X  = (dO S^T) * X (1 - X)  (in place: dx^{l-1} over x^{l-1}; bf16 hi + lo weights, or with precision
 *        IDDGCN_GEMM_BF16 the weights rounded to bf16 as iddgcn_rowgemm_bf16 takes them; fp32 accumulation)
 * X and dO are M x 256 bf16 (16-B aligned), S 256 x 256 fp32; slab holds iddgcn_sigma_tn_ranges(M) * 256 * 256
 * floats of partials (slab_floats is checked); precision: IDDGCN_GEMM_EXACT_F32, _SPLIT_F16 or _BF16X3 (the hi + lo
 * weights) or IDDGCN_GEMM_BF16, anything else IDDGCN_E_BAD_ARG.  D = 256 only. */
int iddgcn_sigma_tn_ranges(long long M);
int iddgcn_sigma_tn_bf16(void* stream, long long M, int d, const void* dO, void* X, const float* S, float* slab,
                         long long slab_floats, float* dS, int precision);

/* ABI 12: the same pass over fp32 tables in the bf16x3 operand mode (the headline's layer-2/3 edge backward, configs
 * 3 / 4; replaces iddgcn_gemm_tn_f32 + iddgcn_rowgemm_f32 with act DSIGMOID at precision IDDGCN_GEMM_BF16X3):
 *   dS = X^T dO (overwritten) and X = (dO S^T) * X (1 - X) in place, every operand split exactly into three bf16
 *   pieces (six products, fp32 accumulation); X is bitwise the row GEMM's sigma' output.
 * X and dO are M x 256 fp32 (16-B aligned); slab holds iddgcn_sigma_tn_ranges(M) * 256 * 256 floats; precision must
 * be IDDGCN_GEMM_BF16X3 (anything else: IDDGCN_E_BAD_ARG).  D = 256 only. */
int iddgcn_sigma_tn_f32(void* stream, long long M, int d, const float* dO, float* X, const float* S, float* slab,
                        long long slab_floats, float* dS, int precision);

/* The run form of iddgcn_combine_f32 (y_idx == v_idx = idx, coefficients per row) writing bf16 out. */
int iddgcn_combine_bf16(void* stream, int M, int d, int R, const float* Y, const int* idx, const float* coef,
                        const float* V, long long v_rel_stride, void* out);

/* iddgcn_distmult_bce_f32 / _heads_f32 with Xt and do_out bf16 (do_out may alias Xt). */
int iddgcn_distmult_bce_bf16(void* stream, long long T, int d, int R, const float* Xh, const int* h_idx,
                             const void* Xt, const int* t_idx, const int* r_idx, const float* rel, const float* y,
                             float scale, float* p_out, float* s_out, float* ds_out, void* do_out,
                             float* drel_slab, float* loss_slab, int n_blocks);
int iddgcn_distmult_bce_heads_bf16(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const int* perm,
                                   const float* Xh, const void* Xt, const int* r_idx, const float* rel,
                                   const float* y, float scale, float* p_out, float* s_out, float* ds_out,
                                   void* do_out, float* dXh, float* drel_slab, float* loss_slab, int n_blocks);

/* iddgcn_tail_seg_reduce_f32 with dO bf16. */
int iddgcn_tail_seg_reduce_bf16(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const int* h_idx,
                                const float* W, const void* dO, const float* P, long long p_rel_stride, float* dP,
                                long long dp_rel_stride, float* dsum, float* dWedge);

/* ABI 9: iddgcn_tail_seg_reduce_bf16 (per-edge W, R = 8, d = 256 only) fused with the head chain's node terms of the
 * same layer (IDDGCN.py:66-77 autodiff, node n):
 *   dP[r][n][:] = sum_{e in seg(n)} W[e][r] dO[e][:]  +  Wn[n][r] * head_dO[n][:]
 *   dsum[n][:]  = sum_{e in seg(n)} dO[e][:]          +  head_dO[n][:]            (if dsum)
 *   dWedge      as iddgcn_tail_seg_reduce_bf16
 *   dwh[n][r]   = <head_dO[n], P[r][n]>                                      (the node's own part of dW_r)
 * so the head backward is then only iddgcn_head_dz_f32 (the R node tables are written once instead of written, read
 * and rewritten, and P and head_dO are not read again).  head_dO: the layer's head seed (n_nodes x d fp32), Wn: its
 * node-level dynamic weights (n_nodes x R), dwh: n_nodes x R output. */
int iddgcn_tail_seg_reduce_head_bf16(void* stream, int n_nodes, int d, int R, const int* seg_ptr, const float* W,
                                     const void* dO, const float* P, long long p_rel_stride, float* dP,
                                     long long dp_rel_stride, float* dsum, float* dWedge, const float* head_dO,
                                     const float* Wn, float* dwh);

/* ABI 9: the rest of iddgcn_head_bwd_node_f32 after iddgcn_tail_seg_reduce_head_bf16, node n:
 *   dW_r = dwh[n][r] + sum_{k in hseg(n)} dWedge[hperm[k]][r];  ds_r = dW_r w_r (1-w_r);
 *   dz[n][j] = s_j (ds_j - sum_r ds_r s_r)                                  (W = Wn, s = Ssm; n_nodes x R each) */
int iddgcn_head_dz_f32(void* stream, int n_nodes, int R, const float* Ssm, const float* W, const int* hseg_ptr,
                       const int* hperm, const float* dWedge, const float* dwh, float* dz);

#ifdef __cplusplus
}
#endif
#endif /* IDDGCN_H_ */
