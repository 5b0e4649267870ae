/*
 * alignn_hip.h — C ABI of libalignn_hip.so, the MI355X (gfx950) ALIGNN message-passing engine.
 *
 * Drop-in boundary: these entry points replace the PyTorch/PyG ops that the
 * reference's hot path launches implicitly.  Each declaration cites the reference call site it
 * replaces.  All tensors are raw device pointers + explicit sizes/strides (elements, not bytes);
 * fp32 data, int32 graph indices (int64 accepted where the reference hands over PyG edge_index).
 * Every function enqueues on `stream` (a hipStream_t passed as void*), allocates nothing,
 * never synchronises, and returns 0 on success or a negative ALIGNN_E* code.  Results are
 * deterministic (no float atomics; CSR segmented reductions).
 */
#ifndef ALIGNN_HIP_H
#define ALIGNN_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ALIGNN_OK 0
#define ALIGNN_E_BAD_SHAPE -1
#define ALIGNN_E_UNSUPPORTED -2
#define ALIGNN_E_HIP -3
#define ALIGNN_E_WORKSPACE -4

/* Library/version and error introspection.  ABI version 2 (round 3): alignn_tconv_fwd / _bwd_dst /
 * _family lost the edge-encoder argument, AlignnGemmArgs lost `counters`. */
#define ALIGNN_ABI_VERSION 3
int alignn_version(void);
const char* alignn_last_error(void);

/* Dropout / jitter randomness: every call site passes a 64-bit site seed; masks are a counter hash
 * of (seed, element), so the backward regenerates them.  alignn_set_step_seed(ptr) registers a
 * device-resident uint64 that kernels launched afterwards mix into their site seed when they run:
 * a step captured once in a HIP graph draws fresh masks on every replay after the caller updates
 * *ptr (NULL = host seeds only).  Process-wide setting. */
void alignn_set_step_seed(const uint64_t* device_ptr);

/* ------------------------------------------------------------------------------------------
 * Dense projections (MFMA f32 32x32x2, exact fp32).  Replaces every nn.Linear / PyG Linear
 * addmm+mm on the path: encoders train.py:350-364, TransformerConv lin_query/key/value/skip/
 * edge (PyG 2.7.0, built at train.py:308/:326), edge_proj train.py:325/:333, feat_proj
 * train.py:368-372, heads train.py:534-535, and their autograd backward (dX, dW).
 *
 *   C[b](m,n) = act( alpha * sum_k A[b](m,k) * B[b](k,n)  + beta * C[b](m,n)
 *                    + bias[b](n) + rowscale[b](m) * bias2[b](n) ) * (mask ? (mask(m,n) > 0) : 1)
 * with A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn], C(m,n) = C[m*scm + n*scn].
 * Fast path: (sak == 1 or sam == 1) and (sbk == 1 or sbn == 1); others fall back to scalar loads.
 * split_k > 1 accumulates fp32 partial slabs in `workspace` (>= split_k*batch*M*N floats) and
 * reduces them in a second kernel in fixed order; split_k = 0 lets the library choose tile shape
 * and split (alignn_gemm_workspace gives the workspace that choice needs).  reduce_batch = 1 sums the batch into C itself
 * (used for weights shared by all layers, e.g. the folded angle-encoder projection).
 * ---------------------------------------------------------------------------------------- */
typedef struct AlignnGemmArgs {
  int64_t M, N, K, batch;
  const float* A; int64_t sam, sak, sab;
  const float* B; int64_t sbk, sbn, sbb;
  float* C; int64_t scm, scn, scb;
  const float* bias; int64_t sbias_b;              /* may be NULL */
  const float* rowscale; int64_t srs_m, srs_b;     /* may be NULL (with bias2) */
  const float* bias2; int64_t sb2_b;
  const float* mask; int64_t smk_m, smk_n;         /* relu-backward mask source, may be NULL */
  float alpha, beta;
  int32_t relu;
  int32_t split_k;
  float* workspace; int64_t workspace_elems;
  int32_t reduce_batch;   /* 1: C = sum over the batch (one output; K % 16 == 0) */
  int32_t tile;           /* 0: automatic; 1: 128x128, 2: 128x64, 3: 64x128, 4: 64x64 (tuning);
                             + ALIGNN_GEMM_BK32 / BK16 / BK64 (stage depth), + ALIGNN_GEMM_BF16 */
  const int32_t* c_rows;  /* optional: logical row r of C is stored at row c_rows[r] (scatter; beta
                             reads the same row).  bias/rowscale/mask stay indexed by r. */
  float* rowsum;          /* optional (ABI 3): rowsum[m] = sum_k A[m][k] in fp32, written by the same
                             launch — the bias gradient db = dY^T 1 of the Linear whose weight gradient
                             is this product dW = dY^T X (train.py's Linear backwards), replacing a
                             separate column-sum pass over dY.  batch == 1, no reduce_batch; with
                             split-K the partial sums take split * M more workspace floats. */
} AlignnGemmArgs;

#define ALIGNN_GEMM_BK32 16
#define ALIGNN_GEMM_BK16 32
#define ALIGNN_GEMM_BK64 128   /* 64-deep stages: 4x fewer global round trips (small grids, long K) */
/* bf16 compute (the reference's CUDA autocast precision, train.py:632-636):
 * A and B are rounded to bf16 (round-to-nearest-even) as they enter the matrix cores
 * (v_mfma_f32_32x32x16_bf16, 16x the f32 MFMA rate); accumulation, epilogue and storage stay fp32. */
#define ALIGNN_GEMM_BF16 64
/* Force the one-stage-in-flight main loop (the pipelined loop — two register sets of loads in
 * flight — is taken automatically when every stage is full and both operands are vectorisable; both
 * give bitwise the same result).  For A/B tests. */
#define ALIGNN_GEMM_NOPIPE 256
/* bf16 storage (config C3, autocast's tensor dtypes, train.py:632-636): the A / B pointer holds bf16
 * elements (widened exactly as they are staged; strides stay in elements, vector loads need 8-byte
 * alignment), or C receives bf16 (RNE of the fp32 epilogue value; write-only: no beta, no mask).
 * Pointers in AlignnGemmArgs are reinterpreted; combine with ALIGNN_GEMM_BF16 arithmetic. */
#define ALIGNN_GEMM_A_BF16 1024
#define ALIGNN_GEMM_B_BF16 2048
#define ALIGNN_GEMM_C_BF16 4096
/* bf16 only, tiled kernels: operands rounded to bf16 as they are staged and kept as bf16 LDS images
 * (half the LDS bytes, one 16-byte read per fragment, no per-fragment conversion); bitwise equal to
 * the fp32 images.  Taken by default when A is k-contiguous (the products over rows; the weight
 * gradients' transposing stores cost more than the images save); LDS16 forces it on, NOLDS16 off. */
#define ALIGNN_GEMM_LDS16 16384
#define ALIGNN_GEMM_NOLDS16 32768
/* Row-streaming bf16 kernel (gemm_rows.hip: W columns in VGPRs, A bands streamed through LDS; K <= 256,
 * N % 256 == 0, taken from 4096 rows up — the environment variable ALIGNN_GEMM_ROWS_MIN_M moves it):
 * ALIGNN_GEMM_ROWS takes it at any M, ALIGNN_GEMM_NOROWS never.  For tests and A/B. */
#define ALIGNN_GEMM_ROWS 65536
#define ALIGNN_GEMM_NOROWS 131072
/* bf16 weight-gradient kernel (gemm_wgrad.hip: A = dY^T and B = X stored row-major over a long K >= 4096,
 * whole 256 x 256 output tiles per workgroup over row chunks, transposed LDS reads, partials through
 * the split-K reduce): taken by default where it applies; ALIGNN_GEMM_NOWGRAD never.  For tests and A/B. */
#define ALIGNN_GEMM_NOWGRAD 262144

int alignn_gemm_f32(const AlignnGemmArgs* args, void* stream);

/* Workspace floats alignn_gemm_f32 needs for these arguments (split_k = 0: the automatic plan on
 * the current device); 0 when no split is used, -1 for invalid shapes. */
int64_t alignn_gemm_workspace(const AlignnGemmArgs* args);

/* Which kernel alignn_gemm_f32 takes (host query, no GPU work): 0 tiled, 2 the bf16 row-streaming
 * kernel (ALIGNN_GEMM_NOROWS), 3 the bf16 weight-gradient kernel (ALIGNN_GEMM_NOWGRAD), -1 invalid
 * arguments (1, the W-in-LDS streaming kernel of rounds 2-4, was removed in round 5: the row kernel
 * takes every product it took, faster; its ALIGNN_GEMM_STREAM / _NOSTREAM bits are gone). */
int alignn_gemm_path(const AlignnGemmArgs* args);

/* ----------------------------------------------------------------------------------------
 * Skinny products (skinny.hip), streamed at HBM rate: the angle encoder's first Linear over the
 * T line-graph edges (train.py:358-364 and its autograd backward) — K or N is the 11 raw angle
 * features.
 *
 *   alignn_linear_smallk_f32:  out[r][c] = act(sum_k X[r][k] W[c][k] + bias[c])   (K <= 16,
 *       N % 4 == 0, out 16-byte aligned with ldo % 4 == 0; otherwise ALIGNN_E_UNSUPPORTED and the
 *       caller uses alignn_gemm_f32).  relu = 1 applies ReLU.
 *   alignn_gemm_tn_smalln_f32: C[m][n] (+)= sum_k A[k][m] X[k][n] (N <= 16) and, when colsum is
 *       not NULL, colsum[m] (+)= sum_k A[k][m]: one pass over A (the weight and bias gradients of
 *       a Linear from its [K, M] output gradient).  Two fixed-order stages (deterministic);
 *       workspace floats from alignn_gemm_tn_smalln_workspace.
 * ---------------------------------------------------------------------------------------- */
int alignn_linear_smallk_f32(const float* X, int64_t ldx, int64_t M, int32_t K, const float* W, int64_t ldw,
                             const float* bias, int64_t N, int32_t relu, float* out, int64_t ldo, void* stream);
/* bf16 output rows: the Linear as bf16 autocast computes it (train.py:554 under :636) — X, W and bias
 * rounded to bf16, the exact products summed in fp32 on the matrix cores (one v_mfma_f32_32x32x16_bf16
 * per 32 x 32 tile), the sum rounded to bf16 (RNE), ReLU on the rounded value: the angle encoder's
 * hidden layer for the bf16-storage attention kernels (config C3).  Its pre-activation is bitwise the
 * one alignn_enc_bwd_bf16 recomputes without the stored layer.  Needs 1 <= K <= 15, N % 32 == 0,
 * N <= 1024, out rows 16-byte aligned (else ALIGNN_E_UNSUPPORTED). */
int alignn_linear_smallk_bf16out(const float* X, int64_t ldx, int64_t M, int32_t K, const float* W, int64_t ldw,
                                 const float* bias, int64_t N, int32_t relu, uint16_t* out, int64_t ldo,
                                 void* stream);
int64_t alignn_gemm_tn_smalln_workspace(int64_t K, int64_t M, int32_t N);
int alignn_gemm_tn_smalln_f32(const float* A, int64_t lda, int64_t K, int64_t M, const float* X, int64_t ldx,
                              int32_t N, float* C, int64_t ldc, float* colsum, int32_t accumulate, float* workspace,
                              int64_t workspace_elems, void* stream);

/* ------------------------------------------------------------------------------------------
 * Angle-encoder backward, deferred (encbwd.hip).  Replaces the autograd backward of the angle
 * encoder's first Linear + ReLU (train.py:358-364) as it is reached from every EdgeUpdateBlock's
 * TransformerConv (train.py:315): instead of each layer's attention backward accumulating the
 * hidden-layer gradient into a [T, D] array (alignn_tconv_bwd_dst with dF), the layers leave their
 * per-edge scalars dz_e / alpha_e and per-target U / Vd, and one pass forms per target-sorted edge t
 *     dpre_t = [W1 x_t + b1 > 0] * sum_{l<L, h<H} dz_l[t,h] U_l[d,h] + alpha_l[t,h] Vd_l[d,h]
 *     dW1 (+)= sum_t dpre_t x_t^T,   db1 (+)= sum_t dpre_t        (d = dst_at[t])
 * The pre-activation uses alignn_linear_smallk_f32's fma order (the forward's ReLU mask exactly).
 * Needs D <= 256 with D % 4 == 0, kin <= 16, H*L <= 16, L <= ALIGNN_ENCBWD_MAX_LAYERS
 * (otherwise ALIGNN_E_UNSUPPORTED: the caller keeps the per-layer dF path).  Fixed grid and
 * summation orders: deterministic.  workspace floats: alignn_enc_bwd_workspace(D, kin).
 * ---------------------------------------------------------------------------------------- */
#define ALIGNN_ENCBWD_MAX_LAYERS 8
typedef struct AlignnEncBwdArgs {
  int64_t n, T;                        /* line-graph nodes (targets) and edges */
  int32_t D, H, L, kin;
  const int32_t* dst_at;               /* [T] target of each target-sorted edge (alignn_graph_prep) */
  const int32_t* off_dst;              /* [n + 1] target segment offsets (alignn_graph_prep) */
  const float* x; int64_t ldx;         /* [T, kin] raw angle features, target-sorted */
  const float* w1; const float* b1;    /* [D, kin], [D] */
  const float* U[ALIGNN_ENCBWD_MAX_LAYERS];      /* per layer [n, H, D] */
  const float* Vd[ALIGNN_ENCBWD_MAX_LAYERS];     /* per layer [n, H, D] */
  const float* dz[ALIGNN_ENCBWD_MAX_LAYERS];     /* per layer [T, H] (alignn_tconv_bwd_dst dz_e) */
  const float* alpha[ALIGNN_ENCBWD_MAX_LAYERS];  /* per layer [T, H] (alignn_tconv_bwd_dst alpha_e) */
  float* dW1; float* db1; int32_t accumulate;
  float* workspace; int64_t workspace_elems;
} AlignnEncBwdArgs;
int64_t alignn_enc_bwd_workspace(int32_t D, int32_t kin);
int alignn_enc_bwd_f32(const AlignnEncBwdArgs* args, void* stream);
/* bf16 storage (config C3, the reference's autocast, train.py:628-636): the same gradients on the
 * matrix cores with bf16 operands and fp32 accumulation, as autocast runs these Linear backwards —
 * per target and chunk of 32 edges G = [dz | alpha'] . [U ; Vd], dpre = G * [f > 0] with f the
 * forward's bf16 hidden layer F16 [T, ldf] itself (ReLU's backward reads its output), and
 * [dW1^T | db1] (+)= dpre^T . [x | 1].  Needs D = 256 (else ALIGNN_E_UNSUPPORTED); same workspace and
 * determinism as alignn_enc_bwd_f32.  F16 == NULL (the line convs recompute the hidden layer,
 * alignn_lg_fwd_x): the mask comes from bf16(relu(W1 x + b1)) recomputed with the forward's arithmetic
 * (a k-ordered fused multiply-add chain, bitwise the stored layer's mask); kin <= 12. */
int alignn_enc_bwd_bf16(const AlignnEncBwdArgs* args, const uint16_t* F16, int64_t ldf, void* stream);

/* Column sums: out[n] (+)= sum_m X[m*ldx + n], m < M, n < N.  Bias gradients of every Linear.
 * Two-stage, fixed order.  workspace >= 256*N floats. */
int alignn_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, int32_t accumulate,
                      float* workspace, void* stream);
/* The same over bf16 X (fp32 sums): the bias gradient of a Linear whose output gradient is stored in
 * bf16 (the skip projection under bf16 storage). */
int alignn_colsum_bf16(const uint16_t* X, int64_t M, int64_t N, int64_t ldx, float* out, int32_t accumulate,
                       float* workspace, void* stream);

/* Weighted column sums of two row-strided [M, N] matrices with per-row weights per column group
 * of width C (N % C == 0; W rows hold N / C weights):
 *   out[j] (+)= sum_r W1[r*lw1 + j/C] X1[r*ld1 + j] + W2[r*lw2 + j/C] X2[r*ld2 + j]
 * The w-bar gradient of a TransformerConv whose edge features pass through a folded Linear
 * (edge_proj, train.py:325/:333; the angle encoder's 2nd Linear, train.py:358-364): per head,
 * sum_n Q_nh sigz_nh + dout_nh sumA_nh.  Two fixed-order stages; workspace >= 256*N floats. */
int alignn_wcolsum2_f32(int64_t M, int64_t N, int32_t C, const float* X1, int64_t ld1, const float* W1, int64_t lw1,
                        const float* X2, int64_t ld2, const float* W2, int64_t lw2, float* out, int32_t accumulate,
                        float* workspace, void* stream);

/* ------------------------------------------------------------------------------------------
 * Graph preparation: CSR neighbour lists in HBM.  Replaces PyG MessagePassing.collect's
 * index_select by edge_index[0]/[1] and the scatter/ index_add by edge_index[1]
 * (TransformerConv propagate, train.py:315/:334).
 *
 * From PyG edge_index (int64 [2, m], row 0 = source j, row 1 = target i) over n nodes:
 *   off_dst[n+1], perm_dst[m]  : edges grouped by target, original edge order kept in a group
 *   src_at[m], dst_at[m]       : endpoints of the edge at each target-sorted position
 *   off_src[n+1], pos_src[m]   : target-sorted positions grouped by source (ascending)
 * workspace >= 2*n + 64 int32.  *err_flag (device int32) is OR-ed with 1 when an index is out of
 * [0, n) (PyG raises IndexError there; the caller checks the flag).
 * ---------------------------------------------------------------------------------------- */
int alignn_graph_prep(const int64_t* edge_index, int64_t m, int64_t n,
                      int32_t* off_dst, int32_t* perm_dst, int32_t* src_at, int32_t* dst_at,
                      int32_t* off_src, int32_t* pos_src,
                      int32_t* workspace, int32_t* err_flag, void* stream);

/* The attention work list (AlignnSchedule.light, every one of the n targets) built on the device
 * from alignn_graph_prep's off_dst, without copying the in-degrees to the host: targets with
 * in-edges, longest in-edge list first within each of `xcds` contiguous id ranges of equal edge
 * count, interleaved range by range in chunks of `chunk` items, then the targets without in-edges
 * (ops.schedule_lists' lists exactly; every target is one work item, so no result depends on the
 * order, only the L2 reuse of the sources' rows).  For callers that bound every in-degree by heavy_threshold on the host (no heavy list: a
 * larger in-degree ORs 2 into *err_flag).  heavy_threshold <= 512, xcds <= 8.  One workgroup. */
int alignn_schedule_build(const int32_t* off_dst, int64_t n, int32_t heavy_threshold, int32_t xcds,
                          int32_t chunk, int32_t* light, int32_t* err_flag, void* stream);

/* rows_out[i, :] = rows_in[idx[i], :] (float, ld in elements).  Used to lay per-edge inputs out
 * in target-sorted order (lg_edge_attr, train.py:553-554) once per batch. */
int alignn_gather_rows_f32(const float* in, int64_t ld_in, const int32_t* idx, int64_t rows,
                           int64_t cols, float* out, int64_t ld_out, void* stream);

/* out[idx[i], :] (+)= in[i, :] (idx distinct).  Scatters rows computed on the compacted set of
 * active nodes (nodes with line-graph edges) back to all nodes. */
int alignn_scatter_rows_f32(const float* in, int64_t ld_in, const int32_t* idx, int64_t rows,
                            int64_t cols, float* out, int64_t ld_out, int32_t accumulate, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused TransformerConv attention (PyG 2.7.0 TransformerConv.message/aggregate + utils.softmax,
 * SURVEY §8a A5), heads H, hidden D = H*C, edge features of dim D projected per head by
 * M_h = W_edge[h] @ P (P = identity for lin_edge on raw features, P = edge_proj.weight for the
 * atom graph) with w̄ = W_edge @ p (p = edge_proj.bias).  The edge-feature GEMM over the m edges
 * is never formed: per target node d the kernel consumes u[d,h] = M_h^T Q[d,h] (an n-row GEMM)
 * and produces S[d,h] = sum_t alpha'_t f_t, which the caller maps back through M_h (exact algebra,
 * DESIGN.md §3).  One wavefront per target segment, online segment softmax.
 *
 * Layouts: QKVR [n, ldq] with Q at col 0, K at D, V at 2D (R at 3D is for the gate kernel);
 * U, S, Vd, Sz: [n, H, D]; F rows of length D at stride ldf, row of edge position t is
 * feat_row[t] (or t when feat_row == NULL).  Stats mstat/den/sumA: [n, H].
 * Dropout on alpha (p = drop_p, training): keep mask from a counter hash of (seed, t, h).
 *
 * Schedule (may be NULL = every target node gets one wavefront): `light` nodes get one wave each,
 * `heavy` nodes (long in-edge lists, e.g. the PyG lg_edge_index offset quirk) a
 * workgroup of four waves that split the edges and merge in fixed order.  Every node must appear
 * in exactly one of the two lists (nodes without in-edges too: their outputs are written as 0).
 * ---------------------------------------------------------------------------------------- */
typedef struct AlignnSchedule {
  const int32_t* light; int64_t n_light;
  const int32_t* heavy; int64_t n_heavy;
  int32_t flags;     /* ALIGNN_SCHED_WAVE_ITEMS or 0 (bit 0 is reserved) */
  int32_t reserved;
} AlignnSchedule;
/* ALIGNN_SCHED_WAVE_ITEMS: `light` is the list of ALL target nodes in launch order (longest
 * in-edge list first), each processed by one single-wave workgroup (lgconv.hip); `heavy` must be
 * empty.  Used for D = 256, H in {1,2,4}, F rows indexed by edge position (feat_row NULL) and, in
 * the backward, no dF; other calls take the light/heavy kernels of tconv.hip.  Arithmetic and
 * outputs are those kernels' (the same dropout masks); sums are formed in a different order. */
#define ALIGNN_SCHED_WAVE_ITEMS 2

int alignn_tconv_fwd(int64_t n, int64_t m, int32_t D, int32_t H,
                     const int32_t* off_dst, const int32_t* src_at, const int32_t* feat_row,
                     const AlignnSchedule* sched,
                     const float* QKVR, int64_t ldq, const float* U, const float* wbar,
                     const float* F, int64_t ldf,
                     float* aggV, float* S, float* sumA, float* mstat, float* den,
                     float drop_p, uint64_t seed, void* stream);

/* Backward, target side: per target node d, recomputes z/alpha and, with dzs = dL/dz / sqrt(C)
 * (z = the scaled score), writes
 *   dQpart[d]  (cols of dQKVR given by dq, ld lddq) = sum_t dzs_t K_src
 *   Sz[d,h] = sum_t dzs f_t,  sigz[d,h] = sum_t dzs
 *   dz_e[t,h] = dzs, alpha_e[t,h] = alpha' (for the source-side pass)
 *   dF[row(t)] (+)= sum_h dzs u[d,h] + alpha' Vd[d,h]   (row(t) = feat_row[t] or t)
 *   accumulate_dF: bit 0 = add to dF, bit 1 = multiply the result by (F[row(t)] > 0) (F is a
 *   ReLU output, e.g. the angle-encoder hidden layer: its backward mask is applied in place),
 *   bit 2 = dF holds bf16 elements, written (RNE) not accumulated (config C3: the gradient of the
 *   bf16 edge features autocast hands edge_proj is a bf16 tensor; rows 8-byte aligned, lddf % 4 == 0)
 * given dout (gradient of the aggregated message, [n, D]), outp (the aggregated message),
 * Vd[d,h] = M_h^T dout[d,h].  dF may be NULL (the line graph defers the angle-encoder backward to
 * alignn_enc_bwd_f32, which recomputes the per-edge gradient there). */
int alignn_tconv_bwd_dst(int64_t n, int64_t m, int32_t D, int32_t H,
                         const int32_t* off_dst, const int32_t* src_at, const int32_t* feat_row,
                         const AlignnSchedule* sched, const float* QKVR, int64_t ldq, const float* U, const float* Vd,
                         const float* wbar, const float* F, int64_t ldf,
                         const float* dout, const float* outp, const float* mstat, const float* den,
                         float* dq, int64_t lddq, float* Sz, float* sigz, float* dz_e, float* alpha_e,
                         float* dF, int64_t lddf, int32_t accumulate_dF,
                         float drop_p, uint64_t seed, void* stream);
/* The same two kernels with the edge-feature rows F in bf16 when f_bf16 = 1 (config C3: the atom
 * graph's edge features are the bond state as the reference's autocast casts it for edge_proj,
 * train.py:325/:333 under :632-636; widened exactly at the load, all arithmetic and every output
 * fp32; D % 4 == 0, ldf % 4 == 0, rows 8-byte aligned).  f_bf16 = 0: alignn_tconv_fwd /
 * alignn_tconv_bwd_dst. */
int alignn_tconv_fwd_ex(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst, const int32_t* src_at,
                        const int32_t* feat_row, const AlignnSchedule* sched, const float* QKVR, int64_t ldq,
                        const float* U, const float* wbar, const void* F, int64_t ldf, int32_t f_bf16, float* aggV,
                        float* S, float* sumA, float* mstat, float* den, float drop_p, uint64_t seed, void* stream);
int alignn_tconv_bwd_dst_ex(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                            const int32_t* src_at, const int32_t* feat_row, const AlignnSchedule* sched,
                            const float* QKVR, int64_t ldq, const float* U, const float* Vd, const float* wbar,
                            const void* F, int64_t ldf, int32_t f_bf16, const float* dout, const float* outp,
                            const float* mstat, const float* den, float* dq, int64_t lddq, float* Sz, float* sigz,
                            float* dz_e, float* alpha_e, float* dF, int64_t lddf, int32_t accumulate_dF,
                            float drop_p, uint64_t seed, void* stream);

/* bf16 storage variant of the line-graph attention (config C3, the reference's autocast precision:
 * the Linear outputs K, V and the angle encoder's hidden layer are bf16, train.py:632-636): the
 * gathered K|V rows (KV16 [n, ldkv], K at col 0, V at col D) and the streamed edge-feature rows
 * (F16 [m, ldf], row of edge position t is t) are bf16; Q, U, Vd, dout, outp, the statistics and
 * every output stay fp32, and all arithmetic is fp32 (bf16 -> fp32 is exact).  Same outputs as
 * alignn_tconv_fwd / alignn_tconv_bwd_dst (dF == NULL).  Needs D = 256, H in {1, 2, 4} and an
 * ALIGNN_SCHED_WAVE_ITEMS schedule listing every target (heavy list empty). */
int alignn_lg_fwd_bf16(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst, const int32_t* src_at,
                       const AlignnSchedule* sched, const float* Q, int64_t ldq, const uint16_t* KV16, int64_t ldkv,
                       const float* U, const float* wbar, const uint16_t* F16, int64_t ldf, float* aggV, float* S,
                       float* sumA, float* mstat, float* den, float drop_p, uint64_t seed, void* stream);
int alignn_lg_bwd_dst_bf16(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst,
                           const int32_t* src_at, const AlignnSchedule* sched, const float* Q, int64_t ldq,
                           const uint16_t* KV16, int64_t ldkv, const float* U, const float* Vd, const float* wbar,
                           const uint16_t* F16, int64_t ldf, const float* dout, const float* outp,
                           const float* mstat, const float* den, float* dq, int64_t lddq, float* Sz, float* sigz,
                           float* dz_e, float* alpha_e, float drop_p, uint64_t seed, void* stream);
/* The line-graph attention with the edge features RECOMPUTED instead of read (replaces the
 * [T, 256] angle hidden layer that train.py:553-554 materialises and every line conv reads,
 * train.py:315): f_t = relu(W1 x_t + b1) of the 11 raw inputs x_t (lg_edge_attr in target-sorted
 * order, rows of ldx = 12 floats, 16-byte aligned; W1 [256, 11], b1 [256] contiguous fp32), computed
 * per edge group on the matrix cores as the same k-ordered fused multiply-add chain as
 * alignn_linear_smallk_f32 (bitwise the stored layer).  KV16 == NULL: fp32 (K|V read from QKV, f in
 * fp32 — config C2); KV16 given: bf16 storage (K|V from KV16, f rounded to bf16 as
 * alignn_linear_smallk_bf16out stores it — config C3).  Same outputs as alignn_lg_fwd_bf16 /
 * alignn_lg_bwd_dst_bf16 on the materialised layer.  Needs D = 256, H = 4, kin = 11 (else
 * ALIGNN_E_UNSUPPORTED) and an ALIGNN_SCHED_WAVE_ITEMS schedule listing every target. */
int alignn_lg_fwd_x(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst, const int32_t* src_at,
                    const AlignnSchedule* sched, const float* QKV, int64_t ldq, const uint16_t* KV16, int64_t ldkv,
                    const float* U, const float* wbar, const float* X, int64_t ldx, int32_t kin, const float* W1,
                    const float* b1, float* aggV, float* S, float* sumA, float* mstat, float* den, float drop_p,
                    uint64_t seed, void* stream);
int alignn_lg_bwd_dst_x(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_dst, const int32_t* src_at,
                        const AlignnSchedule* sched, const float* QKV, int64_t ldq, const uint16_t* KV16,
                        int64_t ldkv, const float* U, const float* Vd, const float* wbar, const float* X, int64_t ldx,
                        int32_t kin, const float* W1, const float* b1, const float* dout, const float* outp,
                        const float* mstat, const float* den, float* dq, int64_t lddq, float* Sz, float* sigz,
                        float* dz_e, float* alpha_e, float drop_p, uint64_t seed, void* stream);
/* dst (bf16, RNE) = src (fp32) for a [rows, cols] block; cols and both leading dimensions multiples
 * of 4, src rows 16-byte aligned. */
int alignn_cast_bf16_f32(const float* src, int64_t lds, int64_t rows, int64_t cols, uint16_t* dst, int64_t ldd,
                         void* stream);

/* Which attention kernel family alignn_tconv_fwd / alignn_tconv_bwd_dst (with dF == NULL) run for
 * these arguments: 3 = single-wave items (lgconv.hip), 2 = light/heavy workgroups (tconv.hip),
 * 0 = unsupported arguments.  A host query: no device work. */
int alignn_tconv_family(int32_t D, int32_t H, const int32_t* feat_row, const float* F,
                        const AlignnSchedule* sched);

/* Backward, source side (replaces the atomic index_add of the gather backward): per source node
 *   dK[s] = sum_{t: src(t)=s} dzs_t Q[dst(t)],  dV[s] = sum alpha'_t dout[dst(t)]
 * written into dQKVR columns D..3D (ld lddq). */
int alignn_tconv_bwd_src(int64_t n, int64_t m, int32_t D, int32_t H,
                         const int32_t* off_src, const int32_t* pos_src, const int32_t* dst_at,
                         const float* QKVR, int64_t ldq, const float* dout,
                         const float* dz_e, const float* alpha_e, float* dKV, int64_t lddkv, void* stream);
/* The same sums (bitwise) given dst_src[i] = dst_at[pos_src[i]], the targets in by-source order
 * (built once per batch): a wave loads each edge's target and position independently and the next
 * edge group's indices while the current group's rows are in flight. */
int alignn_tconv_bwd_src_by(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_src,
                            const int32_t* pos_src, const int32_t* dst_src, const float* QKVR, int64_t ldq,
                            const float* dout, const float* dz_e, const float* alpha_e, float* dKV, int64_t lddkv,
                            void* stream);
/* bf16 storage (config C3: Q is a bf16 Linear output under the reference's autocast, train.py:632-636):
 * the same sums with the gathered target rows read from bf16 copies — Q16 [n, ldq16] and dout16
 * [n, D] — widened exactly at the load (the fp32 entry on the widened rows gives the same bits);
 * these rows are the kernel's traffic, so it halves.  D % 4 == 0, ldq16 % 4 == 0, 8-byte aligned. */
int alignn_tconv_bwd_src_by_bf16(int64_t n, int64_t m, int32_t D, int32_t H, const int32_t* off_src,
                                 const int32_t* pos_src, const int32_t* dst_src, const uint16_t* Q16, int64_t ldq16,
                                 const uint16_t* dout16, const float* dz_e, const float* alpha_e, float* dKV,
                                 int64_t lddkv, void* stream);

/* ------------------------------------------------------------------------------------------
 * Gate + LayerNorm + ReLU + dropout + residual, fused row kernel.  Replaces TransformerConv's
 * beta gate (lin_beta/sigmoid/blend, PyG forward) and train.py:316-317 / :335-336
 * (LayerNorm eps 1e-5, ReLU, Dropout, residual add).
 *   beta = sigmoid(<[o, r, o-r], wbeta>), y = beta r + (1-beta) o, x_new = x + drop(relu(LN(y)))
 * o = outp [n,D], r = R (ldr), x = X (ldx); saves beta/mu/rstd [n].
 * ---------------------------------------------------------------------------------------- */
int alignn_gate_ln_fwd(int64_t n, int32_t D, const float* outp, const float* R, int64_t ldr,
                       const float* wbeta, const float* X, int64_t ldx, const float* ln_w, const float* ln_b,
                       float* Xnew, int64_t ldxn, float* beta, float* mu, float* rstd,
                       float drop_p, uint64_t seed, void* stream);

/* Backward: given dXnew, writes dout [n,D], dR (ldr), and accumulates (+=) the parameter grads
 * d_wbeta[3D], d_ln_w[D], d_ln_b[D] (fixed-order two-stage reduction; workspace >= 1024*5*D). */
int alignn_gate_ln_bwd(int64_t n, int32_t D, const float* dXnew, int64_t lddx, const float* outp,
                       const float* R, int64_t ldr, const float* wbeta, const float* ln_w, const float* ln_b,
                       const float* beta, const float* mu, const float* rstd,
                       float* dout, float* dR, int64_t lddr, float* d_wbeta, float* d_ln_w, float* d_ln_b,
                       float* workspace, float drop_p, uint64_t seed, void* stream);

/* Compacted conv outputs (the line graph's active bonds): o of row r is
 * outp[outp_rows[r]] (outp_rows[r] = -1: o = 0, the exact output of a node without in-edges), and
 * the backward writes dout only at the compacted rows — no zero-filled [n, D] copy of o and no
 * [n, D] dout to gather from.  outp_rows = NULL is the plain entry above. */
int alignn_gate_ln_fwd_rows(int64_t n, int32_t D, const float* outp, const int32_t* outp_rows, const float* R,
                            int64_t ldr, const float* wbeta, const float* X, int64_t ldx, const float* ln_w,
                            const float* ln_b, float* Xnew, int64_t ldxn, float* beta, float* mu, float* rstd,
                            float drop_p, uint64_t seed, void* stream);
/* Workspace floats alignn_gate_ln_bwd(_rows) needs for n rows of width D (-1: bad shape). */
int64_t alignn_gate_ln_bwd_workspace(int64_t n, int32_t D);
int alignn_gate_ln_bwd_rows(int64_t n, int32_t D, const float* dXnew, int64_t lddx, const float* outp,
                            const int32_t* outp_rows, const float* R, int64_t ldr, const float* wbeta,
                            const float* ln_w, const float* ln_b, const float* beta, const float* mu,
                            const float* rstd, float* dout, float* dR, int64_t lddr, float* d_wbeta, float* d_ln_w,
                            float* d_ln_b, float* workspace, float drop_p, uint64_t seed, void* stream);
/* alignn_gate_ln_bwd_rows in two halves, so the parameter-gradient reduction can run on another
 * stream (the caller orders it after the partials and keeps the workspace alive until it ran):
 * _partials writes dout, dR and the per-workgroup partial rows into workspace; _reduce adds the
 * fixed-order sums of those rows to d_wbeta / d_ln_w / d_ln_b (same n, D). */
int alignn_gate_ln_bwd_partials(int64_t n, int32_t D, const float* dXnew, int64_t lddx, const float* outp,
                                const int32_t* outp_rows, const float* R, int64_t ldr, const float* wbeta,
                                const float* ln_w, const float* ln_b, const float* beta, const float* mu,
                                const float* rstd, float* dout, float* dR, int64_t lddr, float* workspace,
                                float drop_p, uint64_t seed, void* stream);
int alignn_gate_ln_bwd_reduce(int64_t n, int32_t D, const float* workspace, float* d_wbeta, float* d_ln_w,
                              float* d_ln_b, void* stream);
/* _partials with an addend: the incoming gradient is dXnew + dX_add ([n, D] contiguous, one fp32 add
 * per element), and that sum is written back to dXnew (it is also the residual's gradient).  The
 * bond state e feeds both the atom block and the next line block (train.py:570-573): the line
 * block's backward folds the atom block's edge-feature gradient in here, so the atom block can run
 * on its own stream (write-only dF) beside the later line block. */
int alignn_gate_ln_bwd_partials_add(int64_t n, int32_t D, float* dXnew, int64_t lddx, const float* dX_add,
                                    const float* outp, const int32_t* outp_rows, const float* R, int64_t ldr,
                                    const float* wbeta, const float* ln_w, const float* ln_b, const float* beta,
                                    const float* mu, const float* rstd, float* dout, float* dR, int64_t lddr,
                                    float* workspace, float drop_p, uint64_t seed, void* stream);
/* bf16 storage forms (config C3; autocast keeps Linear outputs and their gradients in bf16,
 * train.py:632-636): r_bf16 = R is the skip projection's bf16 output; Xnew16 (may be NULL) receives
 * a bf16 copy of the new state, the next Linear's input as autocast casts it; dr_bf16 = dR is written
 * as bf16.  LayerNorm, the gate and every accumulation stay fp32.  bf16 rows: 8-byte aligned,
 * leading dimension % 4 == 0.  alignn_gate_ln_bwd_partials_ex: r_bf16 bit 1 = dX_add holds bf16
 * elements (the atom block's edge-feature gradient under autocast, alignn_tconv_bwd_dst_ex bit 2);
 * bit 2 = dXnew holds no gradient yet (read as zero; needs dX_add, whose values are written to dXnew):
 * the last line block's incoming gradient, which comes from the atom block beside it alone. */
int alignn_gate_ln_fwd_ex(int64_t n, int32_t D, const float* outp, const int32_t* outp_rows, const void* R,
                          int64_t ldr, int32_t r_bf16, const float* wbeta, const float* X, int64_t ldx,
                          const float* ln_w, const float* ln_b, float* Xnew, int64_t ldxn, uint16_t* Xnew16,
                          int64_t ldxn16, float* beta, float* mu, float* rstd, float drop_p, uint64_t seed,
                          void* stream);
/* The same, and (Xa not NULL, needs outp_rows) row r of the new state also written to Xa[outp_rows[r]]
 * wherever outp_rows[r] >= 0: the next line block's gather of the active rows (they are the same
 * rows for every layer), done by the gate kernel that writes the state instead of a separate launch. */
int alignn_gate_ln_fwd_ex2(int64_t n, int32_t D, const float* outp, const int32_t* outp_rows, const void* R,
                           int64_t ldr, int32_t r_bf16, const float* wbeta, const float* X, int64_t ldx,
                           const float* ln_w, const float* ln_b, float* Xnew, int64_t ldxn, uint16_t* Xnew16,
                           int64_t ldxn16, float* Xa, float* beta, float* mu, float* rstd, float drop_p,
                           uint64_t seed, void* stream);
int alignn_gate_ln_bwd_partials_ex(int64_t n, int32_t D, float* dXnew, int64_t lddx, const float* dX_add,
                                   const float* outp, const int32_t* outp_rows, const void* R, int64_t ldr,
                                   int32_t r_bf16, const float* wbeta, const float* ln_w, const float* ln_b,
                                   const float* beta, const float* mu, const float* rstd, float* dout, void* dR,
                                   int64_t lddr, int32_t dr_bf16, float* workspace, float drop_p, uint64_t seed,
                                   void* stream);

/* ------------------------------------------------------------------------------------------
 * Readout (train.py:562-586): global_mean_pool over ptr (PyG, train.py:562), concat with
 * global_x / sg_one_hot (train.py:563-572), dropout (train.py:573).
 * feats [B, D + G]  (G = gdim + sgdim).  Backward scatters dpooled/count to the atoms.
 * ---------------------------------------------------------------------------------------- */
int alignn_readout_feats_fwd(int64_t B, int32_t D, const float* h, const int64_t* ptr,
                             const float* global_x, int32_t gdim, const float* sg, int32_t sgdim,
                             float* feats, float drop_p, uint64_t seed, void* stream);
int alignn_readout_pool_bwd(int64_t B, int64_t N, int32_t D, const float* dfeats, int64_t ldf,
                            const int64_t* ptr, const int64_t* batch, float* dh, int32_t accumulate,
                            float drop_p, uint64_t seed, void* stream);

/* Elementwise dropout (+ optional ReLU-mask backward): y = x * keep/(1-p) [* (ref > 0)] */
int alignn_dropout_f32(int64_t rows, int64_t cols, const float* x, int64_t ldx, float* y, int64_t ldy,
                       const float* relu_ref, int64_t ldr, float drop_p, uint64_t seed, void* stream);

/* Hetero Gaussian NLL (train.py:656-681), forward + gradient in one launch:
 * loss = mean_b mean_t w_b 0.5(lv + (mu-y)^2/e^lv) + l2 * mean((lv/2)^2), lv = clamp(logvar, floor).
 * heads [B, ldh] hold mean at col 0..T-1 and logvar at T..2T-1; y_z = (log y - m)/s.
 * weights [B]: KNN sample weights (train.py:660-674), NULL = 1. */
int alignn_hetero_nll(int64_t B, int32_t T, const float* heads, int64_t ldh, const float* y,
                      const float* weights, const float* log_means, const float* log_stds, float floor, float l2,
                      float* loss, float* dheads, int64_t lddh, void* stream);

/* The same loss as the reference's CUDA step computes it under autocast(bfloat16) (train.py:632-636,
 * :653-681 with use_amp): mean/logvar rounded to bf16 as autocast's Linear returns them, clamp, the
 * target cast, mean - target and 0.5*logvar in bf16, exp/pow/div/means in fp32; dheads = autograd's
 * gradient of those ops (each rounded to its tensor's dtype; logvar's three bf16 gradients summed in
 * autograd's order), unscaled.  Same arguments as alignn_hetero_nll. */
int alignn_hetero_nll_amp(int64_t B, int32_t T, const float* heads, int64_t ldh, const float* y,
                          const float* weights, const float* log_means, const float* log_stds, float floor,
                          float l2, float* loss, float* dheads, int64_t lddh, void* stream);

/* Feature jitter (train.py:641-646): x += std * N(0,1) from a counter-based generator. */
int alignn_add_noise_f32(int64_t n, float* x, float std, uint64_t seed, void* stream);
/* Both jittered feature copies of a step in one launch: dst_k[i] = src_k[i] + std * N(0,1), the same
 * values as copying src_k to dst_k and calling alignn_add_noise_f32(n_k, dst_k, std, seed_k). */
int alignn_noisy_copy2_f32(int64_t n1, const float* src1, float* dst1, uint64_t seed1, int64_t n2,
                           const float* src2, float* dst2, uint64_t seed2, float std, void* stream);

/* ------------------------------------------------------------------------------------------
 * Deep-ensemble inference: moment-matched mixture of M heteroscedastic members,
 * ensemble_collect train.py:875-894, and predict.ensemble_predict's log-normal conversion and
 * 90% interval, predict.py:604-640.
 *   heads: member j's [B, 2T] output (mean | logvar) at heads + j*member_stride, row stride ldh.
 *   var_j = exp(max(logvar_j, floor)); mean = E[mu]; var = E[var_j] + E[mu^2] - mean^2;
 *   std_z = sqrt(max(var, 1e-12)).  With log_means/log_stds [T] (LogTransformer): mean_orig =
 *   exp(mean*s+m), std_lin = sqrt(max((exp(ls^2)-1) exp(2lm+ls^2), 0)), lo90/hi90 = mean_orig -/+
 *   1.6448536269514722 std_lin (lo clipped at 0).  Outputs [B, T]; any may be NULL.
 * ---------------------------------------------------------------------------------------- */
int alignn_ensemble_moments(int32_t M, int64_t B, int32_t T, const float* heads, int64_t member_stride,
                            int64_t ldh, float min_logvar_floor, const float* log_means, const float* log_stds,
                            float* mean_z, float* std_z, float* mean_orig, float* std_lin, float* lo90,
                            float* hi90, void* stream);

/* out[i] = mean over M members of x[j*member_stride + i], i < n (ensemble embeddings,
 * ensemble_collect_embeddings train.py:907-927). */
int alignn_member_mean_f32(int32_t M, int64_t n, const float* x, int64_t member_stride, float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Optimizer step over the flat buffers: clip_grad_norm_(5.0) + fused AdamW with
 * the reference's two param groups (train.py:693-699, :1516-1542).
 * alignn_grad_norm_f32: *norm = ||g||_2 (fixed-order two-stage sum; workspace >= 1024 floats).
 * alignn_adamw_f32: *step += 1; c = min(max_norm / (*norm + 1e-6), 1) (norm NULL: c = 1); g *= c
 * (in place, as clip_grad_norm_); then for i < split lr = lr0 else lr1:
 *   p *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
 *   p -= lr / (1 - b1^step) * m / (sqrt(v) / sqrt(1 - b2^step) + eps).
 * The hyper-parameters are doubles, as the reference's Python floats are: each derived scalar
 * (1 - lr*wd, 1 - b1, 1 - b2, lr / (1 - b1^step), sqrt(1 - b2^step)) is formed in double and rounded
 * to fp32 once, as torch's single-tensor AdamW does (the reference's CPU optimizer).
 * norm and step are device scalars (graph-capturable).
 * ---------------------------------------------------------------------------------------- */
int alignn_grad_norm_f32(const float* g, int64_t n, float* norm, float* workspace, void* stream);
int alignn_adamw_f32(float* p, float* g, float* m, float* v, int64_t n, int64_t split, double lr0, double lr1,
                     double weight_decay, double beta1, double beta2, double eps, const float* norm, float max_norm,
                     float* step, void* stream);
/* alignn_adamw_f32_dev: the same update with the two groups' learning rates read from device memory
 * (lr: double[2] = {lr0, lr1}) when the kernel runs, so a recorded launch plan follows the
 * reference's per-epoch schedule (set_lr before each epoch, train.py:1641-1652, cosine :1215-1232)
 * without being re-recorded. */
int alignn_adamw_f32_dev(float* p, float* g, float* m, float* v, int64_t n, int64_t split, const double* lr,
                         double weight_decay, double beta1, double beta2, double eps, const float* norm,
                         float max_norm, float* step, void* stream);
/* GradScaler semantics of the reference's CUDA step (train.py:690-695: scaler.scale(loss).backward();
 * unscale_; clip_grad_norm_; scaler.step; scaler.update(); scaler built at :1475-1476 with torch's
 * defaults).  scaler: device float[4] = {scale (initially 65536), growth_tracker, found_inf, skipped}.
 * The gradients handed in are the unscaled ones (a power-of-two scale is exact in fp32, so
 * scale-then-unscale only matters where the scaled value overflows).
 * alignn_grad_norm_amp_f32: *norm as alignn_grad_norm_f32 (bitwise the same), and found_inf =
 *   1 if some g[i] * scale is inf or NaN (unscale_'s check), else 0 (workspace >= 2048 floats).
 * alignn_adamw_amp_f32_dev: found_inf set -> no update at all (p, g, m, v and *step unchanged),
 *   scale *= 0.5, growth_tracker = 0, skipped += 1 (scaler.step skips optimizer.step; update backs
 *   off); else the alignn_adamw_f32_dev update, then growth_tracker += 1 and, when it reaches
 *   growth_interval (torch: 2000), scale *= 2 and growth_tracker = 0.  No host synchronisation. */
int alignn_grad_norm_amp_f32(const float* g, int64_t n, float* norm, float* scaler, float* workspace, void* stream);
int alignn_adamw_amp_f32_dev(float* p, float* g, float* m, float* v, int64_t n, int64_t split, const double* lr,
                             double weight_decay, double beta1, double beta2, double eps, const float* norm,
                             float max_norm, float* step, float* scaler, int32_t growth_interval, void* stream);

/* ------------------------------------------------------------------------------------------
 * Batch assembly from a dataset resident in HBM (replaces PyG Collater /
 * Batch.from_data_list, SURVEY §8a A9, over per-sample .pt loads, train.py:132).  All offset
 * arrays are device int64 [G]; graph g's segment src[src_start[g] .. +count[g]) goes to
 * dst[dst_start[g] ..); max_count = max_g count[g] (sizes the grid).
 *   rows:  float rows of `width` values (x, edge_attr, lg_edge_attr, global_x, sg_one_hot, y)
 *   index: two int64 rows (src row stride src_ld, dst row stride dst_ld), + add[g] (PyG's
 *          increment: cumulative num_nodes for edge_index AND lg_edge_index)
 *   batchvec: batch[dst_start[g] + i] = g for i < count[g] (nodes).
 * ---------------------------------------------------------------------------------------- */
int alignn_collate_rows_f32(int32_t G, const float* src, int64_t width, const int64_t* src_start,
                            const int64_t* dst_start, const int64_t* count, int64_t max_count, float* dst,
                            void* stream);
int alignn_collate_index_i64(int32_t G, const int64_t* src, int64_t src_ld, const int64_t* src_start,
                             const int64_t* dst_start, const int64_t* count, const int64_t* add, int64_t max_count,
                             int64_t* dst, int64_t dst_ld, void* stream);
int alignn_collate_batchvec(int32_t G, const int64_t* dst_start, const int64_t* count, int64_t max_count,
                            int64_t* batch, void* stream);
/* The dataset's per-sample transform fused into the row copy (PtGraphDataset.__getitem__,
 * train.py:137-154 and :200-216): a destination row of dst_width values takes the source row's first
 * copy_width values and zeros after them (use_mat2vec / force_node_dim: select, pad, truncate); with
 * mean/std (device fp32, both or neither) each value v becomes (v - mean[k]) / std[k], k = the column
 * (by_row = 0, node features: scalar | mat2vec statistics) or the element's index inside the graph's
 * segment (by_row = 1, global_x: one statistic per global scalar). */
int alignn_collate_rows_std_f32(int32_t G, const float* src, int64_t src_width, const int64_t* src_start,
                                const int64_t* dst_start, const int64_t* count, int64_t max_count, float* dst,
                                int64_t dst_width, int64_t copy_width, const float* mean, const float* stdv,
                                int32_t by_row, void* stream);
/* ok[g] = 0 when graph g's segment holds a NaN or an infinity (PtGraphDataset._is_valid,
 * train.py:174-182; ok preset to 1 by the caller, one launch per float field). */
int alignn_segment_finite_f32(int32_t G, const float* src, int64_t width, const int64_t* start,
                              const int64_t* count, int64_t max_count, int32_t* ok, void* stream);
/* Feature statistics over a selection of J graphs (train.py:1324-1380): fp64 sum and sum of squares
 * per statistic k < K — a column summed over the graph's rows (by_row = 0) or the element at index
 * k of the graph's segment (by_row = 1) — per graph first, then accumulated in selection order.
 * workspace: alignn_feature_stats_workspace(J, K) doubles. */
int64_t alignn_feature_stats_workspace(int32_t J, int64_t K);
int alignn_feature_stats_f64(int32_t J, const float* src, int64_t width, const int64_t* start, const int64_t* count,
                             int64_t K, int32_t by_row, double* sum, double* sq, double* workspace,
                             int64_t workspace_elems, void* stream);
/* Ghost edges of the inert graph that pads a batch to a fixed capacity (a captured plan replays any
 * batch that fits; alignn_mi355x.store.BatchCapacity): for j < count, dst[start + j] =
 * base + (j + 1) % mod (source row) and dst[ld + start + j] = base + j % mod (target row). */
int alignn_ghost_edges_i64(int64_t* dst, int64_t ld, int64_t start, int64_t count, int64_t base, int64_t mod,
                           void* stream);
/* Up to 32 device-to-device copies in one launch (src, dst: HOST arrays of device pointers, 16-byte
 * aligned; bytes: host array, multiples of 4).  Re-binds a captured step to a new batch (the batch
 * fields and its CSR / compaction / schedule cache copied into the captured buffers). */
int alignn_copy_many(int32_t n, const void* const* src, void* const* dst, const int64_t* bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * KNN density weights over graph embeddings (compute_global_knn_weights,
 * train.py:930-1010).  Column standardisation (population std, floor 1e-8) from column sums:
 *   alignn_col_center_sq_f32: out = (Z - colsum/n)^2 (feed to alignn_colsum_f32 for ssq)
 *   alignn_standardize_f32:   out = (Z - colsum/n) / max(sqrt(ssq/n), 1e-8)
 *   alignn_row_sqnorm_f32:    r_i = |Zs_i|^2
 * alignn_knn_select_weights: for query rows row0..row0+rows-1 with G = Zs[rows] Zs^T ([rows, ldg]):
 *   the k nearest j != i by d2 = r_i + r_j - 2 G (ties by index), nbr [rows, k] (may be NULL),
 *   w_raw[i] = (k / (sum sqrt(d2) + eps))^-alpha / (1 + beta * mean_t var_k(Y[nbr, t])).
 *   Y [n, T] (raw targets, as the reference); 1 <= k <= min(64, n-1).
 * ---------------------------------------------------------------------------------------- */
int alignn_col_center_sq_f32(const float* Z, int64_t n, int32_t D, const float* colsum, float* out, void* stream);
int alignn_standardize_f32(const float* Z, int64_t n, int32_t D, const float* colsum, const float* ssq, float* out,
                           void* stream);
int alignn_row_sqnorm_f32(const float* Zs, int64_t n, int32_t D, float* r, void* stream);
int alignn_knn_select_weights(const float* G, int64_t ldg, const float* r, int64_t n, int64_t row0, int64_t rows,
                              int32_t k, const float* Y, int32_t T, float eps, float alpha, float beta, int64_t* nbr,
                              float* w_raw, void* stream);

/* ------------------------------------------------------------------------------------------
 * Launch plans (native step executor).  Replaces the per-batch host loop of train_epoch_hetero
 * (train.py:639-699: model(batch), loss.backward(), clip_grad_norm_, optimizer.step()) once the
 * step has been recorded: the engine's ~300 launches are re-issued from C++, no Python in between.
 * alignn_plan_begin(stream): start recording; every launch of this library is executed as usual
 *   and appended to the plan; `stream` becomes slot 0 (replaced by the replay stream).
 * alignn_plan_note_wait(dst, src): append the ordering edge "dst waits for src's work so far"
 *   (the caller performs the wait itself while recording; no-op when not recording).
 * alignn_plan_end(): finish, returns the plan (NULL on error). alignn_plan_abort(): drop it.
 * alignn_plan_replay(plan, stream): issue the recorded launches and edges (slot 0 -> stream).
 *   Every buffer the recorded step touched must still be allocated at the same address.
 * alignn_plan_info: launches, edges, distinct streams, stored argument bytes.
 * alignn_plan_note_timestamp(stream): while recording, append a timing-event record on `stream`
 *   and return its index (-1 when not recording); alignn_plan_elapsed_ms(plan, i0, i1, &ms): the
 *   device time between two timestamps of the last (completed) replay (roofline probes).
 * alignn_graph_census(hipGraph_t, &kernels, &other): node counts of a captured graph, to check
 *   that a plan recorded during that capture holds every kernel (other == 0).
 * alignn_fill_f32 / alignn_copy_f32: x[0:n] = value; dst[0:n] = src[0:n] (plan-recordable
 *   replacements for torch's zero_/copy_ inside the step).
 * alignn_add_f32: x[0:n] += y[0:n], one fp32 add per element (the atom-graph blocks' edge-feature
 *   gradient folded into the bond-state gradient; replaces the `+=` autograd does where the bond
 *   state e feeds both the atom block and the next line block, train.py:570-573).
 * alignn_set_i64: x[0] = value on the stream — the per-step device seed written before a plan
 *   replay (the reference draws fresh dropout masks every step, train.py:655).
 * ---------------------------------------------------------------------------------------- */
int alignn_plan_begin(void* stream);
int alignn_plan_note_wait(void* dst_stream, void* src_stream);
void* alignn_plan_end(void);
int alignn_plan_abort(void);
int alignn_plan_replay(void* plan, void* stream);
/* alignn_plan_replay_serial(plan, stream): the same launches and timestamps in recorded issue order,
 * all on `stream`, cross-stream edges dropped (issue order satisfies them): each kernel alone on the
 * device, so the plan timestamps give its isolated duration (the bench's roofline probes). */
int alignn_plan_replay_serial(void* plan, void* stream);
int alignn_plan_info(const void* plan, int64_t* launches, int64_t* waits, int64_t* streams, int64_t* arg_bytes);
/* alignn_plan_entries(plan, kind_slot_src, names, cap): the recorded entries in issue order, entry i
 * as kind_slot_src[3i..3i+2] = (kind, stream slot, source slot) — kind 0 kernel (source -1), 1 edge
 * ("slot waits for source's work so far"), 2 timestamp — and names[i] the kernel's name (NULL for
 * edges and timestamps; names may be NULL).  Fills at most cap entries; returns the entry count
 * (-1 for a NULL plan).  Introspection of the step's stream structure (tools/plan_dump.py). */
int64_t alignn_plan_entries(const void* plan, int32_t* kind_slot_src, const char** names, int64_t cap);
int alignn_plan_destroy(void* plan);
int alignn_plan_note_timestamp(void* stream);
int alignn_plan_elapsed_ms(void* plan, int32_t i0, int32_t i1, float* ms);
/* alignn_plan_check_ptrs(plan, ranges, n, &bad_value, &bad_launch, &checked): ownership proof of a
 * recorded plan.  ranges = n pairs [lo, hi) of device byte addresses the caller holds for as long as
 * the plan lives (its workspaces, parameters, batch buffers, the capture's memory pool).  Every
 * non-null pointer argument and every struct-argument word that resolves to device memory must lie
 * in one; otherwise ALIGNN_E_BAD_SHAPE with the offending value and launch index (trainer.capture
 * refuses such a plan).  Recording state and the registered step seed are per host thread. */
int alignn_plan_check_ptrs(const void* plan, const uint64_t* ranges, int64_t n, uint64_t* bad_value,
                           int64_t* bad_launch, int64_t* checked);
/* alignn_plan_refs(plan, ranges, n, hit): hit[i] = 1 when some pointer argument or struct-argument
 * word of the recorded plan lies in [ranges[2i], ranges[2i+1]), else 0 (trainer._rebind copies a new
 * batch only into the captured batch's buffers the plans touch). */
int alignn_plan_refs(const void* plan, const uint64_t* ranges, int64_t n, int32_t* hit);
int alignn_graph_census(void* graph, int64_t* kernels, int64_t* other);
/* alignn_plan_check_deps(plan, hipGraph_t, &bad_from, &bad_to, &edges): the plan's ordering against the
 * graph captured during its recording (kernel nodes matched to launches in creation order): every
 * kernel-to-kernel dependency of the graph (through empty / event nodes too) must be a happens-before
 * of the plan's slot order + noted waits, and every stream slot must be joined into slot 0 at the
 * plan's end.  A cross-stream wait issued without alignn_plan_note_wait fails here (bad_from/bad_to =
 * the launches the plan leaves unordered; bad_to = -1 for an unjoined slot); edges = the kernel
 * dependencies checked. */
int alignn_plan_check_deps(const void* plan, void* graph, int64_t* bad_from, int64_t* bad_to, int64_t* edges);
/* A non-blocking HIP stream of the library's own at `priority` (an execution context's side / aux
 * streams: never one of torch's pooled streams, which may coincide with a capture or loader stream);
 * destroy synchronises it first. */
int alignn_stream_create(int32_t priority, void** out);
/* A stream on a hardware queue of its own (CU-masked stream, every CU enabled; normal priority): for
 * a batch-preparation (loader) stream that must not share in-order dispatch with the step's streams. */
int alignn_stream_create_dedicated(void** out);
int alignn_stream_destroy(void* stream);
int alignn_fill_f32(float* x, int64_t n, float value, void* stream);
int alignn_copy_f32(float* dst, const float* src, int64_t n, void* stream);
int alignn_add_f32(float* x, const float* y, int64_t n, void* stream);
int alignn_set_i64(int64_t* x, int64_t value, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ALIGNN_HIP_H */
