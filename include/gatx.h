/*
 * gatx — MI355X-native GATLayer hot path: C-ABI of libgatx.so.
 *
 * The reference (loodvn/gat-pytorch) is pure Python and has no FFI: its plugin point for this path
 * is the nn.Module `GATLayer` (`models/gat_layer.py:6-148`), picked by `LayerType`
 * (`run_config.py:4-6`) and constructed in `GATModel.__init__` (`models/GATModel.py:69-79`).
 * The Python mirror of that module (gat-pytorch_amd/gatx/layer.py) binds the entry points below
 * with ctypes; each one says which piece of the reference it replaces.
 *
 * Conventions
 *   - All pointers are DEVICE pointers unless stated; all launches go to `stream` (the caller's
 *     current HIP stream); nothing allocates, frees or synchronises, so every call is capturable
 *     into a hipGraph. Scratch memory comes from the caller (`*_workspace_bytes` says how much).
 *   - Node ids and edge positions are int32 (graphs up to 2^31-1 edges/nodes); features are fp32.
 *   - Return value: 0 on success, otherwise a hipError_t code (launch errors are checked after each
 *     launch) or GATX_EINVAL for unsupported shapes. gatx_last_error() gives a message.
 *   - Layout (per layer): NH heads, F features per head, Fp = round_up(F, 4),
 *     Dp = NH*Fp. Wh is [N][Dp] (head-major, each head padded to Fp so a float4 never straddles a
 *     head); S is [N][2*NH] = (s_src | s_dst) per node, the attention logit factors; the augmented
 *     projection weight W_aug is [Dp + 2*NH][F_in].
 */
#ifndef GATX_H
#define GATX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* gatx_stream_t; /* == hipStream_t */

#define GATX_EINVAL 1000
#define GATX_ARGMAX_CAP 1024 /* argmax (edge, head) slots recorded for the max() gradient */
#define GATX_META_WORDS 520  /* int64 words of a graph meta record (8 + 1024 int32 offsets) */

const char* gatx_last_error(void);
int gatx_version(void);
/* Profiling aid (not on the reference path): enqueue one empty dispatch of
 * gatx_region_mark_kernel with `tag` (1..2^20) one-wave workgroups, so the trace's grid size
 * carries the tag. bench.py brackets its timed steps with two of them (the first tagged with the
 * step count), so a rocprofv3 counter pass can select exactly those steps' dispatches by id. */
int gatx_region_mark(uint32_t tag, gatx_stream_t stream);

/* ---------------------------------------------------------------- graph (models/utils.py) */

/* Device-side sizing of the self-loop rewrite, no host sync (replaces the `int(index.max())` of
 * maybe_num_nodes, models/utils.py:70-72, and the `row != col` mask count of
 * add_remaining_self_loops, models/utils.py:58-60). edge_index (2, E): int64 if index_is_int64
 * else int32, rows `ld` elements apart. meta (device int64[GATX_META_WORDS]) = {E2, num_loops,
 * status, min id, max id, input self-loops, nb, chunk} with num_loops = max+1 when
 * add_self_loops, E2 = |edge_index'|, followed by the compaction's per-block offsets (int32, for
 * gatx_graph_build; only the first 8 words are meant for the host).
 * status 1 = a negative id, 2 = an id >= num_nodes: then E2 = num_loops = 0, so every later kernel
 * sees an empty graph (no out-of-bounds access) and the host raises when it reads meta (the
 * reference raises in index_select / scatter_add_). workspace: gatx_graph_meta_workspace_bytes(). */
size_t gatx_graph_meta_workspace_bytes(void);
int gatx_graph_meta(const void* edge_index, int index_is_int64, int64_t E, int64_t ld,
                    int add_self_loops, int64_t num_nodes, int64_t* meta, void* workspace,
                    gatx_stream_t stream);

/* Self-loop rewrite + destination CSR, one pass of device kernels, sized on the device from meta.
 * edge_index' = [edges with src != dst in input order | (i, i) for i < num_loops] when
 * add_self_loops (models/utils.py:47-67), else edge_index unchanged. The host allocates for
 * E_bound >= E (+ num_nodes with self-loops); slots past E2 are padding that sorts after every
 * real slot (col = rowidx = num_nodes there), and rowptr[num_nodes] = E2.
 * Outputs: edge_index_out (nullable) int64[2 * E_bound] holding edge_index' contiguously as
 * (2, E2): sources at [0, E2), destinations at [E2, 2*E2); and the CSR of edge_index' by
 * destination over num_nodes rows, stable in edge_index' order:
 *   rowptr [num_nodes+1], col [E_bound] = source id, rowidx [E_bound] = destination id,
 *   perm [E_bound] = position in edge_index' of each CSR slot.
 * Replaces the per-layer `add_remaining_self_loops` call (models/gat_layer.py:53-54) and the
 * scatter/gather index plumbing of sum_over_neighbourhood / explicit_broadcast. */
size_t gatx_graph_build_workspace_bytes(int64_t E, int64_t E_bound, int64_t num_nodes);
int gatx_graph_build(const void* edge_index, int index_is_int64, int64_t E, int64_t ld,
                     int add_self_loops, int64_t num_nodes, int64_t E_bound, const int64_t* meta,
                     int64_t* edge_index_out, int32_t* rowptr, int32_t* col, int32_t* rowidx,
                     int32_t* perm, void* workspace, size_t workspace_bytes,
                     gatx_stream_t stream);

/* Source-ordered transpose of the CSR built by gatx_graph_build (its padding slots hold
 * num_nodes, so they sort last): srowptr [num_nodes+1], scol [E_bound] = destination id,
 * seid [E_bound] = dst-CSR slot. e2 (= &meta[0]) is kept for the signature; the padding makes it
 * unnecessary. */
size_t gatx_graph_transpose_workspace_bytes(int64_t E_bound, int64_t num_nodes);
int gatx_graph_transpose(const int32_t* col, const int32_t* rowidx, int64_t num_nodes,
                         int64_t E_bound, const int64_t* e2, int32_t* srowptr, int32_t* scol,
                         int32_t* seid, void* workspace, size_t workspace_bytes,
                         gatx_stream_t stream);

/* ---------------------------------------------------------------- projection (gat_layer.py:64) */

/* W_aug [(Dp + 2*NH) x F_in] from W.weight [NH*F x F_in] and a.weight [NH x NH*2F]:
 * rows h*Fp+f = W[h*F+f] (pad rows 0); row Dp+h = (A_src W)[h]; row Dp+NH+h = (A_dst W)[h], where
 * A_src[h][k*F+f] = a[h][k*2F+f], A_dst[h][k*F+f] = a[h][k*2F+F+f] (the src/dst halves of the
 * (E, NH*2F) concatenation of gat_layer.py:76-82). a == NULL (const_attention): no extra rows. */
int gatx_prepare_weights(const float* W, const float* a, int NH, int F, int64_t F_in,
                         float* W_aug, gatx_stream_t stream);
/* Floats the W_aug buffer must hold: (Dp + 2NH) * F_in plus split-K scratch behind it. */
int64_t gatx_prepare_weights_floats(int NH, int F, int64_t F_in, int has_a);
/* gatx_prepare_weights with GATModel's Linear skip folded in (models/GATModel.py:107-110,
 * applied at :136-145 to the same layer input as W): skip_cols rows W_skip_eff follow the
 * Dp + 2NH rows, W_skip_eff[c][i] = mean_h W_skip[h*skip_cols + c][i] over skip_heads row blocks
 * (skip_heads = NH for a head-mean layer: mean_h(x W_h^T) == x (mean_h W_h)^T, :143-145; 1 for
 * concat: a copy, :140-141), written by the same launch. Buffer:
 * gatx_prepare_weights_skip_floats(). W_skip == NULL: gatx_prepare_weights. */
int gatx_prepare_weights_skip(const float* W, const float* a, int NH, int F, int64_t F_in,
                              const float* W_skip, int skip_heads, int64_t skip_cols,
                              float* W_aug, gatx_stream_t stream);
int64_t gatx_prepare_weights_skip_floats(int NH, int F, int64_t F_in, int has_a,
                                         int64_t skip_cols);

/* fp32 GEMM on MFMA (v_mfma_f32_32x32x2_f32): C = A * B (+ C if accumulate).
 * A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn]; one of sam/sak and one of sbk/sbn must
 * be 1. Output column n < n_split goes to C0[m*ldc0 + n], n >= n_split to C1[m*ldc1 + n-n_split].
 * Used for Wh|S = x * W_aug^T (gat_layer.py:64 + the per-edge `a` GEMV of :82 folded into per-node
 * scores), and for the backward's g_x = G_aug * W_aug and g_W_aug = G_aug^T * x. */
int gatx_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam, int64_t sak,
                  const float* B, int64_t sbk, int64_t sbn, float* C0, int64_t ldc0,
                  int64_t n_split, float* C1, int64_t ldc1, int accumulate, void* workspace,
                  size_t workspace_bytes, gatx_stream_t stream);
/* dst[c * ld_dst + r] = src[r * ld_src + c] for r < rows, c < cols (the backward's k-contiguous
 * copy of W_aug, so g_x = G_aug W_aug runs with both operands k-contiguous). */
int gatx_transpose_f32(int64_t rows, int64_t cols, const float* src, int64_t ld_src, float* dst,
                       int64_t ld_dst, gatx_stream_t stream);
/* Arithmetic of every gatx GEMM (process-wide; nothing is read from the environment; default 2):
 * 2 = "f16x3" (default): each fp32 operand split into an fp16 plane and a 2^11-scaled fp16
 *     residual plane, three products on v_mfma_f32_32x32x16_f16 with f32 accumulation — fp32
 *     GEMM accuracy at 2x fewer MFMA cycles than x3; k-contiguous operand pairs only, and a
 *     workgroup whose operand rows leave the fp16 range (row max |a| > 1023 or |b| > 2047, or a
 *     nonzero row max below 2^-13) recomputes its tile as x3; other layouts run x3;
 * 1 = "x3": each fp32 operand split exactly into three bf16 planes, the six partial products
 *     above fp32 resolution on v_mfma_f32_32x32x16_bf16 with f32 accumulation — fp32 GEMM
 *     accuracy at 2.7x fewer MFMA cycles than f32;
 * 0 = "f32": v_mfma_f32_32x32x2_f32. */
void gatx_set_gemm_mode(int mode);
int gatx_get_gemm_mode(void);
/* Pre-split weight planes for the f16x3 GEMMs (gemm_f16p.hip): W (rows x K, row stride ld) as two
 * fp16 planes per element with one power-of-two scale for the whole matrix, a 256-byte header
 * (the scale and per-256-row-tile range flags) and the build's scratch (row maxima; two launches,
 * no memset). Built once per weight version (the
 * projection's W_aug, the backward's W_aug^T) and passed to gatx_gemm_planes; the buffer
 * (gatx_weight_planes_bytes; 0 for a shape that cannot take planes: rows > 15360, the header's
 * tile flags) must be 256-byte aligned. Replaces nothing in the reference: it is
 * how `self.W(x)` (models/gat_layer.py:64) keeps fp32 accuracy on the fp16 matrix cores. */
size_t gatx_weight_planes_bytes(int64_t rows, int64_t K);
int gatx_weight_planes(const float* W, int64_t rows, int64_t K, int64_t ld, void* planes,
                       gatx_stream_t stream);
/* C = A . B^T for k-contiguous A (M x K, row stride lda) and B (N x K, row stride ldb) with B's
 * planes from gatx_weight_planes (NULL: the in-loop split kernel), into up to three column
 * ranges as gatx_projection_gemm3 (C0 below n_split, C1 below n_split2, C2 beyond), optionally
 * accumulating into C0. a != NULL: the forward projection with the node scores fused, exactly
 * gatx_projection_gemm_scores (then C0 is the packed Wh and the only output). gradient != 0:
 * A is a gradient (G_aug): its rows are scaled into the fp16 range (models/gat_layer.py:64's
 * backward, g_x = G_aug W_aug), by its exact max a_rowmax[row] when given (NULL: by its first
 * K-tile's). Shapes the pre-split kernel does not take (other arithmetic modes, unaligned rows,
 * small outputs) run the regular kernels with the same result. */
int gatx_gemm_planes(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                     const float* B, int64_t ldb, const void* b_planes, float* C0, int64_t ldc0,
                     int64_t n_split, float* C1, int64_t ldc1, int64_t n_split2, float* C2,
                     int64_t ldc2, int accumulate, const float* a, int NH, int F, float* S,
                     int gradient, const float* a_rowmax, void* workspace,
                     size_t workspace_bytes, gatx_stream_t stream);
/* The weight gradient C (M x N) = A^T-layout product for row-contiguous A (element (m, k) at
 * A[k * lda + m]) and B (element (n, k) at B[k * ldb + n]): g_W_aug = G_aug^T x with M = the
 * G_aug columns, K = the nodes (models/gat_layer.py:64's weight gradient). a_rowmax[m] = the
 * exact max |A row m| (gatx_absmax_rows_cols' colmax of G_aug): f16x3 arithmetic with those
 * rows scaled into the fp16 range (gemm_f16p.hip); split-K slabs in the workspace
 * (gatx_gemm_splitk_workspace_bytes), summed in a fixed order. Other arithmetic modes / shapes
 * run the x3 / f32 kernels with the same result. */
int gatx_gemm_wgrad(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                    const float* B, int64_t ldb, const float* a_rowmax, float* C, int64_t ldc,
                    void* workspace, size_t workspace_bytes, gatx_stream_t stream);
/* Exact max |x| of every row (rowmax[rows]) and, when colmax != NULL, every column
 * (colmax[cols], cols <= 2048; nan counts as inf) of X (rows x cols, row stride ld): the
 * per-row / per-column power-of-two scales of the f16x3 gradient GEMMs (G_aug's rows for
 * g_x = G_aug W_aug, its columns for g_W_aug = G_aug^T x), in one read of G_aug. */
int gatx_absmax_rows_cols(const float* X, int64_t rows, int64_t cols, int64_t ld, float* rowmax,
                          float* colmax, gatx_stream_t stream);
/* The arithmetic (2 f16x3, 1 x3, 0 f32) the tiled GEMMs run for an operand layout: a_kc / b_kc
 * = whether A's rows / B's columns are k-contiguous (the weight gradient G_aug^T x has neither:
 * f16x3 through gatx_gemm_wgrad with the column maxima; the host takes it unless gatx.tuning
 * f16p=0). */
int gatx_gemm_layout_mode(int a_kc, int b_kc);
/* Diagnostic (not on the reference path): enqueue a copy of the count of f16x3 GEMM workgroups
 * that tripped the range check and recomputed their tile as x3 (each costs ~1.5x its tile) into
 * dst (device uint64[1]); reset != 0 also zeroes the counter. Stream-ordered, capturable. */
int gatx_gemm_fallback_read(uint64_t* dst, int reset, gatx_stream_t stream);
/* Workspace that lets gatx_gemm_f32 / gatx_projection_gemm split the K range of the tiles in
 * their last, partially filled wave (0 = no split for this shape; NULL workspace = never split).
 * The slices are summed in a fixed order by a fix-up kernel, so results stay deterministic. */
size_t gatx_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K);
/* Split-K variant for reductions over many rows (g_W_aug = G_aug^T x, K = #nodes): slabs of
 * partial products in `workspace` (gatx_gemm_splitk_workspace_bytes; 0 = no split needed)
 * summed in a fixed order by a second kernel (deterministic). */
size_t gatx_gemm_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K);
int gatx_gemm_f32_splitk(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                         int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C,
                         int64_t ldc, int accumulate, void* workspace, size_t workspace_bytes,
                         gatx_stream_t stream);


/* Batched split-K: `batch` independent products (A, B, C offset by b*a_bs, b*b_bs, b*c_bs
 * floats), each summed over K in deterministic slabs (the reassociated first layer's per-head
 * weight gradient g_W_h = go_h^T Z_h, K = #nodes). */
size_t gatx_gemm_splitk_batched_workspace_bytes(int64_t batch, int64_t M, int64_t N, int64_t K);
int gatx_gemm_f32_splitk_batched(int64_t batch, int64_t M, int64_t N, int64_t K, const float* A,
                                 int64_t sam, int64_t sak, int64_t a_bs, const float* B,
                                 int64_t sbk, int64_t sbn, int64_t b_bs, float* C, int64_t ldc,
                                 int64_t c_bs, int accumulate, void* workspace,
                                 size_t workspace_bytes, gatx_stream_t stream);

/* gatx_gemm_f32 for the forward projection x . W_aug^T (accumulate = 0); a separate entry point
 * only so profiles can tell the projection launches from the auxiliary products. */
int gatx_projection_gemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                         int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C0,
                         int64_t ldc0, int64_t n_split, float* C1, int64_t ldc1,
                         void* workspace, size_t workspace_bytes, gatx_stream_t stream);
/* The projection with GATModel's Linear skip folded in (models/GATModel.py:107-110 applied at
 * :136-145; the skip reads the same layer input as W, gat_layer.py:64): B = [W_aug; W_skip_eff],
 * columns n < n_split -> C0 (Wh), n_split <= n < n_split2 -> C1 (S), n >= n_split2 -> C2[m*ldc2 +
 * n - n_split2] (the skip output, added by the edge pass epilogue). One launch instead of the
 * projection plus a separate skip GEMM. */
int gatx_projection_gemm3(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                          int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C0,
                          int64_t ldc0, int64_t n_split, float* C1, int64_t ldc1,
                          int64_t n_split2, float* C2, int64_t ldc2, void* workspace,
                          size_t workspace_bytes, gatx_stream_t stream);
/* The projection Wh = x . W^T (C0, packed [M][NH * round4(F)], ldc0 == N) with the per-node
 * logit factors S[m][0..2NH) = (Wh[m] . A_src^T | Wh[m] . A_dst^T) (gatx_node_scores' result,
 * models/gat_layer.py:76-82) reduced in the GEMM's epilogue from the accumulators: no second
 * read of Wh. `a` is the reference's attention vector [NH][2 * NH * F]. Per-column-tile partials
 * are summed in a fixed order (deterministic). Shapes without the fused epilogue (f32
 * arithmetic, small products, NH > 8) run the projection and then gatx_node_scores. Workspace:
 * gatx_projection_scores_workspace_bytes (the tail split's slices plus the partials). */
size_t gatx_projection_scores_workspace_bytes(int64_t M, int64_t N, int64_t K, int NH);
int gatx_projection_gemm_scores(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                                int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C0,
                                int64_t ldc0, const float* a, int NH, int F, float* S,
                                void* workspace, size_t workspace_bytes, gatx_stream_t stream);
/* Its gradient: g_W_skip[h*cols + c][i] = g_eff[c][i] / heads for every head block h. */
int gatx_skip_weight_grad(const float* g_eff, int heads, int64_t cols, int64_t F_in, float* g_W,
                          gatx_stream_t stream);

/* The same for `batch` independent products (batch b offsets A, B, C by b*a_bs, b*b_bs,
 * b*c_bs floats) with a fused epilogue C = elu?(A*B (+C) + bias[b*bias_bs + n] +
 * resid[b*resid_bs + m*resid_ld + n]) (bias / resid nullable): the per-head output projection
 * of the reassociated first layer, with GATModel's skip-add + ELU folded in. */
int gatx_gemm_f32_batched(int64_t batch, int64_t M, int64_t N, int64_t K, const float* A,
                          int64_t sam, int64_t sak, int64_t a_bs, const float* B, int64_t sbk,
                          int64_t sbn, int64_t b_bs, float* C, int64_t ldc, int64_t c_bs,
                          int accumulate, const float* bias, int64_t bias_bs, const float* resid,
                          int64_t resid_ld, int64_t resid_bs, int elu, gatx_stream_t stream);

/* Hub plan for the edge pass (SURVEY §7 "degree skew"): destination segments of more than
 * hub_edges edges are cut into ceil(deg / hub_edges) pieces listed in hubs [hub_bound][4] =
 * (node, piece, pieces, first slot); *hub_count (device) = the number of entries. hub_bound =
 * gatx_graph_hub_bound(E_bound, hub_edges) always suffices. No host sync. */
int64_t gatx_graph_hub_bound(int64_t E_bound, int hub_edges);
int gatx_graph_hub_plan(const int32_t* rowptr, int64_t num_nodes, int hub_edges, int32_t* hubs,
                        int64_t hub_bound, int32_t* hub_count, gatx_stream_t stream);

/* Node blocks (round 5): cut [0, N) into contiguous blocks [segs[k], segs[k+1]), k <
 * *seg_count, that no edge crosses (an edge s -> d covers the boundaries in (min, max]), each at
 * most max_rows nodes, packing the gap-free runs greedily — the graphs of a PyG-style batch
 * (models/GATModel.py's data.x / data.edge_index of a collated batch), found from the CSR alone.
 * *seg_count = -1 (device) when a gap-free run exceeds max_rows, there are more than
 * gatx_graph_segments_max() runs, or N > 2^17. segs: gatx_graph_segments_max() + 2 entries. Two
 * launches, no host sync. Replaces nothing in the reference (it never batches beyond PyG's
 * disjoint union); the LDS-staged edge passes stage one block per workgroup. */
size_t gatx_graph_segments_workspace_bytes(int64_t num_nodes);
int gatx_graph_segments(const int32_t* rowptr, const int32_t* col, int64_t num_nodes,
                        int max_rows, int32_t* segs, int32_t* seg_count, void* workspace,
                        size_t workspace_bytes, gatx_stream_t stream);
int gatx_graph_segments_max(void);

/* ---------------------------------------------------------------- attention + aggregation */

/* Global max M = max_{e,h} s_src[col[e],h] + s_dst[rowidx[e],h]  (gat_layer.py:85), written as an
 * order-preserving uint32 into *M_ord (device). Edge-count convention of every edge-parallel
 * entry point: E2 is the host bound (grid size, strides); e2 (nullable) is the device count
 * (&meta[0] of gatx_graph_meta), and min(E2, *e2) edges are processed. argmax (nullable): its
 * tie counter argmax[0] is reset to 0 for the following gatx_attention_alpha*. workspace:
 * gatx_attention_max_workspace_bytes(). */
size_t gatx_attention_max_workspace_bytes(void);
int gatx_attention_max(const int32_t* col, const int32_t* rowidx, int64_t E2, const int64_t* e2,
                       const float* S, int NH, uint32_t* M_ord, int64_t* argmax,
                       void* workspace, gatx_stream_t stream);

/* Fused edge pass per destination segment (gat_layer.py:85-135), then the attention output:
 *   ex = exp(0.01 * (s_src[src] + s_dst[dst] - M))   (LeakyReLU(0.01) of a non-positive value)
 *   den[n,h] = sum_{e->n} ex;  alpha = ex / (den[dst] + 1e-8)   (no per-segment max: :96-109)
 *   out[n,h,:] = sum_{e->n} alpha~ * Wh[src,h,:]   (alpha~ = dropout(alpha), :113-127)
 *   concat: out [N][NH*F]; else out [N][F] = head mean (:129-132); + bias (:134-135, nullable).
 * alpha is written in edge_index' order ([E2][NH], via perm); den [N][NH] is kept for the
 * backward; argmax = int64[GATX_ARGMAX_CAP + 2]: count, then (csr_slot*NH + h) of raw == M
 * entries, then one scratch slot for gatx_max_backward (zeroed by the caller).
 * const_attention: ex = 1 (S, M, argmax unused). dropout_p > 0 applies the counter-based keep
 * mask dropout_keep(*seed, e', h) (gatx_common.h); seed is a DEVICE uint64 (drawn from torch's
 * generator, so a captured graph draws a fresh one per replay; unused when dropout_p == 0).
 * = gatx_edge_forward_ex + gatx_attention_alpha (E2 exact here). */
int gatx_edge_forward(const float* Wh, const float* S, const uint32_t* M_ord,
                      const int32_t* rowptr, const int32_t* col, const int32_t* rowidx,
                      const int32_t* perm, int64_t num_nodes, int64_t E2, int NH, int F,
                      int concat, int const_attention, const float* bias, float dropout_p,
                      const uint64_t* seed, float* out, float* alpha, float* den, int64_t* argmax,
                      gatx_stream_t stream);

/* The aggregation half, generalised. Source rows are read at rows + src*row_stride +
 * h*head_stride (+ f): row_stride = Dp, head_stride = Fp for Wh; for the reassociated first
 * layer rows = x padded to Fp = round_up(F_in, 4) with head_stride = 0, so the pass aggregates
 * Z[n,h,:] = sum alpha~ x[src,:] (F = that Fp). One work item is (node, group of heads_per_item
 * heads) (<= 0: all heads; at most 8); items are swept in chunks of `chunk` nodes per head group
 * (<= 0: 2048) so one XCD's L2 holds one head group's slice of the rows. A launch covers head
 * groups [group_begin, group_begin + group_count) (group_count <= 0: all).
 * Head mean (concat 0): mean_mode 0 = all heads in one item (heads_per_item = NH); otherwise one
 * head group per launch, launched in order over the groups: 1 = first (out = the group's head
 * sum), 2 = middle (out += it), 3 = last (out = epilogue((out + it) / NH + bias)) — NH > 8, or
 * smaller groups whose row slices stay L2-resident; each pass is deterministic, in stream order.
 * out rows are out_ld floats apart; fused epilogue out = elu?(agg + bias + resid) with resid
 * [N][resid_ld] (nullable) and elu in {0, 1} (GATModel's skip-add + ELU). Writes den. */
int gatx_edge_forward_ex(const float* rows, int64_t row_stride, int64_t head_stride,
                         const float* S, const uint32_t* M_ord, const int32_t* rowptr,
                         const int32_t* col, const int32_t* perm, int64_t num_nodes, int NH,
                         int F, int heads_per_item, int group_begin, int group_count,
                         int mean_mode, int concat, int const_attention,
                         const float* bias, float dropout_p, const uint64_t* seed, float* out,
                         int64_t out_ld, const float* resid, int64_t resid_ld, int elu,
                         float* den, int64_t chunk, gatx_stream_t stream);
/* gatx_edge_forward_ex with hub splitting: segments longer than hub_edges (a plan from
 * gatx_graph_hub_plan over the same rowptr) are aggregated as pieces by their own waves into
 * hub_part (gatx_edge_forward_hub_part_bytes), then summed in piece order and finished by a
 * second kernel — a hub costs ceil(deg / hub_edges) waves in parallel instead of one wave walking
 * every edge. hub_edges = 0: no splitting (exactly gatx_edge_forward_ex). */
size_t gatx_edge_forward_hub_part_bytes(int64_t hub_bound, int num_heads, int out_features,
                                        int heads_per_item, int group_count);
int gatx_edge_forward_hubs(const float* rows, int64_t row_stride, int64_t head_stride,
                           const float* S, const uint32_t* M_ord, const int32_t* rowptr,
                           const int32_t* col, const int32_t* perm, int64_t num_nodes,
                           int num_heads, int out_features, int heads_per_item, int group_begin,
                           int group_count, int mean_mode, int concat, int const_attention,
                           const float* bias, float dropout_p, const uint64_t* seed, float* out,
                           int64_t out_ld, const float* resid, int64_t resid_ld, int elu,
                           float* den, int64_t chunk, int hub_edges, const int32_t* hubs,
                           const int32_t* hub_count, int64_t hub_bound, float* hub_part,
                           gatx_stream_t stream);
/* gatx_edge_forward_hubs with the NEXT layer's input dropout (models/GATModel.py:130, applied
 * to this layer's output) fused after the ELU: out = keep(out_seed, n*OC + c) ? v/(1-out_p) : 0
 * (OC = output width; the mask of gatx_dropout). For the last head-mean pass only. */
int gatx_edge_forward_drop(const float* rows, int64_t row_stride, int64_t head_stride,
                           const float* S, const uint32_t* M_ord, const int32_t* rowptr,
                           const int32_t* col, const int32_t* perm, int64_t num_nodes,
                           int num_heads, int out_features, int heads_per_item, int group_begin,
                           int group_count, int mean_mode, int concat, int const_attention,
                           const float* bias, float dropout_p, const uint64_t* seed, float* out,
                           int64_t out_ld, const float* resid, int64_t resid_ld, int elu,
                           float* den, int64_t chunk, int hub_edges, const int32_t* hubs,
                           const int32_t* hub_count, int64_t hub_bound, float* hub_part,
                           float out_p, const uint64_t* out_seed, gatx_stream_t stream);
/* gatx_edge_forward_drop that leaves out the destinations with skip[n] != 0 (no output, no den:
 * for a caller that serves them another way). skip = NULL: every destination. */
int gatx_edge_forward_skip(const float* rows, int64_t row_stride, int64_t head_stride,
                           const float* S, const uint32_t* M_ord, const int32_t* rowptr,
                           const int32_t* col, const int32_t* perm, int64_t num_nodes,
                           int num_heads, int out_features, int heads_per_item, int group_begin,
                           int group_count, int mean_mode, int concat, int const_attention,
                           const float* bias, float dropout_p, const uint64_t* seed, float* out,
                           int64_t out_ld, const float* resid, int64_t resid_ld, int elu,
                           float* den, int64_t chunk, int hub_edges, const int32_t* hubs,
                           const int32_t* hub_count, int64_t hub_bound, float* hub_part,
                           float out_p, const uint64_t* out_seed, const uint8_t* skip,
                           gatx_stream_t stream);
/* GATModel's input dropout (models/GATModel.py:130, F.dropout) as a counter-based mask on the
 * element index (the attention dropout's splitmix64 hash): y[i] = keep(seed, i) ? x[i]/(1-p) : 0.
 * The gradient is the same call on g_y. In place (y == x) is allowed. */
int gatx_dropout(const float* x, int64_t n, float p, const uint64_t* seed, float* y,
                 gatx_stream_t stream);

/* alpha [E2][NH] in edge_index' order from S, M and den (one thread per CSR slot, all heads of
 * an edge stored together), plus the argmax records (see gatx_edge_forward). */
int gatx_attention_alpha(const int32_t* col, const int32_t* rowidx, const int32_t* perm,
                         int64_t E2, const float* S, const uint32_t* M_ord, const float* den,
                         int NH, int const_attention, float* alpha, int64_t* argmax,
                         gatx_stream_t stream);
/* gatx_attention_alpha iterating edge_index' itself (int64 or int32, row stride ld; ld < 0:
 * the flat (2, E2) layout of gatx_graph_build, ld = the device count): reads each edge's
 * (src, dst) and writes alpha[p] in order (coalesced both ways); rowptr / perm (the CSR) are only
 * read to record a tied argmax by CSR slot, as gatx_attention_alpha does. E2 / e2: the bound and
 * the device count (see gatx_attention_max). */
int gatx_attention_alpha_ei(const void* edge_index, int index_is_int64, int64_t ld, int64_t E2,
                            const int64_t* e2, const float* S, const uint32_t* M_ord,
                            const float* den, int NH, int const_att, const int32_t* rowptr,
                            const int32_t* perm, float* alpha, int64_t* argmax,
                            gatx_stream_t stream);

/* S [N][2NH] = (Wh . A_src^T | Wh . A_dst^T) from Wh [N][Dp] and a.weight — the reference's own
 * association of the logit GEMV (gat_layer.py:76-82), used when folding the scores into the
 * projection GEMM would cost a whole extra column tile. */
int gatx_node_scores(const float* Wh, int64_t num_nodes, int NH, int F, const float* a, float* S,
                     gatx_stream_t stream);

/* Diagnostic ablations of the edge pass for profiling only (results are WRONG when set):
 * bit 1 skip exp (ex = 1). */
void gatx_set_debug(int flags);

/* Copy an [rows x cols] matrix (row stride ld_src) into [rows x ld_dst], zero-filling columns
 * cols..ld_dst-1 (float4-aligned source rows for the gathers). */
int gatx_pad_rows(const float* src, int64_t rows, int64_t cols, int64_t ld_src, float* dst,
                  int64_t ld_dst, gatx_stream_t stream);

/* LDS-staged edge forward (round 5; csrc/edge_lds.hip) for graphs cut into node blocks by
 * gatx_graph_segments(max_rows = gatx_edge_lds_rows()). Two passes replace gatx_edge_forward_*
 * + gatx_attention_alpha_ei on such graphs (models/gat_layer.py:84-135):
 * gatx_edge_records — one wave per destination, all heads: den (bitwise the L2-gather pass's),
 *   alpha in edge_index' order (nullable), max()'s tied argmax entries (nullable; counter reset by
 *   gatx_attention_max), and per (head, CSR slot) an 8-byte record {64 * src, alpha~} in rec
 *   ([NH][E_bound] x 8 B; alpha~ = alpha after the attention dropout). NH <= 8.
 * gatx_edge_lds_forward — concat layers: one workgroup per (node block, head, 16-float chunk)
 *   stages that chunk of every row of its block in LDS and sums alpha~ x row over each
 *   destination's segment, then bias / resid / ELU / the next layer's input dropout as
 *   gatx_edge_forward_drop. rows: Wh with row_stride >= NH * round4(F) floats, 16-byte aligned.
 *   seg_bound: the grid's block bound (>= *seg_count; blocks past the count exit). When the
 *   device count is -1 or exceeds seg_bound (a captured step replayed on edges that no longer cut
 *   into those blocks), the workgroups split the num_nodes rows evenly and gather from global
 *   memory instead: slower, same result. */
int gatx_edge_lds_rows(void);
int gatx_edge_records(const float* S, const uint32_t* M_ord, const int32_t* rowptr,
                      const int32_t* col, const int32_t* perm, int64_t num_nodes,
                      int64_t E_bound, int num_heads, int const_attention, float dropout_p,
                      const uint64_t* seed, void* rec, float* den, float* alpha,
                      long long* argmax, gatx_stream_t stream);
int gatx_edge_lds_forward(const float* rows, int64_t row_stride, const int32_t* rowptr,
                          int64_t num_nodes, const void* rec, int64_t E_bound, const int32_t* segs,
                          const int32_t* seg_count, int64_t seg_bound, int num_heads,
                          int out_features, const float* bias, float* out, int64_t out_ld,
                          const float* resid, int64_t resid_ld, int elu, float out_p,
                          const uint64_t* out_seed, gatx_stream_t stream);
/* gatx_edge_records_src (round 6) — the records of the backward's source pass on the LDS walk
 *   (the autograd of models/gat_layer.py:117-127 w.r.t. Wh is the forward aggregation on the
 *   transposed CSR with go's rows): one wave per source s, per (head, transposed slot j) the
 *   record {64 * scol[j], alpha~} in rec ([NH][E_bound] x 8 B; alpha~ recomputed from S, den,
 *   M_ord and the dropout mask exactly as gatx_edge_backward_src does), and g_s_src[s, h] = the
 *   sum of g_raw ([NH][E_bound], per CSR slot; nullable) over s's out-edges into
 *   G_aug[s * ldg + Dp + h] (skipped with const_attention). Then gatx_edge_lds_forward(rows = go
 *   with row stride NH * F, rowptr = srowptr, rec, ..., out = G_aug, out_ld = ldg, no bias / resid /
 *   ELU / dropout) writes G_aug[s, 0 : NH * F) — concat layers with F % 4 == 0, N < 2^25. */
int gatx_edge_records_src(const float* S, const uint32_t* M_ord, const float* den,
                          const int32_t* srowptr, const int32_t* scol, const int32_t* seid,
                          const int32_t* perm, int64_t num_nodes, int64_t E_bound, int num_heads,
                          int const_attention, float dropout_p, const uint64_t* seed,
                          const float* g_raw, float* G_aug, int64_t ldg, int64_t Dp, void* rec,
                          gatx_stream_t stream);
/* gatx_edge_lds_mean_forward (round 6) — head-mean layers (concat = False, models/gat_layer.py
 *   :128-135: out = mean over heads, then bias): one workgroup per (node block, 16-float chunk,
 *   destination range of <= 768 nodes) stages every head's chunk in turn and adds each head's
 *   alpha~-weighted rows into the same registers, so the mean needs no partials in memory; then
 *   bias / resid / ELU. Same arguments, records (from gatx_edge_records), fallback and limits
 *   as gatx_edge_lds_forward, and 8 * num_heads * E_bound < 2^32; out_p must be 0 (a head-mean
 *   layer that feeds the next layer's input dropout takes gatx_edge_forward_drop). */
int gatx_edge_lds_mean_forward(const float* rows, int64_t row_stride, const int32_t* rowptr,
                               int64_t num_nodes, const void* rec, int64_t E_bound,
                               const int32_t* segs, const int32_t* seg_count, int64_t seg_bound,
                               int num_heads, int out_features, const float* bias, float* out,
                               int64_t out_ld, const float* resid, int64_t resid_ld, int elu,
                               float out_p, const uint64_t* out_seed, gatx_stream_t stream);

/* ---------------------------------------------------------------- backward (autograd of above) */

/* go [N][NH*Fp] (concat) or [N][Fp] (head mean, scaled by 1/NH): the upstream gradient, gated by
 * elu'(out) when the layer's epilogue applied ELU (out = the saved post-ELU output), zero-padded
 * per head. g_pre (nullable) receives the unpadded elu-gated gradient (the residual's gradient). */
int gatx_prepare_go(const float* g_out, const float* out, int64_t num_nodes, int NH, int F,
                    int concat, int elu, float* go, float* g_pre, gatx_stream_t stream);
/* The same with g_pre rows pre_ld floats apart (>= the output width): the folded skip's
 * gradient written straight into its columns of G_aug (gatx_prepare_weights_skip); out_p /
 * out_seed: the layer's output carries the next layer's fused input dropout
 * (gatx_edge_forward_drop): g_out goes through the mask, ELU's derivative from out * (1-p). */
int gatx_prepare_go_ex(const float* g_out, const float* out, int64_t num_nodes, int NH, int F,
                       int concat, int elu, float* go, float* g_pre, int64_t pre_ld,
                       float out_p, const uint64_t* out_seed, gatx_stream_t stream);

/* Destination pass, one wave per (node n, head h):
 *   g_alpha~[e,h] = <go[n,h,:], Wh[src,h,:]>; g_alpha = g_alpha~ * keep/(1-p) + g_alpha_ret
 *   c[n,h] = sum_{e->n} g_alpha * alpha; g_raw'[e,h] = 0.01 * ex * (g_alpha - c) / (den + 1e-8)
 * Writes g_raw' head-major [NH][E2] in CSR order (E2 = the row stride: the host bound) and g_s_dst = sum_e g_raw' into
 * G_aug[n][Dp+NH+h] and gsd [N][NH]. g_alpha_ret (the returned alpha's gradient, edge_index'
 * order) may be NULL. */
int gatx_edge_backward_dst(const float* Wh, const float* S, const uint32_t* M_ord,
                           const float* den, const int32_t* rowptr, const int32_t* col,
                           const int32_t* perm, int64_t num_nodes, int64_t E2, int NH, int F,
                           int concat, float dropout_p, const uint64_t* seed, const float* go,
                           const float* g_alpha_ret, float* g_raw, float* gsd, float* G_aug,
                           int64_t ldg, gatx_stream_t stream);
/* The dst pass over arbitrary gathered rows: g_alpha[e,h] = <go[n, h], rows[src_e] + h *
 * head_stride> over F floats (row_stride / head_stride / go_stride / go_head in floats, all
 * multiples of 4), g_s_dst into G[n][gs_off + NH + h]. With rows = the padded layer input x
 * (head_stride 0) and go = g_Z = go . W_h per head this is the reassociated first layer's
 * backward (<go_h, W_h x_src> == <go_h W_h, x_src>). */
int gatx_edge_backward_dst_ex(const float* rows, int64_t row_stride, int64_t head_stride,
                              const float* S, const uint32_t* M_ord, const float* den,
                              const int32_t* rowptr, const int32_t* col, const int32_t* perm,
                              int64_t num_nodes, int64_t E2, int NH, int F, const float* go,
                              int64_t go_stride, int64_t go_head, float p, const uint64_t* seed,
                              const float* g_alpha_ret, float* g_raw, float* gsd, float* G,
                              int64_t ldg, int64_t gs_off, gatx_stream_t stream);
/* gatx_edge_backward_dst_ex with hub splitting (SURVEY §7 "degree skew"; the backward of the
 * reference's scatter_add_, models/utils.py:17-20 via gat_layer.py:99-127, has no per-degree
 * cliff): destination segments longer than hub_edges (a plan from gatx_graph_hub_plan over the
 * same rowptr) are walked as pieces by parallel waves; the softmax-backward constant c and
 * g_s_dst are combined from per-piece partials in piece order (deterministic) by two follow-up
 * kernels. hub_part: gatx_edge_backward_hub_part_bytes(hub_bound, NH, F, 0). hub_edges = 0: no
 * splitting (exactly gatx_edge_backward_dst_ex). */
size_t gatx_edge_backward_hub_part_bytes(int64_t hub_bound, int num_heads, int out_features,
                                         int src_pass);
int gatx_edge_backward_dst_hubs(const float* rows, int64_t row_stride, int64_t head_stride,
                                const float* S, const uint32_t* M_ord, const float* den,
                                const int32_t* rowptr, const int32_t* col, const int32_t* perm,
                                int64_t num_nodes, int64_t E2, int NH, int F, const float* go,
                                int64_t go_stride, int64_t go_head, float p, const uint64_t* seed,
                                const float* g_alpha_ret, float* g_raw, float* gsd, float* G,
                                int64_t ldg, int64_t gs_off, int hub_edges, const int32_t* hubs,
                                const int32_t* hub_count, int64_t hub_bound, float* hub_part,
                                gatx_stream_t stream);
/* Source-side logit gradients only: G[s][gs_off + h] = sum over s's out-edges (src-CSR) of
 * g_raw'[h][e] + g_corr[s][h] (NULL allowed). No message gradient. NH <= 8. */
int gatx_edge_backward_src_scores(const int32_t* srowptr, const int32_t* seid, int64_t num_nodes,
                                  int64_t E2, int NH, const float* g_raw, const float* g_corr,
                                  float* G, int64_t ldg, int64_t gs_off, gatx_stream_t stream);

/* max() backward (torch splits the gradient evenly over ties): g_M = -sum gsd (two-stage
 * fixed-order reduction); g_M/k is added to G_aug[dst][Dp+NH+h] and to the source side for
 * each recorded argmax entry: into g_corr_src[src,h] ([N][NH], zeroed by the caller, consumed
 * by the src pass) or, with g_corr_src NULL, straight into G_aug[src][Dp+h] (call it after the
 * src pass). Falls back to a full scan of the edges (E2 bound / e2 device count, see
 * gatx_attention_max) when more than GATX_ARGMAX_CAP entries tie. */
size_t gatx_max_backward_workspace_bytes(void);
int gatx_max_backward(const int64_t* argmax, const float* gsd, const float* S,
                      const uint32_t* M_ord, const int32_t* col, const int32_t* rowidx,
                      int64_t num_nodes, int64_t E2, const int64_t* e2, int NH,
                      float* g_corr_src, float* G_aug, int64_t ldg, int64_t Dp, void* workspace,
                      gatx_stream_t stream);

/* Source pass, one wave per (node s, head h): G_aug[s][h*Fp:] = sum_{e: src=s} alpha~[e,h] *
 * go[dst_e,h,:] (the message gradient), G_aug[s][Dp+h] = sum_{e: src=s} g_raw'[e,h] +
 * g_corr_src[s,h] (g_s_src, g_corr_src nullable; skipped for const_attention). */
int gatx_edge_backward_src(const float* S, const uint32_t* M_ord, const float* den,
                           const int32_t* srowptr, const int32_t* scol, const int32_t* seid,
                           const int32_t* perm, int64_t num_nodes, int64_t E2, int NH, int F,
                           int concat, int const_attention, float dropout_p, const uint64_t* seed,
                           const float* go, const float* g_raw, const float* g_corr_src,
                           float* G_aug, int64_t ldg, gatx_stream_t stream);

/* gatx_edge_backward_src with hub splitting: source segments (srowptr) longer than hub_edges
 * (a gatx_graph_hub_plan over srowptr) are accumulated as pieces by parallel waves into partial
 * rows, summed in piece order by a combine kernel (deterministic). hub_part:
 * gatx_edge_backward_hub_part_bytes(hub_bound, NH, F, 1). hub_edges = 0: no splitting. */
int gatx_edge_backward_src_hubs(const float* S, const uint32_t* M_ord, const float* den,
                                const int32_t* srowptr, const int32_t* scol, const int32_t* seid,
                                const int32_t* perm, int64_t num_nodes, int64_t E2, int NH, int F,
                                int concat, int const_attention, float dropout_p,
                                const uint64_t* seed, const float* go, const float* g_raw,
                                const float* g_corr_src, float* G_aug, int64_t ldg, int hub_edges,
                                const int32_t* hubs, const int32_t* hub_count, int64_t hub_bound,
                                float* hub_part, gatx_stream_t stream);

/* From g_W_aug [(Dp+2NH) x F_in] (= G_aug^T x): g_W [NH*F x F_in] and g_a [NH x NH*2F]
 * (a may be NULL for const_attention; then g_a is untouched). */
int gatx_weight_grads(const float* gW_aug, const float* W, const float* a, int NH, int F,
                      int64_t F_in, float* g_W, float* g_a, gatx_stream_t stream);

/* Column sums: out[j] = sum_i X[i*ld + j], j < ncols (bias gradient). */
int gatx_colsum(const float* X, int64_t nrows, int64_t ncols, int64_t ld, float* out,
                gatx_stream_t stream);

/* ---- attention-norm regulariser (models/GATModel.py:189-234, calc_attention_norm) ---- */
/* out[0] = (accumulate ? out[0] : 0) + scale * sum_{e,h} |alpha[e,h] * deg[dst_e] - 1| over one
 * layer's alpha (E2 x NH, edge_index' order); dst = edge_index'[1] (E2 entries, int64 when
 * dst_is64 else int32), deg from the dst-CSR rowptr. scale = 1 / (E2 * num_layers) gives the
 * reference's mean. workspace: gatx_attention_norm_workspace_bytes(). Replaces
 * GATModel.py:195-230. */
size_t gatx_attention_norm_workspace_bytes(void);
int gatx_attention_norm(const float* alpha, int64_t E2, int NH, const void* dst, int dst_is64,
                        const int32_t* rowptr, float scale, int accumulate, float* out,
                        void* workspace, gatx_stream_t stream);
/* All layers in one pass (round 6): alphas[l] (E2 x num_heads[l], l < num_layers <= 8; a host
 * array of device pointers, read at launch) -> out[0] = the per-layer sums in layer order, each
 * times scale — bitwise what num_layers gatx_attention_norm calls (accumulate = l > 0) give.
 * workspace: gatx_attention_norm_multi_workspace_bytes(num_layers). */
size_t gatx_attention_norm_multi_workspace_bytes(int num_layers);
int gatx_attention_norm_multi(const float* const* alphas, const int* num_heads, int num_layers,
                              int64_t E2, const void* dst, int dst_is64, const int32_t* rowptr,
                              float scale, float* out, void* workspace, gatx_stream_t stream);
/* g_alpha[e,h] = g[0] * scale * sign(alpha[e,h] * deg - 1) * deg (g: device scalar). */
int gatx_attention_norm_backward(const float* alpha, int64_t E2, int NH, const void* dst,
                                 int dst_is64, const int32_t* rowptr, const float* g,
                                 float scale, float* g_alpha, gatx_stream_t stream);

/* ---- the task modules' loss (models/ppi_gat.py:11,19; models/pattern_gat.py:11-15) ---- */
/* BCEWithLogitsLoss, mean reduction, pos_weight (1 = none): loss[0] = mean over n of
 * (1 - y) x + lw softplus(-x), lw = 1 + (pos_weight - 1) y; grad[i] = d loss / d x[i] =
 * (lw sigmoid(x) - pos_weight y) / n, written by the same pass for the backward. One launch for
 * n <= 65536, two above (workspace: gatx_bce_logits_workspace_bytes()). Fixed-order sums. */
size_t gatx_bce_logits_workspace_bytes(void);
int gatx_bce_logits(const float* x, const float* y, int64_t n, float pos_weight, float* loss,
                    float* grad, void* workspace, gatx_stream_t stream);
/* out[i] = g[0] * v[i] (g a device scalar: the loss's upstream gradient). */
int gatx_scale_by_scalar(const float* g, const float* v, int64_t n, float* out,
                         gatx_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GATX_H */
