// Forward of the GATLayer attention + aggregation (models/gat_layer.py:74-135) as two HIP
// kernels over the destination-sorted CSR:
//
//  attention_max : M = max over all (edge, head) of s_src[src] + s_dst[dst]   (:85, a grid-wide
//                  dependency: the reference subtracts ONE global max, not a per-segment one)
//  edge_forward  : one wavefront per destination segment. Each edge's projected source row
//                  Wh[src] (padded [NH][Fp]) is streamed once as float4 chunks, weighted by
//                  ex = exp(0.01 (s_src[src] + s_dst[n] - M)) per head and summed in registers,
//                  alongside den = sum ex. The normalisation 1/(den + 1e-8) is applied once per
//                  segment (sum(ex/(den+eps) * v) == sum(ex * v)/(den+eps)), then concat / head
//                  mean / bias, then alpha is written in edge_index' order. No (E, NH, F) tensor
//                  is ever materialised (the reference builds four of them, :70-71, :76, :119).
//
// Also: gatx_prepare_weights (the augmented projection weight, folding `a` into per-node scores).
#include "gatx_common.h"

namespace gatx {
namespace {

// ------------------------------------------------------------------ global max pre-pass
// Two launches: per-block maxima into a partials array (no single-address atomic contention:
// thousands of workgroups hitting one word serialise at the memory side), then one block folds
// them. max is order-independent, so the result is exact and deterministic.
constexpr int kMaxBlocks = 2048;

__global__ void __launch_bounds__(256) attention_max_kernel(const int32_t* __restrict__ col,
                                                            const int32_t* __restrict__ rowidx,
                                                            int64_t E2b, const long long* e2p,
                                                            const float* __restrict__ S, int NH,
                                                            float* __restrict__ part) {
  const int S2 = 2 * NH;
  const int64_t E2 = e2p ? min(E2b, (int64_t)*e2p) : E2b;
  float m = -INFINITY;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E2;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float* ss = S + (int64_t)col[e] * S2;
    const float* sd = S + (int64_t)rowidx[e] * S2 + NH;
    for (int h = 0; h < NH; ++h) m = fmaxf(m, ss[h] + sd[h]);
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    part[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// The same with the head count known: each thread takes 2 edges per round with every index and
// score load of the round issued before any max (the plain loop keeps one edge's dependent
// col -> S chain in flight per thread), score rows as float4 / float2 loads. (Round 6: 2 edges
// per round ran 0.5-0.8 us faster per PPI launch than 4, and 8 was 2-6 us slower: the pass is
// bound by the L2 request rate, and fewer registers keep more waves resident.)
template <int NHC>
__global__ void __launch_bounds__(256) attention_max_vec_kernel(const int32_t* __restrict__ col,
                                                                const int32_t* __restrict__ rowidx,
                                                                int64_t E2b, const long long* e2p,
                                                                const float* __restrict__ S,
                                                                float* __restrict__ part) {
  constexpr int S2 = 2 * NHC, UE = 2;
  const int64_t E2 = e2p ? min(E2b, (int64_t)*e2p) : E2b;
  constexpr int VEC = (NHC % 4 == 0) ? 4 : ((NHC % 2 == 0) ? 2 : 1);
  float m = -INFINITY;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e0 < E2; e0 += UE * stride) {
    int64_t sv[UE], dv[UE];
#pragma unroll
    for (int u = 0; u < UE; ++u) {
      const int64_t e = min(e0 + u * stride, E2 - 1);   // clamped: a repeat cannot raise the max
      sv[u] = col[e];
      dv[u] = rowidx[e];
    }
    float a[UE][NHC], b[UE][NHC];
#pragma unroll
    for (int u = 0; u < UE; ++u)
#pragma unroll
      for (int h = 0; h < NHC; h += VEC) {
        const float* ps = S + sv[u] * S2 + h;
        const float* pd = S + dv[u] * S2 + NHC + h;
        if constexpr (VEC == 4) {
          const float4 x = *(const float4*)ps, y = *(const float4*)pd;
          a[u][h] = x.x; a[u][h + 1] = x.y; a[u][h + 2] = x.z; a[u][h + 3] = x.w;
          b[u][h] = y.x; b[u][h + 1] = y.y; b[u][h + 2] = y.z; b[u][h + 3] = y.w;
        } else if constexpr (VEC == 2) {
          const float2 x = *(const float2*)ps, y = *(const float2*)pd;
          a[u][h] = x.x; a[u][h + 1] = x.y; b[u][h] = y.x; b[u][h + 1] = y.y;
        } else {
          a[u][h] = *ps; b[u][h] = *pd;
        }
      }
#pragma unroll
    for (int u = 0; u < UE; ++u)
#pragma unroll
      for (int h = 0; h < NHC; ++h) m = fmaxf(m, a[u][h] + b[u][h]);
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    part[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__global__ void __launch_bounds__(256) max_final_kernel(const float* __restrict__ part, int nb,
                                                        uint32_t* __restrict__ M_ord,
                                                        long long* __restrict__ argmax) {
  float m = -INFINITY;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) m = fmaxf(m, part[b]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    *M_ord = m > -INFINITY ? float_to_ord(m) : 0u;
    if (argmax) argmax[0] = 0;   // tie counter for attention_alpha (no separate fill)
  }
}

// ------------------------------------------------------------------ fused edge pass
struct EdgeFwdArgs {
  const float* rows;       // gathered source rows: Wh [N][NH][Fp] (or x [N][Fp], head_stride4 0)
  int64_t row_stride4;     // float4s per source row
  int head_stride4;        // float4s between heads inside a source row
  const float* S;
  const uint32_t* M_ord;
  const int32_t* rowptr;
  const int32_t* col;
  const int32_t* perm;
  int64_t N;
  int NH, F, Fp, HS;       // heads, features (output), padded features, heads per work item
  int concat, const_att;
  const float* bias;
  float p_drop;
  const uint64_t* seed;     // device scalar (torch's generator; graph-capturable)
  float* out;
  int64_t out_ld;
  const float* resid;      // fused epilogue: out = elu?(agg + bias + resid)
  int64_t resid_ld;
  int elu;
  // the next layer's input dropout fused after the ELU (models/GATModel.py:130 applied to this
  // output): out = keep(out_seed, n * out_cols + col) ? v / (1 - out_p) : 0
  float out_p;
  const uint64_t* out_seed;
  int64_t out_cols;
  float* den;
  int lds_row;
  int64_t chunk;           // destination nodes per (chunk, head-group) sweep
  int64_t n_items;
  int g_begin, g_count;    // head groups [g_begin, g_begin + g_count) in this launch
  int mean_mode;           // head mean: 0 all heads in one pass; multi-pass over head groups:
                           // 1 first (out = group sum), 2 middle (out += group sum),
                           // 3 last (out = epilogue((out + group sum) / NH + bias))
  int vec_out;             // concat output / resid rows float4-aligned (F % 4 == 0)
  int dbg;                 // diagnostic ablations (gatx_set_debug); 0 in production
  // hub splitting (hub_T > 0): segments of more than hub_T edges are skipped by their own item
  // and processed as pieces of hub_T edges (gatx_graph_hub_plan's list) by the items past
  // n_items_main, each writing an unnormalised partial; edge_hub_combine_kernel sums a hub's
  // pieces in piece order and runs the item's epilogue
  int hub_T;
  const int32_t* hubs;     // [hub_bound][4]: node, piece, pieces, first slot
  const int32_t* hub_count;
  int64_t hub_bound;
  float* hub_part;         // [slot][g_count][HS*Fp + HS]
  int64_t n_items_main;
  int64_t hub_blocks;      // blocks [0, hub_blocks) run hub pieces (hub_bound * g_count waves)
  // destinations the caller serves another way: skip[n] != 0 -> no item
  const uint8_t* skip;
};

int g_debug = 0;

// XCD-contiguous block order: blocks are dealt round-robin to the 8 XCDs (b % 8); hand XCD x
// the x-th contiguous range of work items so one XCD sweeps one (node chunk, head group) at a
// time and its 4 MB L2 holds that head's slice of the gathered rows. Speed only, never results.
__device__ inline int64_t xcd_contiguous(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, xcd = b % 8, j = b / 8;
  return (xcd < r) ? xcd * (q + 1) + j : r * (q + 1) + (xcd - r) * q + j;
}

__device__ inline float out_dropout(float v, const EdgeFwdArgs& g, int64_t n, int64_t col) {
  return dropout_keep(*g.out_seed, n * g.out_cols + col, g.out_p) ? v * (1.f / (1.f - g.out_p))
                                                                   : 0.f;
}

__device__ inline float epilogue(float v, const EdgeFwdArgs& g, int64_t n, int64_t col) {
  if (g.resid) v += g.resid[n * g.resid_ld + col];
  if (g.elu) v = elu_act(v);
  if (g.out_p > 0.f) v = out_dropout(v, g, n, col);
  return v;
}

constexpr int kMaxHS = 8;
typedef float f4v __attribute__((ext_vector_type(4)));   // heads per work item held in registers by the batch phase

__device__ inline int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline float lane_f(float v, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

// Normalisation and epilogue of one (node, head group) item: grp-0 lanes hold the item's
// unnormalised sums acc (chunk q[c] of the HS * Fp row), den_lds its HS softmax denominators.
template <int LPE, int CPL>
__device__ inline void finish_item(const EdgeFwdArgs& g, int64_t n, int h0, int lane, int grp,
                                   const int (&q)[CPL], const bool (&vq)[CPL],
                                   const int (&hl)[CPL], const float4 (&acc)[CPL],
                                   float* row_lds, const float* den_lds) {
  const int NH = g.NH, F = g.F, Fp = g.Fp, HS = g.HS;
  if (grp == 0) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      if (!vq[c]) continue;
      const float inv = 1.f / (den_lds[hl[c]] + kSoftmaxEps);
      const float4 o = acc[c] * inv;
      const int h = h0 + hl[c], f0 = q[c] * 4 - hl[c] * Fp;
      if (g.concat) {
        float* orow = g.out + n * g.out_ld;
        const int64_t cb = (int64_t)h * F + f0;
        if (g.vec_out) {
          // out / resid are streamed once: non-temporal, so they do not evict the gathered rows
          float4 r = g.bias ? *(const float4*)(g.bias + cb) : make_float4(0.f, 0.f, 0.f, 0.f);
          r = add4(o, r);
          if (g.resid) {
            const f4v rv = __builtin_nontemporal_load((const f4v*)(g.resid + n * g.resid_ld + cb));
            r.x += rv[0]; r.y += rv[1]; r.z += rv[2]; r.w += rv[3];
          }
          if (g.elu) {
            r.x = elu_act(r.x);
            r.y = elu_act(r.y);
            r.z = elu_act(r.z);
            r.w = elu_act(r.w);
          }
          if (g.out_p > 0.f) {
            r.x = out_dropout(r.x, g, n, cb);
            r.y = out_dropout(r.y, g, n, cb + 1);
            r.z = out_dropout(r.z, g, n, cb + 2);
            r.w = out_dropout(r.w, g, n, cb + 3);
          }
          const f4v ov = {r.x, r.y, r.z, r.w};
          __builtin_nontemporal_store(ov, (f4v*)(orow + cb));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (f0 + j < F)
              orow[cb + j] = epilogue(get4(o, j) + (g.bias ? g.bias[cb + j] : 0.f), g, n, cb + j);
        }
      } else {
        *(float4*)(row_lds + q[c] * 4) = o;
      }
    }
  }
  wave_lds_sync();
  if (!g.concat) {   // head mean over this item's HS heads (all NH when mean_mode == 0)
    const float inv_nh = 1.f / (float)NH;
    float* orow = g.out + n * g.out_ld;
    for (int f = lane; f < F; f += 64) {
      float sum = 0.f;
      for (int h = 0; h < HS; ++h) sum += row_lds[h * Fp + f];
      if (g.mean_mode == 1) {
        orow[f] = sum;
      } else if (g.mean_mode == 2) {
        orow[f] += sum;
      } else {
        if (g.mean_mode == 3) sum += orow[f];
        orow[f] = epilogue(sum * inv_nh + (g.bias ? g.bias[f] : 0.f), g, n, f);
      }
    }
  }
  if (lane < HS) g.den[n * NH + h0 + lane] = den_lds[lane];
}

// One wavefront per work item = (destination node n, group of HS heads). Edges are taken in
// batches of 64: lane j loads batch edge j's source id (one coalesced load) and computes its HS
// attention weights ex = exp(0.01 (s_src[src] + s_dst[n] - M)) (one gather of s_src per head).
// The gather phase then streams the source rows with no dependent address latency:
//  - LPE == 64 (one edge per wave step): the source id is wave-uniform (readlane -> SGPR, scalar
//    row address); with one head per item (SCALAR_W) so is its weight.
//  - LPE < 64 (narrow rows, 64/LPE edges per step): ids and weights through LDS.
// Lane l of edge group grp owns chunks q = c*LPE + (l % LPE) of the item's HS*Fp/4; chunks past
// the row end load a valid address of the same row and are never stored (branch-free loop).
// Everything that indexes work (item, node, edge range) is made wave-uniform explicitly.
template <int LPE, int CPL, int U, bool SCALAR_W>
__global__ void __launch_bounds__(256) edge_forward_kernel(EdgeFwdArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int EPW = 64 / LPE;
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int grp = lane / LPE, li = lane % LPE;
  // the first hub_blocks blocks (a multiple of 8: dealt round-robin over the XCDs, and
  // dispatched first, so long hub pieces start early) take the hub pieces; the rest the items
  const int64_t hb = g.hub_blocks;
  const bool hub_block = (int64_t)blockIdx.x < hb;
  const int64_t item = hub_block ? g.n_items_main + (int64_t)blockIdx.x * 4 + wave
                                 : xcd_contiguous(blockIdx.x - hb, gridDim.x - hb) * 4 + wave;
  if (!hub_block && item >= g.n_items_main) return;
  const int NG = g.g_count;
  int64_t n;
  int hgl, beg, end;
  int64_t hub_slot = -1;   // >= 0: this wave is one piece of a hub segment
  if (!hub_block) {
    const int64_t per_chunk = g.chunk * NG;
    const int64_t ck = item / per_chunk, rem = item - ck * per_chunk;
    hgl = (int)(rem / g.chunk);
    n = ck * g.chunk + (rem - (int64_t)hgl * g.chunk);
    if (n >= g.N) return;
    if (g.skip && g.skip[n]) return;
    beg = uni(g.rowptr[n]);
    end = uni(g.rowptr[n + 1]);
    if (g.hub_T > 0 && end - beg > g.hub_T) return;   // done in pieces below
  } else {
    const int64_t hi = item - g.n_items_main;
    hgl = (int)(hi / g.hub_bound);
    const int64_t pc = hi - (int64_t)hgl * g.hub_bound;
    if (hgl >= NG || pc >= uni(*g.hub_count)) return;
    const int32_t* hp = g.hubs + 4 * pc;
    n = uni(hp[0]);
    const int p = uni(hp[1]);
    hub_slot = (int64_t)uni(hp[3]) + p;
    beg = uni(g.rowptr[n]) + p * g.hub_T;
    end = min(uni(g.rowptr[n + 1]), beg + g.hub_T);
  }
  const int hg = g.g_begin + hgl;
  const int h0 = hg * g.HS, HS = g.HS;
  const int NH = g.NH, Fp = g.Fp, F4 = Fp / 4, S2 = 2 * NH;
  const int D4 = HS * F4;
  // per-wave LDS: [HS*Fp head-mean staging][HS den][64 src ids][HS*64 edge weights]
  float* row_lds = smem + wave * g.lds_row;
  float* den_lds = row_lds + HS * Fp;
  int* src_lds = (int*)(den_lds + HS);
  float* w_lds = (float*)(src_lds + 64);
  const float M = g.const_att ? 0.f : ord_to_float(*g.M_ord);
  const bool drop = g.p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  const uint64_t seed = drop ? *g.seed : 0ull;
  const float4* __restrict__ rows4 = (const float4*)g.rows;
  const float* __restrict__ S = g.S;
  const int32_t* __restrict__ col = g.col;

  int q[CPL], hl[CPL], off4[CPL];
  bool vq[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    q[c] = c * LPE + li;
    vq[c] = q[c] < D4;
    const int qq = vq[c] ? q[c] : 0;
    hl[c] = qq / F4;
    off4[c] = (h0 + hl[c]) * g.head_stride4 + (qq - hl[c] * F4);
  }
  float sdst[kMaxHS], dnl[kMaxHS];
#pragma unroll
  for (int h = 0; h < kMaxHS; ++h) {
    sdst[h] = (h < HS && !g.const_att) ? S[n * S2 + NH + h0 + h] : 0.f;
    dnl[h] = 0.f;
  }
  float4 acc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);

  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    // batch phase: lane j <-> edge base + j (lanes past the segment reuse its last edge, w = 0)
    const bool valid = lane < cnt;
    const int e = base + min(lane, cnt - 1);
    const int my_src = col[e];
    float my_w0 = 0.f;
    {
      float ssv[kMaxHS];
#pragma unroll
      for (int h = 0; h < kMaxHS; ++h)
        ssv[h] = (h < HS && !g.const_att) ? S[(int64_t)my_src * S2 + h0 + h] : 0.f;
      const int64_t ep = drop ? (int64_t)g.perm[e] : 0;
#pragma unroll
      for (int h = 0; h < kMaxHS; ++h) {
        if (h < HS) {
          float ex = g.const_att ? 1.f : att_exp(ssv[h] + sdst[h], M);
          if (g.dbg & 2) ex = 1.f;
          ex = valid ? ex : 0.f;
          dnl[h] += ex;
          float w = ex;
          if (drop) w = dropout_keep(seed, ep * NH + h0 + h, g.p_drop) ? ex * drop_scale : 0.f;
          if (h == 0) my_w0 = w;
          if (!SCALAR_W) w_lds[h * 64 + lane] = w;
        }
      }
    }
    if (EPW > 1) src_lds[lane] = my_src;
    if (EPW > 1 || !SCALAR_W) wave_lds_sync();
    if constexpr (EPW == 1) {
      for (int j0 = 0; j0 < cnt; j0 += U) {
        const float4* rp[U];
        float wsc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = min(j0 + u, cnt - 1);
          rp[u] = rows4 + (int64_t)__builtin_amdgcn_readlane(my_src, j) * g.row_stride4;
          wsc[u] = (j0 + u < cnt) ? lane_f(my_w0, j) : 0.f;
        }
        float4 v[U][CPL];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int c = 0; c < CPL; ++c)
            v[u][c] = rp[u][off4[c]];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = min(j0 + u, cnt - 1);
          const bool live = j0 + u < cnt;
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const float w = SCALAR_W ? wsc[u] : (live ? w_lds[hl[c] * 64 + j] : 0.f);
            acc[c] = fma4(w, v[u][c], acc[c]);
          }
        }
      }
    } else {
      for (int j0 = grp; j0 < cnt; j0 += EPW * U) {
        int sv[U];
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + u * EPW;
          live[u] = j < cnt;
          sv[u] = src_lds[live[u] ? j : cnt - 1];
        }
        float4 v[U][CPL];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int c = 0; c < CPL; ++c)
            v[u][c] = rows4[(int64_t)sv[u] * g.row_stride4 + off4[c]];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + u * EPW;
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const float w = live[u] ? w_lds[hl[c] * 64 + j] : 0.f;
            acc[c] = fma4(w, v[u][c], acc[c]);
          }
        }
      }
    }
    if (EPW > 1 || !SCALAR_W) wave_lds_sync();
  }
  // softmax denominators: per-lane partials -> wave sums (fixed butterfly order)
#pragma unroll
  for (int h = 0; h < kMaxHS; ++h) {
    if (h < HS) {
      float t = dnl[h];
      for (int off = 1; off < 64; off <<= 1) t += __shfl_xor(t, off);
      dnl[h] = t;
    }
  }
  if (lane < HS) {
    float d = 0.f;
#pragma unroll
    for (int h = 0; h < kMaxHS; ++h)
      if (h == lane) d = dnl[h];
    den_lds[lane] = d;   // to memory at the very end: a store ahead of the epilogue's bias /
                         // residual loads would make them wait for it (shared vmcnt)
  }
  // combine the EPW edge groups (butterfly: every group ends with the totals)
#pragma unroll
  for (int off = LPE; off < 64; off <<= 1) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc[c] = add4(acc[c], shfl_xor4(acc[c], off));
  }
  wave_lds_sync();
  if (hub_slot >= 0) {   // one piece of a hub: its unnormalised partial, finished by the combine
    float* part = g.hub_part + (hub_slot * NG + hgl) * (int64_t)(HS * Fp + HS);
    if (grp == 0) {
#pragma unroll
      for (int c = 0; c < CPL; ++c)
        if (vq[c]) *(float4*)(part + q[c] * 4) = acc[c];
    }
    if (lane < HS) part[HS * Fp + lane] = den_lds[lane];
    return;
  }
  finish_item<LPE, CPL>(g, n, h0, lane, grp, q, vq, hl, acc, row_lds, den_lds);
}

// The edge pass over source rows SHARED by every head (head_stride 0: the reassociated first
// layer aggregates x rows, Z[n,h,:] = sum_e alpha~[e,h] x[src_e,:]). edge_forward_kernel would give
// each (head, chunk) pair its own lane, so the HS lanes of one chunk load the same float4; here a
// lane owns one float4 chunk of the row for ALL HS heads of the item (HS accumulators), so one
// load instruction moves 64/LPE distinct edges' chunks. Per-edge weights of the HS heads sit in
// LDS as one float4 row per edge (a single ds_read_b128 per edge for HS <= 4). Plain epilogue
// (no bias / skip / ELU / output dropout: the reassociated layer's epilogue runs in its output
// GEMM); hub pieces write the generic partial layout [h * Fp + f | den], finished by
// edge_hub_combine_kernel.
template <int LPE, int HSC>
__global__ void __launch_bounds__(256) edge_forward_shared_kernel(EdgeFwdArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // U: row loads in flight per lane (round 6: 2 ran ~2 us faster per PPI launch than 4, and 8 was
  // ~9 us slower; same summation order, so the same bits)
  constexpr int EPW = 64 / LPE, U = 2;
  constexpr int HSP = HSC <= 4 ? 4 : 8;   // weights per edge row in LDS (float4 granules)
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int grp = lane / LPE, li = lane % LPE;
  const int64_t hb = g.hub_blocks;
  const bool hub_block = (int64_t)blockIdx.x < hb;
  const int64_t item = hub_block ? g.n_items_main + (int64_t)blockIdx.x * 4 + wave
                                 : xcd_contiguous(blockIdx.x - hb, gridDim.x - hb) * 4 + wave;
  if (!hub_block && item >= g.n_items_main) return;
  const int NG = g.g_count;
  int64_t n;
  int hgl, beg, end;
  int64_t hub_slot = -1;
  if (!hub_block) {
    const int64_t per_chunk = g.chunk * NG;
    const int64_t ck = item / per_chunk, rem = item - ck * per_chunk;
    hgl = (int)(rem / g.chunk);
    n = ck * g.chunk + (rem - (int64_t)hgl * g.chunk);
    if (n >= g.N) return;
    if (g.skip && g.skip[n]) return;
    beg = uni(g.rowptr[n]);
    end = uni(g.rowptr[n + 1]);
    if (g.hub_T > 0 && end - beg > g.hub_T) return;
  } else {
    const int64_t hi = item - g.n_items_main;
    hgl = (int)(hi / g.hub_bound);
    const int64_t pc = hi - (int64_t)hgl * g.hub_bound;
    if (hgl >= NG || pc >= uni(*g.hub_count)) return;
    const int32_t* hp = g.hubs + 4 * pc;
    n = uni(hp[0]);
    const int p = uni(hp[1]);
    hub_slot = (int64_t)uni(hp[3]) + p;
    beg = uni(g.rowptr[n]) + p * g.hub_T;
    end = min(uni(g.rowptr[n + 1]), beg + g.hub_T);
  }
  const int h0 = (g.g_begin + hgl) * HSC;
  const int NH = g.NH, Fp = g.Fp, F4 = Fp / 4, S2 = 2 * NH;
  // per-wave LDS: [64 src ids][64 x HSP edge weights][HSC den]
  int* src_lds = (int*)(smem + wave * g.lds_row);
  float* w_lds = (float*)(src_lds + 64);
  float* den_lds = w_lds + 64 * HSP;
  const float M = g.const_att ? 0.f : ord_to_float(*g.M_ord);
  const bool drop = g.p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  const uint64_t seed = drop ? *g.seed : 0ull;
  const float4* __restrict__ rows4 = (const float4*)g.rows;
  const bool vq = li < F4;
  const int off4 = vq ? li : 0;
  float sdst[HSC], dnl[HSC];
#pragma unroll
  for (int h = 0; h < HSC; ++h) {
    sdst[h] = g.const_att ? 0.f : g.S[n * S2 + NH + h0 + h];
    dnl[h] = 0.f;
  }
  float4 acc[HSC];
#pragma unroll
  for (int h = 0; h < HSC; ++h) acc[h] = make_float4(0.f, 0.f, 0.f, 0.f);

  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const bool valid = lane < cnt;
    const int e = base + min(lane, cnt - 1);
    const int my_src = g.col[e];
    {
      float w[HSP];
      const int64_t ep = drop ? (int64_t)g.perm[e] : 0;
#pragma unroll
      for (int h = 0; h < HSP; ++h) {
        w[h] = 0.f;
        if (h < HSC) {
          const float ss = g.const_att ? 0.f : g.S[(int64_t)my_src * S2 + h0 + h];
          float ex = g.const_att ? 1.f : att_exp(ss + sdst[h], M);
          ex = valid ? ex : 0.f;
          dnl[h] += ex;
          w[h] = ex;
          if (drop) w[h] = dropout_keep(seed, ep * NH + h0 + h, g.p_drop) ? ex * drop_scale : 0.f;
        }
      }
#pragma unroll
      for (int h = 0; h < HSP; h += 4)
        *(float4*)(w_lds + lane * HSP + h) = make_float4(w[h], w[h + 1], w[h + 2], w[h + 3]);
      src_lds[lane] = my_src;
    }
    wave_lds_sync();
    for (int j0 = grp; j0 < cnt; j0 += EPW * U) {
      int sv[U];
      bool live[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * EPW;
        live[u] = j < cnt;
        sv[u] = src_lds[live[u] ? j : cnt - 1];
      }
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = rows4[(int64_t)sv[u] * g.row_stride4 + off4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = live[u] ? j0 + u * EPW : 0;
        float wv[HSP];
#pragma unroll
        for (int h = 0; h < HSP; h += 4) {
          const float4 t = *(const float4*)(w_lds + j * HSP + h);
          wv[h] = t.x; wv[h + 1] = t.y; wv[h + 2] = t.z; wv[h + 3] = t.w;
        }
#pragma unroll
        for (int h = 0; h < HSC; ++h) acc[h] = fma4(live[u] ? wv[h] : 0.f, v[u], acc[h]);
      }
    }
    wave_lds_sync();
  }
#pragma unroll
  for (int h = 0; h < HSC; ++h) {
    float t = dnl[h];
    for (int o = 1; o < 64; o <<= 1) t += __shfl_xor(t, o);
    dnl[h] = t;
  }
#pragma unroll
  for (int o = LPE; o < 64; o <<= 1) {
#pragma unroll
    for (int h = 0; h < HSC; ++h) acc[h] = add4(acc[h], shfl_xor4(acc[h], o));
  }
  if (hub_slot >= 0) {   // one piece of a hub: the generic partial layout
    float* part = g.hub_part + (hub_slot * NG + hgl) * (int64_t)(HSC * Fp + HSC);
    if (grp == 0 && vq) {
#pragma unroll
      for (int h = 0; h < HSC; ++h) *(float4*)(part + h * Fp + 4 * li) = acc[h];
    }
    if (lane == 0) {
#pragma unroll
      for (int h = 0; h < HSC; ++h) part[HSC * Fp + h] = dnl[h];
    }
    return;
  }
  if (grp == 0 && vq) {
    float* orow = g.out + n * g.out_ld;
#pragma unroll
    for (int h = 0; h < HSC; ++h) {
      const float4 o = acc[h] * (1.f / (dnl[h] + kSoftmaxEps));
      const int64_t cb = (int64_t)(h0 + h) * g.F + 4 * li;
      if (g.vec_out) {
        *(float4*)(orow + cb) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (4 * li + j < g.F) orow[cb + j] = get4(o, j);
      }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < HSC; ++h) g.den[n * NH + h0 + h] = dnl[h];
  }
  (void)den_lds;
}

// Sum a hub's pieces (slots first .. first + pieces - 1, in that order) and finish the item:
// one wave per (hub, head group), the lane layout of edge_forward_kernel<LPE, CPL>.
template <int LPE, int CPL>
__global__ void __launch_bounds__(256) edge_hub_combine_kernel(EdgeFwdArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int grp = lane / LPE, li = lane % LPE;
  const int64_t hi = (int64_t)blockIdx.x * 4 + wave;
  const int NG = g.g_count;
  const int hgl = (int)(hi / g.hub_bound);
  const int64_t pc = hi - (int64_t)hgl * g.hub_bound;
  if (hgl >= NG || pc >= uni(*g.hub_count)) return;
  const int32_t* hp = g.hubs + 4 * pc;
  if (uni(hp[1]) != 0) return;   // one wave per hub: its first piece's entry
  const int64_t n = uni(hp[0]);
  const int pieces = uni(hp[2]), first = uni(hp[3]);
  const int hg = g.g_begin + hgl;
  const int h0 = hg * g.HS, HS = g.HS, Fp = g.Fp, F4 = Fp / 4, D4 = HS * F4;
  float* row_lds = smem + wave * g.lds_row;
  float* den_lds = row_lds + HS * Fp;
  int q[CPL], hl[CPL];
  bool vq[CPL];
  float4 acc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    q[c] = c * LPE + li;
    vq[c] = q[c] < D4;
    hl[c] = (vq[c] ? q[c] : 0) / F4;
    acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float d = 0.f;
  const int64_t W = (int64_t)HS * Fp + HS;
  for (int p = 0; p < pieces; ++p) {
    const float* part = g.hub_part + ((int64_t)(first + p) * NG + hgl) * W;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
      if (vq[c]) acc[c] = add4(acc[c], *(const float4*)(part + q[c] * 4));
    if (lane < HS) d += part[HS * Fp + lane];
  }
  if (lane < HS) den_lds[lane] = d;
  wave_lds_sync();
  finish_item<LPE, CPL>(g, n, h0, lane, grp, q, vq, hl, acc, row_lds, den_lds);
}

// ------------------------------------------------------------------ weights
// W_aug rows Dp.. Dp+2NH-1 = A2 . W with A2 = [A_src; A_dst] (2NH x D), deterministic split-K:
// block (i-chunk of 64 columns, c-chunk of 128 rows of W) -> partial[cb][h2][i].
constexpr int kMaxH2 = 32;
// Block (64 columns i, 16 rows c of W; 4 waves x 4 rows): the row index is wave-uniform, so
// the 2NH coefficients of `a` per row are scalar loads; partial[cb][h2][i] over the block's rows.
constexpr int kWeffRows = 16;
__global__ void __launch_bounds__(256) weff_partial_kernel(const float* __restrict__ W,
                                                           const float* __restrict__ a, int NH,
                                                           int F, int64_t F_in,
                                                           float* __restrict__ partial) {
  __shared__ float red[4][kMaxH2][64];
  const int tx = threadIdx.x & 63;
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t i = blockIdx.x * 64ll + tx;
  const int D = NH * F, H2 = 2 * NH;
  const int c0 = blockIdx.y * kWeffRows + ty * (kWeffRows / 4);
  float acc[kMaxH2];
#pragma unroll
  for (int h = 0; h < kMaxH2; ++h) acc[h] = 0.f;
#pragma unroll
  for (int cc = 0; cc < kWeffRows / 4; ++cc) {
    const int c = c0 + cc;
    if (c >= D) break;
    const float w = (i < F_in) ? W[(int64_t)c * F_in + i] : 0.f;
    const int k = c / F, f = c - k * F;
    const float* ak = a + (int64_t)k * 2 * F + f;
#pragma unroll
    for (int h = 0; h < kMaxH2; ++h) {
      if (h >= H2) break;
      const int hh = h < NH ? h : h - NH;
      acc[h] = fmaf(ak[(int64_t)hh * 2 * D + (h < NH ? 0 : F)], w, acc[h]);
    }
  }
#pragma unroll
  for (int h = 0; h < kMaxH2; ++h)
    if (h < H2) red[ty][h][tx] = acc[h];
  __syncthreads();
  if (ty == 0 && i < F_in) {
    for (int h = 0; h < H2; ++h) {
      float s = (red[0][h][tx] + red[1][h][tx]) + (red[2][h][tx] + red[3][h][tx]);
      partial[((int64_t)blockIdx.y * H2 + h) * F_in + i] = s;
    }
  }
}

// W_aug from W and the split-K partials: blocks [0, ncopy) copy the head-padded W rows and the
// folded skip's rows; the blocks after them give each score-row element one wave, lanes over the
// n_cb partials, fixed-order wave sum (a thread summing its element's 64 partials alone made the
// PPI assembly an 18 us latency chain).
__global__ void __launch_bounds__(256) waug_assemble_kernel(const float* __restrict__ W,
                                                            const float* __restrict__ partial,
                                                            int n_cb, int NH, int F, int Fp,
                                                            int H2, int64_t F_in, int ncopy,
                                                            float* __restrict__ W_aug,
                                                            const float* __restrict__ W_skip,
                                                            int skip_heads, int64_t skip_cols) {
  const int64_t Dp = (int64_t)NH * Fp;
  if ((int)blockIdx.x < ncopy) {
    const int64_t ncp = Dp * F_in, sk = skip_cols * F_in;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < ncp + sk;
         t += (int64_t)ncopy * blockDim.x) {
      float v;
      int64_t dst;
      if (t >= ncp) {   // folded skip rows: mean over the skip's head blocks (a copy for 1)
        const int64_t q = t - ncp;
        v = W_skip[q];
        for (int h = 1; h < skip_heads; ++h) v += W_skip[(int64_t)h * sk + q];
        if (skip_heads > 1) v /= (float)skip_heads;
        dst = (Dp + H2) * F_in + q;
      } else {
        const int64_t r = t / F_in, i = t - r * F_in;
        const int h = (int)(r / Fp), f = (int)(r - (int64_t)h * Fp);
        v = (f < F) ? W[((int64_t)h * F + f) * F_in + i] : 0.f;
        dst = t;
      }
      W_aug[dst] = v;
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t o = ((int64_t)blockIdx.x - ncopy) * 4 + (threadIdx.x >> 6);
  if (o >= (int64_t)H2 * F_in) return;
  const int h2 = (int)(o / F_in);
  const int64_t i = o - (int64_t)h2 * F_in;
  float v = 0.f;
  for (int cb = lane; cb < n_cb; cb += 64) v += partial[((int64_t)cb * H2 + h2) * F_in + i];
  v = group_sum<64>(v);
  if (lane == 0) W_aug[(Dp + h2) * F_in + i] = v;
}

// W_aug in ONE launch for small layers (D = NH*F <= 256; split-K partials + assembly are two
// launches, and small layers are launch-bound). Blocks [0, ncopy) copy the head-padded W rows
// (and the folded skip's rows); the blocks after them give each score-row element
// W_aug[Dp + h2][i] = sum_c A2[h2][c] W[c][i] one wave, lanes over c, fixed-order wave sum.
__global__ void __launch_bounds__(256) waug_direct_kernel(const float* __restrict__ W,
                                                          const float* __restrict__ a, int NH,
                                                          int F, int Fp, int H2, int64_t F_in,
                                                          int ncopy, float* __restrict__ W_aug,
                                                          const float* __restrict__ W_skip,
                                                          int skip_heads, int64_t skip_cols) {
  const int64_t Dp = (int64_t)NH * Fp;
  const int D = NH * F;
  if ((int)blockIdx.x < ncopy) {
    const int64_t ncp = Dp * F_in, sk = skip_cols * F_in;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < ncp + sk;
         t += (int64_t)ncopy * blockDim.x) {
      float v;
      int64_t dst;
      if (t >= ncp) {   // folded skip rows: mean over the skip's head blocks (a copy for 1)
        const int64_t q = t - ncp;
        v = W_skip[q];
        for (int h = 1; h < skip_heads; ++h) v += W_skip[(int64_t)h * sk + q];
        if (skip_heads > 1) v /= (float)skip_heads;
        dst = (Dp + H2) * F_in + q;
      } else {
        const int64_t r = t / F_in, i = t - r * F_in;
        const int h = (int)(r / Fp), f = (int)(r - (int64_t)h * Fp);
        v = (f < F) ? W[((int64_t)h * F + f) * F_in + i] : 0.f;
        dst = t;
      }
      W_aug[dst] = v;
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t o = ((int64_t)blockIdx.x - ncopy) * 4 + (threadIdx.x >> 6);
  if (o >= (int64_t)H2 * F_in) return;
  const int h2 = (int)(o / F_in);
  const int64_t i = o - (int64_t)h2 * F_in;
  const int hh = h2 < NH ? h2 : h2 - NH;
  const float* ah = a + (int64_t)hh * 2 * D + (h2 < NH ? 0 : F);
  float v = 0.f;
  for (int c = lane; c < D; c += 64) {
    const int k = c / F, f = c - k * F;
    v = fmaf(ah[k * 2 * F + f], W[(int64_t)c * F_in + i], v);
  }
  v = group_sum<64>(v);
  if (lane == 0) W_aug[(Dp + h2) * F_in + i] = v;
}

// Its gradient: g_W[(h * cols + c)][i] = g_eff[c][i] / heads for every head block.
__global__ void __launch_bounds__(256) skip_grad_kernel(const float* __restrict__ g_eff,
                                                        int heads, int64_t cols, int64_t F_in,
                                                        float* __restrict__ g_W) {
  const int64_t total = cols * F_in;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < heads * total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t % total;
    g_W[t] = heads > 1 ? g_eff[r] / (float)heads : g_eff[r];
  }
}

__global__ void __launch_bounds__(256) pad_rows_kernel(const float* __restrict__ src,
                                                       int64_t rows, int64_t cols, int64_t lds,
                                                       float* __restrict__ dst, int64_t ldd) {
  const int64_t total = rows * ldd;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / ldd, c = t - r * ldd;
    dst[t] = c < cols ? src[r * lds + c] : 0.f;
  }
}

// S[n] = (Wh[n] . A_src^T | Wh[n] . A_dst^T): the per-node logit factors, in the reference's
// own association (raw = cat(Wh[src], Wh[dst]) . a^T, gat_layer.py:76-82, split per half).
// One wave per node; A2 = [A_src; A_dst] (2NH x Dp, head-padded) staged in LDS once per block.
__global__ void __launch_bounds__(256) node_scores_kernel(const float* __restrict__ Wh,
                                                          int64_t N, int NH, int F, int Fp,
                                                          const float* __restrict__ a,
                                                          float* __restrict__ S) {
  extern __shared__ __attribute__((aligned(16))) float a2[];   // [2NH][Dp]
  const int Dp = NH * Fp, D = NH * F, H2 = 2 * NH;
  for (int t = threadIdx.x; t < H2 * Dp; t += blockDim.x) {
    const int h2 = t / Dp, c = t - h2 * Dp, k = c / Fp, f = c - k * Fp;
    const int hh = h2 < NH ? h2 : h2 - NH;
    a2[t] = f < F ? a[(int64_t)hh * 2 * D + k * 2 * F + (h2 < NH ? 0 : F) + f] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int D4 = Dp / 4;
  for (int64_t n = blockIdx.x * 4ll + wave; n < N; n += gridDim.x * 4ll) {
    const float4* row = (const float4*)(Wh + n * Dp);
    float acc[32];
#pragma unroll
    for (int h = 0; h < 32; ++h) acc[h] = 0.f;
    for (int q = lane; q < D4; q += 64) {
      const float4 v = row[q];
#pragma unroll
      for (int h = 0; h < 32; ++h) {
        if (h >= H2) break;
        const float4 w = *(const float4*)(a2 + h * Dp + 4 * q);
        acc[h] += v.x * w.x + v.y * w.y + v.z * w.z + v.w * w.w;
      }
    }
#pragma unroll
    for (int h = 0; h < 32; ++h) {
      if (h >= H2) break;
      float t = acc[h];
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
      if (lane == 0) S[n * H2 + h] = t;
    }
  }
}

// S from Wh rows with the attention matrix held in registers: one wave per row, lane l owns
// float4 columns q = l + 64c (c < CPL) and the matching slice of every one of the H (= 2NH
// rounded up to a power of two) rows of A2 [2NH][Dp] (a rearranged per column of Wh). The next
// row's loads are issued before the current row's reduce-scatter (reduce_scatter64).
template <int CPL, int H>
__global__ void __launch_bounds__(256) node_scores_reg_kernel(const float* __restrict__ Wh,
                                                              int64_t N, int NH, int F, int Fp,
                                                              const float* __restrict__ a,
                                                              float* __restrict__ S) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = blockIdx.x * 4ll + (threadIdx.x >> 6), nw = gridDim.x * 4ll;
  const int Dp = NH * Fp, D4 = Dp / 4, D = NH * F, H2 = 2 * NH;
  float4 w[CPL][H];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int q = lane + 64 * c;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float e[4] = {0.f, 0.f, 0.f, 0.f};
      if (q < D4 && h < H2) {
        const int hh = h < NH ? h : h - NH;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = 4 * q + j, k = col / Fp, f = col - k * Fp;
          if (f < F) e[j] = a[(int64_t)hh * 2 * D + k * 2 * F + (h < NH ? 0 : F) + f];
        }
      }
      w[c][h] = make_float4(e[0], e[1], e[2], e[3]);
    }
  }
  const float4* __restrict__ W4 = (const float4*)Wh;
  float4 cur[CPL];
  auto load = [&](int64_t n, float4 (&v)[CPL]) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int q = lane + 64 * c;
      v[c] = (n < N && q < D4) ? W4[n * D4 + q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // two rows in flight ahead of the one being reduced (one ahead: 3.8 TB/s at PPI layer 1,
  // where the attention registers leave two waves per SIMD)
  float4 nx[CPL];
  load(wave0, cur);
  load(wave0 + nw, nx);
  for (int64_t n = wave0; n < N; n += nw) {
    float acc[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float t = 0.f;
#pragma unroll
      for (int c = 0; c < CPL; ++c)
        t += cur[c].x * w[c][h].x + cur[c].y * w[c][h].y + cur[c].z * w[c][h].z +
             cur[c].w * w[c][h].w;
      acc[h] = t;
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) cur[c] = nx[c];
    load(n + 2 * nw, nx);
    int h;
    const float tot = reduce_scatter64<H>(acc, lane, h);
    if ((lane & (64 / H - 1)) == 0 && h < H2) S[n * H2 + h] = tot;
  }
}

// alpha in edge_index' order (pre-dropout, as the reference returns and stores it,
// models/gat_layer.py:109-110): alpha[e', h] = ex / (den[dst] + 1e-8), one thread per CSR slot,
// all heads of an edge written together (one random 4*NH-byte store per edge instead of NH
// scattered dwords). Also records the argmax (edge, head) entries for max()'s gradient.
template <int NHC, bool const_att>
__global__ void __launch_bounds__(256) attention_alpha_kernel(
    const int32_t* __restrict__ col, const int32_t* __restrict__ rowidx,
    const int32_t* __restrict__ perm, int64_t E2, const float* __restrict__ S,
    const uint32_t* __restrict__ M_ord, const float* __restrict__ den, int NH_rt,
    float* __restrict__ alpha, long long* __restrict__ argmax) {
  constexpr int VEC = (NHC % 4 == 0) ? 4 : ((NHC % 2 == 0) ? 2 : 1);
  const int NH = NHC > 0 ? NHC : NH_rt, S2 = 2 * NH;
  const float M = const_att ? 0.f : ord_to_float(*M_ord);
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E2;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = col[e], d = rowidx[e];
    float* out = alpha + (int64_t)perm[e] * NH;
    if constexpr (NHC > 0) {
      // constant attention (compile-time) has no score matrix — S is a placeholder — so it is
      // never read
      float ss[NHC], sd[NHC], dn[NHC], a[NHC];
#pragma unroll
      for (int h = 0; h < NHC; h += VEC) {
        if constexpr (VEC == 4) {
          const float4 x = const_att ? float4{} : *(const float4*)(S + s * S2 + h);
          const float4 y = const_att ? float4{} : *(const float4*)(S + d * S2 + NHC + h);
          const float4 z = *(const float4*)(den + d * NHC + h);
          ss[h] = x.x; ss[h + 1] = x.y; ss[h + 2] = x.z; ss[h + 3] = x.w;
          sd[h] = y.x; sd[h + 1] = y.y; sd[h + 2] = y.z; sd[h + 3] = y.w;
          dn[h] = z.x; dn[h + 1] = z.y; dn[h + 2] = z.z; dn[h + 3] = z.w;
        } else if constexpr (VEC == 2) {
          const float2 x = const_att ? float2{} : *(const float2*)(S + s * S2 + h);
          const float2 y = const_att ? float2{} : *(const float2*)(S + d * S2 + NHC + h);
          const float2 z = *(const float2*)(den + d * NHC + h);
          ss[h] = x.x; ss[h + 1] = x.y; sd[h] = y.x; sd[h + 1] = y.y; dn[h] = z.x; dn[h + 1] = z.y;
        } else {
          ss[h] = const_att ? 0.f : S[s * S2 + h];
          sd[h] = const_att ? 0.f : S[d * S2 + NHC + h];
          dn[h] = den[d * NHC + h];
        }
      }
      bool hit = false;
#pragma unroll
      for (int h = 0; h < NHC; ++h) {
        const float raw = ss[h] + sd[h];
        hit |= (!const_att && raw == M);
        a[h] = (const_att ? 1.f : att_exp(raw, M)) / (dn[h] + kSoftmaxEps);
      }
#pragma unroll
      for (int h = 0; h < NHC; h += VEC) {
        if constexpr (VEC == 4) *(float4*)(out + h) = make_float4(a[h], a[h + 1], a[h + 2], a[h + 3]);
        else if constexpr (VEC == 2) *(float2*)(out + h) = make_float2(a[h], a[h + 1]);
        else out[h] = a[h];
      }
      if (hit) {   // rare: record every tied argmax (edge, head) for max()'s gradient
#pragma unroll
        for (int h = 0; h < NHC; ++h)
          if (ss[h] + sd[h] == M) {
            unsigned long long k = atomicAdd((unsigned long long*)argmax, 1ull);
            if (k < GATX_ARGMAX_CAP) argmax[1 + k] = (long long)e * NHC + h;
          }
      }
    } else {
      for (int h = 0; h < NH; ++h) {
        float a;
        if (const_att) {
          a = 1.f / (den[d * NH + h] + kSoftmaxEps);
        } else {
          const float raw = S[s * S2 + h] + S[d * S2 + NH + h];
          a = att_exp(raw, M) / (den[d * NH + h] + kSoftmaxEps);
          if (raw == M) {
            unsigned long long k = atomicAdd((unsigned long long*)argmax, 1ull);
            if (k < GATX_ARGMAX_CAP) argmax[1 + k] = (long long)e * NH + h;
          }
        }
        out[h] = a;
      }
    }
  }
}

// The same in edge_index' order: thread p reads edge p's (src, dst) from edge_index' itself
// (coalesced) and writes alpha[p] (coalesced): the CSR-order kernel above scatters its writes
// through perm (each 4*NH-byte row a separate partial granule). Tied argmax entries are
// recorded by CSR slot as above, found by a scan of dst's segment (ties are rare).
template <int NHC, typename I, bool const_att>
__global__ void __launch_bounds__(256) attention_alpha_ei_kernel(
    const I* __restrict__ ei, int64_t ld_, int64_t E2b, const long long* e2p,
    const float* __restrict__ S,
    const uint32_t* __restrict__ M_ord, const float* __restrict__ den, int NH_rt,
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ perm,
    float* __restrict__ alpha, long long* __restrict__ argmax) {
  const int64_t E2 = e2p ? min(E2b, (int64_t)*e2p) : E2b;
  const int64_t ld = ld_ < 0 ? E2 : ld_;   // flat edge_index' of device-known size
  constexpr int VEC = (NHC % 4 == 0) ? 4 : ((NHC % 2 == 0) ? 2 : 1);
  constexpr int UE = NHC > 0 ? 4 : 1;   // edges per thread per round, all loads issued first
  constexpr int NHA = NHC > 0 ? NHC : 1;
  const int NH = NHC > 0 ? NHC : NH_rt, S2 = 2 * NH;
  const float M = const_att ? 0.f : ord_to_float(*M_ord);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p0 < E2; p0 += UE * stride) {
    if constexpr (NHC > 0) {
      int64_t sv[UE], dv[UE];
#pragma unroll
      for (int u = 0; u < UE; ++u) {
        const int64_t p = min(p0 + u * stride, E2 - 1);
        sv[u] = (int64_t)ei[p];
        dv[u] = (int64_t)ei[ld + p];
      }
      // score and denominator rows as float4 / float2 loads (rows of 2NH / NH floats: aligned
      // whenever NH is a multiple of the vector width; torch's allocations are 256-B aligned)
      float a[UE][NHA], dn[UE][NHA];
#pragma unroll
      for (int u = 0; u < UE; ++u)
#pragma unroll
        for (int h = 0; h < NHC; h += VEC) {
          const float* ps = S + sv[u] * S2 + h;
          const float* pd = S + dv[u] * S2 + NHC + h;
          const float* pn = den + dv[u] * NHC + h;
          if constexpr (VEC == 4) {
            const float4 z = *(const float4*)pn;
            dn[u][h] = z.x; dn[u][h + 1] = z.y; dn[u][h + 2] = z.z; dn[u][h + 3] = z.w;
            if (!const_att) {
              const float4 x = *(const float4*)ps, y = *(const float4*)pd;
              a[u][h] = x.x + y.x; a[u][h + 1] = x.y + y.y;
              a[u][h + 2] = x.z + y.z; a[u][h + 3] = x.w + y.w;
            } else {
              a[u][h] = a[u][h + 1] = a[u][h + 2] = a[u][h + 3] = 0.f;
            }
          } else if constexpr (VEC == 2) {
            const float2 z = *(const float2*)pn;
            dn[u][h] = z.x; dn[u][h + 1] = z.y;
            if (!const_att) {
              const float2 x = *(const float2*)ps, y = *(const float2*)pd;
              a[u][h] = x.x + y.x; a[u][h + 1] = x.y + y.y;
            } else {
              a[u][h] = a[u][h + 1] = 0.f;
            }
          } else {
            dn[u][h] = *pn;
            a[u][h] = const_att ? 0.f : *ps + *pd;
          }
        }
#pragma unroll
      for (int u = 0; u < UE; ++u) {
        const int64_t p = p0 + u * stride;
        if (p >= E2) break;
        float* out = alpha + p * NHC;
        bool hit = false;
        float r[NHA];
#pragma unroll
        for (int h = 0; h < NHC; ++h) {
          hit |= (!const_att && a[u][h] == M);
          r[h] = (const_att ? 1.f : att_exp(a[u][h], M)) / (dn[u][h] + kSoftmaxEps);
        }
#pragma unroll
        for (int h = 0; h < NHC; h += VEC) {
          if constexpr (VEC == 4) *(float4*)(out + h) = make_float4(r[h], r[h + 1], r[h + 2], r[h + 3]);
          else if constexpr (VEC == 2) *(float2*)(out + h) = make_float2(r[h], r[h + 1]);
          else out[h] = r[h];
        }
        if (hit) {   // rare: record every tied argmax (CSR slot, head) for max()'s gradient
          int64_t e = rowptr[dv[u]];
          while (perm[e] != (int32_t)p) ++e;
          for (int h = 0; h < NHC; ++h)
            if (a[u][h] == M) {
              unsigned long long k = atomicAdd((unsigned long long*)argmax, 1ull);
              if (k < GATX_ARGMAX_CAP) argmax[1 + k] = (long long)e * NHC + h;
            }
        }
      }
    } else {
      const int64_t p = p0;
      const int64_t s = (int64_t)ei[p], d = (int64_t)ei[ld + p];
      float* out = alpha + p * NH;
      bool hit = false;
      for (int h = 0; h < NH; ++h) {
        const float raw = const_att ? 0.f : S[s * S2 + h] + S[d * S2 + NH + h];
        hit |= (!const_att && raw == M);
        out[h] = (const_att ? 1.f : att_exp(raw, M)) / (den[d * NH + h] + kSoftmaxEps);
      }
      if (hit) {
        int64_t e = rowptr[d];
        while (perm[e] != (int32_t)p) ++e;
        for (int h = 0; h < NH; ++h)
          if (S[s * S2 + h] + S[d * S2 + NH + h] == M) {
            unsigned long long k = atomicAdd((unsigned long long*)argmax, 1ull);
            if (k < GATX_ARGMAX_CAP) argmax[1 + k] = (long long)e * NH + h;
          }
      }
    }
  }
}

inline unsigned grid_for(int64_t n, int block = 256, int64_t cap = 16384) {
  int64_t g = ceil_div(n > 0 ? n : 1, block);
  return (unsigned)(g < cap ? g : cap);
}

template <int LPE, int CPL>
int launch_edge_forward(unsigned grid, size_t lds, hipStream_t st, const EdgeFwdArgs& g) {
  constexpr int U = CPL <= 1 ? 8 : (CPL <= 4 ? 4 : 2);
  // one head per item with whole 64-lane chunks: every chunk's weight is wave-uniform
  const bool scalar_w = (LPE == 64) && g.HS == 1 && ((g.Fp / 4) % 64 == 0);
  if (scalar_w)
    edge_forward_kernel<LPE, CPL, U, true><<<grid, 256, lds, st>>>(g);
  else
    edge_forward_kernel<LPE, CPL, U, false><<<grid, 256, lds, st>>>(g);
  GATX_LAUNCH_CHECK("edge_forward");
  if (g.hub_T > 0) {
    const int64_t waves = g.hub_bound * g.g_count;
    edge_hub_combine_kernel<LPE, CPL><<<(unsigned)ceil_div(waves, 4), 256, lds, st>>>(g);
    GATX_LAUNCH_CHECK("edge_hub_combine");
  }
  return 0;
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" int gatx_prepare_weights_skip(const float* W, const float* a, int NH, int F,
                                         int64_t F_in, const float* W_skip, int skip_heads,
                                         int64_t skip_cols, float* W_aug, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  if (!W_skip) skip_cols = 0;
  GATX_REQUIRE(skip_cols >= 0 && (skip_cols == 0 || skip_heads >= 1),
               "prepare_weights: bad skip sizes");
  GATX_REQUIRE(NH >= 1 && F >= 1 && F_in >= 1, "prepare_weights: bad sizes");
  const int Fp = (int)round_up(F, 4);
  const int H2 = a ? 2 * NH : 0;
  GATX_REQUIRE(H2 <= kMaxH2, "prepare_weights: num_heads > %d unsupported", kMaxH2 / 2);
  const int D = NH * F;
  const int n_cb = (int)ceil_div(D, kWeffRows);
  if (D <= 256) {   // small layers: one launch (launch-bound at PATTERN size)
    const int ncopy = (int)grid_for(((int64_t)NH * Fp + skip_cols) * F_in, 256, 1024);
    const int64_t nscore = ceil_div((int64_t)H2 * F_in, 4);
    GATX_REQUIRE(ncopy + nscore < (1ll << 31), "prepare_weights: too many blocks");
    waug_direct_kernel<<<(unsigned)(ncopy + nscore), 256, 0, st>>>(
        W, a, NH, F, Fp, H2, F_in, ncopy, W_aug, W_skip, skip_heads, skip_cols);
    GATX_LAUNCH_CHECK("waug_direct");
    return 0;
  }
  float* partial = nullptr;
  if (H2) {
    // split-K partials are staged in the tail of the caller's buffer, which holds
    // gatx_prepare_weights_floats() floats: (Dp + 2NH) * F_in for W_aug + n_cb * 2NH * F_in.
    partial = W_aug + ((int64_t)NH * Fp + H2 + skip_cols) * F_in;
    dim3 g((unsigned)ceil_div(F_in, 64), (unsigned)n_cb);
    weff_partial_kernel<<<g, 256, 0, st>>>(W, a, NH, F, F_in, partial);
    GATX_LAUNCH_CHECK("weff_partial");
  }
  {
    const int ncopy = (int)grid_for(((int64_t)NH * Fp + skip_cols) * F_in, 256, 4096);
    const int64_t nscore = ceil_div((int64_t)H2 * F_in, 4);
    GATX_REQUIRE(ncopy + nscore < (1ll << 31), "prepare_weights: too many blocks");
    waug_assemble_kernel<<<(unsigned)(ncopy + nscore), 256, 0, st>>>(
        W, partial, n_cb, NH, F, Fp, H2, F_in, ncopy, W_aug, W_skip, skip_heads, skip_cols);
  }
  GATX_LAUNCH_CHECK("waug_assemble");
  return 0;
}

extern "C" int gatx_prepare_weights(const float* W, const float* a, int NH, int F, int64_t F_in,
                                    float* W_aug, gatx_stream_t s) {
  return gatx_prepare_weights_skip(W, a, NH, F, F_in, nullptr, 1, 0, W_aug, s);
}

extern "C" int gatx_skip_weight_grad(const float* g_eff, int heads, int64_t cols, int64_t F_in,
                                     float* g_W, gatx_stream_t s) {
  GATX_REQUIRE(heads >= 1 && cols >= 0 && F_in >= 0, "skip_weight_grad: bad sizes");
  if (cols == 0 || F_in == 0) return 0;
  skip_grad_kernel<<<grid_for(heads * cols * F_in), 256, 0, (hipStream_t)s>>>(g_eff, heads, cols,
                                                                              F_in, g_W);
  GATX_LAUNCH_CHECK("skip_grad");
  return 0;
}

extern "C" int64_t gatx_prepare_weights_skip_floats(int NH, int F, int64_t F_in, int has_a,
                                                   int64_t skip_cols) {
  const int64_t Fp = round_up(F, 4), H2 = has_a ? 2 * NH : 0;
  return (NH * Fp + H2 + skip_cols + ceil_div((int64_t)NH * F, kWeffRows) * H2) * F_in;
}

extern "C" int64_t gatx_prepare_weights_floats(int NH, int F, int64_t F_in, int has_a) {
  const int64_t Fp = round_up(F, 4), H2 = has_a ? 2 * NH : 0;
  return (NH * Fp + H2 + ceil_div((int64_t)NH * F, kWeffRows) * H2) * F_in;
}

extern "C" void gatx_set_debug(int flags) { g_debug = flags; }

extern "C" int gatx_node_scores(const float* Wh, int64_t N, int NH, int F, const float* a,
                                float* S, gatx_stream_t s) {
  const int Fp = (int)round_up(F, 4);
  GATX_REQUIRE(2 * NH <= kMaxH2, "node_scores: num_heads > %d unsupported", kMaxH2 / 2);
  if (N == 0) return 0;
  hipStream_t st = (hipStream_t)s;
  const int cpl = (int)ceil_div((int64_t)NH * Fp / 4, 64);
  int H = 2;
  while (H < 2 * NH) H *= 2;
  if (cpl <= 4 && cpl * H <= 32) {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(N, 4), 512);
#define GATX_NS(C, HH)                                                                         \
  if (cpl == C && H == HH) {                                                                   \
    node_scores_reg_kernel<C, HH><<<grid, 256, 0, st>>>(Wh, N, NH, F, Fp, a, S);               \
    GATX_LAUNCH_CHECK("node_scores");                                                          \
    return 0;                                                                                  \
  }
    GATX_NS(1, 2) GATX_NS(1, 4) GATX_NS(1, 8) GATX_NS(1, 16) GATX_NS(1, 32)
    GATX_NS(2, 2) GATX_NS(2, 4) GATX_NS(2, 8) GATX_NS(2, 16)
    GATX_NS(3, 2) GATX_NS(3, 4) GATX_NS(3, 8)
    GATX_NS(4, 2) GATX_NS(4, 4) GATX_NS(4, 8)
#undef GATX_NS
  }
  const size_t lds = (size_t)2 * NH * NH * Fp * sizeof(float);
  GATX_REQUIRE(lds <= 64 * 1024, "node_scores: attention vector too large for LDS");
  node_scores_kernel<<<(unsigned)std::min<int64_t>(ceil_div(N, 4), 1024), 256, lds, st>>>(
      Wh, N, NH, F, Fp, a, S);
  GATX_LAUNCH_CHECK("node_scores");
  return 0;
}

extern "C" int gatx_attention_alpha(const int32_t* col, const int32_t* rowidx,
                                    const int32_t* perm, int64_t E2, const float* S,
                                    const uint32_t* M_ord, const float* den, int NH,
                                    int const_att, float* alpha, int64_t* argmax,
                                    gatx_stream_t s) {
  if (E2 == 0) return 0;
  hipStream_t st = (hipStream_t)s;
  const unsigned grid = grid_for(E2, 256, 8192);
#define GATX_AL(C)                                                                             \
  do {                                                                                         \
    if (const_att) attention_alpha_kernel<C, true><<<grid, 256, 0, st>>>(                      \
        col, rowidx, perm, E2, S, M_ord, den, NH, alpha, (long long*)argmax);                  \
    else attention_alpha_kernel<C, false><<<grid, 256, 0, st>>>(                               \
        col, rowidx, perm, E2, S, M_ord, den, NH, alpha, (long long*)argmax);                  \
  } while (0)
  // the head-count variants load score / den rows and store alpha rows as vectors: only for
  // 16-byte aligned buffers (an offset view falls back to the scalar variant)
  const bool al = ((uintptr_t)S % 16) == 0 && ((uintptr_t)den % 16) == 0 &&
                  ((uintptr_t)alpha % 16) == 0;
  switch (al ? NH : 0) {
    case 1: GATX_AL(1); break; case 2: GATX_AL(2); break; case 4: GATX_AL(4); break;
    case 6: GATX_AL(6); break; case 8: GATX_AL(8); break; default: GATX_AL(0); break;
  }
#undef GATX_AL
  GATX_LAUNCH_CHECK("attention_alpha");
  return 0;
}

extern "C" int gatx_attention_alpha_ei(const void* edge_index, int is64, int64_t ld, int64_t E2,
                                       const int64_t* e2, const float* S, const uint32_t* M_ord,
                                       const float* den, int NH, int const_att,
                                       const int32_t* rowptr, const int32_t* perm, float* alpha,
                                       int64_t* argmax, gatx_stream_t s) {
  if (E2 == 0) return 0;
  GATX_REQUIRE(ld >= 0 || e2 != nullptr, "attention_alpha_ei: ld < 0 needs the device count");
  hipStream_t st = (hipStream_t)s;
  const unsigned grid = grid_for(ceil_div(E2, 4), 256, 8192);   // 4 edges per thread
  const long long* e2p = (const long long*)e2;
#define GATX_AE(C, I)                                                                          \
  do {                                                                                         \
    if (const_att) attention_alpha_ei_kernel<C, I, true><<<grid, 256, 0, st>>>(                \
        (const I*)edge_index, ld, E2, e2p, S, M_ord, den, NH, rowptr, perm, alpha,             \
        (long long*)argmax);                                                                   \
    else attention_alpha_ei_kernel<C, I, false><<<grid, 256, 0, st>>>(                         \
        (const I*)edge_index, ld, E2, e2p, S, M_ord, den, NH, rowptr, perm, alpha,             \
        (long long*)argmax);                                                                   \
  } while (0)
  // the head-count variants load score / den rows and store alpha rows as vectors
  const bool al = ((uintptr_t)S % 16) == 0 && ((uintptr_t)den % 16) == 0 &&
                  ((uintptr_t)alpha % 16) == 0;
#define GATX_AEI(I)                                                                            \
  switch (al ? NH : 0) {                                                                       \
    case 1: GATX_AE(1, I); break; case 2: GATX_AE(2, I); break; case 4: GATX_AE(4, I); break;  \
    case 6: GATX_AE(6, I); break; case 8: GATX_AE(8, I); break; default: GATX_AE(0, I); break; \
  }
  if (is64) { GATX_AEI(int64_t) } else { GATX_AEI(int32_t) }
#undef GATX_AEI
#undef GATX_AE
  GATX_LAUNCH_CHECK("attention_alpha_ei");
  return 0;
}

extern "C" int gatx_pad_rows(const float* src, int64_t rows, int64_t cols, int64_t ld_src,
                             float* dst, int64_t ld_dst, gatx_stream_t s) {
  GATX_REQUIRE(ld_dst >= cols, "pad_rows: destination narrower than source");
  if (rows == 0) return 0;
  pad_rows_kernel<<<grid_for(rows * ld_dst), 256, 0, (hipStream_t)s>>>(src, rows, cols, ld_src,
                                                                       dst, ld_dst);
  GATX_LAUNCH_CHECK("pad_rows");
  return 0;
}

extern "C" int gatx_attention_max(const int32_t* col, const int32_t* rowidx, int64_t E2,
                                  const int64_t* e2, const float* S, int NH, uint32_t* M_ord,
                                  int64_t* argmax, void* workspace, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(E2, 256), kMaxBlocks));
  float* part = (float*)workspace;
  const long long* e2p = (const long long*)e2;
  // S rows are float4/float2-aligned when 2*NH is a multiple of the vector width
  const bool al = ((uintptr_t)S % 16) == 0;
  if (E2 > 0 && al && NH == 4) attention_max_vec_kernel<4><<<nb, 256, 0, st>>>(col, rowidx, E2, e2p, S, part);
  else if (E2 > 0 && al && NH == 8) attention_max_vec_kernel<8><<<nb, 256, 0, st>>>(col, rowidx, E2, e2p, S, part);
  else if (E2 > 0 && al && NH == 6) attention_max_vec_kernel<6><<<nb, 256, 0, st>>>(col, rowidx, E2, e2p, S, part);
  else if (E2 > 0 && al && NH == 2) attention_max_vec_kernel<2><<<nb, 256, 0, st>>>(col, rowidx, E2, e2p, S, part);
  else if (E2 > 0 && NH == 1) attention_max_vec_kernel<1><<<nb, 256, 0, st>>>(col, rowidx, E2, e2p, S, part);
  else attention_max_kernel<<<nb, 256, 0, st>>>(col, rowidx, E2, e2p, S, NH, part);
  GATX_LAUNCH_CHECK("attention_max");
  max_final_kernel<<<1, 256, 0, st>>>(part, nb, M_ord, (long long*)argmax);
  GATX_LAUNCH_CHECK("attention_max_final");
  return 0;
}

extern "C" size_t gatx_attention_max_workspace_bytes(void) { return sizeof(float) * kMaxBlocks; }

extern "C" int gatx_edge_forward_ex(
    const float* rows, int64_t row_stride, int64_t head_stride, const float* S,
    const uint32_t* M_ord, const int32_t* rowptr, const int32_t* col, const int32_t* perm,
    int64_t N, int NH, int F, int heads_per_item, int group_begin, int group_count,
    int mean_mode, int concat, int const_att, const float* bias,
    float p, const uint64_t* seed, float* out, int64_t out_ld, const float* resid, int64_t resid_ld,
    int elu, float* den, int64_t chunk, gatx_stream_t s) {
  return gatx_edge_forward_hubs(rows, row_stride, head_stride, S, M_ord, rowptr, col, perm, N,
                                NH, F, heads_per_item, group_begin, group_count, mean_mode,
                                concat, const_att, bias, p, seed, out, out_ld, resid, resid_ld,
                                elu, den, chunk, 0, nullptr, nullptr, 0, nullptr, s);
}

extern "C" size_t gatx_edge_forward_hub_part_bytes(int64_t hub_bound, int NH, int F,
                                                   int heads_per_item, int group_count) {
  const int HS = heads_per_item <= 0 ? NH : heads_per_item;
  const int64_t W = (int64_t)HS * round_up(F, 4) + HS;
  return (size_t)hub_bound * (group_count > 0 ? group_count : NH / HS) * W * sizeof(float);
}

extern "C" int gatx_edge_forward_drop(
    const float* rows, int64_t row_stride, int64_t head_stride, const float* S,
    const uint32_t* M_ord, const int32_t* rowptr, const int32_t* col, const int32_t* perm,
    int64_t N, int NH, int F, int heads_per_item, int group_begin, int group_count,
    int mean_mode, int concat, int const_att, const float* bias,
    float p, const uint64_t* seed, float* out, int64_t out_ld, const float* resid, int64_t resid_ld,
    int elu, float* den, int64_t chunk, int hub_edges, const int32_t* hubs,
    const int32_t* hub_count, int64_t hub_bound, float* hub_part, float out_p,
    const uint64_t* out_seed, gatx_stream_t s) {
  return gatx_edge_forward_skip(rows, row_stride, head_stride, S, M_ord, rowptr, col, perm, N, NH,
                                F, heads_per_item, group_begin, group_count, mean_mode, concat,
                                const_att, bias, p, seed, out, out_ld, resid, resid_ld, elu, den,
                                chunk, hub_edges, hubs, hub_count, hub_bound, hub_part, out_p,
                                out_seed, nullptr, s);
}

extern "C" int gatx_edge_forward_skip(
    const float* rows, int64_t row_stride, int64_t head_stride, const float* S,
    const uint32_t* M_ord, const int32_t* rowptr, const int32_t* col, const int32_t* perm,
    int64_t N, int NH, int F, int heads_per_item, int group_begin, int group_count,
    int mean_mode, int concat, int const_att, const float* bias,
    float p, const uint64_t* seed, float* out, int64_t out_ld, const float* resid, int64_t resid_ld,
    int elu, float* den, int64_t chunk, int hub_edges, const int32_t* hubs,
    const int32_t* hub_count, int64_t hub_bound, float* hub_part, float out_p,
    const uint64_t* out_seed, const uint8_t* skip, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  GATX_REQUIRE(out_p >= 0.f && out_p < 1.f, "edge_forward: output dropout must be in [0, 1)");
  GATX_REQUIRE(out_p == 0.f || out_seed != nullptr,
               "edge_forward: output dropout needs its device seed");
  GATX_REQUIRE(out_p == 0.f || mean_mode == 0 || mean_mode == 3,
               "edge_forward: output dropout belongs to the last head-mean pass");
  GATX_REQUIRE(NH >= 1 && F >= 1, "edge_forward: bad sizes");
  GATX_REQUIRE(concat || bias == nullptr || NH == 1,
               "edge_forward: bias with head-mean needs num_heads == 1");
  const int HS = heads_per_item <= 0 ? NH : heads_per_item;
  GATX_REQUIRE(NH % HS == 0, "edge_forward: heads_per_item must divide num_heads");
  const int NGall = NH / HS;
  if (group_count <= 0) { group_begin = 0; group_count = NGall; }
  GATX_REQUIRE(group_begin >= 0 && group_begin + group_count <= NGall,
               "edge_forward: head groups out of range");
  GATX_REQUIRE(mean_mode >= 0 && mean_mode <= 3, "edge_forward: bad mean_mode");
  GATX_REQUIRE(concat || (mean_mode == 0 ? HS == NH : group_count == 1),
               "edge_forward: head mean in one pass needs all heads in one item, multi-pass "
               "one head group per launch");
  GATX_REQUIRE(!concat || mean_mode == 0, "edge_forward: mean_mode needs concat == 0");
  GATX_REQUIRE(mean_mode == 0 || mean_mode == 3 || (resid == nullptr && !elu && !bias),
               "edge_forward: the epilogue belongs to the last head-mean pass");
  GATX_REQUIRE(row_stride % 4 == 0 && head_stride % 4 == 0 && ((uintptr_t)rows % 16) == 0,
               "edge_forward: source rows must be float4-aligned");
  GATX_REQUIRE(p >= 0.f && p < 1.f, "edge_forward: dropout must be in [0, 1)");
  GATX_REQUIRE(p == 0.f || seed != nullptr, "edge_forward: dropout needs the device seed");
  if (N == 0) return 0;
  const int Fp = (int)round_up(F, 4);
  const int64_t D4 = (int64_t)HS * Fp / 4;
  const RowGeom rg = row_geom(D4);
  GATX_REQUIRE(rg.cpl <= 8, "edge_forward: heads_per_item*out_features > 2048 unsupported");
  EdgeFwdArgs g;
  g.rows = rows; g.row_stride4 = row_stride / 4; g.head_stride4 = (int)(head_stride / 4);
  g.S = S; g.M_ord = M_ord; g.rowptr = rowptr; g.col = col; g.perm = perm;
  g.N = N; g.NH = NH; g.F = F; g.Fp = Fp; g.HS = HS; g.concat = concat; g.const_att = const_att;
  g.bias = bias; g.p_drop = p; g.seed = seed; g.out = out; g.out_ld = out_ld;
  g.resid = resid; g.resid_ld = resid_ld; g.elu = elu;
  g.out_p = out_p; g.out_seed = out_seed; g.out_cols = concat ? (int64_t)NH * F : F;
  g.den = den;
  g.skip = skip;
  g.vec_out = concat && (F & 3) == 0 && out_ld % 4 == 0 && ((uintptr_t)out % 16) == 0 &&
              (!resid || (resid_ld % 4 == 0 && ((uintptr_t)resid % 16) == 0)) &&
              (!bias || ((uintptr_t)bias % 16) == 0);
  GATX_REQUIRE(HS <= kMaxHS, "edge_forward: more than %d heads per work item", kMaxHS);
  g.lds_row = (int)round_up((int64_t)HS * Fp + HS + 64 + (int64_t)HS * 64, 4);
  g.chunk = chunk > 0 ? chunk : 2048;
  g.dbg = g_debug;
  g.g_begin = group_begin; g.g_count = group_count; g.mean_mode = concat ? 0 : mean_mode;
  g.n_items_main = ceil_div(N, g.chunk) * g.chunk * group_count;
  g.hub_T = 0; g.hubs = nullptr; g.hub_count = nullptr; g.hub_bound = 0; g.hub_part = nullptr;
  if (hub_edges > 0 && hub_bound > 0) {
    GATX_REQUIRE(hubs && hub_count && hub_part, "edge_forward: hub splitting needs its buffers");
    g.hub_T = hub_edges; g.hubs = hubs; g.hub_count = hub_count; g.hub_bound = hub_bound;
    g.hub_part = hub_part;
  }
  g.n_items = g.n_items_main + g.hub_bound * group_count;
  g.hub_blocks = round_up(ceil_div(g.hub_bound * group_count, 4), 8);
  const size_t lds = (size_t)4 * g.lds_row * sizeof(float);
  GATX_REQUIRE(lds <= 160 * 1024, "edge_forward: row too wide for LDS staging");
  const int64_t blocks = g.hub_blocks + ceil_div(g.n_items_main, 4);
  GATX_REQUIRE(blocks < (1ll << 31), "edge_forward: too many work items");
  const unsigned grid = (unsigned)blocks;
  // rows shared by every head (the reassociated first layer): one lane per chunk for all heads
  if (head_stride == 0 && concat && !resid && !elu && !bias && out_p == 0.f &&
      Fp / 4 <= 64 && (HS == 1 || HS == 2 || HS == 4 || HS == 8)) {
    int lpe = 1;
    while (lpe < Fp / 4) lpe <<= 1;
    EdgeFwdArgs gs = g;
    const int hsp = HS <= 4 ? 4 : 8;
    gs.lds_row = 64 + 64 * hsp + 8;
    const size_t slds = (size_t)4 * gs.lds_row * sizeof(float);
#define GATX_SH(L)                                                                             \
  do {                                                                                         \
    if (HS == 1) edge_forward_shared_kernel<L, 1><<<grid, 256, slds, st>>>(gs);                \
    else if (HS == 2) edge_forward_shared_kernel<L, 2><<<grid, 256, slds, st>>>(gs);           \
    else if (HS == 4) edge_forward_shared_kernel<L, 4><<<grid, 256, slds, st>>>(gs);           \
    else edge_forward_shared_kernel<L, 8><<<grid, 256, slds, st>>>(gs);                        \
  } while (0)
    switch (lpe) {
      case 1: GATX_SH(1); break; case 2: GATX_SH(2); break; case 4: GATX_SH(4); break;
      case 8: GATX_SH(8); break; case 16: GATX_SH(16); break; case 32: GATX_SH(32); break;
      default: GATX_SH(64); break;
    }
#undef GATX_SH
    GATX_LAUNCH_CHECK("edge_forward_shared");
    if (g.hub_T > 0) {   // the generic combine over the generic partial layout
      const unsigned cg = (unsigned)ceil_div(g.hub_bound * g.g_count, 4);
#define GATX_HC(L, C) edge_hub_combine_kernel<L, C><<<cg, 256, lds, st>>>(g)
      if (rg.lpe == 64) {
        switch (rg.cpl) {
          case 1: GATX_HC(64, 1); break; case 2: GATX_HC(64, 2); break;
          case 3: GATX_HC(64, 3); break; case 4: GATX_HC(64, 4); break;
          case 5: GATX_HC(64, 5); break; case 6: GATX_HC(64, 6); break;
          case 7: GATX_HC(64, 7); break; default: GATX_HC(64, 8); break;
        }
      } else {
        switch (rg.lpe) {
          case 1: GATX_HC(1, 1); break; case 2: GATX_HC(2, 1); break; case 4: GATX_HC(4, 1); break;
          case 8: GATX_HC(8, 1); break; case 16: GATX_HC(16, 1); break; default: GATX_HC(32, 1); break;
        }
      }
#undef GATX_HC
      GATX_LAUNCH_CHECK("edge_hub_combine");
    }
    return 0;
  }
#define GATX_EF(L, C) return launch_edge_forward<L, C>(grid, lds, st, g)
  if (rg.lpe == 64) {
    switch (rg.cpl) {
      case 1: GATX_EF(64, 1); case 2: GATX_EF(64, 2); case 3: GATX_EF(64, 3);
      case 4: GATX_EF(64, 4); case 5: GATX_EF(64, 5); case 6: GATX_EF(64, 6);
      case 7: GATX_EF(64, 7); default: GATX_EF(64, 8);
    }
  }
  switch (rg.lpe) {
    case 1: GATX_EF(1, 1); case 2: GATX_EF(2, 1); case 4: GATX_EF(4, 1);
    case 8: GATX_EF(8, 1); case 16: GATX_EF(16, 1); default: GATX_EF(32, 1);
  }
#undef GATX_EF
}

extern "C" int gatx_edge_forward(const float* Wh, const float* S, const uint32_t* M_ord,
                                 const int32_t* rowptr, const int32_t* col,
                                 const int32_t* rowidx, const int32_t* perm, int64_t N,
                                 int64_t E2, int NH, int F, int concat, int const_att,
                                 const float* bias, float p,
                                 const uint64_t* seed, float* out, float* alpha, float* den,
                                 int64_t* argmax, gatx_stream_t s) {
  const int64_t Fp = round_up(F, 4);
  GATX_CALL(gatx_edge_forward_ex(Wh, NH * Fp, Fp, S, M_ord, rowptr, col, perm, N, NH, F,
                                 concat ? 0 : NH, 0, 0, 0, concat, const_att, bias, p, seed, out,
                                 concat ? (int64_t)NH * F : F, nullptr, 0, 0, den, 0, s));
  return gatx_attention_alpha(col, rowidx, perm, E2, S, M_ord, den, NH, const_att,
                              alpha, argmax, s);
}

extern "C" int gatx_edge_forward_hubs(
    const float* rows, int64_t row_stride, int64_t head_stride, const float* S,
    const uint32_t* M_ord, const int32_t* rowptr, const int32_t* col, const int32_t* perm,
    int64_t N, int NH, int F, int heads_per_item, int group_begin, int group_count,
    int mean_mode, int concat, int const_att, const float* bias,
    float p, const uint64_t* seed, float* out, int64_t out_ld, const float* resid, int64_t resid_ld,
    int elu, float* den, int64_t chunk, int hub_edges, const int32_t* hubs,
    const int32_t* hub_count, int64_t hub_bound, float* hub_part, gatx_stream_t s) {
  return gatx_edge_forward_drop(rows, row_stride, head_stride, S, M_ord, rowptr, col, perm, N, NH,
                                F, heads_per_item, group_begin, group_count, mean_mode, concat,
                                const_att, bias, p, seed, out, out_ld, resid, resid_ld, elu, den,
                                chunk, hub_edges, hubs, hub_count, hub_bound, hub_part, 0.f,
                                nullptr, s);
}

namespace gatx {
namespace {
// GATModel's input dropout (models/GATModel.py:130) as a counter-based mask on the element
// index, the same hash as the attention dropout and the fused epilogue's: y = keep ? x / (1 - p)
// : 0. Its own backward (the gradient takes the same mask and scale).
__global__ void __launch_bounds__(256) dropout_kernel(const float* __restrict__ x, int64_t n,
                                                      float p, const uint64_t* __restrict__ seed,
                                                      float* __restrict__ y) {
  const uint64_t sd = *seed;
  const float scale = 1.f / (1.f - p);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x)
    y[t] = dropout_keep(sd, t, p) ? x[t] * scale : 0.f;
}
}  // namespace
}  // namespace gatx

extern "C" int gatx_dropout(const float* x, int64_t n, float p, const uint64_t* seed, float* y,
                            gatx_stream_t s) {
  GATX_REQUIRE(n >= 0 && p >= 0.f && p < 1.f, "dropout: bad arguments");
  GATX_REQUIRE(seed != nullptr, "dropout: needs the device seed");
  if (n == 0) return 0;
  dropout_kernel<<<grid_for(n), 256, 0, (hipStream_t)s>>>(x, n, p, seed, y);
  GATX_LAUNCH_CHECK("dropout");
  return 0;
}
