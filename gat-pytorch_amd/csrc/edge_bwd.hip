// Backward of the GATLayer attention + aggregation: the closed form of torch autograd through
// models/gat_layer.py:64-135, as passes over the two CSR orders.
//
//   prepare_go  go = g_out * elu'(out) (fused-epilogue layers), scaled 1/NH for head-mean layers,
//               written head-padded [N][NH][Fp] (or [N][Fp] for head-mean) so every later gather is
//               an aligned float4; optionally also the residual's gradient.
//   dst pass    one wave per (destination n, head h): g_alpha~[e] = <go[n,h,:], Wh[src_e,h,:]>
//               (go in registers, Wh rows gathered with a wave-uniform scalar address, the dot
//               reduced with DPP + permlane swaps), then softmax backward:
//               c = sum_e g_alpha alpha, g_raw'[e] = 0.01 ex (g_alpha - c) / (den + 1e-8),
//               g_s_dst[n,h] = sum_e g_raw'  (g_raw' stored head-major [NH][E2] in CSR order).
//   max bwd     g_M = -sum g_raw' (= -sum g_s_dst), split evenly over the argmax entries.
//   src pass    one wave per (source s, head h): the message gradient sum alpha~ go[dst] (go rows
//               gathered like the forward gathers Wh rows) and g_s_src = sum g_raw' + max share,
//               written as one row of G_aug = [g_Wh | g_s_src | g_s_dst]. Head-mean layers
//               (go one row per node, shared by every head) use one wave per source for all
//               heads, so each go[dst] row is gathered once per edge instead of NH times.
// The weight/input gradients then come from two MFMA GEMMs on G_aug (gemm.hip) and
// gatx_weight_grads. No float atomics on the data path: every sum has a fixed order (bitwise
// reproducible), except the tie-split of max()'s gradient when several argmax entries share a node.
#include "gatx_common.h"

namespace gatx {
namespace {

inline unsigned grid_for(int64_t n, int block = 256, int64_t cap = 16384) {
  int64_t g = ceil_div(n > 0 ? n : 1, block);
  return (unsigned)(g < cap ? g : cap);
}

__device__ inline int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline float lane_f(float v, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}
__device__ inline int64_t xcd_contiguous(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, xcd = b % 8, j = b / 8;
  return (xcd < r) ? xcd * (q + 1) + j : r * (q + 1) + (xcd - r) * q + j;
}

// (node, head) work item -> n, h with chunked sweeps (one head over `chunk` nodes at a time).
__device__ inline bool decode_item(int64_t item, int64_t N, int NH, int64_t chunk, int64_t& n,
                                   int& h) {
  const int64_t per_chunk = chunk * NH;
  const int64_t ck = item / per_chunk, rem = item - ck * per_chunk;
  h = (int)(rem / chunk);
  n = ck * chunk + (rem - (int64_t)h * chunk);
  return n < N;
}

// go [N][GW] (GW = NH*Fp concat, Fp head-mean): elu-gated, 1/NH-scaled, head-padded g_out.
__global__ void __launch_bounds__(256) prepare_go_kernel(const float* __restrict__ g_out,
                                                         const float* __restrict__ out,
                                                         int64_t N, int NH, int F, int Fp,
                                                         int concat, int elu,
                                                         float* __restrict__ go,
                                                         float* __restrict__ g_pre,
                                                         int64_t pre_ld, float out_p,
                                                         const uint64_t* __restrict__ out_seed) {
  const int OC = concat ? NH * F : F, GW = concat ? NH * Fp : Fp;
  const float scale = concat ? 1.f : 1.f / (float)NH;
  // the next layer's input dropout fused into this layer's epilogue: out holds the dropped
  // output, g_out its gradient — take the mask's gradient, and ELU's from out * (1 - p)
  const uint64_t osd = out_p > 0.f ? *out_seed : 0ull;
  const float oscale = out_p > 0.f ? 1.f / (1.f - out_p) : 1.f;
  const int64_t total = N * GW;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = t / GW;
    const int c = (int)(t - n * GW), h = c / Fp, f = c - h * Fp;
    float v = 0.f;
    if (f < F) {
      const int64_t src = n * OC + (concat ? h * F + f : f);
      v = g_out[src];
      if (out_p > 0.f) v = dropout_keep(osd, src, out_p) ? v * oscale : 0.f;
      if (elu) {
        const float o = out_p > 0.f ? out[src] * (1.f - out_p) : out[src];
        v = o > 0.f ? v : v * (o + 1.f);   // d elu(x) = elu(x) + 1 for x <= 0
      }
      if (g_pre) g_pre[n * pre_ld + (concat ? h * F + f : f)] = v;
    }
    go[t] = v * scale;
  }
}

// The same for F % 4 == 0 (Fp == F: go has g_out's layout): float4 streams, 4 per thread per
// round with all loads issued before any store (loads and stores share vmcnt). g_pre == go is
// allowed (the caller then reads the residual gradient from go).
__global__ void __launch_bounds__(256) prepare_go_vec_kernel(const float4* __restrict__ g_out,
                                                             const float4* __restrict__ out,
                                                             int64_t n4, int elu, float scale,
                                                             float4* go, float4* g_pre) {
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t0 < n4; t0 += U * stride) {
    float4 v[U], o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t t = t0 + u * stride;
      if (t < n4) {
        v[u] = g_out[t];
        if (elu) o[u] = out[t];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t t = t0 + u * stride;
      if (t >= n4) continue;
      float4 w = v[u];
      if (elu) {   // d elu(x) = elu(x) + 1 for x <= 0
        w.x = o[u].x > 0.f ? w.x : w.x * (o[u].x + 1.f);
        w.y = o[u].y > 0.f ? w.y : w.y * (o[u].y + 1.f);
        w.z = o[u].z > 0.f ? w.z : w.z * (o[u].z + 1.f);
        w.w = o[u].w > 0.f ? w.w : w.w * (o[u].w + 1.f);
      }
      if (g_pre && g_pre != go) g_pre[t] = w;
      go[t] = make_float4(w.x * scale, w.y * scale, w.z * scale, w.w * scale);
    }
  }
}

struct BwdArgs {
  const float* Wh;      // [N][Dp]
  const float* go;      // prepared upstream gradient rows
  int64_t go_stride4;   // float4s per go row
  int go_head4;         // float4s between heads in a go row (0 for head-mean)
  const float* S;
  const uint32_t* M_ord;
  const float* den;
  const int32_t* rowptr;   // dst CSR (dst pass) / src CSR (src pass)
  const int32_t* col;      // src of each dst-CSR slot / dst of each src-CSR slot
  const int32_t* seid;     // src pass: dst-CSR slot of each src-CSR slot
  const int32_t* perm;
  int64_t N, E2;
  int NH, F, Fp, const_att;
  float p_drop;
  const uint64_t* seed;    // device scalar
  const float* g_alpha_ret;
  float* g_raw;            // [NH][E2] head-major, dst-CSR order
  float* gsd;              // [N][NH] compact copy of g_s_dst (for max()'s gradient)
  const float* g_corr;     // [N][NH] max() share for the src pass
  float* G_aug;
  int64_t ldg, chunk, n_items;
  int64_t row_stride4;     // dst pass: float4s per gathered row (Wh: Dp/4; x rows: Fin_p/4)
  int64_t head_stride4;    // float4s between heads in a gathered row (0: one row for all heads)
  int64_t gs_off;          // column of g_s_src in G_aug (g_s_dst at gs_off + NH)
  // hub splitting (hub_T > 0): segments of more than hub_T edges are skipped by their own item
  // and processed as pieces of hub_T edges (gatx_graph_hub_plan over this pass's CSR) by the
  // waves of the first hub_blocks blocks (dispatched first, dealt over the XCDs), each leaving a
  // partial in hub_part; follow-up kernels combine a hub's pieces in piece order.
  int hub_T;
  const int32_t* hubs;     // [hub_bound][4]: node, piece, pieces, first slot
  const int32_t* hub_count;
  int64_t hub_bound;
  float* hub_part;         // dst: [2][hub_bound][NH]; src: [hub_bound][NH][Fp + 4]
  int64_t hub_blocks;
};

// Work of one wave of a hub-split pass: a regular item (slot < 0) or one piece of a hub (slot =
// its plan entry). Returns false when the wave has nothing to do.
__device__ inline bool hub_piece(const BwdArgs& g, int wave, int64_t& n, int& h, int& beg,
                                 int& end, int64_t& slot) {
  const int64_t hi = (int64_t)blockIdx.x * 4 + wave;
  h = (int)(hi / g.hub_bound);
  const int64_t pc = hi - (int64_t)h * g.hub_bound;
  if (h >= g.NH || pc >= uni(*g.hub_count)) return false;
  const int32_t* hp = g.hubs + 4 * pc;
  n = uni(hp[0]);
  const int p = uni(hp[1]);
  slot = pc;
  beg = uni(g.rowptr[n]) + p * g.hub_T;
  end = min(uni(g.rowptr[n + 1]), beg + g.hub_T);
  return true;
}

// dst pass: one wave per (destination n, head h); LPE lanes per edge over the head's Fp/4
// chunks (CPL per lane), 64/LPE edges per step.
template <int LPE, int CPL>
__global__ void __launch_bounds__(256) edge_bwd_dst_kernel(BwdArgs g) {
  constexpr int EPW = 64 / LPE;
  constexpr int U = CPL <= 1 ? 4 : 2;
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int grp = lane / LPE, li = lane % LPE;
  const int64_t hb = g.hub_blocks;
  int64_t n, slot = -1;
  int h, beg, end;
  if ((int64_t)blockIdx.x < hb) {   // one piece of a hub: sweep 1 only (g_alpha, partial c)
    if (!hub_piece(g, wave, n, h, beg, end, slot)) return;
  } else {
    const int64_t item = xcd_contiguous(blockIdx.x - hb, gridDim.x - hb) * 4 + wave;
    if (item >= g.n_items) return;
    if (!decode_item(item, g.N, g.NH, g.chunk, n, h)) return;
    beg = uni(g.rowptr[n]);
    end = uni(g.rowptr[n + 1]);
    if (g.hub_T > 0 && end - beg > g.hub_T) return;   // done in pieces
  }
  const bool keep0 = slot < 0;   // a piece stores every g_alpha for the hub kernels
  const int NH = g.NH, Fp = g.Fp, F4 = Fp / 4, S2 = 2 * NH;
  const int64_t E2 = g.E2;
  const float M = ord_to_float(*g.M_ord);
  const bool drop = g.p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  const uint64_t seed = drop ? *g.seed : 0ull;
  const float4* __restrict__ Wh4 = (const float4*)g.Wh;
  const float4* __restrict__ go4 = (const float4*)g.go;

  int off4[CPL];
  bool vq[CPL];
  float4 gv[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int q = c * LPE + li;
    vq[c] = q < F4;
    off4[c] = (int)(h * g.head_stride4) + (vq[c] ? q : 0);
    gv[c] = vq[c] ? go4[n * g.go_stride4 + h * g.go_head4 + q] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float sdst = g.S[n * S2 + NH + h];
  const float dinv = 1.f / (g.den[n * NH + h] + kSoftmaxEps);
  float* __restrict__ graw = g.g_raw + (int64_t)h * E2;
  __shared__ int src_sh[4][64];
  __shared__ float dot_sh[4][64];
  int* src_lds = src_sh[wave];
  float* dot_lds = dot_sh[wave];

  // sweep 1: g_alpha per edge, c = sum g_alpha * alpha. The first 64 edges' g_alpha and exp
  // stay in registers for sweep 2 (at PPI that is every edge of nearly every node); later
  // batches go through g_raw. Besides the reload, a store ahead of sweep 2's loads would make
  // them wait for it to reach memory (loads and stores share vmcnt).
  float c_acc = 0.f, ga0 = 0.f, ex0 = 0.f;
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const bool valid = lane < cnt;
    const int e = base + min(lane, cnt - 1);
    const int my_src = g.col[e];
    const float ex = att_exp(g.S[(int64_t)my_src * S2 + h] + sdst, M);
    if (EPW > 1) src_lds[lane] = my_src;
    if (EPW > 1) wave_lds_sync();
    float my_dot = 0.f;
    // U rows in flight per lane group: all loads of a step issue before any reduction
    for (int j0 = grp; j0 < cnt; j0 += EPW * U) {
      float4 v[U][CPL];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = min(j0 + u * EPW, cnt - 1);
        const int sj = (EPW == 1) ? __builtin_amdgcn_readlane(my_src, jj) : src_lds[jj];
        const float4* rp = Wh4 + (int64_t)sj * g.row_stride4;
#pragma unroll
        for (int c = 0; c < CPL; ++c) v[u][c] = rp[off4[c]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = j0 + u * EPW;
        float p = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c)
          p += gv[c].x * v[u][c].x + gv[c].y * v[u][c].y + gv[c].z * v[u][c].z +
               gv[c].w * v[u][c].w;
        p = group_sum<LPE>(p);
        if (EPW == 1) {
          if (lane == jj) my_dot = p;
        } else if (li == 0 && jj < cnt) {
          dot_lds[jj] = p;
        }
      }
    }
    if (EPW > 1) {
      wave_lds_sync();
      my_dot = dot_lds[lane];
      wave_lds_sync();
    }
    if (valid) {
      float ga = my_dot;
      if (drop) ga = dropout_keep(seed, (int64_t)g.perm[e] * NH + h, g.p_drop) ? ga * drop_scale : 0.f;
      if (g.g_alpha_ret) ga += g.g_alpha_ret[(int64_t)g.perm[e] * NH + h];
      if (base == beg && keep0) {
        ga0 = ga;
        ex0 = ex;
      } else {
        graw[e] = ga;
      }
      c_acc += ga * ex * dinv;
    }
  }
  const float cc = group_sum<64>(c_acc);
  if (!keep0) {   // the piece's share of c; edge_bwd_dst_hub_kernel finishes the hub
    if (lane == 0) g.hub_part[slot * NH + h] = cc;
    return;
  }
  // sweep 2 (same lane <-> edge map, so each lane re-reads only its own stores)
  float gsum = 0.f;
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    if (e < end) {
      const bool first = base == beg;
      const float ex = first ? ex0 : att_exp(g.S[(int64_t)g.col[e] * S2 + h] + sdst, M);
      const float gr = kLeakySlope * ex * ((first ? ga0 : graw[e]) - cc) * dinv;
      graw[e] = gr;
      gsum += gr;
    }
  }
  gsum = group_sum<64>(gsum);
  if (lane == 0) {
    g.G_aug[n * g.ldg + g.gs_off + NH + h] = gsum;
    g.gsd[n * NH + h] = gsum;
  }
}

// Sweep 2 of a hub-split destination segment, one wave per piece: c = the hub's piece partials
// summed in piece order, then g_raw' of the piece's edges (from the g_alpha sweep 1 stored) and
// the piece's share of g_s_dst into hub_part[hub_bound + slot].
__global__ void __launch_bounds__(256) edge_bwd_dst_hub_kernel(BwdArgs g) {
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  int64_t n, slot;
  int h, beg, end;
  if (!hub_piece(g, wave, n, h, beg, end, slot)) return;
  const int NH = g.NH, S2 = 2 * NH;
  const int32_t* hp = g.hubs + 4 * slot;
  const int pieces = uni(hp[2]), first = uni(hp[3]);
  float cc = 0.f;
  for (int q = 0; q < pieces; ++q) cc += g.hub_part[(int64_t)(first + q) * NH + h];
  const float M = ord_to_float(*g.M_ord);
  const float sdst = g.S[n * S2 + NH + h];
  const float dinv = 1.f / (g.den[n * NH + h] + kSoftmaxEps);
  float* __restrict__ graw = g.g_raw + (int64_t)h * g.E2;
  float gsum = 0.f;
  for (int e = beg + lane; e < end; e += 64) {
    const float ex = att_exp(g.S[(int64_t)g.col[e] * S2 + h] + sdst, M);
    const float gr = kLeakySlope * ex * (graw[e] - cc) * dinv;
    graw[e] = gr;
    gsum += gr;
  }
  gsum = group_sum<64>(gsum);
  if (lane == 0) g.hub_part[g.hub_bound * NH + slot * NH + h] = gsum;
}

// g_s_dst of a hub: its pieces' shares summed in piece order (one wave per hub and head: the
// wave of the hub's first piece).
__global__ void __launch_bounds__(256) edge_bwd_dst_hub_finish_kernel(BwdArgs g) {
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  int64_t n, slot;
  int h, beg, end;
  if (!hub_piece(g, wave, n, h, beg, end, slot)) return;
  const int32_t* hp = g.hubs + 4 * slot;
  if (uni(hp[1]) != 0) return;
  const int NH = g.NH, pieces = uni(hp[2]);
  float gsum = 0.f;
  for (int q = 0; q < pieces; ++q) gsum += g.hub_part[g.hub_bound * NH + (slot + q) * NH + h];
  if (lane == 0) {
    g.G_aug[n * g.ldg + g.gs_off + NH + h] = gsum;
    g.gsd[n * NH + h] = gsum;
  }
}

// Source-side logit gradients only (no message gradient; the reassociated first layer, whose
// input needs no gradient): G[s][gs_off + h] = sum over s's out-edges of g_raw'[h] + max share.
// One wave per source, lanes over its edges, fixed-order wave sums.
template <int NHC>
__global__ void __launch_bounds__(256) src_scores_kernel(const int32_t* __restrict__ srowptr,
                                                         const int32_t* __restrict__ seid,
                                                         int64_t N, int64_t E2, int NH_rt,
                                                         const float* __restrict__ g_raw,
                                                         const float* __restrict__ g_corr,
                                                         float* __restrict__ G, int64_t ldg,
                                                         int64_t gs_off) {
  const int NH = NHC > 0 ? NHC : NH_rt;
  const int lane = threadIdx.x & 63;
  const int64_t s = blockIdx.x * 4ll + uni(threadIdx.x >> 6);
  if (s >= N) return;
  const int beg = uni(srowptr[s]), end = uni(srowptr[s + 1]);
  float acc[8];
#pragma unroll
  for (int h = 0; h < 8; ++h) acc[h] = 0.f;
  for (int j = beg + lane; j < end; j += 64) {
    const int64_t e = seid[j];
#pragma unroll
    for (int h = 0; h < 8; ++h)
      if (h < NH) acc[h] += g_raw[(int64_t)h * E2 + e];
  }
#pragma unroll
  for (int h = 0; h < 8; ++h) {
    if (h >= NH) break;
    const float v = group_sum<64>(acc[h]);
    if (lane == 0) G[s * ldg + gs_off + h] = v + (g_corr ? g_corr[s * NH + h] : 0.f);
  }
}

// max() backward: g_M = -sum_{n,h} g_s_dst[n,h] (two-stage fixed-order reduction of the compact
// g_s_dst copy), split evenly over the k tied argmax entries recorded by the forward.
constexpr int kSumBlocks = 1024;

__global__ void __launch_bounds__(256) sum_partial_kernel(const float* __restrict__ x, int64_t n,
                                                          float* __restrict__ part) {
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    s += x[i];
  s = group_sum<64>(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) max_bwd_kernel(const float* __restrict__ part, int nb,
                                                      const long long* __restrict__ argmax,
                                                      const int32_t* __restrict__ col,
                                                      const int32_t* __restrict__ rowidx, int NH,
                                                      float* __restrict__ g_corr_src,
                                                      float* __restrict__ G_aug, int64_t ldg,
                                                      int64_t Dp, float* __restrict__ gm_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) s += part[b];
  s = group_sum<64>(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float total = (red[0] + red[1]) + (red[2] + red[3]);
  const long long k = argmax[0];
  if (k <= 0) return;
  const float share = -total / (float)k;
  gm_out[0] = share;
  if (k > GATX_ARGMAX_CAP) return;   // handled by the full-scan kernel
  for (long long j = 0; j < k; ++j) {   // sequential: k is small (ties)
    const long long ent = argmax[1 + j];
    const long long e = ent / NH;
    const int h = (int)(ent - e * NH);
    if (g_corr_src) g_corr_src[(int64_t)col[e] * NH + h] += share;
    else G_aug[(int64_t)col[e] * ldg + Dp + h] += share;   // after the src pass wrote g_s_src
    G_aug[(int64_t)rowidx[e] * ldg + Dp + NH + h] += share;
  }
}

// Fallback when more than GATX_ARGMAX_CAP entries tie: rescan every (edge, head).
__global__ void __launch_bounds__(256) max_bwd_scan_kernel(const float* __restrict__ S,
                                                           const uint32_t* __restrict__ M_ord,
                                                           const int32_t* __restrict__ col,
                                                           const int32_t* __restrict__ rowidx,
                                                           int64_t E2b, const long long* e2p,
                                                           int NH,
                                                           const long long* __restrict__ argmax,
                                                           const float* __restrict__ gm,
                                                           float* __restrict__ g_corr_src,
                                                           float* __restrict__ G_aug,
                                                           int64_t ldg, int64_t Dp) {
  if (argmax[0] <= GATX_ARGMAX_CAP) return;
  const int64_t E2 = e2p ? min(E2b, (int64_t)*e2p) : E2b;
  const float M = ord_to_float(*M_ord), share = gm[0];
  const int S2 = 2 * NH;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < E2 * NH;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / NH;
    const int h = (int)(t - e * NH);
    const int64_t s = col[e], d = rowidx[e];
    if (S[s * S2 + h] + S[d * S2 + NH + h] == M) {
      if (g_corr_src) atomicAdd(&g_corr_src[s * NH + h], share);
      else atomicAdd(&G_aug[s * ldg + Dp + h], share);
      atomicAdd(&G_aug[d * ldg + Dp + NH + h], share);
    }
  }
}

// src pass: one wave per (source s, head h); gathers go rows of the destinations with weights
// alpha~ = keep * exp(0.01 (s_src[s] + s_dst[d] - M)) / (den[d] + 1e-8) computed lane-parallel
// per 64-edge batch (the forward's structure with the roles of src and dst swapped).
template <int LPE, int CPL>
__global__ void __launch_bounds__(256) edge_bwd_src_kernel(BwdArgs g) {
  constexpr int EPW = 64 / LPE;
  constexpr int U = CPL <= 1 ? 8 : (CPL <= 2 ? 4 : 2);
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int grp = lane / LPE, li = lane % LPE;
  const int64_t hb = g.hub_blocks;
  int64_t s, slot = -1;
  int h, beg, end;
  if ((int64_t)blockIdx.x < hb) {   // one piece of a hub source: a partial row
    if (!hub_piece(g, wave, s, h, beg, end, slot)) return;
  } else {
    const int64_t item = xcd_contiguous(blockIdx.x - hb, gridDim.x - hb) * 4 + wave;
    if (item >= g.n_items) return;
    if (!decode_item(item, g.N, g.NH, g.chunk, s, h)) return;
    beg = uni(g.rowptr[s]);
    end = uni(g.rowptr[s + 1]);
    if (g.hub_T > 0 && end - beg > g.hub_T) return;   // done in pieces
  }
  const int NH = g.NH, Fp = g.Fp, F4 = Fp / 4, S2 = 2 * NH;
  const int64_t Dp = (int64_t)NH * Fp, E2 = g.E2;
  const float M = g.const_att ? 0.f : ord_to_float(*g.M_ord);
  const bool drop = g.p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  const uint64_t seed = drop ? *g.seed : 0ull;
  const float4* __restrict__ go4 = (const float4*)g.go;
  __shared__ int src_sh[4][64];
  __shared__ float w_sh[4][64];
  int* src_lds = src_sh[wave];
  float* w_lds = w_sh[wave];

  int off4[CPL];
  bool vq[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int q = c * LPE + li;
    vq[c] = q < F4;
    off4[c] = h * g.go_head4 + (vq[c] ? q : 0);
  }
  const float ssrc = g.const_att ? 0.f : g.S[s * S2 + h];
  float4 acc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  float gs = 0.f;
  const float* __restrict__ graw = g.g_raw ? g.g_raw + (int64_t)h * E2 : nullptr;

  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const bool valid = lane < cnt;
    const int j = base + min(lane, cnt - 1);
    const int d = g.col[j];
    const int e = g.seid[j];
    float w = 0.f;
    if (valid) {
      const float ex = g.const_att ? 1.f : att_exp(ssrc + g.S[(int64_t)d * S2 + NH + h], M);
      w = ex / (g.den[(int64_t)d * NH + h] + kSoftmaxEps);
      if (drop) w = dropout_keep(seed, (int64_t)g.perm[e] * NH + h, g.p_drop) ? w * drop_scale : 0.f;
      if (graw) gs += graw[e];
    }
    if (EPW > 1) {
      src_lds[lane] = d;
      w_lds[lane] = w;
      wave_lds_sync();
    }
    if constexpr (EPW == 1) {
      for (int j0 = 0; j0 < cnt; j0 += U) {
        const float4* rp[U];
        float wsc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int jj = min(j0 + u, cnt - 1);
          rp[u] = go4 + (int64_t)__builtin_amdgcn_readlane(d, jj) * g.go_stride4;
          wsc[u] = (j0 + u < cnt) ? lane_f(w, jj) : 0.f;
        }
        float4 v[U][CPL];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int c = 0; c < CPL; ++c) v[u][c] = rp[u][off4[c]];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int c = 0; c < CPL; ++c) acc[c] = fma4(wsc[u], v[u][c], acc[c]);
      }
    } else {
      for (int j0 = grp; j0 < cnt; j0 += EPW * U) {
        float4 v[U][CPL];
        float wj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int jj = j0 + u * EPW;
          const int jc = min(jj, cnt - 1);
          const float4* rp = go4 + (int64_t)src_lds[jc] * g.go_stride4;
          wj[u] = jj < cnt ? w_lds[jc] : 0.f;
#pragma unroll
          for (int c = 0; c < CPL; ++c) v[u][c] = rp[off4[c]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int c = 0; c < CPL; ++c) acc[c] = fma4(wj[u], v[u][c], acc[c]);
      }
      wave_lds_sync();
    }
  }
#pragma unroll
  for (int off = LPE; off < 64; off <<= 1) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc[c] = add4(acc[c], shfl_xor4(acc[c], off));
  }
  if (slot >= 0) {   // a hub piece: [Fp row | g_s_src share] partial for the combine kernel
    float* part = g.hub_part + (slot * NH + h) * (int64_t)(Fp + 4);
    if (grp == 0) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int q = c * LPE + li;
        if (q < F4) *(float4*)(part + 4 * q) = acc[c];
      }
    }
    if (!g.const_att) {
      gs = group_sum<64>(gs);
      if (lane == 0) part[Fp] = gs;
    }
    return;
  }
  float* row = g.G_aug + s * g.ldg;
  if (grp == 0) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int q = c * LPE + li;
      if (q < F4) *(float4*)(row + (int64_t)h * Fp + 4 * q) = acc[c];
    }
  }
  if (!g.const_att) {
    gs = group_sum<64>(gs);
    if (lane == 0) row[Dp + h] = gs + (g.g_corr ? g.g_corr[s * NH + h] : 0.f);
  }
}

// A hub source's row of G_aug: its pieces' partial rows summed in piece order (one wave per hub
// and head: the wave of the hub's first piece), plus max()'s share.
__global__ void __launch_bounds__(256) edge_bwd_src_hub_combine_kernel(BwdArgs g) {
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  int64_t s, slot;
  int h, beg, end;
  if (!hub_piece(g, wave, s, h, beg, end, slot)) return;
  const int32_t* hp = g.hubs + 4 * slot;
  if (uni(hp[1]) != 0) return;
  const int NH = g.NH, Fp = g.Fp, F4 = Fp / 4, pieces = uni(hp[2]);
  const int64_t W = Fp + 4, Dp = (int64_t)NH * Fp;
  const float* part = g.hub_part + (slot * NH + h) * W;
  float* row = g.G_aug + s * g.ldg;
  for (int q = lane; q < F4; q += 64) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < pieces; ++p) acc = add4(acc, *(const float4*)(part + p * NH * W + 4 * q));
    *(float4*)(row + (int64_t)h * Fp + 4 * q) = acc;
  }
  if (!g.const_att && lane == 0) {
    float gs = 0.f;
    for (int p = 0; p < pieces; ++p) gs += part[p * NH * W + Fp];
    row[Dp + h] = gs + (g.g_corr ? g.g_corr[s * NH + h] : 0.f);
  }
}

// src pass of a head-mean layer: go is one row per node for every head (the mean's gradient
// go / NH), so one wave per SOURCE node takes all NH heads: each go[dst] row is gathered once
// and accumulated with the NH weights of the edge, instead of once per (source, head) item
// (NH-fold fewer gathered bytes and NH-fold fewer items). Same per-head summation order as
// edge_bwd_src_kernel.
template <int LPE, int CPL>
__global__ void __launch_bounds__(256) edge_bwd_src_mean_kernel(BwdArgs g) {
  constexpr int EPW = 64 / LPE, NHM = 8;
  // rows in flight per lane (round 6: 2 instead of 8 at CPL 1, PPI L2: 166 -> 151-154 us, windowed
  // train traces on one box; the gathers are L2-request-bound and fewer registers keep more
  // waves resident; the same summation order, so the same bits)
  constexpr int U = CPL <= 1 ? 2 : (CPL <= 2 ? 4 : 2);
  const int lane = threadIdx.x & 63;
  const int wave = uni(threadIdx.x >> 6);
  const int grp = lane / LPE, li = lane % LPE;
  const int64_t s = xcd_contiguous(blockIdx.x, gridDim.x) * 4 + wave;
  if (s >= g.N) return;
  const int NH = g.NH, Fp = g.Fp, F4 = Fp / 4, S2 = 2 * NH;
  const int64_t Dp = (int64_t)NH * Fp, E2 = g.E2;
  const float M = g.const_att ? 0.f : ord_to_float(*g.M_ord);
  const bool drop = g.p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  const uint64_t seed = drop ? *g.seed : 0ull;
  const float4* __restrict__ go4 = (const float4*)g.go;
  __shared__ int src_sh[4][64];
  __shared__ float w_sh[4][NHM][64];
  int* src_lds = src_sh[wave];
  float (*w_lds)[64] = w_sh[wave];

  int off4[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int q = c * LPE + li;
    off4[c] = q < F4 ? q : 0;
  }
  float ssrc[NHM], gs[NHM];
  float4 acc[NHM][CPL];
#pragma unroll
  for (int h = 0; h < NHM; ++h) {
    ssrc[h] = (h < NH && !g.const_att) ? g.S[s * S2 + h] : 0.f;
    gs[h] = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc[h][c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float* __restrict__ graw = g.g_raw;

  const int beg = uni(g.rowptr[s]), end = uni(g.rowptr[s + 1]);
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const bool valid = lane < cnt;
    const int j = base + min(lane, cnt - 1);
    const int d = g.col[j];
    const int e = g.seid[j];
    const int64_t ep = drop ? (int64_t)g.perm[e] : 0;
#pragma unroll
    for (int h = 0; h < NHM; ++h) {
      if (h >= NH) break;
      float w = 0.f;
      if (valid) {
        const float ex = g.const_att ? 1.f : att_exp(ssrc[h] + g.S[(int64_t)d * S2 + NH + h], M);
        w = ex / (g.den[(int64_t)d * NH + h] + kSoftmaxEps);
        if (drop) w = dropout_keep(seed, ep * NH + h, g.p_drop) ? w * drop_scale : 0.f;
        if (graw) gs[h] += graw[(int64_t)h * E2 + e];
      }
      w_lds[h][lane] = w;
    }
    src_lds[lane] = d;
    wave_lds_sync();
    for (int j0 = grp; j0 < cnt; j0 += EPW * U) {
      float4 v[U][CPL];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float4* rp = go4 + (int64_t)src_lds[min(j0 + u * EPW, cnt - 1)] * g.go_stride4;
#pragma unroll
        for (int c = 0; c < CPL; ++c) v[u][c] = rp[off4[c]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jr = j0 + u * EPW;
        const bool live = jr < cnt;
        const int jc = live ? jr : 0;
#pragma unroll
        for (int h = 0; h < NHM; ++h) {
          if (h >= NH) break;
          const float wv = live ? w_lds[h][jc] : 0.f;
#pragma unroll
          for (int c = 0; c < CPL; ++c) acc[h][c] = fma4(wv, v[u][c], acc[h][c]);
        }
      }
    }
    wave_lds_sync();
  }
  float* row = g.G_aug + s * g.ldg;
#pragma unroll
  for (int h = 0; h < NHM; ++h) {
    if (h >= NH) break;
#pragma unroll
    for (int off = LPE; off < 64; off <<= 1) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[h][c] = add4(acc[h][c], shfl_xor4(acc[h][c], off));
    }
    if (grp == 0) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int q = c * LPE + li;
        if (q < F4) *(float4*)(row + (int64_t)h * Fp + 4 * q) = acc[h][c];
      }
    }
  }
  if (!g.const_att) {
#pragma unroll
    for (int h = 0; h < NHM; ++h) {
      if (h >= NH) break;
      const float v = group_sum<64>(gs[h]);
      if (lane == 0) row[Dp + h] = v + (g.g_corr ? g.g_corr[s * NH + h] : 0.f);
    }
  }
}

// g_W[c][i] = gW_aug[pad(c)][i] + sum_h2 A2[h2][c] * gW_aug[Dp + h2][i]
__global__ void __launch_bounds__(256) gw_kernel(const float* __restrict__ gW_aug,
                                                 const float* __restrict__ a, int NH, int F,
                                                 int Fp, int64_t F_in, float* __restrict__ g_W) {
  const int D = NH * F;
  const int64_t Dp = (int64_t)NH * Fp;
  const int64_t total = (int64_t)D * F_in;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = t / F_in, i = t - c * F_in;
    const int k = (int)(c / F), f = (int)(c - (int64_t)k * F);
    float v = gW_aug[((int64_t)k * Fp + f) * F_in + i];
    if (a) {
      for (int h = 0; h < NH; ++h) {
        const float* ar = a + (int64_t)h * 2 * D + k * 2 * F + f;
        v = fmaf(ar[0], gW_aug[(Dp + h) * F_in + i], v);
        v = fmaf(ar[F], gW_aug[(Dp + NH + h) * F_in + i], v);
      }
    }
    g_W[t] = v;
  }
}

// g_a[h][k*2F + f (+F)] = sum_i gW_aug[Dp + h (+NH)][i] * W[k*F + f][i]; one workgroup per W
// row c, its 4 waves splitting F_in, then a fixed-order combine of the 4 wave sums.
template <int H2C>
__global__ void __launch_bounds__(256) ga_kernel(const float* __restrict__ gW_aug,
                                                 const float* __restrict__ W, int NH, int F,
                                                 int Fp, int64_t F_in, float* __restrict__ g_a) {
  __shared__ float red[4][H2C];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int D = NH * F, H2 = 2 * NH;
  const int64_t Dp = (int64_t)NH * Fp;
  const int c = blockIdx.x;
  const int k = c / F, f = c - k * F;
  float acc[H2C];
#pragma unroll
  for (int h = 0; h < H2C; ++h) acc[h] = 0.f;
  for (int64_t i = threadIdx.x; i < F_in; i += 256) {
    const float w = W[(int64_t)c * F_in + i];
#pragma unroll
    for (int h = 0; h < H2C; ++h)
      if (h < H2) acc[h] = fmaf(gW_aug[(Dp + h) * F_in + i], w, acc[h]);
  }
#pragma unroll
  for (int h = 0; h < H2C; ++h) {
    const float v = group_sum<64>(acc[h]);
    if (lane == 0) red[wave][h] = v;
  }
  __syncthreads();
  if (threadIdx.x < H2) {
    const int h = threadIdx.x;
    const float v = (red[0][h] + red[1][h]) + (red[2][h] + red[3][h]);
    const int hh = h < NH ? h : h - NH;
    g_a[(int64_t)hh * 2 * D + k * 2 * F + (h < NH ? 0 : F) + f] = v;
  }
}

// gw_kernel and ga_kernel as ONE launch (small layers are launch-bound): blocks [0, ngw) do the
// g_W elements grid-stride over those blocks, blocks ngw.. one W row each of g_a.
template <int H2C>
__global__ void __launch_bounds__(256) weight_grads_kernel(const float* __restrict__ gW_aug,
                                                           const float* __restrict__ W,
                                                           const float* __restrict__ a, int NH,
                                                           int F, int Fp, int64_t F_in, int ngw,
                                                           float* __restrict__ g_W,
                                                           float* __restrict__ g_a) {
  const int D = NH * F;
  const int64_t Dp = (int64_t)NH * Fp;
  if ((int)blockIdx.x < ngw) {
    const int64_t total = (int64_t)D * F_in;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)ngw * blockDim.x) {
      const int64_t c = t / F_in, i = t - c * F_in;
      const int k = (int)(c / F), f = (int)(c - (int64_t)k * F);
      float v = gW_aug[((int64_t)k * Fp + f) * F_in + i];
      if (a) {
        for (int h = 0; h < NH; ++h) {
          const float* ar = a + (int64_t)h * 2 * D + k * 2 * F + f;
          v = fmaf(ar[0], gW_aug[(Dp + h) * F_in + i], v);
          v = fmaf(ar[F], gW_aug[(Dp + NH + h) * F_in + i], v);
        }
      }
      g_W[t] = v;
    }
    return;
  }
  // g_a[h][k*2F + f (+F)] = sum_i gW_aug[Dp + h (+NH)][i] * W[c][i], c = k*F + f (ga_kernel)
  __shared__ float red[4][H2C];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int H2 = 2 * NH;
  const int c = (int)blockIdx.x - ngw;
  const int k = c / F, f = c - k * F;
  float acc[H2C];
#pragma unroll
  for (int h = 0; h < H2C; ++h) acc[h] = 0.f;
  for (int64_t i = threadIdx.x; i < F_in; i += 256) {
    const float w = W[(int64_t)c * F_in + i];
#pragma unroll
    for (int h = 0; h < H2C; ++h)
      if (h < H2) acc[h] = fmaf(gW_aug[(Dp + h) * F_in + i], w, acc[h]);
  }
#pragma unroll
  for (int h = 0; h < H2C; ++h) {
    const float v = group_sum<64>(acc[h]);
    if (lane == 0) red[wave][h] = v;
  }
  __syncthreads();
  if (threadIdx.x < H2) {
    const int h = threadIdx.x;
    const float v = (red[0][h] + red[1][h]) + (red[2][h] + red[3][h]);
    const int hh = h < NH ? h : h - NH;
    g_a[(int64_t)hh * 2 * D + k * 2 * F + (h < NH ? 0 : F) + f] = v;
  }
}

// max() backward for small graphs in ONE launch (sum_partial + max_bwd + the tie-overflow scan):
// one 1024-thread block sums g_s_dst in a fixed order (thread-strided sums, then a fixed tree),
// applies the share to the recorded argmax entries, and rescans the edges itself in the rare
// case of more than GATX_ARGMAX_CAP ties.
__global__ void __launch_bounds__(1024) max_bwd_small_kernel(
    const float* __restrict__ gsd, int64_t n, const long long* __restrict__ argmax,
    const float* __restrict__ S, const uint32_t* __restrict__ M_ord,
    const int32_t* __restrict__ col, const int32_t* __restrict__ rowidx, int64_t E2b,
    const long long* e2p, int NH, float* __restrict__ g_corr_src, float* __restrict__ G_aug,
    int64_t ldg, int64_t Dp, float* __restrict__ gm_out) {
  __shared__ float red[16];
  __shared__ float share_s;
  float sum = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) sum += gsd[i];
  sum = group_sum<64>(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  const long long k = argmax[0];
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w];
    share_s = k > 0 ? -t / (float)k : 0.f;
    if (k > 0) gm_out[0] = share_s;
  }
  __syncthreads();
  if (k <= 0) return;
  const float share = share_s;
  if (k <= GATX_ARGMAX_CAP) {
    if (threadIdx.x == 0) {
      for (long long j = 0; j < k; ++j) {   // sequential: k is small (ties)
        const long long ent = argmax[1 + j];
        const long long e = ent / NH;
        const int h = (int)(ent - e * NH);
        if (g_corr_src) g_corr_src[(int64_t)col[e] * NH + h] += share;
        else G_aug[(int64_t)col[e] * ldg + Dp + h] += share;
        G_aug[(int64_t)rowidx[e] * ldg + Dp + NH + h] += share;
      }
    }
    return;
  }
  const int64_t E2 = e2p ? min(E2b, (int64_t)*e2p) : E2b;
  const float M = ord_to_float(*M_ord);
  const int S2 = 2 * NH;
  for (int64_t t = threadIdx.x; t < E2 * NH; t += 1024) {
    const int64_t e = t / NH;
    const int h = (int)(t - e * NH);
    const int64_t s = col[e], d = rowidx[e];
    if (S[s * S2 + h] + S[d * S2 + NH + h] == M) {
      if (g_corr_src) atomicAdd(&g_corr_src[s * NH + h], share);
      else atomicAdd(&G_aug[s * ldg + Dp + h], share);
      atomicAdd(&G_aug[d * ldg + Dp + NH + h], share);
    }
  }
}

__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ X, int64_t nrows,
                                                     int64_t ncols, int64_t ld,
                                                     float* __restrict__ out) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t j = blockIdx.x * 64ll + tx;
  float s = 0.f;
  if (j < ncols)
    for (int64_t i = ty; i < nrows; i += 4) s += X[i * ld + j];
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && j < ncols) out[j] = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}

struct Geom {
  int lpe, cpl;
};
// lanes per edge for one head's Fp/4 chunks (power of two <= 64), chunks per lane
inline Geom head_geom(int F4) {
  if (F4 >= 64) return {64, (int)ceil_div(F4, 64)};
  int l = 1;
  while (l < F4) l <<= 1;
  return {l, 1};
}

constexpr int64_t kChunk = 2048;

}  // namespace
}  // namespace gatx

using namespace gatx;

#define GATX_DISPATCH_HEAD(gm, KERNEL, grid, args)                                             \
  do {                                                                                         \
    if ((gm).lpe == 64) {                                                                      \
      switch ((gm).cpl) {                                                                      \
        case 1: KERNEL<64, 1><<<grid, 256, 0, st>>>(args); break;                              \
        case 2: KERNEL<64, 2><<<grid, 256, 0, st>>>(args); break;                              \
        case 3: KERNEL<64, 3><<<grid, 256, 0, st>>>(args); break;                              \
        default: KERNEL<64, 4><<<grid, 256, 0, st>>>(args); break;                             \
      }                                                                                        \
    } else {                                                                                   \
      switch ((gm).lpe) {                                                                      \
        case 1: KERNEL<1, 1><<<grid, 256, 0, st>>>(args); break;                               \
        case 2: KERNEL<2, 1><<<grid, 256, 0, st>>>(args); break;                               \
        case 4: KERNEL<4, 1><<<grid, 256, 0, st>>>(args); break;                               \
        case 8: KERNEL<8, 1><<<grid, 256, 0, st>>>(args); break;                               \
        case 16: KERNEL<16, 1><<<grid, 256, 0, st>>>(args); break;                             \
        default: KERNEL<32, 1><<<grid, 256, 0, st>>>(args); break;                             \
      }                                                                                        \
    }                                                                                          \
  } while (0)

extern "C" int gatx_prepare_go_ex(const float* g_out, const float* out, int64_t N, int NH,
                                  int F, int concat, int elu, float* go, float* g_pre,
                                  int64_t pre_ld, float out_p, const uint64_t* out_seed,
                                  gatx_stream_t s) {
  GATX_REQUIRE(out_p >= 0.f && out_p < 1.f && (out_p == 0.f || out_seed),
               "prepare_go: output dropout needs p in [0, 1) and its device seed");
  if (N == 0) return 0;
  const int64_t OC = concat ? (int64_t)NH * F : F;
  GATX_REQUIRE(pre_ld >= OC, "prepare_go: g_pre row stride below the output width");
  const int Fp = (int)round_up(F, 4);
  const int64_t GW = concat ? (int64_t)NH * Fp : Fp;
  GATX_REQUIRE(!elu || out, "prepare_go: elu needs the forward output");
  GATX_REQUIRE(g_pre != go || (concat && F % 4 == 0),
               "prepare_go: g_pre may alias go only for concat layers with F % 4 == 0");
  const bool aligned = ((uintptr_t)g_out % 16 == 0) && ((uintptr_t)go % 16 == 0) &&
                       (!elu || (uintptr_t)out % 16 == 0) && ((uintptr_t)g_pre % 16 == 0);
  if (F % 4 == 0 && aligned && pre_ld == OC && out_p == 0.f) {
    const int64_t n4 = N * GW / 4;
    prepare_go_vec_kernel<<<grid_for(ceil_div(n4, 4), 256, 8192), 256, 0, (hipStream_t)s>>>(
        (const float4*)g_out, (const float4*)out, n4, elu, concat ? 1.f : 1.f / (float)NH,
        (float4*)go, (float4*)g_pre);
    GATX_LAUNCH_CHECK("prepare_go");
    return 0;
  }
  prepare_go_kernel<<<grid_for(N * GW), 256, 0, (hipStream_t)s>>>(g_out, out, N, NH, F, Fp,
                                                                  concat, elu, go, g_pre,
                                                                  pre_ld, out_p, out_seed);
  GATX_LAUNCH_CHECK("prepare_go");
  return 0;
}

extern "C" int gatx_prepare_go(const float* g_out, const float* out, int64_t N, int NH, int F,
                               int concat, int elu, float* go, float* g_pre, gatx_stream_t s) {
  return gatx_prepare_go_ex(g_out, out, N, NH, F, concat, elu, go, g_pre,
                            concat ? (int64_t)NH * F : F, 0.f, nullptr, s);
}

extern "C" size_t gatx_edge_backward_hub_part_bytes(int64_t hub_bound, int NH, int F,
                                                    int src_pass) {
  const int64_t Fp = round_up(F, 4);
  return (size_t)hub_bound * NH * (src_pass ? Fp + 4 : 2) * sizeof(float);
}

namespace gatx {
namespace {
// Hub fields of BwdArgs; false when the buffers are missing.
bool set_hubs(BwdArgs& a, int hub_edges, const int32_t* hubs, const int32_t* hub_count,
              int64_t hub_bound, float* hub_part) {
  a.hub_T = 0; a.hubs = nullptr; a.hub_count = nullptr; a.hub_bound = 0; a.hub_part = nullptr;
  a.hub_blocks = 0;
  if (hub_edges <= 0 || hub_bound <= 0) return true;
  if (!hubs || !hub_count || !hub_part) return false;
  a.hub_T = hub_edges; a.hubs = hubs; a.hub_count = hub_count; a.hub_bound = hub_bound;
  a.hub_part = hub_part;
  // a multiple of 8 blocks: dealt round-robin over the XCDs, dispatched first
  a.hub_blocks = round_up(ceil_div(hub_bound * a.NH, 4), 8);
  return true;
}
}  // namespace
}  // namespace gatx

extern "C" int gatx_edge_backward_dst_hubs(const float* rows, int64_t row_stride,
                                           int64_t head_stride, const float* S,
                                           const uint32_t* M_ord, const float* den,
                                           const int32_t* rowptr, const int32_t* col,
                                           const int32_t* perm, int64_t N, int64_t E2, int NH,
                                           int F, const float* go, int64_t go_stride,
                                           int64_t go_head, float p, const uint64_t* seed,
                                           const float* g_alpha, float* g_raw, float* gsd,
                                           float* G, int64_t ldg, int64_t gs_off, int hub_edges,
                                           const int32_t* hubs, const int32_t* hub_count,
                                           int64_t hub_bound, float* hub_part, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  if (N == 0) return 0;
  const int Fp = (int)round_up(F, 4);
  GATX_REQUIRE(row_stride % 4 == 0 && head_stride % 4 == 0 && go_stride % 4 == 0 &&
                   go_head % 4 == 0 && ((uintptr_t)rows % 16) == 0 && ((uintptr_t)go % 16) == 0,
               "edge_backward_dst: rows / go must be float4-aligned");
  const Geom gm = head_geom(Fp / 4);
  GATX_REQUIRE(gm.cpl <= 4, "edge_backward: out_features > 1024 unsupported");
  BwdArgs a{};
  a.Wh = rows; a.go = go;
  a.go_stride4 = go_stride / 4;
  a.go_head4 = (int)(go_head / 4);
  a.row_stride4 = row_stride / 4;
  a.head_stride4 = head_stride / 4;
  a.gs_off = gs_off;
  a.S = S; a.M_ord = M_ord; a.den = den; a.rowptr = rowptr; a.col = col; a.perm = perm;
  a.N = N; a.E2 = E2; a.NH = NH; a.F = F; a.Fp = Fp; a.p_drop = p; a.seed = seed;
  a.g_alpha_ret = g_alpha; a.g_raw = g_raw; a.gsd = gsd; a.G_aug = G; a.ldg = ldg;
  a.chunk = kChunk;
  a.n_items = ceil_div(N, kChunk) * kChunk * NH;
  GATX_REQUIRE(set_hubs(a, hub_edges, hubs, hub_count, hub_bound, hub_part),
               "edge_backward_dst: hub splitting needs its plan and partial buffer");
  const unsigned grid = (unsigned)(a.hub_blocks + ceil_div(a.n_items, 4));
  GATX_DISPATCH_HEAD(gm, edge_bwd_dst_kernel, grid, a);
  GATX_LAUNCH_CHECK("edge_bwd_dst");
  if (a.hub_T > 0) {
    const unsigned hg = (unsigned)ceil_div(a.hub_bound * NH, 4);
    edge_bwd_dst_hub_kernel<<<hg, 256, 0, st>>>(a);
    GATX_LAUNCH_CHECK("edge_bwd_dst_hub");
    edge_bwd_dst_hub_finish_kernel<<<hg, 256, 0, st>>>(a);
    GATX_LAUNCH_CHECK("edge_bwd_dst_hub_finish");
  }
  return 0;
}

extern "C" int gatx_edge_backward_dst_ex(const float* rows, int64_t row_stride,
                                         int64_t head_stride, const float* S,
                                         const uint32_t* M_ord, const float* den,
                                         const int32_t* rowptr, const int32_t* col,
                                         const int32_t* perm, int64_t N, int64_t E2, int NH, int F,
                                         const float* go, int64_t go_stride, int64_t go_head,
                                         float p, const uint64_t* seed, const float* g_alpha,
                                         float* g_raw, float* gsd, float* G, int64_t ldg,
                                         int64_t gs_off, gatx_stream_t s) {
  return gatx_edge_backward_dst_hubs(rows, row_stride, head_stride, S, M_ord, den, rowptr, col,
                                     perm, N, E2, NH, F, go, go_stride, go_head, p, seed, g_alpha,
                                     g_raw, gsd, G, ldg, gs_off, 0, nullptr, nullptr, 0, nullptr,
                                     s);
}

extern "C" int gatx_edge_backward_dst(const float* Wh, const float* S, const uint32_t* M_ord,
                                      const float* den, const int32_t* rowptr,
                                      const int32_t* col, const int32_t* perm, int64_t N,
                                      int64_t E2, int NH, int F, int concat, float p,
                                      const uint64_t* seed, const float* go, const float* g_alpha,
                                      float* g_raw, float* gsd, float* G_aug, int64_t ldg,
                                      gatx_stream_t s) {
  const int64_t Fp = round_up(F, 4), Dp = NH * Fp;
  return gatx_edge_backward_dst_ex(Wh, Dp, Fp, S, M_ord, den, rowptr, col, perm, N, E2, NH, F,
                                   go, concat ? Dp : Fp, concat ? Fp : 0, p, seed, g_alpha,
                                   g_raw, gsd, G_aug, ldg, Dp, s);
}

extern "C" int gatx_edge_backward_src_scores(const int32_t* srowptr, const int32_t* seid,
                                             int64_t N, int64_t E2, int NH, const float* g_raw,
                                             const float* g_corr, float* G, int64_t ldg,
                                             int64_t gs_off, gatx_stream_t s) {
  GATX_REQUIRE(NH >= 1 && NH <= 8, "edge_backward_src_scores: 1..8 heads");
  if (N == 0) return 0;
  hipStream_t st = (hipStream_t)s;
  const unsigned grid = (unsigned)ceil_div(N, 4);
#define GATX_SS(C) src_scores_kernel<C><<<grid, 256, 0, st>>>(srowptr, seid, N, E2, NH, g_raw, \
                                                             g_corr, G, ldg, gs_off)
  switch (NH) {
    case 1: GATX_SS(1); break; case 2: GATX_SS(2); break; case 4: GATX_SS(4); break;
    case 8: GATX_SS(8); break; default: GATX_SS(0); break;
  }
#undef GATX_SS
  GATX_LAUNCH_CHECK("edge_bwd_src_scores");
  return 0;
}

extern "C" size_t gatx_max_backward_workspace_bytes(void) {
  return sizeof(float) * kSumBlocks;
}

extern "C" int gatx_max_backward(const int64_t* argmax, const float* gsd, const float* S,
                                 const uint32_t* M_ord, const int32_t* col, const int32_t* rowidx,
                                 int64_t N, int64_t E2, const int64_t* e2, int NH,
                                 float* g_corr_src, float* G_aug, int64_t ldg, int64_t Dp,
                                 void* workspace, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  // the g_M share is parked right after the argmax records (the buffer holds CAP + 2 int64s)
  float* gm = (float*)(argmax + 1 + GATX_ARGMAX_CAP);
  float* part = (float*)workspace;
  if (N * NH <= (1 << 16)) {   // small graphs: one launch instead of three
    max_bwd_small_kernel<<<1, 1024, 0, st>>>(gsd, N * NH, (const long long*)argmax, S, M_ord, col,
                                             rowidx, E2, (const long long*)e2, NH, g_corr_src,
                                             G_aug, ldg, Dp, gm);
    GATX_LAUNCH_CHECK("max_bwd_small");
    return 0;
  }
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(N * NH, 256), kSumBlocks));
  sum_partial_kernel<<<nb, 256, 0, st>>>(gsd, N * NH, part);
  GATX_LAUNCH_CHECK("gsd_sum");
  max_bwd_kernel<<<1, 256, 0, st>>>(part, nb, (const long long*)argmax, col, rowidx, NH,
                                    g_corr_src, G_aug, ldg, Dp, gm);
  GATX_LAUNCH_CHECK("max_bwd");
  max_bwd_scan_kernel<<<grid_for(E2 * NH, 256, 4096), 256, 0, st>>>(
      S, M_ord, col, rowidx, E2, (const long long*)e2, NH, (const long long*)argmax, gm,
      g_corr_src, G_aug, ldg, Dp);
  GATX_LAUNCH_CHECK("max_bwd_scan");
  return 0;
}

extern "C" int gatx_edge_backward_src_hubs(const float* S, const uint32_t* M_ord,
                                           const float* den, const int32_t* srowptr,
                                           const int32_t* scol, const int32_t* seid,
                                           const int32_t* perm, int64_t N, int64_t E2, int NH,
                                           int F, int concat, int const_att, float p,
                                           const uint64_t* seed, const float* go,
                                           const float* g_raw, const float* g_corr_src,
                                           float* G_aug, int64_t ldg, int hub_edges,
                                           const int32_t* hubs, const int32_t* hub_count,
                                           int64_t hub_bound, float* hub_part, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  if (N == 0) return 0;
  const int Fp = (int)round_up(F, 4);
  const Geom gm = head_geom(Fp / 4);
  GATX_REQUIRE(gm.cpl <= 4, "edge_backward: out_features > 1024 unsupported");
  GATX_REQUIRE(ldg % 4 == 0, "edge_backward: G_aug row stride must be a multiple of 4");
  BwdArgs a{};
  a.go = go;
  a.go_stride4 = concat ? (int64_t)NH * Fp / 4 : Fp / 4;
  a.go_head4 = concat ? Fp / 4 : 0;
  a.S = S; a.M_ord = M_ord; a.den = den; a.rowptr = srowptr; a.col = scol; a.seid = seid;
  a.perm = perm; a.N = N; a.E2 = E2; a.NH = NH; a.F = F; a.Fp = Fp; a.const_att = const_att;
  a.p_drop = p; a.seed = seed; a.g_raw = const_att ? nullptr : (float*)g_raw;
  a.g_corr = g_corr_src; a.G_aug = G_aug; a.ldg = ldg;
  a.chunk = kChunk;
  GATX_REQUIRE(set_hubs(a, hub_edges, hubs, hub_count, hub_bound, hub_part),
               "edge_backward_src: hub splitting needs its plan and partial buffer");
  // head-mean: one item per source, all heads (hub-split graphs take the per-head items, which
  // also serve head-mean layers: go_head4 = 0)
  if (!concat && NH <= 8 && a.hub_T == 0) {
    const unsigned grid = (unsigned)ceil_div(N, 4);
    GATX_DISPATCH_HEAD(gm, edge_bwd_src_mean_kernel, grid, a);
    GATX_LAUNCH_CHECK("edge_bwd_src_mean");
    return 0;
  }
  a.n_items = ceil_div(N, kChunk) * kChunk * NH;
  const unsigned grid = (unsigned)(a.hub_blocks + ceil_div(a.n_items, 4));
  GATX_DISPATCH_HEAD(gm, edge_bwd_src_kernel, grid, a);
  GATX_LAUNCH_CHECK("edge_bwd_src");
  if (a.hub_T > 0) {
    edge_bwd_src_hub_combine_kernel<<<(unsigned)ceil_div(a.hub_bound * NH, 4), 256, 0, st>>>(a);
    GATX_LAUNCH_CHECK("edge_bwd_src_hub_combine");
  }
  return 0;
}

extern "C" int gatx_edge_backward_src(const float* S, const uint32_t* M_ord, const float* den,
                                      const int32_t* srowptr, const int32_t* scol,
                                      const int32_t* seid, const int32_t* perm, int64_t N,
                                      int64_t E2, int NH, int F, int concat, int const_att,
                                      float p, const uint64_t* seed, const float* go,
                                      const float* g_raw, const float* g_corr_src, float* G_aug,
                                      int64_t ldg, gatx_stream_t s) {
  return gatx_edge_backward_src_hubs(S, M_ord, den, srowptr, scol, seid, perm, N, E2, NH, F,
                                     concat, const_att, p, seed, go, g_raw, g_corr_src, G_aug,
                                     ldg, 0, nullptr, nullptr, 0, nullptr, s);
}

extern "C" int gatx_weight_grads(const float* gW_aug, const float* W, const float* a, int NH,
                                 int F, int64_t F_in, float* g_W, float* g_a, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  const int Fp = (int)round_up(F, 4);
  GATX_REQUIRE(!a || 2 * NH <= 32, "weight_grads: num_heads > 16 unsupported");
  if (a && (int64_t)NH * F * F_in <= (1 << 22)) {   // small layers: one launch for both
    const int ngw = (int)grid_for((int64_t)NH * F * F_in, 256, 1024);
    const unsigned grid = (unsigned)(ngw + NH * F);
    if (2 * NH <= 8) weight_grads_kernel<8><<<grid, 256, 0, st>>>(gW_aug, W, a, NH, F, Fp, F_in, ngw, g_W, g_a);
    else if (2 * NH <= 16) weight_grads_kernel<16><<<grid, 256, 0, st>>>(gW_aug, W, a, NH, F, Fp, F_in, ngw, g_W, g_a);
    else weight_grads_kernel<32><<<grid, 256, 0, st>>>(gW_aug, W, a, NH, F, Fp, F_in, ngw, g_W, g_a);
    GATX_LAUNCH_CHECK("weight_grads");
    return 0;
  }
  gw_kernel<<<grid_for((int64_t)NH * F * F_in), 256, 0, st>>>(gW_aug, a, NH, F, Fp, F_in, g_W);
  GATX_LAUNCH_CHECK("gw");
  if (a) {
    const unsigned D = (unsigned)(NH * F);
    if (2 * NH <= 8) ga_kernel<8><<<D, 256, 0, st>>>(gW_aug, W, NH, F, Fp, F_in, g_a);
    else if (2 * NH <= 16) ga_kernel<16><<<D, 256, 0, st>>>(gW_aug, W, NH, F, Fp, F_in, g_a);
    else ga_kernel<32><<<D, 256, 0, st>>>(gW_aug, W, NH, F, Fp, F_in, g_a);
    GATX_LAUNCH_CHECK("ga");
  }
  return 0;
}

extern "C" int gatx_colsum(const float* X, int64_t nrows, int64_t ncols, int64_t ld, float* out,
                           gatx_stream_t s) {
  if (ncols == 0) return 0;
  colsum_kernel<<<(unsigned)ceil_div(ncols, 64), 256, 0, (hipStream_t)s>>>(X, nrows, ncols, ld,
                                                                           out);
  GATX_LAUNCH_CHECK("colsum");
  return 0;
}
