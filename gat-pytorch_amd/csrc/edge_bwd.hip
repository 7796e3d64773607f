// Backward of the GATLayer attention + aggregation: the closed form of torch autograd through
// models/gat_layer.py:64-135, as passes over the two CSR orders.
//
//   dst pass  (per destination n, one wave): g_alpha~ = <go[n,h,:], Wh[src,h,:]> per edge & head
//             (go row held in registers, Wh[src] streamed), softmax backward
//             c = sum g_alpha * alpha, g_raw' = 0.01 * ex * (g_alpha - c) / (den + 1e-8),
//             g_s_dst = sum_e g_raw', and a per-workgroup partial of sum g_raw' for max()'s grad.
//   max bwd   g_M = -sum g_raw' split evenly over the argmax entries recorded by the forward.
//   src pass  (per source s, one wave): the message gradient sum alpha~ * go[dst] (go rows
//             streamed) and g_s_src = sum_e g_raw' + the max() correction, written as one row of
//             G_aug = [g_Wh | g_s_src | g_s_dst], the gradient of the augmented projection.
// The weight/input gradients then come from two MFMA GEMMs on G_aug (gemm.hip) and
// gatx_weight_grads, which maps g_W_aug back onto W.weight and a.weight.
// No float atomics on the data path: every sum has a fixed order (bitwise reproducible), except
// the tie-split of max()'s gradient when several argmax entries share a node.
#include "gatx_common.h"

namespace gatx {
namespace {

inline unsigned grid_for(int64_t n, int block = 256, int64_t cap = 16384) {
  int64_t g = ceil_div(n > 0 ? n : 1, block);
  return (unsigned)(g < cap ? g : cap);
}

// Load chunk q (4 features of head h) of the upstream gradient row of node n, in the padded
// [NH][Fp] layout; f >= F reads as 0. Head-mean layers broadcast g_out[n, :F] / NH to all heads.
__device__ inline float4 load_go(const float* __restrict__ g_out, int64_t n, int q, int NH, int F,
                                 int Fp, int concat, float inv_nh) {
  const int h = (q * 4) / Fp, f0 = q * 4 - h * Fp;
  const float* row = concat ? g_out + n * (int64_t)(NH * F) + h * F : g_out + n * (int64_t)F;
  float4 v;
  if ((F & 3) == 0) {
    v = *(const float4*)(row + f0);
  } else {
    v.x = (f0 + 0 < F) ? row[f0 + 0] : 0.f;
    v.y = (f0 + 1 < F) ? row[f0 + 1] : 0.f;
    v.z = (f0 + 2 < F) ? row[f0 + 2] : 0.f;
    v.w = (f0 + 3 < F) ? row[f0 + 3] : 0.f;
  }
  return concat ? v : v * inv_nh;
}

template <int LPE, int CPL>
__global__ void __launch_bounds__(256)
edge_bwd_dst_kernel(const float* __restrict__ Wh, const float* __restrict__ S,
                    const uint32_t* __restrict__ M_ord, const float* __restrict__ den,
                    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                    const int32_t* __restrict__ perm, int64_t N, int NH, int F, int Fp,
                    int concat, float p_drop, uint64_t seed, const float* __restrict__ g_out,
                    const float* __restrict__ g_alpha_ret, float* __restrict__ g_raw,
                    float* __restrict__ G_aug, int64_t ldg, float* __restrict__ partials) {
  __shared__ float part_lds[4];
  constexpr int EPW = 64 / LPE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / LPE, li = lane % LPE;
  const int D4 = NH * Fp / 4, F4 = Fp / 4, S2 = 2 * NH;
  const int64_t Dp = (int64_t)NH * Fp;
  const float M = ord_to_float(*M_ord);
  const bool drop = p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const float inv_nh = 1.f / (float)NH;
  const float4* __restrict__ Wh4 = (const float4*)Wh;
  // lane li < NH of every edge group owns head li for the per-(edge, head) scalars
  const bool owner = li < NH;
  const int hl = owner ? li : 0;

  int q[CPL], hc[CPL];
  bool vq[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    q[c] = c * LPE + li;
    vq[c] = q[c] < D4;
    hc[c] = vq[c] ? q[c] / F4 : -1;
  }
  float wave_part = 0.f;

  for (int64_t n = blockIdx.x * 4ll + wave; n < N; n += gridDim.x * 4ll) {
    const int beg = rowptr[n], end = rowptr[n + 1];
    float4 go[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c)
      go[c] = vq[c] ? load_go(g_out, n, q[c], NH, F, Fp, concat, inv_nh)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    const float sdst = S[n * S2 + NH + hl];
    const float dinv = 1.f / (den[n * NH + hl] + kSoftmaxEps);
    // loop 1: g_alpha per (edge, head) and c = sum g_alpha * alpha
    float c_acc = 0.f;
    for (int e = beg + grp; e < end; e += EPW) {
      const int64_t s = col[e];
      float pc[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        pc[c] = 0.f;
        if (!vq[c]) continue;
        const float4 v = Wh4[s * D4 + q[c]];
        pc[c] = go[c].x * v.x + go[c].y * v.y + go[c].z * v.z + go[c].w * v.w;
      }
      float mine = 0.f;
      for (int h = 0; h < NH; ++h) {   // per-head sum over the group's lanes
        float t = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) t += (hc[c] == h) ? pc[c] : 0.f;
#pragma unroll
        for (int off = 1; off < LPE; off <<= 1) t += __shfl_xor(t, off);
        if (li == h) mine = t;
      }
      if (owner) {
        const float alpha = att_exp(S[s * S2 + hl] + sdst, M) * dinv;
        float ga = mine;
        if (drop) ga = dropout_keep(seed, (int64_t)perm[e] * NH + hl, p_drop) ? ga * drop_scale : 0.f;
        if (g_alpha_ret) ga += g_alpha_ret[(int64_t)perm[e] * NH + hl];
        g_raw[(int64_t)e * NH + hl] = ga;   // g_alpha for now; the same lane rewrites it below
        c_acc += ga * alpha;
      }
    }
#pragma unroll
    for (int off = LPE; off < 64; off <<= 1) c_acc += __shfl_xor(c_acc, off);
    // loop 2 (same lane <-> (edge, head) map as loop 1): g_raw' and g_s_dst = sum_e g_raw'
    float gsum = 0.f;
    if (owner) {
      for (int e = beg + grp; e < end; e += EPW) {
        const float ex = att_exp(S[(int64_t)col[e] * S2 + hl] + sdst, M);
        const float ga = g_raw[(int64_t)e * NH + hl];
        const float gr = kLeakySlope * ex * (ga - c_acc) * dinv;
        g_raw[(int64_t)e * NH + hl] = gr;
        gsum += gr;
      }
    }
#pragma unroll
    for (int off = LPE; off < 64; off <<= 1) gsum += __shfl_xor(gsum, off);
    if (grp == 0 && owner) G_aug[n * ldg + Dp + NH + hl] = gsum;
    // wave-level partial of sum g_raw' (for max()'s gradient), fixed order
    float hs = (grp == 0 && owner) ? gsum : 0.f;
    for (int off = 1; off < 64; off <<= 1) hs += __shfl_xor(hs, off);
    wave_part += hs;
  }
  if (lane == 0) part_lds[wave] = wave_part;
  __syncthreads();
  if (threadIdx.x == 0)
    partials[blockIdx.x] = (part_lds[0] + part_lds[1]) + (part_lds[2] + part_lds[3]);
}

// max() backward: g_M = -sum(g_raw'), split evenly over the k tied argmax entries.
__global__ void __launch_bounds__(256) max_bwd_kernel(const float* __restrict__ partials,
                                                      int64_t n_part,
                                                      const long long* __restrict__ argmax,
                                                      const int32_t* __restrict__ col,
                                                      const int32_t* __restrict__ rowidx, int NH,
                                                      float* __restrict__ g_corr_src,
                                                      float* __restrict__ G_aug, int64_t ldg,
                                                      int64_t Dp, float* __restrict__ gm_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n_part; i += blockDim.x) s += partials[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
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
    g_corr_src[(int64_t)col[e] * NH + h] += share;
    G_aug[(int64_t)rowidx[e] * ldg + Dp + NH + h] += share;
  }
}

// Fallback when more than GATX_ARGMAX_CAP entries tie: rescan every (edge, head).
__global__ void __launch_bounds__(256) max_bwd_scan_kernel(const float* __restrict__ S,
                                                           const uint32_t* __restrict__ M_ord,
                                                           const int32_t* __restrict__ col,
                                                           const int32_t* __restrict__ rowidx,
                                                           int64_t E2, int NH,
                                                           const long long* __restrict__ argmax,
                                                           const float* __restrict__ gm,
                                                           float* __restrict__ g_corr_src,
                                                           float* __restrict__ G_aug,
                                                           int64_t ldg, int64_t Dp) {
  if (argmax[0] <= GATX_ARGMAX_CAP) return;
  const float M = ord_to_float(*M_ord), share = gm[0];
  const int S2 = 2 * NH;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < E2 * NH;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / NH;
    const int h = (int)(t - e * NH);
    const int64_t s = col[e], d = rowidx[e];
    if (S[s * S2 + h] + S[d * S2 + NH + h] == M) {
      atomicAdd(&g_corr_src[s * NH + h], share);
      atomicAdd(&G_aug[d * ldg + Dp + NH + h], share);
    }
  }
}

template <int LPE, int CPL>
__global__ void __launch_bounds__(256)
edge_bwd_src_kernel(const float* __restrict__ S, const uint32_t* __restrict__ M_ord,
                    const float* __restrict__ den, const int32_t* __restrict__ srowptr,
                    const int32_t* __restrict__ scol, const int32_t* __restrict__ seid,
                    const int32_t* __restrict__ perm, int64_t N, int NH, int F, int Fp,
                    int concat, int const_att, float p_drop, uint64_t seed,
                    const float* __restrict__ g_out, const float* __restrict__ g_raw,
                    const float* __restrict__ g_corr_src, float* __restrict__ G_aug,
                    int64_t ldg) {
  constexpr int EPW = 64 / LPE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / LPE, li = lane % LPE;
  const int D4 = NH * Fp / 4, F4 = Fp / 4, S2 = 2 * NH;
  const int64_t Dp = (int64_t)NH * Fp;
  const float M = const_att ? 0.f : ord_to_float(*M_ord);
  const bool drop = p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const float inv_nh = 1.f / (float)NH;

  int q[CPL], hc[CPL];
  bool vq[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    q[c] = c * LPE + li;
    vq[c] = q[c] < D4;
    hc[c] = vq[c] ? q[c] / F4 : 0;
  }

  for (int64_t s = blockIdx.x * 4ll + wave; s < N; s += gridDim.x * 4ll) {
    const int beg = srowptr[s], end = srowptr[s + 1];
    float ssrc[CPL];
    float4 acc[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      ssrc[c] = const_att ? 0.f : S[s * S2 + hc[c]];
      acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float gs = 0.f;
    for (int j = beg + grp; j < end; j += EPW) {
      const int64_t d = scol[j];
      const int64_t e = seid[j];
      const int64_t ep = drop ? (int64_t)perm[e] : 0;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        if (!vq[c]) continue;
        const float4 g = load_go(g_out, d, q[c], NH, F, Fp, concat, inv_nh);
        const float ex = const_att ? 1.f : att_exp(ssrc[c] + S[d * S2 + NH + hc[c]], M);
        float w = ex / (den[d * NH + hc[c]] + kSoftmaxEps);
        if (drop) w = dropout_keep(seed, ep * NH + hc[c], p_drop) ? w * drop_scale : 0.f;
        acc[c] = fma4(w, g, acc[c]);
      }
      if (!const_att && li < NH) gs += g_raw[e * NH + li];
    }
#pragma unroll
    for (int off = LPE; off < 64; off <<= 1) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) acc[c] = add4(acc[c], shfl_xor4(acc[c], off));
      gs += __shfl_xor(gs, off);
    }
    if (grp == 0) {
      float* row = G_aug + s * ldg;
#pragma unroll
      for (int c = 0; c < CPL; ++c)
        if (vq[c]) *(float4*)(row + q[c] * 4) = acc[c];
      if (!const_att && li < NH) row[Dp + li] = gs + g_corr_src[s * NH + li];
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

// g_a[h][k*2F + f (+F)] = sum_i gW_aug[Dp + h (+NH)][i] * W[k*F + f][i]; one wave per W row c.
__global__ void __launch_bounds__(256) ga_kernel(const float* __restrict__ gW_aug,
                                                 const float* __restrict__ W, int NH, int F,
                                                 int Fp, int64_t F_in, float* __restrict__ g_a) {
  const int lane = threadIdx.x & 63;
  const int D = NH * F;
  const int64_t Dp = (int64_t)NH * Fp;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= D) return;
  const int k = c / F, f = c - k * F;
  float acc[32];
#pragma unroll
  for (int h = 0; h < 32; ++h) acc[h] = 0.f;
  for (int64_t i = lane; i < F_in; i += 64) {
    const float w = W[(int64_t)c * F_in + i];
#pragma unroll
    for (int h = 0; h < 32; ++h)
      if (h < 2 * NH) acc[h] = fmaf(gW_aug[(Dp + h) * F_in + i], w, acc[h]);
  }
#pragma unroll
  for (int h = 0; h < 32; ++h) {
    if (h >= 2 * NH) break;
    float v = acc[h];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) {
      const int hh = h < NH ? h : h - NH;
      g_a[(int64_t)hh * 2 * D + k * 2 * F + (h < NH ? 0 : F) + f] = v;
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

template <int LPE, int CPL>
int launch_bwd_dst(unsigned grid, hipStream_t st, const float* Wh, const float* S,
                   const uint32_t* M_ord, const float* den, const int32_t* rowptr,
                   const int32_t* col, const int32_t* perm, int64_t N, int NH, int F, int Fp,
                   int concat, float p, uint64_t seed, const float* g_out, const float* g_alpha,
                   float* g_raw, float* G_aug, int64_t ldg, float* partials) {
  edge_bwd_dst_kernel<LPE, CPL><<<grid, 256, 0, st>>>(Wh, S, M_ord, den, rowptr, col, perm, N, NH,
                                                      F, Fp, concat, p, seed, g_out, g_alpha,
                                                      g_raw, G_aug, ldg, partials);
  GATX_LAUNCH_CHECK("edge_bwd_dst");
  return 0;
}

template <int LPE, int CPL>
int launch_bwd_src(unsigned grid, hipStream_t st, const float* S, const uint32_t* M_ord,
                   const float* den, const int32_t* srowptr, const int32_t* scol,
                   const int32_t* seid, const int32_t* perm, int64_t N, int NH, int F, int Fp,
                   int concat, int const_att, float p, uint64_t seed, const float* g_out,
                   const float* g_raw, const float* g_corr, float* G_aug, int64_t ldg) {
  edge_bwd_src_kernel<LPE, CPL><<<grid, 256, 0, st>>>(S, M_ord, den, srowptr, scol, seid, perm,
                                                      N, NH, F, Fp, concat, const_att, p, seed,
                                                      g_out, g_raw, g_corr, G_aug, ldg);
  GATX_LAUNCH_CHECK("edge_bwd_src");
  return 0;
}

constexpr int64_t kDstGridCap = 8192;

}  // namespace
}  // namespace gatx

using namespace gatx;

#define GATX_DISPATCH_GEOM(g, MACRO)                                                           \
  do {                                                                                         \
    if ((g).lpe == 64) {                                                                       \
      switch ((g).cpl) {                                                                       \
        case 1: MACRO(64, 1); case 2: MACRO(64, 2); case 3: MACRO(64, 3);                      \
        case 4: MACRO(64, 4); case 5: MACRO(64, 5); case 6: MACRO(64, 6);                      \
        case 7: MACRO(64, 7); default: MACRO(64, 8);                                           \
      }                                                                                        \
    }                                                                                          \
    switch ((g).lpe) {                                                                         \
      case 1: MACRO(1, 1); case 2: MACRO(2, 1); case 4: MACRO(4, 1);                           \
      case 8: MACRO(8, 1); case 16: MACRO(16, 1); default: MACRO(32, 1);                       \
    }                                                                                          \
  } while (0)

extern "C" int64_t gatx_edge_backward_dst_partials(int64_t N) {
  return std::max<int64_t>(1, std::min<int64_t>(ceil_div(N, 4), kDstGridCap));
}

extern "C" int gatx_edge_backward_dst(const float* Wh, const float* S, const uint32_t* M_ord,
                                      const float* den, const int32_t* rowptr,
                                      const int32_t* col, const int32_t* perm, int64_t N, int NH,
                                      int F, int concat, float p, uint64_t seed,
                                      const float* g_out, const float* g_alpha, float* g_raw,
                                      float* G_aug, int64_t ldg, float* partials,
                                      gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  const int Fp = (int)round_up(F, 4);
  const RowGeom g = row_geom((int64_t)NH * Fp / 4);
  GATX_REQUIRE(g.cpl <= 8, "edge_backward: num_heads*out_features > 2048 unsupported");
  GATX_REQUIRE(NH <= 64 && NH <= g.lpe, "edge_backward: num_heads too large");
  const unsigned grid = (unsigned)gatx_edge_backward_dst_partials(N);
  if (N == 0) {
    hipError_t r = hipMemsetAsync(partials, 0, sizeof(float), st);
    return (int)r;
  }
#define GATX_BD(L, C)                                                                          \
  return launch_bwd_dst<L, C>(grid, st, Wh, S, M_ord, den, rowptr, col, perm, N, NH, F, Fp,    \
                              concat, p, seed, g_out, g_alpha, g_raw, G_aug, ldg, partials)
  GATX_DISPATCH_GEOM(g, GATX_BD);
#undef GATX_BD
}

extern "C" int gatx_max_backward(const float* partials, int64_t n_partials,
                                 const int64_t* argmax, const float* S, const uint32_t* M_ord,
                                 const int32_t* col, const int32_t* rowidx, int64_t E2, int NH,
                                 float* g_corr_src, float* G_aug, int64_t ldg, int64_t Dp,
                                 gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  // the g_M share is parked right after the argmax records (the buffer holds CAP + 2 int64s)
  float* gm = (float*)(argmax + 1 + GATX_ARGMAX_CAP);
  max_bwd_kernel<<<1, 256, 0, st>>>(partials, n_partials, (const long long*)argmax, col, rowidx,
                                    NH, g_corr_src, G_aug, ldg, Dp, gm);
  GATX_LAUNCH_CHECK("max_bwd");
  max_bwd_scan_kernel<<<grid_for(E2 * NH, 256, 4096), 256, 0, st>>>(
      S, M_ord, col, rowidx, E2, NH, (const long long*)argmax, gm, g_corr_src, G_aug, ldg, Dp);
  GATX_LAUNCH_CHECK("max_bwd_scan");
  return 0;
}

extern "C" int gatx_edge_backward_src(const float* S, const uint32_t* M_ord, const float* den,
                                      const int32_t* srowptr, const int32_t* scol,
                                      const int32_t* seid, const int32_t* perm, int64_t N, int NH,
                                      int F, int concat, int const_att, float p, uint64_t seed,
                                      const float* g_out, const float* g_raw,
                                      const float* g_corr_src, float* G_aug, int64_t ldg,
                                      gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  if (N == 0) return 0;
  const int Fp = (int)round_up(F, 4);
  const RowGeom g = row_geom((int64_t)NH * Fp / 4);
  GATX_REQUIRE(g.cpl <= 8, "edge_backward: num_heads*out_features > 2048 unsupported");
  GATX_REQUIRE(ldg % 4 == 0, "edge_backward: G_aug row stride must be a multiple of 4");
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(N, 4), 65536);
#define GATX_BS(L, C)                                                                          \
  return launch_bwd_src<L, C>(grid, st, S, M_ord, den, srowptr, scol, seid, perm, N, NH, F,    \
                              Fp, concat, const_att, p, seed, g_out, g_raw, g_corr_src, G_aug, \
                              ldg)
  GATX_DISPATCH_GEOM(g, GATX_BS);
#undef GATX_BS
}

extern "C" int gatx_weight_grads(const float* gW_aug, const float* W, const float* a, int NH,
                                 int F, int64_t F_in, float* g_W, float* g_a, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  const int Fp = (int)round_up(F, 4);
  GATX_REQUIRE(!a || 2 * NH <= 32, "weight_grads: num_heads > 16 unsupported");
  gw_kernel<<<grid_for((int64_t)NH * F * F_in), 256, 0, st>>>(gW_aug, a, NH, F, Fp, F_in, g_W);
  GATX_LAUNCH_CHECK("gw");
  if (a) {
    ga_kernel<<<(unsigned)ceil_div((int64_t)NH * F, 4), 256, 0, st>>>(gW_aug, W, NH, F, Fp, F_in,
                                                                      g_a);
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
