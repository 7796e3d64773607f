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
__global__ void __launch_bounds__(256) attention_max_kernel(const int32_t* __restrict__ col,
                                                            const int32_t* __restrict__ rowidx,
                                                            int64_t E2,
                                                            const float* __restrict__ S, int NH,
                                                            uint32_t* M_ord) {
  const int S2 = 2 * NH;
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
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) m = fmaxf(m, red[k]);
    if (m > -INFINITY) atomicMax(M_ord, float_to_ord(m));
  }
}

// ------------------------------------------------------------------ fused edge pass
// LPE lanes per edge, CPL float4 chunks per lane; lane l of edge group g owns chunks
// q = c*LPE + (l % LPE), c < CPL, of the padded row (D4 = NH*Fp/4 chunks; head of q = q/(Fp/4)).
template <int LPE, int CPL>
__global__ void __launch_bounds__(256)
edge_forward_kernel(const float* __restrict__ Wh, const float* __restrict__ S,
                    const uint32_t* __restrict__ M_ord, const int32_t* __restrict__ rowptr,
                    const int32_t* __restrict__ col, const int32_t* __restrict__ perm,
                    int64_t N, int NH, int F, int Fp, int concat, int const_att,
                    const float* __restrict__ bias, float p_drop, uint64_t seed,
                    float* __restrict__ out, float* __restrict__ alpha,
                    float* __restrict__ den_out, long long* __restrict__ argmax, int lds_row) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int EPW = 64 / LPE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / LPE, li = lane % LPE;
  const int D4 = NH * Fp / 4, F4 = Fp / 4, S2 = 2 * NH;
  float* row_lds = smem + wave * lds_row;      // Dp floats (head-mean staging)
  float* den_lds = row_lds + NH * Fp;          // NH floats
  const float M = const_att ? 0.f : ord_to_float(*M_ord);
  const bool drop = p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - p_drop) : 1.f;
  const float4* __restrict__ Wh4 = (const float4*)Wh;

  int q[CPL], hc[CPL];
  bool vq[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    q[c] = c * LPE + li;
    vq[c] = q[c] < D4;
    hc[c] = vq[c] ? q[c] / F4 : 0;
  }

  for (int64_t n = blockIdx.x * 4ll + wave; n < N; n += gridDim.x * 4ll) {
    const int beg = rowptr[n], end = rowptr[n + 1];
    float sd[CPL], dn[CPL];
    float4 acc[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      sd[c] = const_att ? 0.f : S[n * S2 + NH + hc[c]];
      dn[c] = 0.f;
      acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int e = beg + grp; e < end; e += EPW) {
      const int64_t s = col[e];
      const int64_t ep = drop ? (int64_t)perm[e] : 0;
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        if (!vq[c]) continue;
        const float4 v = Wh4[s * D4 + q[c]];
        const float ex = const_att ? 1.f : att_exp(S[s * S2 + hc[c]] + sd[c], M);
        dn[c] += ex;
        float w = ex;
        if (drop) w = dropout_keep(seed, ep * NH + hc[c], p_drop) ? ex * drop_scale : 0.f;
        acc[c] = fma4(w, v, acc[c]);
      }
    }
    // combine the EPW edge groups (butterfly: every group ends with the totals)
#pragma unroll
    for (int off = LPE; off < 64; off <<= 1) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        acc[c] = add4(acc[c], shfl_xor4(acc[c], off));
        dn[c] += __shfl_xor(dn[c], off);
      }
    }
    if (grp == 0) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        if (!vq[c]) continue;
        const float inv = 1.f / (dn[c] + kSoftmaxEps);
        const float4 o = acc[c] * inv;
        const int h = hc[c], f0 = q[c] * 4 - h * Fp;
        if (f0 == 0) {
          den_lds[h] = dn[c];
          den_out[n * NH + h] = dn[c];
        }
        if (concat) {
          float* orow = out + n * (int64_t)(NH * F) + h * F;
          if ((F & 3) == 0) {
            float4 b = bias ? *(const float4*)(bias + h * F + f0) : make_float4(0.f, 0.f, 0.f, 0.f);
            *(float4*)(orow + f0) = add4(o, b);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (f0 + j < F) orow[f0 + j] = get4(o, j) + (bias ? bias[h * F + f0 + j] : 0.f);
          }
        } else {
          *(float4*)(row_lds + q[c] * 4) = o;
        }
      }
    }
    wave_lds_sync();
    if (!concat) {
      const float inv_nh = 1.f / (float)NH;
      for (int f = lane; f < F; f += 64) {
        float sum = 0.f;
        for (int h = 0; h < NH; ++h) sum += row_lds[h * Fp + f];
        out[n * F + f] = sum * inv_nh + (bias ? bias[f] : 0.f);
      }
    }
    // alpha in edge_index' order (pre-dropout, as the reference returns/stores it, :109-110)
    const int pairs = (end - beg) * NH;
    for (int idx = lane; idx < pairs; idx += 64) {
      const int eo = idx / NH, h = idx - eo * NH;
      const int e = beg + eo;
      float a;
      if (const_att) {
        a = 1.f / (den_lds[h] + kSoftmaxEps);
      } else {
        const float raw = S[(int64_t)col[e] * S2 + h] + S[n * S2 + NH + h];
        a = att_exp(raw, M) / (den_lds[h] + kSoftmaxEps);
        if (raw == M) {
          unsigned long long k = atomicAdd((unsigned long long*)argmax, 1ull);
          if (k < GATX_ARGMAX_CAP) argmax[1 + k] = (long long)e * NH + h;
        }
      }
      alpha[(int64_t)perm[e] * NH + h] = a;
    }
    wave_lds_sync();
  }
}

// ------------------------------------------------------------------ weights
// W_aug rows Dp.. Dp+2NH-1 = A2 . W with A2 = [A_src; A_dst] (2NH x D), deterministic split-K:
// block (i-chunk of 64 columns, c-chunk of 128 rows of W) -> partial[cb][h2][i].
constexpr int kMaxH2 = 32;
__global__ void __launch_bounds__(256) weff_partial_kernel(const float* __restrict__ W,
                                                           const float* __restrict__ a, int NH,
                                                           int F, int64_t F_in,
                                                           float* __restrict__ partial) {
  __shared__ float red[4][kMaxH2][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t i = blockIdx.x * 64ll + tx;
  const int D = NH * F, H2 = 2 * NH;
  const int c0 = blockIdx.y * 128 + ty * 32;
  float acc[kMaxH2];
#pragma unroll
  for (int h = 0; h < kMaxH2; ++h) acc[h] = 0.f;
  for (int cc = 0; cc < 32; ++cc) {
    const int c = c0 + cc;
    if (c >= D) break;
    const float w = (i < F_in) ? W[(int64_t)c * F_in + i] : 0.f;
    const int k = c / F, f = c - k * F;
#pragma unroll
    for (int h = 0; h < kMaxH2; ++h) {
      if (h >= H2) break;
      const int hh = h < NH ? h : h - NH;
      const float av = a[(int64_t)hh * 2 * D + k * 2 * F + (h < NH ? 0 : F) + f];
      acc[h] = fmaf(av, w, acc[h]);
    }
  }
#pragma unroll
  for (int h = 0; h < kMaxH2; ++h)
    if (h < H2) red[ty][h][tx] = acc[h];
  __syncthreads();
  if (ty == 0 && i < F_in) {
    for (int h = 0; h < H2; ++h) {
      float s = red[0][h][tx] + red[1][h][tx] + red[2][h][tx] + red[3][h][tx];
      partial[((int64_t)blockIdx.y * H2 + h) * F_in + i] = s;
    }
  }
}

__global__ void __launch_bounds__(256) waug_assemble_kernel(const float* __restrict__ W,
                                                            const float* __restrict__ partial,
                                                            int n_cb, int NH, int F, int Fp,
                                                            int H2, int64_t F_in,
                                                            float* __restrict__ W_aug) {
  const int64_t Dp = (int64_t)NH * Fp;
  const int64_t total = (Dp + H2) * F_in;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / F_in, i = t - r * F_in;
    float v;
    if (r < Dp) {
      const int h = (int)(r / Fp), f = (int)(r - (int64_t)h * Fp);
      v = (f < F) ? W[((int64_t)h * F + f) * F_in + i] : 0.f;
    } else {
      const int h2 = (int)(r - Dp);
      v = 0.f;
      for (int cb = 0; cb < n_cb; ++cb) v += partial[((int64_t)cb * H2 + h2) * F_in + i];
    }
    W_aug[t] = v;
  }
}

inline unsigned grid_for(int64_t n, int block = 256, int64_t cap = 16384) {
  int64_t g = ceil_div(n > 0 ? n : 1, block);
  return (unsigned)(g < cap ? g : cap);
}

template <int LPE, int CPL>
int launch_edge_forward(unsigned grid, size_t lds, hipStream_t st, const float* Wh,
                        const float* S, const uint32_t* M_ord, const int32_t* rowptr,
                        const int32_t* col, const int32_t* perm, int64_t N, int NH, int F, int Fp,
                        int concat, int const_att, const float* bias, float p, uint64_t seed,
                        float* out, float* alpha, float* den, int64_t* argmax, int lds_row) {
  edge_forward_kernel<LPE, CPL><<<grid, 256, lds, st>>>(Wh, S, M_ord, rowptr, col, perm, N, NH,
                                                        F, Fp, concat, const_att, bias, p, seed,
                                                        out, alpha, den, (long long*)argmax,
                                                        lds_row);
  GATX_LAUNCH_CHECK("edge_forward");
  return 0;
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" int gatx_prepare_weights(const float* W, const float* a, int NH, int F, int64_t F_in,
                                    float* W_aug, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  GATX_REQUIRE(NH >= 1 && F >= 1 && F_in >= 1, "prepare_weights: bad sizes");
  const int Fp = (int)round_up(F, 4);
  const int H2 = a ? 2 * NH : 0;
  GATX_REQUIRE(H2 <= kMaxH2, "prepare_weights: num_heads > %d unsupported", kMaxH2 / 2);
  const int D = NH * F;
  const int n_cb = (int)ceil_div(D, 128);
  float* partial = nullptr;
  if (H2) {
    // split-K partials are staged in the tail of the caller's buffer, which holds
    // gatx_prepare_weights_floats() floats: (Dp + 2NH) * F_in for W_aug + n_cb * 2NH * F_in.
    partial = W_aug + ((int64_t)NH * Fp + H2) * F_in;
    dim3 g((unsigned)ceil_div(F_in, 64), (unsigned)n_cb);
    weff_partial_kernel<<<g, 256, 0, st>>>(W, a, NH, F, F_in, partial);
    GATX_LAUNCH_CHECK("weff_partial");
  }
  waug_assemble_kernel<<<grid_for(((int64_t)NH * Fp + H2) * F_in), 256, 0, st>>>(
      W, partial, n_cb, NH, F, Fp, H2, F_in, W_aug);
  GATX_LAUNCH_CHECK("waug_assemble");
  return 0;
}

extern "C" int64_t gatx_prepare_weights_floats(int NH, int F, int64_t F_in, int has_a) {
  const int64_t Fp = round_up(F, 4), H2 = has_a ? 2 * NH : 0;
  return (NH * Fp + H2 + ceil_div((int64_t)NH * F, 128) * H2) * F_in;
}

extern "C" int gatx_attention_max(const int32_t* col, const int32_t* rowidx, int64_t E2,
                                  const float* S, int NH, uint32_t* M_ord, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  hipError_t r = hipMemsetAsync(M_ord, 0, sizeof(uint32_t), st);
  if (r != hipSuccess) { set_error("memset: %s", hipGetErrorString(r)); return (int)r; }
  if (E2 == 0) return 0;
  attention_max_kernel<<<grid_for(E2, 256, 4096), 256, 0, st>>>(col, rowidx, E2, S, NH, M_ord);
  GATX_LAUNCH_CHECK("attention_max");
  return 0;
}

extern "C" int gatx_edge_forward(const float* Wh, const float* S, const uint32_t* M_ord,
                                 const int32_t* rowptr, const int32_t* col, const int32_t* perm,
                                 int64_t N, int NH, int F, int concat, int const_att,
                                 const float* bias, float p, uint64_t seed, float* out,
                                 float* alpha, float* den, int64_t* argmax, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  GATX_REQUIRE(NH >= 1 && F >= 1, "edge_forward: bad sizes");
  GATX_REQUIRE(concat || bias == nullptr || NH == 1,
               "edge_forward: bias with head-mean needs num_heads == 1");
  if (N == 0) return 0;
  const int Fp = (int)round_up(F, 4);
  const int64_t D4 = (int64_t)NH * Fp / 4;
  const RowGeom g = row_geom(D4);
  GATX_REQUIRE(g.cpl <= 8, "edge_forward: num_heads*out_features > 2048 unsupported");
  GATX_REQUIRE(p >= 0.f && p < 1.f, "edge_forward: dropout must be in [0, 1)");
  const int lds_row = (int)round_up((int64_t)NH * Fp + NH, 4);
  const size_t lds = (size_t)4 * lds_row * sizeof(float);
  GATX_REQUIRE(lds <= 160 * 1024, "edge_forward: row too wide for LDS staging");
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(N, 4), 65536);
#define GATX_EF(L, C)                                                                          \
  return launch_edge_forward<L, C>(grid, lds, st, Wh, S, M_ord, rowptr, col, perm, N, NH, F,   \
                                   Fp, concat, const_att, bias, p, seed, out, alpha, den,      \
                                   argmax, lds_row)
  if (g.lpe == 64) {
    switch (g.cpl) {
      case 1: GATX_EF(64, 1); case 2: GATX_EF(64, 2); case 3: GATX_EF(64, 3);
      case 4: GATX_EF(64, 4); case 5: GATX_EF(64, 5); case 6: GATX_EF(64, 6);
      case 7: GATX_EF(64, 7); default: GATX_EF(64, 8);
    }
  }
  switch (g.lpe) {
    case 1: GATX_EF(1, 1); case 2: GATX_EF(2, 1); case 4: GATX_EF(4, 1);
    case 8: GATX_EF(8, 1); case 16: GATX_EF(16, 1); default: GATX_EF(32, 1);
  }
#undef GATX_EF
}
