// Attention-norm regulariser of GATModel.calc_attention_norm (models/GATModel.py:189-234),
// fused over the CSR of edge_index':
//   norm_l = sum_{e,h} | alpha_l[e,h] * deg[dst_e] - 1 | / E'     (torch.norm(p=1) / E', :224-225)
//   result = mean over layers                                          (:230)
// deg[dst] is the in-degree over edge_index' (the reference's scatter of ones over
// edge_index[1], :195-200) = rowptr[dst+1] - rowptr[dst]. One pass per layer reads alpha once
// in edge_index' order instead of building (E', NH) temporaries.
// The gradient is sign(alpha*deg - 1) * deg * g / (E' * L) (torch's |x|' = sgn x, 0 at 0).
// Sums: per-thread partials, a fixed-order block tree and one fixed-order final pass, so the
// result is bitwise reproducible.
#include "gatx_common.h"

namespace gatx {
namespace {

constexpr int kNormBlocks = 1024;

__device__ inline float deg_of(const int32_t* __restrict__ rowptr, int32_t d) {
  return (float)(rowptr[d + 1] - rowptr[d]);
}

// alpha * deg - 1 with the product and the difference each rounded, as torch's two fp32 ops:
// an FMA would return the exact residual where the reference gets 0 (and a zero gradient).
__device__ inline float excess(float a, float deg) {
#pragma clang fp contract(off)
  const float p = a * deg;
  return p - 1.f;
}

// Edges are visited in edge_index' order (alpha rows read contiguously); the destination id
// comes from edge_index'[1] (int64 or int32), its degree from the L2-resident rowptr.
template <typename I>
__global__ void __launch_bounds__(256) attn_norm_partial_kernel(
    const float* __restrict__ alpha, int64_t E2, int NH, const I* __restrict__ dst,
    const int32_t* __restrict__ rowptr, float* __restrict__ part) {
  float s = 0.f;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E2;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float deg = deg_of(rowptr, (int32_t)dst[e]);
    const float* a = alpha + e * NH;
    for (int h = 0; h < NH; ++h) s += fabsf(excess(a[h], deg));
  }
  s = group_sum<64>(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) attn_norm_final_kernel(const float* __restrict__ part,
                                                              int nb, float scale, int accumulate,
                                                              float* __restrict__ out) {
  float s = 0.f;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) s += part[b];
  s = group_sum<64>(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
    out[0] = accumulate ? out[0] + v : v;
  }
}

template <typename I>
__global__ void __launch_bounds__(256) attn_norm_backward_kernel(
    const float* __restrict__ alpha, int64_t E2, int NH, const I* __restrict__ dst,
    const int32_t* __restrict__ rowptr, const float* __restrict__ g, float scale,
    float* __restrict__ g_alpha) {
  const float gs = g[0] * scale;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E2;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float deg = deg_of(rowptr, (int32_t)dst[e]);
    for (int h = 0; h < NH; ++h) {
      const float t = excess(alpha[e * NH + h], deg);
      const float sg = t > 0.f ? 1.f : (t < 0.f ? -1.f : 0.f);
      g_alpha[e * NH + h] = gs * sg * deg;
    }
  }
}

// All layers in one pass (round 6): the layers share edge_index' and rowptr, so one read of dst and
// of the degrees serves them all. Per layer the same per-thread partials, grid and block tree as
// attn_norm_partial_kernel, so every layer's sum is bitwise the per-layer launch's.
constexpr int kNormMaxLayers = 8;
struct NormLayers {
  const float* alpha[kNormMaxLayers];
  int nh[kNormMaxLayers];
};

template <typename I>
__global__ void __launch_bounds__(256) attn_norm_multi_partial_kernel(
    NormLayers L, int nl, int64_t E2, const I* __restrict__ dst,
    const int32_t* __restrict__ rowptr, float* __restrict__ part) {
  float s[kNormMaxLayers];
#pragma unroll
  for (int l = 0; l < kNormMaxLayers; ++l) s[l] = 0.f;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E2;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float deg = deg_of(rowptr, (int32_t)dst[e]);
#pragma unroll
    for (int l = 0; l < kNormMaxLayers; ++l) {
      if (l >= nl) break;
      const float* a = L.alpha[l] + e * L.nh[l];
      for (int h = 0; h < L.nh[l]; ++h) s[l] += fabsf(excess(a[h], deg));
    }
  }
  __shared__ float red[kNormMaxLayers][4];
#pragma unroll
  for (int l = 0; l < kNormMaxLayers; ++l) {
    if (l >= nl) break;
    const float t = group_sum<64>(s[l]);
    if ((threadIdx.x & 63) == 0) red[l][threadIdx.x >> 6] = t;
  }
  __syncthreads();
  if (threadIdx.x < nl)
    part[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] =
        (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

// the layers' finals in layer order: out = v_0, then out + v_1, ... (as the per-layer launches
// with accumulate)
__global__ void __launch_bounds__(256) attn_norm_multi_final_kernel(const float* __restrict__ part,
                                                                    int nb, int nl, float scale,
                                                                    float* __restrict__ out) {
#pragma clang fp contract(off)   // v = sum * scale rounded, then acc + v: the per-layer finals' ops
  __shared__ float red[4];
  float acc = 0.f;
  for (int l = 0; l < nl; ++l) {
    float s = 0.f;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) s += part[(int64_t)l * nb + b];
    s = group_sum<64>(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    const float v = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
    acc = l == 0 ? v : acc + v;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = acc;
}

inline unsigned grid_for(int64_t n, int64_t cap) {
  const int64_t g = ceil_div(n > 0 ? n : 1, 256);
  return (unsigned)(g < cap ? g : cap);
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" size_t gatx_attention_norm_workspace_bytes(void) {
  return sizeof(float) * kNormBlocks;
}

extern "C" int gatx_attention_norm(const float* alpha, int64_t E2, int NH, const void* dst,
                                   int dst_is64, const int32_t* rowptr, float scale,
                                   int accumulate, float* out, void* workspace,
                                   gatx_stream_t s) {
  GATX_REQUIRE(E2 >= 0 && NH >= 1, "attention_norm: bad sizes");
  hipStream_t st = (hipStream_t)s;
  const unsigned nb = grid_for(E2, kNormBlocks);
  float* part = (float*)workspace;
  if (dst_is64)
    attn_norm_partial_kernel<int64_t><<<nb, 256, 0, st>>>(alpha, E2, NH, (const int64_t*)dst,
                                                          rowptr, part);
  else
    attn_norm_partial_kernel<int32_t><<<nb, 256, 0, st>>>(alpha, E2, NH, (const int32_t*)dst,
                                                          rowptr, part);
  GATX_LAUNCH_CHECK("attention_norm");
  attn_norm_final_kernel<<<1, 256, 0, st>>>(part, (int)nb, scale, accumulate, out);
  GATX_LAUNCH_CHECK("attention_norm_final");
  return 0;
}

extern "C" size_t gatx_attention_norm_multi_workspace_bytes(int num_layers) {
  return sizeof(float) * kNormBlocks * (size_t)(num_layers > 0 ? num_layers : 1);
}

extern "C" int gatx_attention_norm_multi(const float* const* alphas, const int* num_heads,
                                         int num_layers, int64_t E2, const void* dst,
                                         int dst_is64, const int32_t* rowptr, float scale,
                                         float* out, void* workspace, gatx_stream_t s) {
  GATX_REQUIRE(E2 >= 0 && num_layers >= 1 && num_layers <= kNormMaxLayers,
               "attention_norm_multi: bad sizes");
  NormLayers L{};
  for (int l = 0; l < num_layers; ++l) {
    GATX_REQUIRE(alphas[l] != nullptr && num_heads[l] >= 1, "attention_norm_multi: bad layer");
    L.alpha[l] = alphas[l];
    L.nh[l] = num_heads[l];
  }
  hipStream_t st = (hipStream_t)s;
  const unsigned nb = grid_for(E2, kNormBlocks);
  float* part = (float*)workspace;
  if (dst_is64)
    attn_norm_multi_partial_kernel<int64_t><<<nb, 256, 0, st>>>(L, num_layers, E2,
                                                                (const int64_t*)dst, rowptr, part);
  else
    attn_norm_multi_partial_kernel<int32_t><<<nb, 256, 0, st>>>(L, num_layers, E2,
                                                                (const int32_t*)dst, rowptr, part);
  GATX_LAUNCH_CHECK("attention_norm_multi");
  attn_norm_multi_final_kernel<<<1, 256, 0, st>>>(part, (int)nb, num_layers, scale, out);
  GATX_LAUNCH_CHECK("attention_norm_multi_final");
  return 0;
}

extern "C" int gatx_attention_norm_backward(const float* alpha, int64_t E2, int NH,
                                            const void* dst, int dst_is64,
                                            const int32_t* rowptr, const float* g, float scale,
                                            float* g_alpha, gatx_stream_t s) {
  GATX_REQUIRE(E2 >= 0 && NH >= 1, "attention_norm_backward: bad sizes");
  if (E2 == 0) return 0;
  hipStream_t st = (hipStream_t)s;
  if (dst_is64)
    attn_norm_backward_kernel<int64_t><<<grid_for(E2, 8192), 256, 0, st>>>(
        alpha, E2, NH, (const int64_t*)dst, rowptr, g, scale, g_alpha);
  else
    attn_norm_backward_kernel<int32_t><<<grid_for(E2, 8192), 256, 0, st>>>(
        alpha, E2, NH, (const int32_t*)dst, rowptr, g, scale, g_alpha);
  GATX_LAUNCH_CHECK("attention_norm_backward");
  return 0;
}
