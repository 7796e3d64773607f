// The task modules' loss, fused: BCEWithLogitsLoss (mean; optional pos_weight) of PPI_GAT
// (models/ppi_gat.py:11,19) and PatternGAT (models/pattern_gat.py:11-15). torch runs it as ~10
// elementwise / reduction launches forward and ~9 backward; at PATTERN's batch of 8 graphs (952
// logits) each is a ~4 us launch. Here: one launch computes the mean loss AND d(loss)/d(logit)
// (the gradient is local, so it is produced in the same pass and kept for the backward), one
// launch scales it by the upstream gradient. Fixed-order reductions: bitwise reproducible.
//   lw = 1 + (p - 1) y;  l = (1 - y) x + lw (log1p(exp(-|x|)) + max(-x, 0));  mean over n
//   dl/dx = (lw sigmoid(x) - p y) / n          (torch's binary_cross_entropy_with_logits)
#include "gatx_common.h"

namespace gatx {
namespace {

constexpr int kLossBlocks = 1024;

__device__ inline void bce_elem(float x, float y, float pw, float inv_n, float& l, float& g) {
  const float lw = 1.f + (pw - 1.f) * y;
  const float sp = log1pf(__expf(-fabsf(x))) + fmaxf(-x, 0.f);   // softplus(-x)
  l = (1.f - y) * x + lw * sp;
  const float sig = 1.f / (1.f + __expf(-x));
  g = (lw * sig - pw * y) * inv_n;
}

// fixed-order block sum of one value per thread (blockDim.x a multiple of 64)
__device__ inline float block_sum(float v, float* red) {
  v = group_sum<64>(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < nw; ++i) t += red[i];
  return t;   // valid in thread 0
}

__global__ void __launch_bounds__(1024) bce_small_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ y, int64_t n,
                                                         float pw, float* __restrict__ loss,
                                                         float* __restrict__ grad) {
  __shared__ float red[16];
  const float inv_n = 1.f / (float)n;
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    float l, g;
    bce_elem(x[i], y[i], pw, inv_n, l, g);
    grad[i] = g;
    s += l;
  }
  const float t = block_sum(s, red);
  if (threadIdx.x == 0) loss[0] = t * inv_n;
}

// Four elements per thread per round, all loads issued first (the loop is load-latency bound).
__global__ void __launch_bounds__(256) bce_partial_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ y, int64_t n,
                                                          float pw, float* __restrict__ part,
                                                          float* __restrict__ grad) {
  __shared__ float red[4];
  const float inv_n = 1.f / (float)n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float s = 0.f;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < n; i0 += 4 * stride) {
    float xv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * stride;
      xv[u] = i < n ? x[i] : 0.f;
      yv[u] = i < n ? y[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n) {
        float l, g;
        bce_elem(xv[u], yv[u], pw, inv_n, l, g);
        grad[i] = g;
        s += l;
      }
    }
  }
  const float t = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void __launch_bounds__(256) bce_final_kernel(const float* __restrict__ part, int nb,
                                                        int64_t n, float* __restrict__ loss) {
  __shared__ float red[4];
  float s = 0.f;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) s += part[b];
  const float t = block_sum(s, red);
  if (threadIdx.x == 0) loss[0] = t / (float)n;
}

__global__ void __launch_bounds__(256) scale_by_scalar_kernel(const float* __restrict__ g,
                                                              const float* __restrict__ v,
                                                              int64_t n, float* __restrict__ out) {
  const float s = g[0];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = s * v[i];
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" size_t gatx_bce_logits_workspace_bytes(void) { return sizeof(float) * kLossBlocks; }

extern "C" int gatx_bce_logits(const float* x, const float* y, int64_t n, float pos_weight,
                               float* loss, float* grad, void* workspace, gatx_stream_t s) {
  GATX_REQUIRE(n >= 1, "bce_logits: empty input");
  GATX_REQUIRE(x && y && loss && grad, "bce_logits: null buffer");
  hipStream_t st = (hipStream_t)s;
  if (n <= (1 << 16)) {
    bce_small_kernel<<<1, 1024, 0, st>>>(x, y, n, pos_weight, loss, grad);
    GATX_LAUNCH_CHECK("bce_small");
    return 0;
  }
  GATX_REQUIRE(workspace, "bce_logits: workspace needed above 65536 elements");
  const int nb = (int)std::min<int64_t>(ceil_div(n, 256), kLossBlocks);
  bce_partial_kernel<<<nb, 256, 0, st>>>(x, y, n, pos_weight, (float*)workspace, grad);
  GATX_LAUNCH_CHECK("bce_partial");
  bce_final_kernel<<<1, 256, 0, st>>>((const float*)workspace, nb, n, loss);
  GATX_LAUNCH_CHECK("bce_final");
  return 0;
}

extern "C" int gatx_scale_by_scalar(const float* g, const float* v, int64_t n, float* out,
                                    gatx_stream_t s) {
  if (n == 0) return 0;
  const int nb = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
  scale_by_scalar_kernel<<<nb, 256, 0, (hipStream_t)s>>>(g, v, n, out);
  GATX_LAUNCH_CHECK("scale_by_scalar");
  return 0;
}
