// Internal helpers shared by the gatx HIP translation units (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/gatx.h"

namespace gatx {

constexpr int kWave = 64;            // CDNA wavefront
constexpr float kLeakySlope = 0.01f; // nn.LeakyReLU() default (models/gat_layer.py:87)
constexpr float kSoftmaxEps = 1e-8f; // models/gat_layer.py:109

void set_error(const char* fmt, ...);

// Check the launch that was just enqueued; returns from the calling entry point on failure.
#define GATX_LAUNCH_CHECK(what)                                                    \
  do {                                                                             \
    hipError_t _e = hipGetLastError();                                             \
    if (_e != hipSuccess) {                                                        \
      ::gatx::set_error("%s: %s", what, hipGetErrorString(_e));                    \
      return (int)_e;                                                              \
    }                                                                              \
  } while (0)

#define GATX_REQUIRE(cond, ...)                                                    \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      ::gatx::set_error(__VA_ARGS__);                                              \
      return GATX_EINVAL;                                                          \
    }                                                                              \
  } while (0)

#define GATX_CALL(expr)                                                            \
  do {                                                                             \
    int _r = (expr);                                                               \
    if (_r != 0) return _r;                                                        \
  } while (0)

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// Order-preserving float <-> uint32 map: a < b (as floats, no NaN) <=> ord(a) < ord(b).
// uint 0 is below every float, so a zero-filled word is the identity of atomicMax.
__device__ inline uint32_t float_to_ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord_to_float(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(u);
}

// Attention-dropout keep mask: element (e, h) of alpha in edge_index' order is kept iff
// u >= p, u = top 24 bits of splitmix64(seed + (e*NH + h + 1) * gamma) / 2^24.
// Counter-based, so forward and backward (and the CPU oracle) regenerate the same mask.
__device__ inline bool dropout_keep(uint64_t seed, int64_t idx, float p) {
  uint64_t z = seed + (uint64_t)(idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  float u = (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
  return u >= p;
}

// exp of the reference's shifted, LeakyReLU'd logit: 0.01 * (raw - M) (raw - M <= 0 always).
__device__ inline float att_exp(float raw, float M) { return __expf(kLeakySlope * (raw - M)); }

// ELU (GATModel's activation, nn.ELU(alpha=1)) for the fused epilogues: v > 0 ? v : expm1(v),
// with expm1 as a degree-5 Taylor polynomial above -1/16 (relative error < 1e-8) and
// exp2(v log2 e) - 1 below (v_exp_f32; the result is then >= 0.06 in magnitude, error ~1e-7).
// About ten VALU operations per element against ocml's expm1f, which made the ELU epilogue of
// the first layer's output projection VALU-bound (46 M elements per PPI step).
__device__ inline float elu_act(float v) {
  const float p = v * (1.f + v * (0.5f + v * (1.f / 6.f + v * (1.f / 24.f + v * (1.f / 120.f)))));
  const float e = __builtin_amdgcn_exp2f(v * 1.44269504088896341f) - 1.f;
  return v > 0.f ? v : (v > -0.0625f ? p : e);
}

// elu_act of two elements, branch-free, the polynomial in packed fp32: the same expression,
// contracted into the same fma chain as elu_act's (fp-contract), so bit-identical per component.
// The compiler turns the scalar form's selects into an exec-masked branch per element around the
// exp and the polynomial; in an epilogue of 128 elements per lane that is a few hundred scalar
// branch instructions beside the VALU work.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ inline f32x2 elu_act2(f32x2 v) {
  const f32x2 p = v * ((f32x2)(1.f) + v * ((f32x2)(0.5f) + v * ((f32x2)(1.f / 6.f) +
                  v * ((f32x2)(1.f / 24.f) + v * (f32x2)(1.f / 120.f)))));
  const f32x2 w = v * (f32x2)(1.44269504088896341f);
  const float e0 = __builtin_amdgcn_exp2f(w.x) - 1.f, e1 = __builtin_amdgcn_exp2f(w.y) - 1.f;
  f32x2 r;
  r.x = v.x > 0.f ? v.x : (v.x > -0.0625f ? p.x : e0);
  r.y = v.y > 0.f ? v.y : (v.y > -0.0625f ? p.y : e1);
  return r;
}

__device__ inline float4 operator*(float4 a, float s) {
  return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}
__device__ inline float4 fma4(float s, float4 a, float4 c) {
  return make_float4(fmaf(s, a.x, c.x), fmaf(s, a.y, c.y), fmaf(s, a.z, c.z), fmaf(s, a.w, c.w));
}
__device__ inline float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ inline float4 shfl_xor4(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m),
                     __shfl_xor(v.w, m));
}
__device__ inline float get4(const float4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// n 32-bit words set to 0 (the library's zero fill: no hipMemsetAsync inside a captured step)
static __global__ void zero_words_kernel(uint32_t* p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0u;
}

// Intra-wave LDS hand-off: order this wave's LDS writes before its later LDS reads.
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Edge-kernel lane geometry for a padded row of D4 float4 chunks: LPE lanes per edge
// (power of two), CPL float4 chunks per lane, 64/LPE edges in flight per wave.
struct RowGeom {
  int lpe, cpl;
};
inline RowGeom row_geom(int64_t D4) {
  if (D4 >= 64) return {64, (int)ceil_div(D4, 64)};
  int l = 1;
  while (l < D4) l <<= 1;
  return {l, 1};
}

template <int CTRL>
__device__ inline float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// Sum over aligned groups of L lanes (L = 1..64); every lane of a group gets the group's total.
// xor 1/2 via quad_perm, 4/8 via row half-mirror / mirror (valid once the smaller groups agree),
// 16/32 via the gfx950 permlane swaps (r[0] + r[1] = own + partner).
template <int L>
__device__ inline float group_sum(float v) {
  if (L >= 2) v += dpp<0xB1>(v);
  if (L >= 4) v += dpp<0x4E>(v);
  if (L >= 8) v += dpp<0x141>(v);
  if (L >= 16) v += dpp<0x140>(v);
  if (L >= 32) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if (L >= 64) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  return v;
}

// Reduce-scatter of H values (H a power of two <= 64) over the 64 lanes: returns, in every
// lane, the wave-wide sum of v[h] for h = h_of_lane (h = the top log2(H) lane bits read as
// 32->H/2, 16->H/4, ...; lanes sharing those bits hold the same total). log2(H) exchange steps
// (each halves the values a lane keeps) + 6 - log2(H) plain butterfly steps: H/2 + ... + 1
// cross-lane moves plus the plain ones, instead of 6 per value. Partners at each level differ
// exactly in that level's lane bit (permlane swaps for 32/16, mirrors for 8/4, quad perms).
template <int H>
__device__ inline float reduce_scatter64(float (&v)[H], int lane, int& h) {
  int cnt = H;
  h = 0;
#pragma unroll
  for (int lev = 0; lev < 6; ++lev) {
    const int bit = 5 - lev;
    const bool up = (lane >> bit) & 1;
    if (cnt > 1) {
      const int half = cnt / 2;
#pragma unroll
      for (int j = 0; j < half; ++j) {
        const float x0 = v[j], x1 = v[half + j];
        if (lev < 2) {
          auto r = lev == 0 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(x0),
                                                               __float_as_uint(x1), false, false)
                            : __builtin_amdgcn_permlane16_swap(__float_as_uint(x0),
                                                               __float_as_uint(x1), false, false);
          v[j] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
        } else {
          const float send = up ? x0 : x1;
          float recv;
          if (lev == 2) recv = dpp<0x140>(send);
          else if (lev == 3) recv = dpp<0x141>(send);
          else if (lev == 4) recv = dpp<0x4E>(send);
          else recv = dpp<0xB1>(send);
          v[j] = (up ? x1 : x0) + recv;
        }
      }
      if (up) h += half;
      cnt = half;
    } else {
      float x = v[0];
      if (lev < 2) {
        auto r = lev == 0 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(x),
                                                             __float_as_uint(x), false, false)
                          : __builtin_amdgcn_permlane16_swap(__float_as_uint(x),
                                                             __float_as_uint(x), false, false);
        x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
      } else if (lev == 2) x += dpp<0x140>(x);
      else if (lev == 3) x += dpp<0x141>(x);
      else if (lev == 4) x += dpp<0x4E>(x);
      else x += dpp<0xB1>(x);
      v[0] = x;
    }
  }
  return v[0];
}

}  // namespace gatx
