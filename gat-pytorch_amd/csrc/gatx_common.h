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

}  // namespace gatx
