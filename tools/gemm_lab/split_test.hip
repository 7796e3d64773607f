#include <hip/hip_runtime.h>
#include <stdint.h>
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ inline void split_pair_s(float x, float y, float c, uint32_t& h, uint32_t& l) {
  const float yx = x * c, yy = y * c;
  const _Float16 hx = (_Float16)yx, hy = (_Float16)yy;
  const _Float16 lx = (_Float16)__builtin_fmaf((float)hx, -1.0f, yx);
  const _Float16 ly = (_Float16)__builtin_fmaf((float)hy, -1.0f, yy);
  f16x2 hv = {hx, hy}, lv = {lx, ly};
  h = __builtin_bit_cast(uint32_t, hv);
  l = __builtin_bit_cast(uint32_t, lv);
}
__global__ void k(const float4* in, uint2* oh, uint2* ol, const float* cs) {
  float4 v = in[threadIdx.x];
  float c = cs[threadIdx.x];
  uint32_t h0, l0, h1, l1;
  split_pair_s(v.x, v.y, c, h0, l0);
  split_pair_s(v.z, v.w, c, h1, l1);
  oh[threadIdx.x] = make_uint2(h0, h1);
  ol[threadIdx.x] = make_uint2(l0, l1);
}
