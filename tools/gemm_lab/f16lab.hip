// GEMM lab (tuning only, not part of libgatx.so): an f16x3 mainloop with the weight operand
// pre-split into fp16 planes and the activation split in the loop by v_fma_mix, the hi planes
// carrying the 2^11 factor (A x 64, B x 32), so the MFMA phase has no scaling multiplies.
//   C[M][N] = A[M][K] . B[N][K]^T, A fp32 k-contiguous, B given as planes (lab_split_b).
// Built standalone (tools/gemm_lab/build.sh) and timed against the library kernel by
// tools/gemm_lab/run_lab.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int TBM = 256, TBN = 256, NT = 512, WGM = 2, WGN = 4, MB = 4, NB = 2;

// One fp16 plane image of 256 rows x BK k: 16-byte (8-k) slots, slot-major; odd slots' rows XOR'd
// by 12 (conflict-free ds_read_b128 fragment reads, as gemm_x3.hip's PlaneImg).
template <int BK>
struct Img {
  static constexpr int BYTES = 256 * BK * 2;
  static __device__ inline int off(int r, int k) {
    const int s = k >> 3;
    return s * (256 * 16) + ((r ^ ((s & 1) * 12)) << 4) + ((k & 4) << 1);
  }
};

__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void* base, int64_t bytes) {
  const int nr = (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nr, 0x00020000);
}

// h = fp16_rn(x c), l = fp16_rn(x c - h) for a pair (x in the low halves): four v_fma_mix.
__device__ inline void split_mix(float x, float y, float c, uint32_t& h, uint32_t& l) {
  asm volatile(
      "v_fma_mixlo_f16 %0, %2, %4, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h), "=&v"(l)
      : "v"(x), "v"(y), "v"(c));
}

__device__ inline void tile_of(int64_t b, int64_t T, int64_t tiles_n, int64_t& tm, int64_t& tn) {
  const int64_t q = T / 8, r = T % 8;
  const int64_t xcd = b % 8, j = b / 8;
  const int64_t t = (xcd < r) ? xcd * (q + 1) + j : r * (q + 1) + (xcd - r) * q + j;
  tm = t / tiles_n;
  tn = t % tiles_n;
}

struct LabArgs {
  const float* A; int64_t lda;
  const uint16_t* Bp; int64_t brow;   // planes: row n at Bp + n * brow bytes: [K/8][2][8] fp16
  int64_t M, N, K;
  float* C; int64_t ldc;
  float binv;                          // 2^-11 / sB
  int* bad;                            // rows out of the fp16 range seen (lab: counted only)
};

template <int BK, bool SCALE>
__global__ void __launch_bounds__(NT, 1) f16v2_kernel(LabArgs g) {
  using I = Img<BK>;
  constexpr int PB = I::BYTES;
  constexpr int STAGE = 4 * PB;               // A_h A_l B_h B_l
  constexpr int NVA = BK / 8, NVB = BK / 8;   // float4 (A) / 16-B (B) loads per thread
  constexpr int TPR = BK / 4;                 // threads per row in staging
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 256 * 4];
  float* inv = (float*)(smem + 2 * STAGE);

  const int64_t T = ((g.M + TBM - 1) / TBM) * ((g.N + TBN - 1) / TBN);
  int64_t tm, tn;
  tile_of(blockIdx.x, T, (g.N + TBN - 1) / TBN, tm, tn);
  const int64_t m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  const int64_t arows = g.M - m0 < TBM ? g.M - m0 : TBM;
  const int64_t brows = g.N - n0 < TBN ? g.N - n0 : TBN;
  const auto ra = rsrc(g.A + m0 * g.lda, arows * g.lda * 4);
  const auto rb = rsrc((const char*)g.Bp + n0 * g.brow, brows * g.brow);
  // per-thread global byte offsets and LDS byte offsets of its staging pieces
  int voa[NVA], vob[NVB], oa[NVA], ob[NVB];
#pragma unroll
  for (int c = 0; c < NVA; ++c) {
    const int idx = tid + NT * c;
    const int r = idx / TPR, k = 4 * (idx % TPR);
    voa[c] = (r * (int)g.lda + k) * 4;
    oa[c] = I::off(r, k);
  }
#pragma unroll
  for (int c = 0; c < NVB; ++c) {
    const int idx = tid + NT * c;
    const int r = idx / TPR, j = idx % TPR;   // slot j >> 1, plane j & 1
    vob[c] = r * (int)g.brow + (j >> 1) * 32 + (j & 1) * 16;
    ob[c] = (2 + (j & 1)) * PB + I::off(r, 8 * (j >> 1));
  }
  float4 va[NVA];
  uint4 vb[NVB];
  auto load = [&](int kt) {
#pragma unroll
    for (int c = 0; c < NVA; ++c)
      va[c] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, voa[c], kt * BK * 4, 0));
#pragma unroll
    for (int c = 0; c < NVB; ++c)
      vb[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb, vob[c], kt * BK * 4, 0));
  };
  float cs[NVA], amax[NVA];
#pragma unroll
  for (int c = 0; c < NVA; ++c) { cs[c] = 64.f; amax[c] = 0.f; }
  auto store = [&](char* st) {
#pragma unroll
    for (int c = 0; c < NVA; ++c) {
      const float4 v = va[c];
      amax[c] = fmaxf(amax[c], fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      uint32_t h0, l0, h1, l1;
      split_mix(v.x, v.y, cs[c], h0, l0);
      split_mix(v.z, v.w, cs[c], h1, l1);
      *(uint2*)(st + oa[c]) = make_uint2(h0, h1);
      *(uint2*)(st + PB + oa[c]) = make_uint2(l0, l1);
    }
#pragma unroll
    for (int c = 0; c < NVB; ++c) *(uint4*)(st + ob[c]) = vb[c];
  };
  floatx16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (int)(g.K / BK);
  load(0);
  if constexpr (SCALE) {
#pragma unroll
    for (int c = 0; c < NVA; ++c) {
      const float4 v = va[c];
      float m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
#pragma unroll
      for (int o = 1; o < TPR; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
      int e = 0;
      (void)frexpf(m, &e);
      const float sc = (m > 0.f && m <= 3.0e38f) ? ldexpf(1.f, 8 - e) : 1.f;
      cs[c] = 64.f * sc;
      if ((tid % TPR) == 0) inv[(tid + NT * c) / TPR] = 1.f / sc;
    }
  } else {
    if (tid < 256) inv[tid] = 1.f;
  }
  store(smem);
  if (nk > 1) load(1);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
#pragma unroll
    for (int q = 0; q < BK / 16; ++q) {
      f16x8 fa[MB][2], fb[NB][2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int x = 0; x < MB; ++x)
          fa[x][p] = *(const f16x8*)(cur + p * PB +
                                     I::off(wm * (MB * 32) + x * 32 + (lane & 31), 16 * q + 8 * (lane >> 5)));
#pragma unroll
        for (int x = 0; x < NB; ++x)
          fb[x][p] = *(const f16x8*)(cur + (2 + p) * PB +
                                     I::off(wn * (NB * 32) + x * 32 + (lane & 31), 16 * q + 8 * (lane >> 5)));
      }
      if (q == 0) {
        if (kt + 1 < nk) store(nxt);
        if (kt + 2 < nk) load(kt + 2);
      }
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][1], fa[mi][0], acc[mi][ni], 0, 0, 0);
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][1], acc[mi][ni], 0, 0, 0);
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][0], acc[mi][ni], 0, 0, 0);
    }
    __syncthreads();
  }
  // range check (lab: count only): a row max over 1023 (64 a_h must be a finite fp16) or a
  // nonzero row max below 2^-9 (its residual plane would be subnormal)
  bool bad = false;
#pragma unroll
  for (int c = 0; c < NVA; ++c) {
    float m = amax[c];
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
    const float s = cs[c] * (1.f / 64.f);
    bad |= !(m * s <= 1023.f) || (m > 0.f && m * s < 0x1p-9f);
  }
  if (__syncthreads_or(bad) && tid == 0) atomicAdd(g.bad, 1);
  const int lr = lane & 31, lc = 4 * (lane >> 5);
#pragma unroll
  for (int mi = 0; mi < MB; ++mi) {
    const int rl = wm * (MB * 32) + mi * 32 + lr;
    const int64_t row = m0 + rl;
    if (row >= g.M) continue;
    const float f = inv[rl] * g.binv;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * (NB * 32) + ni * 32 + 8 * j + lc;
        if (col + 3 < g.N) {
          *(float4*)(g.C + row * g.ldc + col) =
              make_float4(acc[mi][ni][4 * j] * f, acc[mi][ni][4 * j + 1] * f,
                          acc[mi][ni][4 * j + 2] * f, acc[mi][ni][4 * j + 3] * f);
        }
      }
    }
  }
}

// v3: the same staging with 32-deep K-tiles, the MFMA phase on v_mfma_f32_16x16x32_f16 (one
// instruction per plane pair covers the whole K-tile; the guide measures ~1.12-1.15x the FLOP/s of
// 32x32x16 under load at equal cycles, from the clock the chip holds). Wave tile 128 x 64 =
// 8 x 4 blocks of 16 x 16; A fragments read just in time per 16-row block (register budget).
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <bool SCALE>
__global__ void __launch_bounds__(NT, 1) f16v3_kernel(LabArgs g) {
  constexpr int BK = 32;
  using I = Img<BK>;
  constexpr int PB = I::BYTES;
  constexpr int STAGE = 4 * PB;
  constexpr int NVA = BK / 8, NVB = BK / 8, TPR = BK / 4;
  constexpr int M16 = 8, N16 = 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 256 * 4];
  float* inv = (float*)(smem + 2 * STAGE);
  const int64_t T = ((g.M + TBM - 1) / TBM) * ((g.N + TBN - 1) / TBN);
  int64_t tm, tn;
  tile_of(blockIdx.x, T, (g.N + TBN - 1) / TBN, tm, tn);
  const int64_t m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int64_t arows = g.M - m0 < TBM ? g.M - m0 : TBM;
  const int64_t brows = g.N - n0 < TBN ? g.N - n0 : TBN;
  const auto ra = rsrc(g.A + m0 * g.lda, arows * g.lda * 4);
  const auto rb = rsrc((const char*)g.Bp + n0 * g.brow, brows * g.brow);
  int voa[NVA], vob[NVB], oa[NVA], ob[NVB];
#pragma unroll
  for (int c = 0; c < NVA; ++c) {
    const int idx = tid + NT * c;
    const int r = idx / TPR, k = 4 * (idx % TPR), j = idx % TPR;
    voa[c] = (r * (int)g.lda + k) * 4;
    oa[c] = I::off(r, k);
    vob[c] = r * (int)g.brow + (j >> 1) * 32 + (j & 1) * 16;
    ob[c] = (2 + (j & 1)) * PB + I::off(r, 8 * (j >> 1));
  }
  float4 va[NVA];
  uint4 vb[NVB];
  auto load = [&](int kt) {
#pragma unroll
    for (int c = 0; c < NVA; ++c)
      va[c] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, voa[c], kt * BK * 4, 0));
#pragma unroll
    for (int c = 0; c < NVB; ++c)
      vb[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb, vob[c], kt * BK * 4, 0));
  };
  float cs[NVA], amax[NVA];
#pragma unroll
  for (int c = 0; c < NVA; ++c) { cs[c] = 64.f; amax[c] = 0.f; }
  auto store = [&](char* st) {
#pragma unroll
    for (int c = 0; c < NVA; ++c) {
      const float4 v = va[c];
      amax[c] = fmaxf(amax[c], fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      uint32_t h0, l0, h1, l1;
      split_mix(v.x, v.y, cs[c], h0, l0);
      split_mix(v.z, v.w, cs[c], h1, l1);
      *(uint2*)(st + oa[c]) = make_uint2(h0, h1);
      *(uint2*)(st + PB + oa[c]) = make_uint2(l0, l1);
    }
#pragma unroll
    for (int c = 0; c < NVB; ++c) *(uint4*)(st + ob[c]) = vb[c];
  };
  floatx4 acc[M16][N16];
#pragma unroll
  for (int i = 0; i < M16; ++i)
#pragma unroll
    for (int j = 0; j < N16; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = (int)(g.K / BK);
  load(0);
  if constexpr (SCALE) {
#pragma unroll
    for (int c = 0; c < NVA; ++c) {
      const float4 v = va[c];
      float m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
#pragma unroll
      for (int o = 1; o < TPR; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
      int e = 0;
      (void)frexpf(m, &e);
      const float sc = (m > 0.f && m <= 3.0e38f) ? ldexpf(1.f, 8 - e) : 1.f;
      cs[c] = 64.f * sc;
      if ((tid % TPR) == 0) inv[(tid + NT * c) / TPR] = 1.f / sc;
    }
  } else {
    if (tid < 256) inv[tid] = 1.f;
  }
  store(smem);
  if (nk > 1) load(1);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    f16x8 fb[N16][2];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int x = 0; x < N16; ++x)
        fb[x][p] = *(const f16x8*)(cur + (2 + p) * PB + I::off(wn * 64 + x * 16 + fr, fk));
    f16x8 fa0[2], fa1[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) fa0[p] = *(const f16x8*)(cur + p * PB + I::off(wm * 128 + fr, fk));
    if (kt + 1 < nk) store(nxt);
    if (kt + 2 < nk) load(kt + 2);
#pragma unroll
    for (int mi = 0; mi < M16; ++mi) {
      if (mi + 1 < M16) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
          fa1[p] = *(const f16x8*)(cur + p * PB + I::off(wm * 128 + (mi + 1) * 16 + fr, fk));
      }
#pragma unroll
      for (int ni = 0; ni < N16; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[ni][1], fa0[0], acc[mi][ni], 0, 0, 0);
#pragma unroll
      for (int ni = 0; ni < N16; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[ni][0], fa0[1], acc[mi][ni], 0, 0, 0);
#pragma unroll
      for (int ni = 0; ni < N16; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[ni][0], fa0[0], acc[mi][ni], 0, 0, 0);
      fa0[0] = fa1[0];
      fa0[1] = fa1[1];
    }
    __syncthreads();
  }
  bool bad = false;
#pragma unroll
  for (int c = 0; c < NVA; ++c) {
    float m = amax[c];
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
    const float s = cs[c] * (1.f / 64.f);
    bad |= !(m * s <= 1023.f) || (m > 0.f && m * s < 0x1p-9f);
  }
  if (__syncthreads_or(bad) && tid == 0) atomicAdd(g.bad, 1);
  // lane -> output row (lane & 15) of the block, registers -> 4 consecutive columns
#pragma unroll
  for (int mi = 0; mi < M16; ++mi) {
    const int rl = wm * 128 + mi * 16 + fr;
    const int64_t row = m0 + rl;
    if (row >= g.M) continue;
    const float f = inv[rl] * g.binv;
#pragma unroll
    for (int ni = 0; ni < N16; ++ni) {
      const int64_t col = n0 + wn * 64 + ni * 16 + 4 * (lane >> 4);
      if (col + 3 < g.N)
        *(float4*)(g.C + row * g.ldc + col) =
            make_float4(acc[mi][ni][0] * f, acc[mi][ni][1] * f, acc[mi][ni][2] * f, acc[mi][ni][3] * f);
    }
  }
}

// v4: BOTH operands pre-split into planes in memory (A as a producer would write them: Ah =
// fp16(64 a), Al = fp16(64 a - Ah), the B planes' row layout), so the K-loop stages both by plain
// 16-byte copies — no VALU split, no fp32 operand traffic: how much of the f16x3 GEMM's time the
// in-loop split of the activations costs (tuning only).
template <int BK>
__global__ void __launch_bounds__(NT, 1) f16v4_kernel(LabArgs g, const uint16_t* Ap) {
  using I = Img<BK>;
  constexpr int PB = I::BYTES;
  constexpr int STAGE = 4 * PB;
  constexpr int NV = BK / 8, TPR = BK / 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int64_t T = ((g.M + TBM - 1) / TBM) * ((g.N + TBN - 1) / TBN);
  int64_t tm, tn;
  tile_of(blockIdx.x, T, (g.N + TBN - 1) / TBN, tm, tn);
  const int64_t m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int64_t arows = g.M - m0 < TBM ? g.M - m0 : TBM;
  const int64_t brows = g.N - n0 < TBN ? g.N - n0 : TBN;
  const auto ra = rsrc((const char*)Ap + m0 * g.brow, arows * g.brow);   // (A rows: K * 4 bytes)
  const auto rb = rsrc((const char*)g.Bp + n0 * g.brow, brows * g.brow);
  int vo[NV], oa[NV], ob[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int idx = tid + NT * c;
    const int r = idx / TPR, j = idx % TPR;
    vo[c] = r * (int)g.brow + (j >> 1) * 32 + (j & 1) * 16;
    oa[c] = (j & 1) * PB + I::off(r, 8 * (j >> 1));
    ob[c] = (2 + (j & 1)) * PB + I::off(r, 8 * (j >> 1));
  }
  uint4 va[NV], vb[NV];
  auto load = [&](int kt) {
#pragma unroll
    for (int c = 0; c < NV; ++c)
      va[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, vo[c], kt * BK * 4, 0));
#pragma unroll
    for (int c = 0; c < NV; ++c)
      vb[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb, vo[c], kt * BK * 4, 0));
  };
  auto store = [&](char* st) {
#pragma unroll
    for (int c = 0; c < NV; ++c) *(uint4*)(st + oa[c]) = va[c];
#pragma unroll
    for (int c = 0; c < NV; ++c) *(uint4*)(st + ob[c]) = vb[c];
  };
  floatx16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (int)(g.K / BK);
  load(0);
  store(smem);
  if (nk > 1) load(1);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
#pragma unroll
    for (int q = 0; q < BK / 16; ++q) {
      f16x8 fa[MB][2], fb[NB][2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int x = 0; x < MB; ++x)
          fa[x][p] = *(const f16x8*)(cur + p * PB +
                                     I::off(wm * (MB * 32) + x * 32 + (lane & 31), 16 * q + 8 * (lane >> 5)));
#pragma unroll
        for (int x = 0; x < NB; ++x)
          fb[x][p] = *(const f16x8*)(cur + (2 + p) * PB +
                                     I::off(wn * (NB * 32) + x * 32 + (lane & 31), 16 * q + 8 * (lane >> 5)));
      }
      if (q == 0) {
        if (kt + 1 < nk) store(nxt);
        if (kt + 2 < nk) load(kt + 2);
      }
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][1], fa[mi][0], acc[mi][ni], 0, 0, 0);
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][1], acc[mi][ni], 0, 0, 0);
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][0], acc[mi][ni], 0, 0, 0);
    }
    __syncthreads();
  }
  const int lr = lane & 31, lc = 4 * (lane >> 5);
#pragma unroll
  for (int mi = 0; mi < MB; ++mi) {
    const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
    if (row >= g.M) continue;
    const float f = g.binv;   // (Ah = fp16(64 a): the v2 scaling)
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * (NB * 32) + ni * 32 + 8 * j + lc;
        if (col + 3 < g.N) {
          *(float4*)(g.C + row * g.ldc + col) =
              make_float4(acc[mi][ni][4 * j] * f, acc[mi][ni][4 * j + 1] * f,
                          acc[mi][ni][4 * j + 2] * f, acc[mi][ni][4 * j + 3] * f);
        }
      }
    }
  }
}

// v5: both operands as planes (v4), staged by LDS-DMA (global_load_lds_dwordx4, no VGPR round
// trip) into a ring of 4 K-tile buffers (3 tiles in flight), one raw barrier per K-tile behind a
// counted vmcnt (never 0 in the steady state): the guide's "3-buf span" structure.
// LDS image per buffer: [A | B][plane][slot of 8 k][256 rows][16 B] (rows contiguous: the 32x32x16
// fragment reads are conflict-free without a swizzle).
constexpr int V5_BUF = 2 * 2 * 2 * 256 * 16;   // 32 KB: 2 operands x 2 planes x 2 slots
__device__ inline void v5_issue(const char* __restrict__ Ap, const char* __restrict__ Bp, int64_t brow,
                                int64_t m0, int64_t n0, int64_t M, int64_t N, int kt, char* buf,
                                int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gi = wave * 4 + i;          // 32 wave-instructions per buffer
    const int op = gi >> 4;               // 0 = A, 1 = B
    const int c0 = (gi & 15) * 64;        // first chunk of this instruction
    const int row = (c0 & 255) + lane, slot = (c0 >> 8) & 1, plane = c0 >> 9;
    const int64_t r0 = op ? n0 : m0, rmax = op ? N : M;
    int64_t gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;       // rows past the matrix: a valid row, never stored
    const char* src = (op ? Bp : Ap) + gr * brow + ((int64_t)kt * 2 + slot) * 32 + plane * 16;
    char* dst = buf + op * (V5_BUF / 2) + plane * (2 * 256 * 16) + slot * (256 * 16) + (c0 & 255) * 16;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

__global__ void __launch_bounds__(NT, 1) f16v5_kernel(LabArgs g, const uint16_t* Ap) {
  __shared__ __attribute__((aligned(16))) char smem[4 * V5_BUF];
  const int64_t T = ((g.M + TBM - 1) / TBM) * ((g.N + TBN - 1) / TBN);
  int64_t tm, tn;
  tile_of(blockIdx.x, T, (g.N + TBN - 1) / TBN, tm, tn);
  const int64_t m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const char* A = (const char*)Ap;
  const char* B = (const char*)g.Bp;
  floatx16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (int)(g.K / 16);
  for (int t = 0; t < 3 && t < nk; ++t)
    v5_issue(A, B, g.brow, m0, n0, g.M, g.N, t, smem + t * V5_BUF, wave, lane);
  const int fr = lane & 31, fs = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (this wave's DMAs: the later tiles' 4 each may stay in flight), then every
    // wave's (the barrier); the barrier also retires every read of tile kt - 1's buffer
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 3 < nk)
      v5_issue(A, B, g.brow, m0, n0, g.M, g.N, kt + 3, smem + ((kt + 3) & 3) * V5_BUF, wave, lane);
    const char* cur = smem + (kt & 3) * V5_BUF;
    f16x8 fa[MB][2], fb[NB][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int x = 0; x < MB; ++x)
        fa[x][p] = *(const f16x8*)(cur + p * (2 * 256 * 16) + fs * (256 * 16) +
                                   (wm * (MB * 32) + x * 32 + fr) * 16);
#pragma unroll
      for (int x = 0; x < NB; ++x)
        fb[x][p] = *(const f16x8*)(cur + V5_BUF / 2 + p * (2 * 256 * 16) + fs * (256 * 16) +
                                   (wn * (NB * 32) + x * 32 + fr) * 16);
    }
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][1], fa[mi][0], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][1], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][0], acc[mi][ni], 0, 0, 0);
  }
  const int lr = lane & 31, lc = 4 * (lane >> 5);
#pragma unroll
  for (int mi = 0; mi < MB; ++mi) {
    const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
    if (row >= g.M) continue;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * (NB * 32) + ni * 32 + 8 * j + lc;
        if (col + 3 < g.N)
          *(float4*)(g.C + row * g.ldc + col) =
              make_float4(acc[mi][ni][4 * j] * g.binv, acc[mi][ni][4 * j + 1] * g.binv,
                          acc[mi][ni][4 * j + 2] * g.binv, acc[mi][ni][4 * j + 3] * g.binv);
      }
    }
  }
}

// v6: v2 (weight planes + in-loop activation split, BK 16) as a ping-pong: the block's two wave
// groups (waves 0-3 = output rows 0-127, waves 4-7 = rows 128-255; one wave of each per SIMD) run
// the same loop one barrier apart, so one group's MFMA phase overlaps the other's memory phase
// (fragment reads, LDS stores of the next tile with the split, global loads of the one after).
// Per K-tile each wave: MEM | raw barrier | MATH | raw barrier. Group 1 starts one barrier late;
// group 0 ends with one extra, so every s_barrier pairs group 0's n-th call with group 1's n-th.
// Buffer reuse: a wave stores tile i+1 into buffer (i+1)&1 after the barrier that follows every
// wave's reads of tile i-1 (see the lab notes in DESIGN.md §8).
// LDSB: the block's LDS allocation in bytes (>= 64 KB; the library kernel's is 99.5 KB, sized
// for its fused x3 fallback) — a probe of whether the allocation alone costs time.
template <int LDSB = 65536>
__global__ void __launch_bounds__(NT, 1) f16v6_kernel(LabArgs g) {
  constexpr int BK = 16;
  using I = Img<BK>;
  constexpr int PB = I::BYTES;
  constexpr int STAGE = 4 * PB;
  constexpr int NVA = BK / 8, NVB = BK / 8, TPR = BK / 4;
  static_assert(LDSB >= 2 * STAGE, "LDS allocation below the two stages");
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int64_t T = ((g.M + TBM - 1) / TBM) * ((g.N + TBN - 1) / TBN);
  int64_t tm, tn;
  tile_of(blockIdx.x, T, (g.N + TBN - 1) / TBN, tm, tn);
  const int64_t m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int64_t arows = g.M - m0 < TBM ? g.M - m0 : TBM;
  const int64_t brows = g.N - n0 < TBN ? g.N - n0 : TBN;
  const auto ra = rsrc(g.A + m0 * g.lda, arows * g.lda * 4);
  const auto rb = rsrc((const char*)g.Bp + n0 * g.brow, brows * g.brow);
  int voa[NVA], vob[NVB], oa[NVA], ob[NVB];
#pragma unroll
  for (int c = 0; c < NVA; ++c) {
    const int idx = tid + NT * c;
    const int r = idx / TPR, k = 4 * (idx % TPR), j = idx % TPR;
    voa[c] = (r * (int)g.lda + k) * 4;
    oa[c] = I::off(r, k);
    vob[c] = r * (int)g.brow + (j >> 1) * 32 + (j & 1) * 16;
    ob[c] = (2 + (j & 1)) * PB + I::off(r, 8 * (j >> 1));
  }
  float4 va[NVA];
  uint4 vb[NVB];
  auto load = [&](int kt) {
#pragma unroll
    for (int c = 0; c < NVA; ++c)
      va[c] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, voa[c], kt * BK * 4, 0));
#pragma unroll
    for (int c = 0; c < NVB; ++c)
      vb[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb, vob[c], kt * BK * 4, 0));
  };
  auto store = [&](char* st) {
#pragma unroll
    for (int c = 0; c < NVA; ++c) {
      const float4 v = va[c];
      uint32_t h0, l0, h1, l1;
      split_mix(v.x, v.y, 64.f, h0, l0);
      split_mix(v.z, v.w, 64.f, h1, l1);
      *(uint2*)(st + oa[c]) = make_uint2(h0, h1);
      *(uint2*)(st + PB + oa[c]) = make_uint2(l0, l1);
    }
#pragma unroll
    for (int c = 0; c < NVB; ++c) *(uint4*)(st + ob[c]) = vb[c];
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  floatx16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (int)(g.K / BK);
  load(0);
  store(smem);
  if (nk > 1) load(1);
  barrier();                 // tile 0 staged by everyone
  if (wm == 1) barrier();    // group 1 runs one barrier behind
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    // MEM: this tile's fragments, the next tile's stores, the loads of the one after
    f16x8 fa[MB][2], fb[NB][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int x = 0; x < MB; ++x)
        fa[x][p] = *(const f16x8*)(cur + p * PB +
                                   I::off(wm * (MB * 32) + x * 32 + (lane & 31), 8 * (lane >> 5)));
#pragma unroll
      for (int x = 0; x < NB; ++x)
        fb[x][p] = *(const f16x8*)(cur + (2 + p) * PB +
                                   I::off(wn * (NB * 32) + x * 32 + (lane & 31), 8 * (lane >> 5)));
    }
    if (kt + 1 < nk) store(nxt);
    if (kt + 2 < nk) load(kt + 2);
    barrier();
    // MATH
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][1], fa[mi][0], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][1], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][0], acc[mi][ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
  }
  if (wm == 0) barrier();    // balance group 1's extra barrier
  const int lr = lane & 31, lc = 4 * (lane >> 5);
#pragma unroll
  for (int mi = 0; mi < MB; ++mi) {
    const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
    if (row >= g.M) continue;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * (NB * 32) + ni * 32 + 8 * j + lc;
        if (col + 3 < g.N)
          *(float4*)(g.C + row * g.ldc + col) =
              make_float4(acc[mi][ni][4 * j] * g.binv, acc[mi][ni][4 * j + 1] * g.binv,
                          acc[mi][ni][4 * j + 2] * g.binv, acc[mi][ni][4 * j + 3] * g.binv);
      }
    }
  }
}

// v7: v6 with the activations pre-split too (A planes copied like B's; tuning only).
__global__ void __launch_bounds__(NT, 1) f16v7_kernel(LabArgs g, const uint16_t* Ap) {
  constexpr int BK = 16;
  using I = Img<BK>;
  constexpr int PB = I::BYTES;
  constexpr int STAGE = 4 * PB;
  constexpr int NVA = BK / 8, NVB = BK / 8, TPR = BK / 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int64_t T = ((g.M + TBM - 1) / TBM) * ((g.N + TBN - 1) / TBN);
  int64_t tm, tn;
  tile_of(blockIdx.x, T, (g.N + TBN - 1) / TBN, tm, tn);
  const int64_t m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int64_t arows = g.M - m0 < TBM ? g.M - m0 : TBM;
  const int64_t brows = g.N - n0 < TBN ? g.N - n0 : TBN;
  const auto ra = rsrc((const char*)Ap + m0 * g.brow, arows * g.brow);
  const auto rb = rsrc((const char*)g.Bp + n0 * g.brow, brows * g.brow);
  int voa[NVA], vob[NVB], oa[NVA], ob[NVB];
#pragma unroll
  for (int c = 0; c < NVA; ++c) {
    const int idx = tid + NT * c;
    const int r = idx / TPR, j = idx % TPR;
    voa[c] = r * (int)g.brow + (j >> 1) * 32 + (j & 1) * 16;
    oa[c] = (j & 1) * PB + I::off(r, 8 * (j >> 1));
    vob[c] = voa[c];
    ob[c] = (2 + (j & 1)) * PB + I::off(r, 8 * (j >> 1));
  }
  uint4 va[NVA];
  uint4 vb[NVB];
  auto load = [&](int kt) {
#pragma unroll
    for (int c = 0; c < NVA; ++c)
      va[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra, voa[c], kt * BK * 4, 0));
#pragma unroll
    for (int c = 0; c < NVB; ++c)
      vb[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb, vob[c], kt * BK * 4, 0));
  };
  auto store = [&](char* st) {
#pragma unroll
    for (int c = 0; c < NVA; ++c) *(uint4*)(st + oa[c]) = va[c];
#pragma unroll
    for (int c = 0; c < NVB; ++c) *(uint4*)(st + ob[c]) = vb[c];
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  floatx16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (int)(g.K / BK);
  load(0);
  store(smem);
  if (nk > 1) load(1);
  barrier();                 // tile 0 staged by everyone
  if (wm == 1) barrier();    // group 1 runs one barrier behind
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    // MEM: this tile's fragments, the next tile's stores, the loads of the one after
    f16x8 fa[MB][2], fb[NB][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int x = 0; x < MB; ++x)
        fa[x][p] = *(const f16x8*)(cur + p * PB +
                                   I::off(wm * (MB * 32) + x * 32 + (lane & 31), 8 * (lane >> 5)));
#pragma unroll
      for (int x = 0; x < NB; ++x)
        fb[x][p] = *(const f16x8*)(cur + (2 + p) * PB +
                                   I::off(wn * (NB * 32) + x * 32 + (lane & 31), 8 * (lane >> 5)));
    }
    if (kt + 1 < nk) store(nxt);
    if (kt + 2 < nk) load(kt + 2);
    barrier();
    // MATH
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][1], fa[mi][0], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][1], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][0], acc[mi][ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
  }
  if (wm == 0) barrier();    // balance group 1's extra barrier
  const int lr = lane & 31, lc = 4 * (lane >> 5);
#pragma unroll
  for (int mi = 0; mi < MB; ++mi) {
    const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
    if (row >= g.M) continue;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * (NB * 32) + ni * 32 + 8 * j + lc;
        if (col + 3 < g.N)
          *(float4*)(g.C + row * g.ldc + col) =
              make_float4(acc[mi][ni][4 * j] * g.binv, acc[mi][ni][4 * j + 1] * g.binv,
                          acc[mi][ni][4 * j + 2] * g.binv, acc[mi][ni][4 * j + 3] * g.binv);
      }
    }
  }
}

// v8: v7's ping-pong over v5's LDS-DMA ring: 4 K-tile buffers, tiles kt+1..kt+3 in flight while
// tile kt is read, no VGPR round trip for the staging. Per K-tile each wave: MEM (issue tile kt+3's
// DMA into the buffer tile kt-1 used, fragment reads of tile kt, counted vmcnt that retires tile
// kt+1) | raw barrier | MATH at raised priority | raw barrier; group 1 one barrier behind.
//   RAW: a wave's vmcnt for tile kt+1 precedes the barrier that ends its MEM(kt); group 0 reads
//        kt+1 after b(2kt+2), which both groups' MEM(kt) precede; group 1 after b(2kt+3).
//   WAR: tile kt-1's buffer is refilled in MEM(kt), after b(2kt) (group 0) / b(2kt+1) (group 1);
//        the last reads of it end MEM1(kt-1), before b(2kt), with lgkmcnt(0).
// ASPLIT: the activations arrive as fp32 ([4 quads of 4 k][256 rows][16 B]) and are split into
// the hi / lo fp16 fragments right after the fragment reads (v_fma_mix), in the MEM phase that
// the other group's MFMAs cover; otherwise both operands are planes (v5's image).
constexpr int V8_BUF = 32768;
template <bool ASPLIT>
__device__ inline void v8_issue(const char* __restrict__ A, int64_t lda4, const char* __restrict__ Bp,
                                int64_t brow, int64_t m0, int64_t n0, int64_t M, int64_t N, int kt,
                                char* buf, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gi = wave * 4 + i;          // 32 wave-instructions per buffer, 1 KB each
    const int op = gi >> 4;               // 0 = A (waves 0-3), 1 = B (waves 4-7)
    // LDS image per operand: [256 rows][4 chunks of 16 B] (one K-tile row = 64 B), chunk c of
    // row r holding the row's 16-B piece c ^ ((r >> 2) & 3); an instruction moves 16 whole rows
    // (4 lanes per row: 16 lines touched, not 64) into 1 KB of LDS
    char* dst = buf + gi * 1024;
    const int row = (gi & 15) * 16 + (lane >> 2), c = lane & 3;
    const int w = c ^ ((row >> 2) & 3);
    const int64_t r0 = op ? n0 : m0, rmax = op ? N : M;
    int64_t gr = r0 + row;
    gr = gr < rmax ? gr : rmax - 1;   // rows past the matrix: a valid row, never stored
    // piece w of the K-tile: planes [slot][plane][8 fp16] or fp32 [quad][4]: both 16 w bytes in
    const char* src = (op == 0 ? A + gr * (ASPLIT ? lda4 : brow) : Bp + gr * brow) +
                      (int64_t)kt * 64 + w * 16;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

template <bool ASPLIT>
__global__ void __launch_bounds__(NT, 1) f16v8_kernel(LabArgs g, const uint16_t* Ap) {
  __shared__ __attribute__((aligned(16))) char smem[4 * V8_BUF];
  const int64_t T = ((g.M + TBM - 1) / TBM) * ((g.N + TBN - 1) / TBN);
  int64_t tm, tn;
  tile_of(blockIdx.x, T, (g.N + TBN - 1) / TBN, tm, tn);
  const int64_t m0 = tm * TBM, n0 = tn * TBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const char* A = ASPLIT ? (const char*)g.A : (const char*)Ap;
  const int64_t lda4 = g.lda * 4;
  const char* B = (const char*)g.Bp;
  floatx16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (int)(g.K / 16);
  auto issue = [&](int t) {
    v8_issue<ASPLIT>(A, lda4, B, g.brow, m0, n0, g.M, g.N, t,
                     smem + (t & 3) * V8_BUF, wave, lane);
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  for (int t = 0; t < 3 && t < nk; ++t) issue(t);
  if (nk >= 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (nk == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();                 // tile 0 landed for everyone
  if (wm == 1) barrier();    // group 1 runs one barrier behind
  const int fr = lane & 31, fs = lane >> 5, sw = (fr >> 2) & 3;
  const float ca = 64.f;
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_char*)smem;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 3 < nk) issue(kt + 3);
    const char* cur = smem + (kt & 3) * V8_BUF;
    f16x8 fa[MB][2], fb[NB][2];
    // fragment (row r, 16-B piece w) at r * 64 + ((w ^ sw) * 16), sw = (r >> 2) & 3 = (fr >> 2) & 3
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int x = 0; x < NB; ++x)
        fb[x][p] = *(const f16x8*)(cur + V8_BUF / 2 + (wn * (NB * 32) + x * 32 + fr) * 64 +
                                   (((2 * fs + p) ^ sw) * 16));
    if (ASPLIT) {
      // the fp32 activation fragments by inline-asm ds_read: read as plain loads, the compiler
      // drained vmcnt (every DMA in flight) before them; the asm reads carry no such wait, the
      // counted vmcnt + barrier order them (RAW note above)
      typedef float f32x4 __attribute__((ext_vector_type(4)));
      f32x4 u[MB], v[MB];
      const uint32_t rbase = lds_base + (uint32_t)((kt & 3) * V8_BUF) + (wm * (MB * 32) + fr) * 64;
      const uint32_t a0 = rbase + (((2 * fs) ^ sw) * 16), a1 = rbase + (((2 * fs + 1) ^ sw) * 16);
#pragma unroll
      for (int x = 0; x < MB; ++x)
        asm volatile("ds_read_b128 %0, %2 offset:%4\n\tds_read_b128 %1, %3 offset:%4"
                     : "=&v"(u[x]), "=&v"(v[x])
                     : "v"(a0), "v"(a1), "i"(x * 2048)
                     : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int x = 0; x < MB; ++x) {
        uint32_t h[4], l[4];
        split_mix(u[x].x, u[x].y, ca, h[0], l[0]);
        split_mix(u[x].z, u[x].w, ca, h[1], l[1]);
        split_mix(v[x].x, v[x].y, ca, h[2], l[2]);
        split_mix(v[x].z, v[x].w, ca, h[3], l[3]);
        fa[x][0] = __builtin_bit_cast(f16x8, make_uint4(h[0], h[1], h[2], h[3]));
        fa[x][1] = __builtin_bit_cast(f16x8, make_uint4(l[0], l[1], l[2], l[3]));
      }
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int x = 0; x < MB; ++x)
          fa[x][p] = *(const f16x8*)(cur + (wm * (MB * 32) + x * 32 + fr) * 64 +
                                     (((2 * fs + p) ^ sw) * 16));
    }
    // retire tile kt+1 (this wave's DMAs of the later tiles stay in flight)
    if (kt + 3 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][1], fa[mi][0], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][1], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][0], acc[mi][ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
  }
  if (wm == 0) barrier();    // balance group 1's extra barrier
  const int lr = lane & 31, lc = 4 * (lane >> 5);
#pragma unroll
  for (int mi = 0; mi < MB; ++mi) {
    const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
    if (row >= g.M) continue;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t col = n0 + wn * (NB * 32) + ni * 32 + 8 * j + lc;
        if (col + 3 < g.N)
          *(float4*)(g.C + row * g.ldc + col) =
              make_float4(acc[mi][ni][4 * j] * g.binv, acc[mi][ni][4 * j + 1] * g.binv,
                          acc[mi][ni][4 * j + 2] * g.binv, acc[mi][ni][4 * j + 3] * g.binv);
      }
    }
  }
}

// B planes: row n, slot s (8 k): fp16 h[8] = fp16(32 sB b), then l[8] = fp16(32 sB b - h).
__global__ void split_b_kernel(const float* B, int64_t N, int64_t K, int64_t ldb, float c,
                               uint16_t* Bp, int64_t brow) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;   // (row, slot)
  const int64_t slots = K / 8;
  if (i >= N * slots) return;
  const int64_t n = i / slots, s = i % slots;
  const float* p = B + n * ldb + 8 * s;
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split_mix(p[2 * j], p[2 * j + 1], c, h[j], l[j]);
  uint4* d = (uint4*)((char*)Bp + n * brow + s * 32);
  d[0] = make_uint4(h[0], h[1], h[2], h[3]);
  d[1] = make_uint4(l[0], l[1], l[2], l[3]);
}

}  // namespace

extern "C" int lab_split_b(const float* B, int64_t N, int64_t K, int64_t ldb, float c,
                           uint16_t* Bp, hipStream_t s) {
  const int64_t n = N * (K / 8);
  split_b_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(B, N, K, ldb, c, Bp, K * 4);
  return (int)hipGetLastError();
}

extern "C" int lab_gemm_pp(int bk, const float* A_unused, const uint16_t* Ap, const uint16_t* Bp,
                           int64_t M, int64_t N, int64_t K, float binv, float* C, int64_t ldc,
                           hipStream_t s) {
  (void)A_unused;
  LabArgs g{nullptr, K, Bp, K * 4, M, N, K, C, ldc, binv, nullptr};
  const unsigned grid = (unsigned)(((M + 255) / 256) * ((N + 255) / 256));
  if (bk == 5) f16v5_kernel<<<grid, NT, 0, s>>>(g, Ap);
  else if (bk == 7) f16v7_kernel<<<grid, NT, 0, s>>>(g, Ap);
  else if (bk == 8) f16v8_kernel<false><<<grid, NT, 0, s>>>(g, Ap);
  else if (bk == 32) f16v4_kernel<32><<<grid, NT, 0, s>>>(g, Ap);
  else f16v4_kernel<16><<<grid, NT, 0, s>>>(g, Ap);
  return (int)hipGetLastError();
}

extern "C" int lab_gemm(int bk, int scale, const float* A, int64_t lda, const uint16_t* Bp,
                        int64_t M, int64_t N, int64_t K, float binv, float* C, int64_t ldc,
                        int* bad, hipStream_t s) {
  LabArgs g{A, lda, Bp, K * 4, M, N, K, C, ldc, binv, bad};
  const unsigned grid = (unsigned)(((M + 255) / 256) * ((N + 255) / 256));
  if (bk == 6) {   // v6: the ping-pong form of v2 (BK 16, no scaling)
    f16v6_kernel<><<<grid, NT, 0, s>>>(g);
  } else if (bk == 60) {   // v6 with the library kernel's 99.5 KB LDS allocation
    f16v6_kernel<99584><<<grid, NT, 0, s>>>(g);
  } else if (bk == 8) {   // v8 with the activation split in the MEM phase
    f16v8_kernel<true><<<grid, NT, 0, s>>>(g, nullptr);
  } else if (bk == 33) {   // v3: 32-deep K-tiles on 16x16x32 MFMAs
    if (scale) f16v3_kernel<true><<<grid, NT, 0, s>>>(g);
    else f16v3_kernel<false><<<grid, NT, 0, s>>>(g);
  } else if (bk == 16) {
    if (scale) f16v2_kernel<16, true><<<grid, NT, 0, s>>>(g);
    else f16v2_kernel<16, false><<<grid, NT, 0, s>>>(g);
  } else {
    if (scale) f16v2_kernel<32, true><<<grid, NT, 0, s>>>(g);
    else f16v2_kernel<32, false><<<grid, NT, 0, s>>>(g);
  }
  return (int)hipGetLastError();
}
