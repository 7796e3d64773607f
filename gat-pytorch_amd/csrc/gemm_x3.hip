// fp32 GEMM as a three-way bf16 split on v_mfma_f32_32x32x16_bf16, and the f16x3 arithmetic
// (gemm_x3_impl.h holds the mainloops and the epilogue).
#include "gemm_x3_impl.h"

namespace gatx {
namespace {
using namespace gk;

// Workgroups that tripped the range check and recomputed their tile as x3 (~1.5x the tile's
// cost), counted since the last gatx_gemm_fallback_read with reset: a perf cliff on operands out
// of the fp16 range (e.g. a trained weight row below 2^-13) shows up here, not only in timings.
__device__ unsigned long long g_f16_fallback_tiles = 0;

__global__ void fallback_read_kernel(unsigned long long* dst, int reset) {
  if (threadIdx.x == 0) {
    dst[0] = __hip_atomic_load(&g_f16_fallback_tiles, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (reset) __hip_atomic_store(&g_f16_fallback_tiles, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


template <bool A_KC, bool B_KC, bool VEC, int TAG, int CFG>
__global__ void __launch_bounds__(X3Cfg<CFG>::NT, X3Cfg<CFG>::MINB) gemm_x3_kernel(GemmArgs g,
                                                                                   int arith) {
  using C = X3Cfg<CFG>;
  constexpr int STAGE = 3 * 2 * (C::TBM + C::TBN) * C::BK;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int64_t T = g.tiles_m * g.tiles_n;
  int64_t tm, tn, kb, K;
  int tail_z = -1;
  int64_t tail_ti = 0;
  if (g.tail_s > 1 && (int64_t)blockIdx.x >= g.dp_blocks) {
    const int64_t j = blockIdx.x - g.dp_blocks;
    tail_ti = j % g.tail_rem;
    tail_z = (int)(j / g.tail_rem);
    const int64_t lin = g.dp_blocks + tail_ti;
    tm = lin / g.tiles_n;
    tn = lin - tm * g.tiles_n;
    kb = tail_z * g.k_per_split;
    K = min(g.K, kb + g.k_per_split);
  } else if (g.tail_s > 1) {
    tile_of(blockIdx.x, g.dp_blocks, g.tiles_n, tm, tn);
    kb = 0;
    K = g.K;
  } else {
    tile_of(blockIdx.x, T, g.tiles_n, tm, tn);
    kb = blockIdx.z * g.k_per_split;
    K = min(g.K, kb + g.k_per_split);
  }
  const int64_t m0 = tm * C::TBM, n0 = tn * C::TBN;
  const float* __restrict__ A = g.A + blockIdx.y * g.a_bs;
  const float* __restrict__ B = g.B + blockIdx.y * g.b_bs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  floatx16 acc[C::MB][C::NB];
#pragma unroll
  for (int i = 0; i < C::MB; ++i)
#pragma unroll
    for (int j = 0; j < C::NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int64_t nk = K > kb ? ceil_div(K - kb, C::BK) : 0;
  if (nk > 0) {
    bool x3 = true;
    if constexpr (A_KC && B_KC) if (arith == 2) {
      // row scaling for the gradient GEMMs (TAG != 0: A = G_aug, rows ~1e-7); the forward
      // projection's activations are in range as they come (a row that is not takes the fallback)
      constexpr bool SCALE = TAG != 0;
      const bool bad =
          VEC ? f16_mainloop<A_KC, B_KC, false, CFG, SCALE>(g, A, B, m0, n0, kb, K, nk, smem, wm,
                                                             wn, lane, acc)
              : f16_mainloop<A_KC, B_KC, true, CFG, SCALE>(g, A, B, m0, n0, kb, K, nk, smem, wm,
                                                            wn, lane, acc);
      x3 = __syncthreads_or(bad);   // the workgroup's tiles out of fp16 range: redo as x3
      if (x3 && threadIdx.x == 0)
        __hip_atomic_fetch_add(&g_f16_fallback_tiles, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // undo 2^11 and the row / column scales: lane -> row, register 4j + i -> column (the
      // transposed product's layout, write_tile_t)
      constexpr int STAGE16 = 2 * 2 * (C::TBM + C::TBN) * C::BK;
      const float* inv = (const float*)(smem + 2 * STAGE16);
      const int lr = lane & 31, lc = 4 * (lane >> 5);
      (void)lc;
#pragma unroll
      for (int i = 0; i < C::MB; ++i) {
        const float ra = SCALE ? inv[wm * (C::MB * 32) + i * 32 + lr] * 0x1p-11f : 0x1p-11f;
#pragma unroll
        for (int j = 0; j < C::NB; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = x3 ? 0.f : acc[i][j][r] * ra;
      }
      __syncthreads();   // the scales are read before a fallback or the epilogue reuses the LDS
    }
    if (x3) {
      if (VEC)
        x3_mainloop<A_KC, B_KC, false, CFG>(g, A, B, m0, n0, kb, K, nk, smem, wm, wn, lane, acc);
      else
        x3_mainloop<A_KC, B_KC, true, CFG>(g, A, B, m0, n0, kb, K, nk, smem, wm, wn, lane, acc);
    }
  }
  write_tile_t<C::MB, C::NB, C::TBM, C::TBN>(g, acc, tail_z, tail_ti, m0, n0, wm, wn, lane);
  // (tail slices are scored by tail_fixup_scores_kernel once summed)
  if constexpr (TAG == 0)
    if (g.s_part && tail_z < 0)
      scores_tile<C::MB, C::NB, C::TBM, C::TBN, C::WGN>(g, acc, m0, n0, tn, wm, wn, lane, smem);
}

}  // namespace

int launch_gemm_x3(const gk::GemmArgs& g, bool a_kc, bool b_kc, int batch, int tag,
                   hipStream_t stream) {
  const int64_t tiles = g.tiles_m * g.tiles_n;
  const int64_t gx = g.tail_s > 1 ? g.dp_blocks + g.tail_rem * g.tail_s : tiles;
  dim3 grid((unsigned)gx, (unsigned)batch, (unsigned)g.splits);
  const int cfg = g.bm == 256 ? 1 : 0;
  const int arith = gatx_get_gemm_mode();   // 1: bf16 split (x3), 2: fp16 split (f16x3)
#define GATX_X3_V(AK, BKC, V, TG)                                                             \
  do {                                                                                        \
    if (cfg == 1) gemm_x3_kernel<AK, BKC, V, TG, 1><<<grid, 512, 0, stream>>>(g, arith);         \
    else gemm_x3_kernel<AK, BKC, V, TG, 0><<<grid, 256, 0, stream>>>(g, arith);                  \
  } while (0)
#define GATX_X3_T(AK, BKC, V)                                                                 \
  do {                                                                                        \
    if (tag == 0) GATX_X3_V(AK, BKC, V, 0);                                                   \
    else if (tag == 2) GATX_X3_V(AK, BKC, V, 2);                                              \
    else GATX_X3_V(AK, BKC, V, 1);                                                            \
  } while (0)
#define GATX_X3_GO(AK, BKC)                                                                   \
  do {                                                                                        \
    if (g.a_vec && g.b_vec) GATX_X3_T(AK, BKC, true);                                         \
    else GATX_X3_T(AK, BKC, false);                                                           \
  } while (0)
  if (a_kc && b_kc) GATX_X3_GO(true, true);
  else if (a_kc) GATX_X3_GO(true, false);
  else if (b_kc) GATX_X3_GO(false, true);
  else GATX_X3_GO(false, false);
#undef GATX_X3_GO
#undef GATX_X3_T
#undef GATX_X3_V
  GATX_LAUNCH_CHECK("gemm_x3");
  return 0;
}

int read_f16_fallbacks(unsigned long long* dst, int reset, hipStream_t stream) {
  fallback_read_kernel<<<1, 64, 0, stream>>>(dst, reset);
  GATX_LAUNCH_CHECK("gatx_gemm_fallback_read");
  return 0;
}

const void* gemm_x3_occupancy_fn(int cfg) {
  return cfg ? reinterpret_cast<const void*>(&gemm_x3_kernel<true, true, true, 0, 1>)
             : reinterpret_cast<const void*>(&gemm_x3_kernel<true, true, true, 0, 0>);
}

}  // namespace gatx
