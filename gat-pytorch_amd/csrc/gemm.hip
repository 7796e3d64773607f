// fp32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate;
// gfx950 has no xf32, and the f32 MFMA runs at the f32 vector peak, 157 TF).
//
// Replaces the projection `self.W(x)` of models/gat_layer.py:64 — with the attention vector
// folded in as 2*NH extra output columns (W_aug, see gatx_prepare_weights), so the same launch
// also produces the per-node logit factors s_src / s_dst that stand in for the per-edge
// (E, NH*2F) x a^T GEMV of :76-82 — and the two backward products g_x and g_W.
//
// Tile: 128 x 128 x 16 per 256-thread workgroup, 4 waves as 2 x 2, each wave 64 x 64 = 2 x 2
// MFMA blocks of 32 x 32 (16 accumulators each). Operands are staged global -> registers ->
// LDS ([k][m] and [k][n] images, so each MFMA operand read is 32 consecutive floats per lane
// half: conflict-free ds_read_b32); the next K-tile's global loads are issued before the
// current tile's MFMAs so their latency hides under 32 MFMAs per wave.
#include "gatx_common.h"

namespace gatx {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 16, PAD = 4, LDT = BM + PAD;

// Stage an (rows x BK) tile whose K index is contiguous in memory: thread t loads row t/2,
// k = (t&1)*8 .. +7, and writes them transposed into img[k][row].
struct KContig {
  static __device__ inline void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                     int64_t rmax, int64_t k0, int64_t K, bool vec,
                                     float (&v)[8]) {
    const int t = threadIdx.x;
    const int64_t r = r0 + (t >> 1);
    const int64_t k = k0 + (t & 1) * 8;
    const float* p = P + r * ld + k;
    if (r < rmax && vec && k + 8 <= K) {
      float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (r < rmax && k + j < K) ? p[j] : 0.f;
    }
  }
  static __device__ inline void store(float* img, const float (&v)[8]) {
    const int t = threadIdx.x;
    const int r = t >> 1, kb = (t & 1) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) img[(kb + j) * LDT + r] = v[j];
  }
};

// Stage a tile whose row (M or N) index is contiguous: thread t loads k = t/16,
// rows (t&15)*8 .. +7, and writes them straight into img[k][row..row+7].
struct RContig {
  static __device__ inline void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                     int64_t rmax, int64_t k0, int64_t K, bool vec,
                                     float (&v)[8]) {
    const int t = threadIdx.x;
    const int64_t k = k0 + (t >> 4);
    const int64_t r = r0 + (t & 15) * 8;
    const float* p = P + k * ld + r;
    if (k < K && vec && r + 8 <= rmax) {
      float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (k < K && r + j < rmax) ? p[j] : 0.f;
    }
  }
  static __device__ inline void store(float* img, const float (&v)[8]) {
    const int t = threadIdx.x;
    const int k = t >> 4, r = (t & 15) * 8;
    *(float4*)&img[k * LDT + r] = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)&img[k * LDT + r + 4] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// A_KC: A is k-contiguous (sak == 1, ld = sam) else m-contiguous (sam == 1, ld = sak).
// B_NC: B is n-contiguous (sbn == 1, ld = sbk) else k-contiguous (sbk == 1, ld = sbn).
template <bool A_KC, bool B_NC>
__global__ void __launch_bounds__(256, 2)
gemm_f32_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
                const float* __restrict__ B, int64_t ldb, float* __restrict__ C0, int64_t ldc0,
                int64_t n_split, float* __restrict__ C1, int64_t ldc1, int accumulate,
                int a_vec, int b_vec, int64_t tiles_n) {
  __shared__ __attribute__((aligned(16))) float As[BK * LDT];
  __shared__ __attribute__((aligned(16))) float Bs[BK * LDT];
  using AL = typename std::conditional<A_KC, KContig, RContig>::type;
  using BL = typename std::conditional<B_NC, RContig, KContig>::type;

  const int64_t tile = blockIdx.x;
  const int64_t m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float va[8], vb[8];
  const int64_t nk = ceil_div(K, BK);
  AL::load(A, lda, m0, M, 0, K, a_vec, va);
  BL::load(B, ldb, n0, N, 0, K, b_vec, vb);
  for (int64_t kt = 0; kt < nk; ++kt) {
    __syncthreads();
    AL::store(As, va);
    BL::store(Bs, vb);
    __syncthreads();
    if (kt + 1 < nk) {
      AL::load(A, lda, m0, M, (kt + 1) * BK, K, a_vec, va);
      BL::load(B, ldb, n0, N, (kt + 1) * BK, K, b_vec, vb);
    }
    const int kl = lane >> 5, il = lane & 31;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a0 = As[(kk + kl) * LDT + wm * 64 + il];
      float a1 = As[(kk + kl) * LDT + wm * 64 + 32 + il];
      float b0 = Bs[(kk + kl) * LDT + wn * 64 + il];
      float b1 = Bs[(kk + kl) * LDT + wn * 64 + 32 + il];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }

  // C/D map of a 32x32 f32 MFMA block: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int64_t col = n0 + wn * 64 + ni * 32 + (lane & 31);
      if (col >= N) continue;
      float* Cb;
      int64_t ldc, c;
      if (col < n_split) { Cb = C0; ldc = ldc0; c = col; }
      else { Cb = C1; ldc = ldc1; c = col - n_split; }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M) {
          float* p = Cb + row * ldc + c;
          *p = accumulate ? *p + acc[mi][ni][r] : acc[mi][ni][r];
        }
      }
    }
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" int gatx_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                             int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C0,
                             int64_t ldc0, int64_t n_split, float* C1, int64_t ldc1,
                             int accumulate, gatx_stream_t s) {
  GATX_REQUIRE(M >= 0 && N >= 0 && K >= 0, "gemm: negative size");
  if (M == 0 || N == 0) return 0;
  GATX_REQUIRE(sak == 1 || sam == 1, "gemm: A needs a unit stride");
  GATX_REQUIRE(sbn == 1 || sbk == 1, "gemm: B needs a unit stride");
  GATX_REQUIRE(n_split >= N || C1 != nullptr, "gemm: split output needs C1");
  const bool a_kc = (sak == 1);
  const int64_t lda = a_kc ? sam : sak;
  const bool b_nc = (sbn == 1);
  const int64_t ldb = b_nc ? sbk : sbn;
  auto aligned = [](const void* p, int64_t ld) {
    return ((uintptr_t)p % 16 == 0) && (ld % 4 == 0);
  };
  const int a_vec = aligned(A, lda), b_vec = aligned(B, ldb);
  const int64_t tiles_n = ceil_div(N, BN), tiles = ceil_div(M, BM) * tiles_n;
  GATX_REQUIRE(tiles < (1ll << 31), "gemm: too many tiles");
  hipStream_t stream = (hipStream_t)s;
  if (K == 0) {
    GATX_REQUIRE(accumulate, "gemm: K == 0 needs accumulate (output would be zero)");
    return 0;
  }
#define GATX_GEMM_LAUNCH(AK, BN_)                                                              \
  gemm_f32_kernel<AK, BN_><<<(unsigned)tiles, 256, 0, stream>>>(                               \
      M, N, K, A, lda, B, ldb, C0, ldc0, n_split, C1, ldc1, accumulate, a_vec, b_vec, tiles_n)
  if (a_kc && b_nc) GATX_GEMM_LAUNCH(true, true);
  else if (a_kc) GATX_GEMM_LAUNCH(true, false);
  else if (b_nc) GATX_GEMM_LAUNCH(false, true);
  else GATX_GEMM_LAUNCH(false, false);
#undef GATX_GEMM_LAUNCH
  GATX_LAUNCH_CHECK("gemm_f32");
  return 0;
}
