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

constexpr int BK = 32, PAD = 4;

// Stage a (ROWS x BK) tile whose K index is contiguous in memory into img[k][row] (transposed).
// THREADS threads, EPT = ROWS*BK/THREADS consecutive k per thread.
template <int ROWS, int THREADS>
struct KContig {
  static constexpr int EPT = ROWS * BK / THREADS, TPR = BK / EPT, LD = ROWS + PAD;
  static __device__ inline void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                     int64_t rmax, int64_t k0, int64_t K, bool vec,
                                     float (&v)[EPT]) {
    const int t = threadIdx.x;
    const int64_t r = r0 + t / TPR;
    const int64_t k = k0 + (t % TPR) * EPT;
    const float* p = P + r * ld + k;
    if (r < rmax && vec && k + EPT <= K) {
#pragma unroll
      for (int j = 0; j < EPT / 4; ++j) {
        const float4 a = *(const float4*)(p + 4 * j);
        v[4 * j] = a.x; v[4 * j + 1] = a.y; v[4 * j + 2] = a.z; v[4 * j + 3] = a.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) v[j] = (r < rmax && k + j < K) ? p[j] : 0.f;
    }
  }
  static __device__ inline void store(float* img, const float (&v)[EPT]) {
    const int t = threadIdx.x;
    const int r = t / TPR, kb = (t % TPR) * EPT;
#pragma unroll
    for (int j = 0; j < EPT; ++j) img[(kb + j) * LD + r] = v[j];
  }
};

// Stage a tile whose row (M or N) index is contiguous straight into img[k][row].
template <int ROWS, int THREADS>
struct RContig {
  static constexpr int EPT = ROWS * BK / THREADS, TPK = ROWS / EPT, LD = ROWS + PAD;
  static __device__ inline void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                     int64_t rmax, int64_t k0, int64_t K, bool vec,
                                     float (&v)[EPT]) {
    const int t = threadIdx.x;
    const int64_t k = k0 + t / TPK;
    const int64_t r = r0 + (t % TPK) * EPT;
    const float* p = P + k * ld + r;
    if (k < K && vec && r + EPT <= rmax) {
#pragma unroll
      for (int j = 0; j < EPT / 4; ++j) {
        const float4 a = *(const float4*)(p + 4 * j);
        v[4 * j] = a.x; v[4 * j + 1] = a.y; v[4 * j + 2] = a.z; v[4 * j + 3] = a.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) v[j] = (k < K && r + j < rmax) ? p[j] : 0.f;
    }
  }
  static __device__ inline void store(float* img, const float (&v)[EPT]) {
    const int t = threadIdx.x;
    const int k = t / TPK, r = (t % TPK) * EPT;
#pragma unroll
    for (int j = 0; j < EPT / 4; ++j)
      *(float4*)&img[k * LD + r + 4 * j] = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2],
                                                        v[4 * j + 3]);
  }
};

struct GemmArgs {
  int64_t M, N, K;
  const float* A; int64_t lda, a_bs;
  const float* B; int64_t ldb, b_bs;
  float* C0; int64_t ldc0, c0_bs;
  int64_t n_split;
  float* C1; int64_t ldc1, c1_bs;
  int accumulate, a_vec, b_vec;
  int64_t tiles_m, tiles_n;
  // epilogue on C0 columns: C = elu?(acc (+C) + bias[col] + resid[row][col])
  const float* bias; int64_t bias_bs;
  const float* resid; int64_t resid_ld, resid_bs;
  int elu;
  int64_t k_per_split; int splits; float* partial;
};

// Deterministic split-K combine: C = epilogue(sum over slabs in slab order), one pass.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(GemmArgs g, int batch) {
  const int64_t MN = g.M * g.N, total = MN * batch;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / MN, mn = t - b * MN, row = mn / g.N, col = mn - row * g.N;
    float v = 0.f;
    for (int z = 0; z < g.splits; ++z) v += g.partial[((int64_t)z * batch + b) * MN + mn];
    float* Cb;
    int64_t ldc, c;
    const bool first = col < g.n_split;
    if (first) { Cb = g.C0 + b * g.c0_bs; ldc = g.ldc0; c = col; }
    else { Cb = g.C1 + b * g.c1_bs; ldc = g.ldc1; c = col - g.n_split; }
    float* p = Cb + row * ldc + c;
    if (g.accumulate) v += *p;
    if (first) {
      if (g.bias) v += g.bias[b * g.bias_bs + c];
      if (g.resid) v += g.resid[b * g.resid_bs + row * g.resid_ld + c];
      if (g.elu) v = v > 0.f ? v : expm1f(v);
    }
    *p = v;
  }
}

// Workgroup -> output tile. Workgroups are dealt round-robin over the 8 XCDs (b % 8), so give
// XCD x a contiguous run of m-major tiles: an A row-tile (x rows) is then fetched into one XCD's
// L2 and reused there by all its n-tiles. Placement only changes speed, never results.
__device__ inline void tile_of(int64_t b, int64_t T, int64_t tiles_n, int64_t& tm, int64_t& tn) {
  const int64_t q = T / 8, r = T % 8;
  const int64_t xcd = b % 8, j = b / 8;
  const int64_t t = (xcd < r) ? xcd * (q + 1) + j : r * (q + 1) + (xcd - r) * q + j;
  tm = t / tiles_n;
  tn = t % tiles_n;
}

// Block tile (64*WM) x 128 x 32, 2*WM waves as WM x 2; each wave owns a 64 x 64 sub-tile =
// 2 x 2 MFMA blocks of 32 x 32. A_KC: A is k-contiguous (sak == 1, ld = sam) else m-contiguous;
// B_NC: B is n-contiguous (sbn == 1, ld = sbk) else k-contiguous.
// TAG only separates the symbol names of the call sites in profiles (0 = forward projection,
// 1 = auxiliary products, 2 = split-K weight gradient); the code is identical.
template <bool A_KC, bool B_NC, int WM, int TAG>
__global__ void __launch_bounds__(128 * WM, 2) gemm_f32_kernel(GemmArgs g) {
  constexpr int BM = 64 * WM, BN = 128, THREADS = 128 * WM;
  using AL = typename std::conditional<A_KC, KContig<BM, THREADS>, RContig<BM, THREADS>>::type;
  using BL = typename std::conditional<B_NC, RContig<BN, THREADS>, KContig<BN, THREADS>>::type;
  constexpr int LDA = BM + PAD, LDB = BN + PAD;
  __shared__ __attribute__((aligned(16))) float As[BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[BK * LDB];

  const int64_t T = g.tiles_m * g.tiles_n;
  int64_t tm, tn;
  tile_of(blockIdx.x, T, g.tiles_n, tm, tn);
  const int64_t m0 = tm * BM, n0 = tn * BN;
  const float* __restrict__ A = g.A + blockIdx.y * g.a_bs;
  const float* __restrict__ B = g.B + blockIdx.y * g.b_bs;
  const int64_t M = g.M, N = g.N;
  // split-K: slice blockIdx.z covers k in [kb, ke) and writes its own partial slab
  const int64_t kb = blockIdx.z * g.k_per_split;
  const int64_t K = min(g.K, kb + g.k_per_split);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float va[AL::EPT], vb[BL::EPT];
  const int64_t nk = ceil_div(K - kb, BK);
  AL::load(A, g.lda, m0, M, kb, K, g.a_vec, va);
  BL::load(B, g.ldb, n0, N, kb, K, g.b_vec, vb);
  for (int64_t kt = 0; kt < nk; ++kt) {
    __syncthreads();
    AL::store(As, va);
    BL::store(Bs, vb);
    __syncthreads();
    if (kt + 1 < nk) {
      AL::load(A, g.lda, m0, M, kb + (kt + 1) * BK, K, g.a_vec, va);
      BL::load(B, g.ldb, n0, N, kb + (kt + 1) * BK, K, g.b_vec, vb);
    }
    const int kl = lane >> 5, il = lane & 31;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a0 = As[(kk + kl) * LDA + wm * 64 + il];
      const float a1 = As[(kk + kl) * LDA + wm * 64 + 32 + il];
      const float b0 = Bs[(kk + kl) * LDB + wn * 64 + il];
      const float b1 = Bs[(kk + kl) * LDB + wn * 64 + 32 + il];
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
      const bool first = col < g.n_split;
      if (g.splits > 1) {   // partial slab z: plain [M][N] store, reduced by splitk_reduce_kernel
        float* P = g.partial + ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * M * N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < M) P[row * N + col] = acc[mi][ni][r];
        }
        continue;
      }
      if (first) { Cb = g.C0 + blockIdx.y * g.c0_bs; ldc = g.ldc0; c = col; }
      else { Cb = g.C1 + blockIdx.y * g.c1_bs; ldc = g.ldc1; c = col - g.n_split; }
      const float bcol = (first && g.bias) ? g.bias[blockIdx.y * g.bias_bs + c] : 0.f;
      const float* rs = (first && g.resid) ? g.resid + blockIdx.y * g.resid_bs + c : nullptr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M) {
          float* p = Cb + row * ldc + c;
          float v = g.accumulate ? *p + acc[mi][ni][r] : acc[mi][ni][r];
          if (first) {
            v += bcol;
            if (rs) v += rs[row * g.resid_ld];
            if (g.elu) v = v > 0.f ? v : expm1f(v);
          }
          *p = v;
        }
      }
    }
}

template <int WM, int TAG>
int launch_gemm(const GemmArgs& g0, bool a_kc, bool b_nc, int batch, hipStream_t stream) {
  GemmArgs g = g0;
  g.tiles_m = ceil_div(g.M, 64 * WM);
  g.tiles_n = ceil_div(g.N, 128);
  const int64_t tiles = g.tiles_m * g.tiles_n;
  GATX_REQUIRE(tiles < (1ll << 31) && batch < 65536, "gemm: too many tiles");
  dim3 grid((unsigned)tiles, (unsigned)batch, (unsigned)g.splits);
  constexpr int TH = 128 * WM;
  if (a_kc && b_nc) gemm_f32_kernel<true, true, WM, TAG><<<grid, TH, 0, stream>>>(g);
  else if (a_kc) gemm_f32_kernel<true, false, WM, TAG><<<grid, TH, 0, stream>>>(g);
  else if (b_nc) gemm_f32_kernel<false, true, WM, TAG><<<grid, TH, 0, stream>>>(g);
  else gemm_f32_kernel<false, false, WM, TAG><<<grid, TH, 0, stream>>>(g);
  GATX_LAUNCH_CHECK("gemm_f32");
  if (g.splits > 1) {
    const int64_t total = g.M * g.N * batch;
    const unsigned rg = (unsigned)std::min<int64_t>(ceil_div(total, 256), 8192);
    splitk_reduce_kernel<<<rg, 256, 0, stream>>>(g, batch);
    GATX_LAUNCH_CHECK("splitk_reduce");
  }
  return 0;
}

// Split K when the output alone cannot fill the chip (g_W = G^T x: ~70 tiles, K = #nodes):
// aim for >= 512 workgroups with >= 1024 k per slice.
int choose_splits(int64_t tiles, int64_t K) {
  int s = 1;
  while (tiles * s < 512 && K / (s * 2) >= 1024 && s < 32) s *= 2;
  return s;
}

int g_gemm_wm = 0;   // 0: choose by shape; 2 or 4 forces the 128- or 256-row tile

}  // namespace
}  // namespace gatx

using namespace gatx;

static int gemm_impl(int64_t M, int64_t N, int64_t K, int batch, const float* A, int64_t sam,
                     int64_t sak, int64_t a_bs, const float* B, int64_t sbk, int64_t sbn,
                     int64_t b_bs, float* C0, int64_t ldc0, int64_t c0_bs, int64_t n_split,
                     float* C1, int64_t ldc1, int64_t c1_bs, int accumulate, const float* bias,
                     int64_t bias_bs, const float* resid, int64_t resid_ld, int64_t resid_bs,
                     int elu, void* workspace, size_t workspace_bytes, int tag,
                     hipStream_t stream) {
  GATX_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "gemm: negative size");
  if (M == 0 || N == 0) return 0;
  GATX_REQUIRE(sak == 1 || sam == 1, "gemm: A needs a unit stride");
  GATX_REQUIRE(sbn == 1 || sbk == 1, "gemm: B needs a unit stride");
  GATX_REQUIRE(n_split >= N || C1 != nullptr, "gemm: split output needs C1");
  GATX_REQUIRE(K > 0 || accumulate, "gemm: K == 0 needs accumulate (output would be zero)");
  if (K == 0) return 0;
  GemmArgs g;
  const bool a_kc = (sak == 1);
  const bool b_nc = (sbn == 1);
  g.M = M; g.N = N; g.K = K;
  g.A = A; g.lda = a_kc ? sam : sak; g.a_bs = a_bs;
  g.B = B; g.ldb = b_nc ? sbk : sbn; g.b_bs = b_bs;
  g.C0 = C0; g.ldc0 = ldc0; g.c0_bs = c0_bs; g.n_split = n_split;
  g.C1 = C1; g.ldc1 = ldc1; g.c1_bs = c1_bs;
  g.accumulate = accumulate;
  g.bias = bias; g.bias_bs = bias_bs;
  g.resid = resid; g.resid_ld = resid_ld; g.resid_bs = resid_bs;
  g.elu = elu;
  g.splits = 1; g.k_per_split = K; g.partial = nullptr;
  auto aligned = [](const void* p, int64_t ld, int64_t bs) {
    return ((uintptr_t)p % 16 == 0) && (ld % 4 == 0) && (bs % 4 == 0);
  };
  g.a_vec = aligned(A, g.lda, a_bs);
  g.b_vec = aligned(B, g.ldb, b_bs);
  static const int env_wm = [] {
    const char* e = getenv("GATX_GEMM_WM");
    return e ? atoi(e) : 0;
  }();
  int wm = g_gemm_wm ? g_gemm_wm : env_wm;
  if (wm == 0) wm = 2;
  if (workspace) {
    const int64_t tiles = ceil_div(M, 64 * wm) * ceil_div(N, 128) * batch;
    int sp = choose_splits(tiles, K);
    while (sp > 1 && (size_t)sp * batch * M * N * sizeof(float) > workspace_bytes) sp /= 2;
    if (sp > 1) {
      g.splits = sp;
      g.k_per_split = round_up(ceil_div(K, sp), BK);
      g.splits = (int)ceil_div(K, g.k_per_split);
      g.partial = (float*)workspace;
    }
  }
  if (wm == 4) return launch_gemm<4, 1>(g, a_kc, b_nc, batch, stream);   // tuning only
  if (tag == 0) return launch_gemm<2, 0>(g, a_kc, b_nc, batch, stream);
  if (tag == 2) return launch_gemm<2, 2>(g, a_kc, b_nc, batch, stream);
  return launch_gemm<2, 1>(g, a_kc, b_nc, batch, stream);
}

extern "C" void gatx_set_gemm_rows(int rows) { g_gemm_wm = rows / 64; }

extern "C" int gatx_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                             int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C0,
                             int64_t ldc0, int64_t n_split, float* C1, int64_t ldc1,
                             int accumulate, gatx_stream_t s) {
  return gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C0, ldc0, 0, n_split, C1, ldc1, 0,
                   accumulate, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, 1, (hipStream_t)s);
}

extern "C" int gatx_projection_gemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                                    int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                                    float* C0, int64_t ldc0, int64_t n_split, float* C1,
                                    int64_t ldc1, gatx_stream_t s) {
  return gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C0, ldc0, 0, n_split, C1, ldc1, 0,
                   0, nullptr, 0, nullptr, 0, 0, 0, nullptr, 0, 0, (hipStream_t)s);
}

extern "C" int gatx_gemm_f32_batched(int64_t batch, int64_t M, int64_t N, int64_t K,
                                     const float* A, int64_t sam, int64_t sak, int64_t a_bs,
                                     const float* B, int64_t sbk, int64_t sbn, int64_t b_bs,
                                     float* C, int64_t ldc, int64_t c_bs, int accumulate,
                                     const float* bias, int64_t bias_bs, const float* resid,
                                     int64_t resid_ld, int64_t resid_bs, int elu,
                                     gatx_stream_t s) {
  return gemm_impl(M, N, K, (int)batch, A, sam, sak, a_bs, B, sbk, sbn, b_bs, C, ldc, c_bs, N,
                   nullptr, 0, 0, accumulate, bias, bias_bs, resid, resid_ld, resid_bs, elu,
                   nullptr, 0, 1, (hipStream_t)s);
}

extern "C" size_t gatx_gemm_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ceil_div(M, 128) * ceil_div(N, 128);
  const int sp = choose_splits(tiles, K);
  return sp > 1 ? (size_t)sp * M * N * sizeof(float) : 0;
}

extern "C" int gatx_gemm_f32_splitk(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                                    int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                                    float* C, int64_t ldc, int accumulate, void* workspace,
                                    size_t workspace_bytes, gatx_stream_t s) {
  return gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C, ldc, 0, N, nullptr, 0, 0,
                   accumulate, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 2,
                   (hipStream_t)s);
}
