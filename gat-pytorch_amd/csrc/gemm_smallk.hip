// Small-K GEMM with the fused epilogue, in the split-bf16 ("x3") arithmetic of gemm_x3.hip:
// C_b = elu?(A_b B_b + bias_b + resid_b) for K <= 64 and N <= 256 — the reassociated first
// layer's per-head output projection (PPI layer 0: 4 heads x (44900 x 50) . (50 x 256), then
// GATModel's ELU; models/gat_layer.py:64 applied after the aggregation, see functional.py).
//
// The tiled GEMM is the wrong shape for this product: with K = 50 a 256 x 256 tile does four
// K-steps of MFMA work and then writes 256 KB, so its workgroups alternate between an idle
// memory system and idle matrix cores (148 us for 184 MB of output). Here each workgroup owns
// one batch entry's whole B (<= 256 x 64), split once into its three bf16 planes and kept in
// LDS (96 KB) for the life of the workgroup; its 8 waves then stream 32-row blocks of A: each
// wave loads its rows' K values once (8 consecutive k per lane = one MFMA fragment), splits
// them in registers, and sweeps the column blocks two at a time, storing each pair of finished
// 32 x 32 blocks while the next pair's MFMAs run. A is read once, C written once.
#include "gemm_common.h"

namespace gatx {
namespace {
using namespace gk;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int SK_WAVES = 8, SK_KMAX = 64, SK_NMAX = 256;
constexpr int SK_KSLOTS = SK_KMAX / 8;
constexpr int SK_PLANE = SK_KSLOTS * SK_NMAX * 16;   // bytes per bf16 plane of B

__device__ inline uint32_t sk_cvt_pk(float a, float b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  bf2 v = {(__bf16)a, (__bf16)b};
  uint32_t u = __builtin_bit_cast(uint32_t, v);
  asm("" : "+v"(u));
  return u;
}

// 8 floats -> their three bf16 planes (x = h + m + l exactly; gemm_x3.hip's split), 16 B each.
__device__ inline void sk_split8(const float (&v)[8], uint4& h, uint4& m, uint4& l) {
  uint32_t hh[4], mm[4], ll[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x = v[2 * j], y = v[2 * j + 1];
    hh[j] = sk_cvt_pk(x, y);
    const float rx = x - __uint_as_float(hh[j] << 16), ry = y - __uint_as_float(hh[j] & 0xffff0000u);
    mm[j] = sk_cvt_pk(rx, ry);
    ll[j] = sk_cvt_pk(rx - __uint_as_float(mm[j] << 16), ry - __uint_as_float(mm[j] & 0xffff0000u));
  }
  h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  m = make_uint4(mm[0], mm[1], mm[2], mm[3]);
  l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// A row-major (k-contiguous, lda), B as rows of k (ldb: B(k, n) = B[n * ldb + k]). VEC: A rows
// 16-byte aligned (lda % 4 == 0, aligned base), so full 8-k groups load as two float4.
template <bool VEC, bool ELU>
__global__ void __launch_bounds__(64 * SK_WAVES, 1) gemm_smallk_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char wl[3 * SK_PLANE];
  __shared__ float bias_l[SK_NMAX];
  const int b = blockIdx.y;
  const float* __restrict__ A = g.A + b * g.a_bs;
  const float* __restrict__ B = g.B + b * g.b_bs;
  const int K = (int)g.K, N = (int)g.N;
  const int64_t M = g.M;
  const int ncb = (N + 31) / 32;

  // B -> three bf16 planes in LDS, [plane][k / 8][n][8 k]: a fragment read (32 columns at one
  // k-slot per half-wave) is 512 contiguous bytes per half-wave
  for (int t = threadIdx.x; t < ncb * 32 * SK_KSLOTS; t += 64 * SK_WAVES) {
    const int n = t / SK_KSLOTS, kc = t % SK_KSLOTS;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kc * 8 + j;
      v[j] = (n < N && k < K) ? B[(int64_t)n * g.ldb + k] : 0.f;
    }
    uint4 h, m, l;
    sk_split8(v, h, m, l);
    const int o = (kc * SK_NMAX + n) * 16;
    *(uint4*)(wl + o) = h;
    *(uint4*)(wl + SK_PLANE + o) = m;
    *(uint4*)(wl + 2 * SK_PLANE + o) = l;
  }
  for (int t = threadIdx.x; t < SK_NMAX; t += 64 * SK_WAVES)
    bias_l[t] = (g.bias && t < N) ? g.bias[b * g.bias_bs + t] : 0.f;
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int nks = (K + 15) / 16;
  const int64_t nrb = (M + 31) / 32;
  // Raw A values of a row block: 8 consecutive k per lane and k16 step (one MFMA fragment).
  // The next row block's values are fetched before this one's stores: loads and stores share
  // vmcnt, so a load issued after the stores would wait for all of them to reach memory.
  float raw[SK_KMAX / 16][8];
  auto fetch = [&](int64_t rb) {
    const int64_t row = rb * 32 + (lane & 31);
    const float* ar = A + (row < M ? row : M - 1) * g.lda;
#pragma unroll
    for (int s = 0; s < SK_KMAX / 16; ++s) {
      if (s >= nks) break;
      const int k0 = 16 * s + 8 * half;
      if (VEC && k0 + 8 <= K) {
        const float4 p = *(const float4*)(ar + k0), q = *(const float4*)(ar + k0 + 4);
        raw[s][0] = p.x; raw[s][1] = p.y; raw[s][2] = p.z; raw[s][3] = p.w;
        raw[s][4] = q.x; raw[s][5] = q.y; raw[s][6] = q.z; raw[s][7] = q.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) raw[s][j] = k0 + j < K ? ar[k0 + j] : 0.f;
      }
    }
  };
  int64_t rb = (int64_t)blockIdx.x * SK_WAVES + wave;
  const int64_t rstep = (int64_t)gridDim.x * SK_WAVES;
  if (rb < nrb) fetch(rb);
  for (; rb < nrb; rb += rstep) {
    bf16x8 fa[SK_KMAX / 16][3];
#pragma unroll
    for (int s = 0; s < SK_KMAX / 16; ++s) {
      if (s >= nks) break;
      uint4 h, m, l;
      sk_split8(raw[s], h, m, l);
      fa[s][0] = __builtin_bit_cast(bf16x8, h);
      fa[s][1] = __builtin_bit_cast(bf16x8, m);
      fa[s][2] = __builtin_bit_cast(bf16x8, l);
    }
    if (rb + rstep < nrb) fetch(rb + rstep);
    for (int cb = 0; cb < ncb; cb += 2) {
      floatx16 acc[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      const int nb = cb + 1 < ncb ? 2 : 1;
#pragma unroll
      for (int s = 0; s < SK_KMAX / 16; ++s) {
        if (s >= nks) break;
        bf16x8 fb[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fb[i][p] = *(const bf16x8*)(wl + p * SK_PLANE +
                                        ((2 * s + half) * SK_NMAX + (cb + i) * 32 + (lane & 31)) * 16);
        // small terms first: (l,h) (h,l) (m,m) (m,h) (h,m) (h,h), as gemm_x3_kernel
        constexpr int PLA[6] = {2, 0, 1, 1, 0, 0};
        constexpr int PLB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][PLA[t]], fb[i][PLB[t]], acc[i],
                                                             0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i >= nb) break;
        // epilogue (no residual / accumulate on this path): elu?(acc + bias); the bias comes
        // from LDS, so no global load waits behind this wave's earlier stores. Interior blocks
        // (every row and column inside the matrix) take a straight-line path of 16 stores with
        // ELU a compile-time choice: per-element bound checks and a runtime ELU test had made
        // each store its own exec-masked branch.
        const int col = (cb + i) * 32 + (lane & 31);
        const int colc = col < N ? col : N - 1;
        const float bv = bias_l[colc];
        float* base = g.C0 + b * g.c0_bs + colc;
        const int64_t row0 = rb * 32 + 4 * half;
        if (row0 + 27 < M && (cb + i) * 32 + 32 <= N) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float v = acc[i][r] + bv;
            if (ELU) v = elu_act(v);
            base[(row0 + (r & 3) + 8 * (r >> 2)) * g.ldc0] = v;
          }
        } else if (col < N) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int64_t row = row0 + (r & 3) + 8 * (r >> 2);
            if (row >= M) continue;
            float v = acc[i][r] + bv;
            if (ELU) v = elu_act(v);
            base[row * g.ldc0] = v;
          }
        }
      }
    }
  }
}

}  // namespace

bool gemm_smallk_fits(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc, int accumulate,
                      bool resid) {
  return a_kc && b_kc && !accumulate && !resid && K >= 1 && K <= SK_KMAX && N >= 1 && N <= SK_NMAX &&
         M >= 32 * SK_WAVES;
}

int launch_gemm_smallk(const gk::GemmArgs& g, int batch, hipStream_t stream) {
  GATX_REQUIRE(g.K <= SK_KMAX && g.N <= SK_NMAX && batch < 65536, "gemm_smallk: shape");
  // one 96-KB workgroup per CU: ~256 workgroups over the batch entries, each sweeping its
  // entry's 32-row blocks
  const int64_t nrb = ceil_div(g.M, 32);
  const int64_t per = std::max<int64_t>(1, 256 / batch);
  const unsigned gx = (unsigned)std::min<int64_t>(per, ceil_div(nrb, SK_WAVES));
  dim3 grid(gx, (unsigned)batch);
  const bool vec = ((uintptr_t)g.A % 16 == 0) && g.lda % 4 == 0 && g.a_bs % 4 == 0;
  if (vec && g.elu) gemm_smallk_kernel<true, true><<<grid, 64 * SK_WAVES, 0, stream>>>(g);
  else if (vec) gemm_smallk_kernel<true, false><<<grid, 64 * SK_WAVES, 0, stream>>>(g);
  else if (g.elu) gemm_smallk_kernel<false, true><<<grid, 64 * SK_WAVES, 0, stream>>>(g);
  else gemm_smallk_kernel<false, false><<<grid, 64 * SK_WAVES, 0, stream>>>(g);
  GATX_LAUNCH_CHECK("gemm_smallk");
  return 0;
}

}  // namespace gatx
