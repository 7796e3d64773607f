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
// VST: C rows 16-byte aligned (ldc0, c0_bs % 4 == 0, aligned base) for the float4 stores.
// CB column blocks per pass (4 measured slower: 256 VGPRs, 74 vs 68 us on PPI layer 0).
template <bool VEC, bool ELU, bool VST, bool FULLN = false, int CB = 2>
__global__ void __launch_bounds__(64 * SK_WAVES, 1) gemm_smallk_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char wl[3 * SK_PLANE];
  __shared__ __attribute__((aligned(16))) float bias_l[SK_NMAX];
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
      if (VEC) {
        // unconditional float4 loads (a float4 starting below K stays inside the row: K <= lda,
        // lda % 4 == 0; one starting at or past K reads k = 0 instead), the k >= K lanes zeroed
        // in split_raw: a scalar fallback here wrote registers with vector loads still in
        // flight, which cost an s_waitcnt vmcnt(0) — all this wave's earlier stores — per block
        const float4 p = *(const float4*)(ar + (k0 < K ? k0 : 0));
        const float4 q = *(const float4*)(ar + (k0 + 4 < K ? k0 + 4 : 0));
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
  // the first block's loads are waited for here, so the loop head sees only the back edge's
  // pending loads (issued before a static number of stores when FULLN)
  if (FULLN) __builtin_amdgcn_s_waitcnt(0);
  for (; rb < nrb; rb += rstep) {
    bf16x8 fa[SK_KMAX / 16][3];
#pragma unroll
    for (int s = 0; s < SK_KMAX / 16; ++s) {
      if (s >= nks) break;
      if (VEC) {
#pragma unroll
        for (int j = 0; j < 8; ++j) raw[s][j] = 16 * s + 8 * half + j < K ? raw[s][j] : 0.f;
      }
      uint4 h, m, l;
      sk_split8(raw[s], h, m, l);
      fa[s][0] = __builtin_bit_cast(bf16x8, h);
      fa[s][1] = __builtin_bit_cast(bf16x8, m);
      fa[s][2] = __builtin_bit_cast(bf16x8, l);
    }
    if (rb + rstep < nrb) fetch(rb + rstep);
#pragma unroll
    for (int cb = 0; cb < (FULLN ? SK_NMAX / 32 : ncb); cb += CB) {
      // the bias of this lane's columns (registers 4j..4j+3 are columns cb*32 + 8j + 4*(l >> 5)
      // + 0..3, see the epilogue), read from LDS ahead of the MFMAs. (Starting the accumulators
      // at the bias instead cost accuracy: 8.8e-7 vs 3.3e-7 relative on tests' 5612 x 256 x 50
      // case — the small plane products are then aligned to the bias' exponent.)
      float4 bv[CB][4];
#pragma unroll
      for (int i = 0; i < CB; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[i][j] = *(const float4*)&bias_l[(cb + i) * 32 + 4 * half + 8 * j];
      floatx16 acc[CB];
#pragma unroll
      for (int i = 0; i < CB; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      const int nb = FULLN ? CB : (ncb - cb < CB ? ncb - cb : CB);
#pragma unroll
      for (int s = 0; s < SK_KMAX / 16; ++s) {
        if (s >= nks) break;
        bf16x8 fb[CB][3];
#pragma unroll
        for (int i = 0; i < CB; ++i)
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
          for (int i = 0; i < CB; ++i)   // C^T = B^T A^T: lane = output row, registers = columns
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[i][PLB[t]], fa[s][PLA[t]], acc[i],
                                                             0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        if (i >= nb) break;
        // epilogue (no residual / accumulate on this path): elu?(acc + bias). The product is
        // formed transposed (B^T A^T), so lane l holds output row rb*32 + (l & 31) and registers
        // 4j..4j+3 the four consecutive columns cb*32 + 8j + 4*(l >> 5) + 0..3: one 16-byte store
        // each, four per block instead of sixteen 4-byte ones (the 4-byte stores of the untransposed
        // layout kept the vector memory pipe busy 4x as long per output byte).
        int64_t row = rb * 32 + (lane & 31);
        if (FULLN) {
          // rows past M store row M - 1's values again (fetch clamped their A rows to M - 1, so
          // the values are identical): every block issues exactly four stores, the store count
          // per row block is static, and the next block's A loads (issued before these stores)
          // are waited for with vmcnt(#stores) instead of vmcnt(0) — a wait on all of this
          // wave's stores reaching memory
          row = row < M ? row : M - 1;
        } else if (row >= M) {
          continue;
        }
        const int c0 = (cb + i) * 32 + 4 * half;
        float* base = g.C0 + b * g.c0_bs + row * g.ldc0;
        if (FULLN || (VST && (cb + i) * 32 + 32 <= N)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f32x2 lo = {acc[i][4 * j] + bv[i][j].x, acc[i][4 * j + 1] + bv[i][j].y};
            f32x2 hi = {acc[i][4 * j + 2] + bv[i][j].z, acc[i][4 * j + 3] + bv[i][j].w};
            if (ELU) { lo = elu_act2(lo); hi = elu_act2(hi); }
            *(float4*)(base + c0 + 8 * j) = make_float4(lo.x, lo.y, hi.x, hi.y);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int col = c0 + 8 * (r >> 2) + (r & 3);
            if (col >= N) continue;
            float v = acc[i][r] + bias_l[col];
            if (ELU) v = elu_act(v);
            base[col] = v;
          }
        }
      }
    }
  }
}

// Small-N GEMM, the same arithmetic: C_b = A_b B_b for N <= 64 and K <= 256, A k-contiguous and
// B stored n-contiguous (B(k, n) = B[k * ldb + n]), no epilogue — the reassociated first
// layer's backward g_Z[n, h] = go[n, h] . W_h (functional._reassoc_backward; PPI layer 0: 4 heads
// x (44900 x 256) . (256 x 52)). On the tiled x3 kernel that product ran 91 us for 221 MB of
// traffic: a 128 x 128 tile over 52 columns wastes 59% of its MFMA work and stages A through LDS
// for a single column tile. Here, as gemm_smallk_kernel, each workgroup keeps its entry's whole
// B (256 k x 64 columns) as three bf16 planes in LDS (96 KB) and its 8 waves stream 32-row
// blocks of A straight from HBM into MFMA fragments, 64 k per chunk, the next chunk's loads
// issued before this chunk's MFMAs; A is read once and C written once.
constexpr int SN_WAVES = 8, SN_KMAX = 256, SN_NMAX = 64;
constexpr int SN_KSLOTS = SN_KMAX / 8;
constexpr int SN_PLANE = SN_KSLOTS * SN_NMAX * 16;   // bytes per bf16 plane of B
constexpr int SN_CHUNK = 4;                            // k16 steps per chunk of A

// VEC: A rows 16-byte aligned and K % 8 == 0 (float4 loads of whole 8-k groups).
// VST: C rows 16-byte aligned and N % 4 == 0 (float4 stores).
template <bool VEC, bool VST>
__global__ void __launch_bounds__(64 * SN_WAVES, 1) gemm_smalln_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char wl[3 * SN_PLANE];
  const int b = blockIdx.y;
  const float* __restrict__ A = g.A + b * g.a_bs;
  const float* __restrict__ B = g.B + b * g.b_bs;
  const int K = (int)g.K, N = (int)g.N;
  const int64_t M = g.M;
  const int ncb = (N + 31) / 32;

  // B -> [plane][k / 8][n][8 k] (gemm_smallk_kernel's layout); consecutive threads take
  // consecutive n, i.e. consecutive addresses of one row of B
  for (int t = threadIdx.x; t < SN_KSLOTS * SN_NMAX; t += 64 * SN_WAVES) {
    const int kc = t / SN_NMAX, n = t % SN_NMAX;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kc * 8 + j;
      v[j] = (n < N && k < K) ? B[(int64_t)k * g.ldb + n] : 0.f;
    }
    uint4 h, m, l;
    sk_split8(v, h, m, l);
    const int o = (kc * SN_NMAX + n) * 16;
    *(uint4*)(wl + o) = h;
    *(uint4*)(wl + SN_PLANE + o) = m;
    *(uint4*)(wl + 2 * SN_PLANE + o) = l;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int nks = (K + 15) / 16;
  const int nch = (nks + SN_CHUNK - 1) / SN_CHUNK;
  const int64_t nrb = (M + 31) / 32;
  // one chunk of a row block's A: 8 consecutive k per lane and k16 step (one MFMA fragment);
  // rows past M read row M - 1 (not stored)
  auto fetch = [&](int64_t rb, int c, float (&r)[SN_CHUNK][8]) {
    const int64_t row = rb * 32 + (lane & 31);
    const float* ar = A + (row < M ? row : M - 1) * g.lda;
#pragma unroll
    for (int s = 0; s < SN_CHUNK; ++s) {
      const int k0 = 16 * (SN_CHUNK * c + s) + 8 * half;
      if (VEC) {   // (a group at or past K loads k = 0..7 and is zeroed at its split)
        const float4 p = *(const float4*)(ar + (k0 < K ? k0 : 0));
        const float4 q = *(const float4*)(ar + (k0 < K ? k0 + 4 : 4));
        r[s][0] = p.x; r[s][1] = p.y; r[s][2] = p.z; r[s][3] = p.w;
        r[s][4] = q.x; r[s][5] = q.y; r[s][6] = q.z; r[s][7] = q.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[s][j] = k0 + j < K ? ar[k0 + j] : 0.f;
      }
    }
  };
  // row blocks dealt wave-major (block x, then x + gridDim.x, ...): every workgroup gets a
  // share when the blocks are fewer than the waves (PPI: 351 per head for 512 waves)
  int64_t rb = (int64_t)wave * gridDim.x + blockIdx.x;
  const int64_t rstep = (int64_t)gridDim.x * SN_WAVES;
  float cur[SN_CHUNK][8], nxt[SN_CHUNK][8];
  if (rb < nrb) fetch(rb, 0, cur);
  for (; rb < nrb; rb += rstep) {
    floatx16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll
    for (int c = 0; c < SN_KMAX / (16 * SN_CHUNK); ++c) {
      if (c >= nch) break;
      if (c + 1 < nch) fetch(rb, c + 1, nxt);
      else if (rb + rstep < nrb) fetch(rb + rstep, 0, nxt);
      bf16x8 fa[SN_CHUNK][3];
#pragma unroll
      for (int s = 0; s < SN_CHUNK; ++s) {
        if (VEC && 16 * (SN_CHUNK * c + s) + 8 * half >= K) {
#pragma unroll
          for (int j = 0; j < 8; ++j) cur[s][j] = 0.f;
        }
        uint4 h, m, l;
        sk_split8(cur[s], h, m, l);
        fa[s][0] = __builtin_bit_cast(bf16x8, h);
        fa[s][1] = __builtin_bit_cast(bf16x8, m);
        fa[s][2] = __builtin_bit_cast(bf16x8, l);
      }
#pragma unroll
      for (int s = 0; s < SN_CHUNK; ++s) {
        const int ks = SN_CHUNK * c + s;
        if (ks >= nks) break;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (i >= ncb) break;
          bf16x8 fb[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fb[p] = *(const bf16x8*)(wl + p * SN_PLANE +
                                     ((2 * ks + half) * SN_NMAX + i * 32 + (lane & 31)) * 16);
          // small terms first: (l,h) (h,l) (m,m) (m,h) (h,m) (h,h), as gemm_smallk_kernel
          constexpr int PLA[6] = {2, 0, 1, 1, 0, 0};
          constexpr int PLB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
          for (int t = 0; t < 6; ++t)   // C^T = B^T A^T: lane = output row, registers = columns
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[PLB[t]], fa[s][PLA[t]], acc[i],
                                                             0, 0, 0);
        }
      }
#pragma unroll
      for (int s = 0; s < SN_CHUNK; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[s][j] = nxt[s][j];
    }
    // lane l: output row rb*32 + (l & 31); registers 4j..4j+3: columns i*32 + 8j + 4*(l >> 5) + 0..3
    const int64_t row = rb * 32 + (lane & 31);
    if (row < M) {
      float* base = g.C0 + b * g.c0_bs + row * g.ldc0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i >= ncb) break;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = i * 32 + 8 * j + 4 * half;
          if (VST) {
            if (col < N)
              *(float4*)(base + col) =
                  make_float4(acc[i][4 * j], acc[i][4 * j + 1], acc[i][4 * j + 2], acc[i][4 * j + 3]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (col + r < N) base[col + r] = acc[i][4 * j + r];
          }
        }
      }
    }
  }
}

// Weight gradient over rows, the same arithmetic: C_b = A_b^T B_b with both operands stored
// row-contiguous (A(m, k) = A[k * lda + m], B(k, n) = B[k * ldb + n]), M <= 256, N <= 64 and a
// long K (the rows): the reassociated first layer's g_W_h = go_h^T Z_h (functional.
// _reassoc_backward; PPI layer 0: 4 heads x (256 x 44900) . (44900 x 52)), which the tiled
// split-K kernel ran at 74 us for 221 MB. One workgroup per (K slice, batch entry); wave w owns
// output rows 32w..32w+31 and both 32-column blocks (32 accumulator registers). Per chunk of 64
// rows the workgroup stages B's chunk once as bf16 planes in LDS (double-buffered, 48 KB: every
// wave needs all of it) while each wave loads its own A columns straight into MFMA fragments
// (lane = output row, 8 consecutive k = rows of A: 128 contiguous bytes per half-wave and row);
// the next chunk's loads are issued before this chunk's MFMAs. Slice partials go to [z][b][M][N]
// slabs summed in slice order by splitk_reduce_kernel (deterministic).
constexpr int TN_WAVES = 8, TN_MMAX = 256, TN_NMAX = 64, TN_ROWS = 64;
constexpr int TN_KSLOTS = TN_ROWS / 8;
constexpr int TN_PLANE = TN_KSLOTS * TN_NMAX * 16;   // bytes per bf16 plane of a B chunk

__global__ void __launch_bounds__(64 * TN_WAVES, 1) gemm_tn_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char bl[2][3 * TN_PLANE];
  const int b = blockIdx.y, z = blockIdx.x;
  const float* __restrict__ A = g.A + b * g.a_bs;
  const float* __restrict__ B = g.B + b * g.b_bs;
  const int M = (int)g.M, N = (int)g.N;
  const int64_t k0 = (int64_t)z * g.k_per_split;
  const int64_t k1 = min(g.K, k0 + g.k_per_split);
  const int ncb = (N + 31) / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int m = wave * 32 + (lane & 31);
  const bool mact = wave * 32 < M;
  // this thread's B staging item: k-slot ks (8 rows), column bn
  const int ks = threadIdx.x / TN_NMAX, bn = threadIdx.x % TN_NMAX;
  float braw[8], araw[4][8];
  // unconditional loads from clamped addresses (a conditional load is a branch, and the
  // compiler waited vmcnt(0) at every join: 131 us for this product). Rows past M and columns
  // past N only feed outputs that are never stored; rows of the K tail are zeroed in B alone,
  // when its chunk is staged (a select here would wait for each load at once)
  const float* __restrict__ Bc = B + (bn < N ? bn : N - 1);
  const float* __restrict__ Ac = A + (m < M ? m : M - 1);
  auto fetch = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t r = r0 + 8 * ks + j;
      braw[j] = Bc[(r < k1 ? r : k1 - 1) * g.ldb];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t r = r0 + 16 * s + 8 * half + j;
        araw[s][j] = Ac[(r < k1 ? r : k1 - 1) * g.lda];
      }
  };
  floatx16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  const int64_t nch = k1 > k0 ? ceil_div(k1 - k0, (int64_t)TN_ROWS) : 0;
  if (nch > 0) fetch(k0);
  for (int64_t c = 0; c < nch; ++c) {
    char* buf = bl[c & 1];
    {
      const int64_t r0 = k0 + c * TN_ROWS + 8 * ks;
#pragma unroll
      for (int j = 0; j < 8; ++j) braw[j] = r0 + j < k1 ? braw[j] : 0.f;
      uint4 h, mm, l;
      sk_split8(braw, h, mm, l);
      const int o = (ks * TN_NMAX + bn) * 16;
      *(uint4*)(buf + o) = h;
      *(uint4*)(buf + TN_PLANE + o) = mm;
      *(uint4*)(buf + 2 * TN_PLANE + o) = l;
    }
    bf16x8 fa[4][3];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      uint4 h, mm, l;
      sk_split8(araw[s], h, mm, l);
      fa[s][0] = __builtin_bit_cast(bf16x8, h);
      fa[s][1] = __builtin_bit_cast(bf16x8, mm);
      fa[s][2] = __builtin_bit_cast(bf16x8, l);
    }
    // (one barrier per chunk: a wave writes buffer c & 1 again only after the barrier of chunk
    // c + 1, which every wave reaches after its reads of chunk c)
    __syncthreads();
    if (c + 1 < nch) fetch(k0 + (c + 1) * TN_ROWS);
    if (mact) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (i >= ncb) break;
          bf16x8 fb[3];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fb[p] = *(const bf16x8*)(buf + p * TN_PLANE +
                                     ((2 * s + half) * TN_NMAX + i * 32 + (lane & 31)) * 16);
          constexpr int PLA[6] = {2, 0, 1, 1, 0, 0};
          constexpr int PLB[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
          for (int t = 0; t < 6; ++t)   // lane = output column, registers = rows
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][PLA[t]], fb[PLB[t]], acc[i],
                                                             0, 0, 0);
        }
    }
  }
  if (!mact) return;
  // lane l: column i*32 + (l & 31); register r: row wave*32 + 8(r >> 2) + 4(l >> 5) + (r & 3)
  float* P = g.partial + ((int64_t)z * gridDim.y + b) * (int64_t)M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int col = i * 32 + (lane & 31);
    if (i >= ncb || col >= N) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wave * 32 + 8 * (r >> 2) + 4 * half + (r & 3);
      if (row < M) P[(int64_t)row * N + col] = acc[i][r];
    }
  }
}

}  // namespace

bool gemm_tn_fits(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc) {
  return !a_kc && !b_kc && M > 8 && M <= TN_MMAX && N >= 1 && N <= TN_NMAX && K >= 4096;
}

// Slices: ~256 workgroups over the batch entries, each slice at least 512 rows; needs
// slices x batch x M x N floats of workspace for the partials (returns 0: not launched).
int launch_gemm_tn(gk::GemmArgs g, int batch, void* workspace, size_t workspace_bytes,
                   hipStream_t stream) {
  GATX_REQUIRE(g.M <= TN_MMAX && g.N <= TN_NMAX && batch < 65536, "gemm_tn: shape");
  int64_t sp = std::max<int64_t>(2, std::min<int64_t>(256 / batch, g.K / 512));
  while (sp > 1 && (!workspace || (size_t)sp * batch * g.M * g.N * sizeof(float) > workspace_bytes))
    --sp;
  if (sp < 2) return 0;
  g.k_per_split = round_up(ceil_div(g.K, sp), (int64_t)TN_ROWS);
  g.splits = (int)ceil_div(g.K, g.k_per_split);
  g.partial = (float*)workspace;
  gemm_tn_kernel<<<dim3((unsigned)g.splits, (unsigned)batch), 64 * TN_WAVES, 0, stream>>>(g);
  GATX_LAUNCH_CHECK("gemm_tn");
  launch_splitk_reduce(g, batch, stream);
  GATX_LAUNCH_CHECK("splitk_reduce");
  return 1;
}

bool gemm_smalln_fits(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc, int accumulate,
                      bool epilogue) {
  return a_kc && !b_kc && !accumulate && !epilogue && K > SK_KMAX && K <= SN_KMAX && N >= 1 &&
         N <= SN_NMAX && M >= 32 * SN_WAVES;
}

int launch_gemm_smalln(const gk::GemmArgs& g, int batch, hipStream_t stream) {
  GATX_REQUIRE(g.K <= SN_KMAX && g.N <= SN_NMAX && batch < 65536, "gemm_smalln: shape");
  const int64_t nrb = ceil_div(g.M, 32);
  const int64_t per = std::max<int64_t>(1, 256 / batch);
  const unsigned gx = (unsigned)std::min<int64_t>(per, nrb);
  dim3 grid(gx, (unsigned)batch);
  const bool vec = ((uintptr_t)g.A % 16 == 0) && g.lda % 4 == 0 && g.a_bs % 4 == 0 && g.K % 8 == 0;
  const bool vst = ((uintptr_t)g.C0 % 16 == 0) && g.ldc0 % 4 == 0 && g.c0_bs % 4 == 0 &&
                   g.N % 4 == 0;
  if (vec && vst) gemm_smalln_kernel<true, true><<<grid, 64 * SN_WAVES, 0, stream>>>(g);
  else if (vec) gemm_smalln_kernel<true, false><<<grid, 64 * SN_WAVES, 0, stream>>>(g);
  else if (vst) gemm_smalln_kernel<false, true><<<grid, 64 * SN_WAVES, 0, stream>>>(g);
  else gemm_smalln_kernel<false, false><<<grid, 64 * SN_WAVES, 0, stream>>>(g);
  GATX_LAUNCH_CHECK("gemm_smalln");
  return 0;
}

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
  const bool vst = ((uintptr_t)g.C0 % 16 == 0) && g.ldc0 % 4 == 0 && g.c0_bs % 4 == 0;
#define GATX_SK(V, E)                                                                          \
  do {                                                                                         \
    if (vst && g.N == SK_NMAX)                                                                 \
      gemm_smallk_kernel<V, E, true, true><<<grid, 64 * SK_WAVES, 0, stream>>>(g);             \
    else if (vst) gemm_smallk_kernel<V, E, true><<<grid, 64 * SK_WAVES, 0, stream>>>(g);       \
    else gemm_smallk_kernel<V, E, false><<<grid, 64 * SK_WAVES, 0, stream>>>(g);               \
  } while (0)
  if (vec && g.elu) GATX_SK(true, true);
  else if (vec) GATX_SK(true, false);
  else if (g.elu) GATX_SK(false, true);
  else GATX_SK(false, false);
#undef GATX_SK
  GATX_LAUNCH_CHECK("gemm_smallk");
  return 0;
}

}  // namespace gatx
