// fp32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate;
// gfx950 has no xf32, and the f32 MFMA runs at the f32 vector peak, 157 TF).
//
// Replaces the projection `self.W(x)` of models/gat_layer.py:64 — with the attention vector
// folded in as 2*NH extra output columns (W_aug, see gatx_prepare_weights), so the same launch
// also produces the per-node logit factors s_src / s_dst that stand in for the per-edge
// (E, NH*2F) x a^T GEMV of :76-82 — and the two backward products g_x and g_W.
//
// Tile 128 x 128 x 16 per 256-thread workgroup, 4 waves as 2 x 2, each wave 64 x 64 = 2 x 2 MFMA
// blocks of 32 x 32. Two LDS stages (one barrier per K-tile): tile kt+1 is fetched into
// registers before tile kt's MFMAs and stored into the other stage after them. An operand whose
// K index is contiguous in memory is staged as a [row][k] image (float4 copies, 36-float rows:
// conflict-free ds_read_b128); a row-contiguous one as a [k][row] image. Within each group of 8
// k, lane half h feeds k = 8g + 4h + j to MFMA step j, so one 16-byte read gives a lane its
// operands for 4 MFMAs; the next group's fragments are read while the current group's MFMAs run.
// Occupancy 4 workgroups per CU (40 KB LDS, <= 128 VGPRs each); the last partial wave of tiles
// can be split along K (tail split) so it does not leave most of the chip idle. A barrier-free
// variant streaming each wave's fragments from L1/L2 into registers (no LDS) reached only 74 TF
// on the same shapes (TA-bound), so operands are shared through LDS.
#include "gemm_common.h"

#include <string.h>

namespace gatx {
namespace {
using namespace gk;

// Deterministic split-K combine: C = epilogue(sum over slabs in slab order), one pass.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(GemmArgs g, int batch) {
  const int64_t MN = g.M * g.N, total = MN * batch;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / MN, mn = t - b * MN, row = mn / g.N, col = mn - row * g.N;
    // slabs summed in order z = 0, 1, ...; eight loads issued before their adds (a small output
    // split 64 ways waited one load latency per slab)
    const float* p = g.partial + b * MN + mn;
    const int64_t zs = (int64_t)batch * MN;
    float v = 0.f;
    int z = 0;
    for (; z + 8 <= g.splits; z += 8) {
      float x[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = p[(z + i) * zs];
#pragma unroll
      for (int i = 0; i < 8; ++i) v += x[i];
    }
    for (; z < g.splits; ++z) v += p[z * zs];
    store_out(g, b, row, col, v);
  }
}

// The same reduction four columns at a time for a plain output (one batch entry, one output
// range, no bias / residual / ELU; N % 4 == 0, C0 16-byte aligned, ldc0 % 4 == 0): float4 slab
// loads, slabs summed in the same order (z ascending), so the result equals splitk_reduce_kernel's.
__global__ void __launch_bounds__(256) splitk_reduce4_kernel(GemmArgs g) {
  const int64_t MN = g.M * g.N, total4 = MN / 4, n4 = g.N / 4;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total4;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t / n4, col = 4 * (t - row * n4);
    const float* p = g.partial + row * g.N + col;
    float4 v = *(const float4*)p;
    int z = 1;
    for (; z + 4 <= g.splits; z += 4) {
      const float4 a = *(const float4*)(p + (int64_t)z * MN);
      const float4 b = *(const float4*)(p + (int64_t)(z + 1) * MN);
      const float4 c = *(const float4*)(p + (int64_t)(z + 2) * MN);
      const float4 d = *(const float4*)(p + (int64_t)(z + 3) * MN);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
      v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
      v.x += c.x; v.y += c.y; v.z += c.z; v.w += c.w;
      v.x += d.x; v.y += d.y; v.z += d.z; v.w += d.w;
    }
    for (; z < g.splits; ++z) {
      const float4 a = *(const float4*)(p + (int64_t)z * MN);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    float* o = g.C0 + row * g.ldc0 + col;
    if (g.accumulate) {
      const float4 c = *(const float4*)o;
      v.x += c.x; v.y += c.y; v.z += c.z; v.w += c.w;
    }
    *(float4*)o = v;
  }
}

inline bool reduce4_ok(const GemmArgs& g, int batch) {
  return batch == 1 && g.N % 4 == 0 && g.n_split >= g.N && !g.bias && !g.resid && !g.elu &&
         g.ldc0 % 4 == 0 && (uintptr_t)g.C0 % 16 == 0;
}

}  // namespace

// (outside the anonymous namespace: gemm_smallk.hip's split-K kernel reduces through it too)
void launch_splitk_reduce(const GemmArgs& g, int batch, hipStream_t stream) {
  if (reduce4_ok(g, batch)) {
    const int64_t total4 = g.M * g.N / 4;
    splitk_reduce4_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total4, 256), 8192), 256, 0,
                            stream>>>(g);
  } else {
    const int64_t total = g.M * g.N * batch;
    splitk_reduce_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 8192), 256, 0,
                           stream>>>(g, batch);
  }
}

namespace {

// Skinny weight gradients: C = A^T B with both operands row-contiguous (A(m, k) = A[k lda + m],
// B(k, n) = B[k ldb + n]), at most 8 output rows and a long K (PPI's first-layer score gradient
// G_s^T x: 8 x 50 over 44,900 nodes, which the 128 x 128 x3 tiles ran in 60 us for 11 MB of
// operands). Plain fp32 on the VALU: lane = output column (256-B row segments per wave), the 16
// waves of a block interleave this split's K range, four rows in flight each, A's <= 8 values
// per row wave-uniform; waves summed in fixed order through LDS into the split's slab.
constexpr int kSkinnyRows = 8;
__global__ void __launch_bounds__(1024) gemm_skinny_rc_kernel(GemmArgs g) {
  constexpr int T = kSkinnyRows, NW = 16, U = 4;
  __shared__ float red[NW][T][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t n = blockIdx.x * 64ll + lane;
  const int z = blockIdx.y;
  const int64_t kb = (int64_t)z * g.k_per_split, ke = min(g.K, kb + g.k_per_split);
  const bool nv = n < g.N;
  const int M = (int)g.M;
  float acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = 0.f;
  for (int64_t k0 = kb + wave; k0 < ke; k0 += (int64_t)NW * U) {
    float b[U], a[U][T];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = k0 + (int64_t)u * NW;
      const bool ok = k < ke;
      const int64_t kk = ok ? k : kb;
      b[u] = g.B[kk * g.ldb + (nv ? n : 0)];
      if (!ok || !nv) b[u] = 0.f;
#pragma unroll
      for (int t = 0; t < T; ++t) a[u][t] = (t < M && ok) ? g.A[kk * g.lda + t] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t] = fmaf(a[u][t], b[u], acc[t]);
  }
#pragma unroll
  for (int t = 0; t < T; ++t) red[wave][t][lane] = acc[t];
  __syncthreads();
  if (threadIdx.x < T * 64) {
    const int t = threadIdx.x / 64, c = threadIdx.x % 64;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][t][c];
    const int64_t col = blockIdx.x * 64ll + c;
    if (t < M && col < g.N) {
      if (g.splits > 1) g.partial[(int64_t)z * g.M * g.N + t * g.N + col] = v;
      else store_out(g, 0, t, col, v);
    }
  }
}

// Split-K reduction with one wave per output element: lane l sums slabs l, l + 64, ... in order,
// then a fixed butterfly over the lanes (deterministic; for small outputs over many slabs, where
// a thread per element waited one load latency per slab).
__global__ void __launch_bounds__(256) splitk_reduce_lanes_kernel(GemmArgs g) {
  const int lane = threadIdx.x & 63;
  const int64_t MN = g.M * g.N;
  const int64_t t = blockIdx.x * 4ll + (threadIdx.x >> 6);
  if (t >= MN) return;   // (whole waves: t is wave-uniform)
  float v = 0.f;
  for (int z = lane; z < g.splits; z += 64) v += g.partial[(int64_t)z * MN + t];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (lane == 0) store_out(g, 0, t / g.N, t % g.N, v);
}

// Tiny products (K <= 64, M N K <= 2^25 multiply-adds: PATTERN's projections) on the VALU in
// plain fp32: the tiled MFMA kernels spend 10-14 us there on prologue,
// barriers and a handful of K-tiles for a few MFLOP, while this is launch-bound (~3 us). Each
// output (b, m, n) is owned by a group of L lanes splitting K (k = li, li + L, ...; fma chain per
// lane, then a fixed-order group_sum<L>), so the result is deterministic and fp32-faithful (exact
// fp32 products). Control flow is wave-uniform: a wave walks its outputs together and the lanes
// of finished groups contribute zeros.
template <int L>
__global__ void __launch_bounds__(256) gemm_tiny_kernel(GemmArgs g, int batch, int a_kc,
                                                        int b_kc) {
  constexpr int GPW = 64 / L;   // output groups per wave
  const int64_t MN = g.M * g.N, total = MN * batch;
  const int lane = threadIdx.x & 63, grp = lane / L, li = lane % L;
  const int64_t wave = blockIdx.x * 4ll + (threadIdx.x >> 6), nwaves = gridDim.x * 4ll;
  for (int64_t base = wave * GPW; base < total; base += nwaves * GPW) {
    const int64_t o = base + grp;
    const bool valid = o < total;
    const int64_t oc = valid ? o : total - 1;
    const int64_t b = oc / MN, mn = oc - b * MN, m = mn / g.N, n = mn - m * g.N;
    const float* __restrict__ A = g.A + b * g.a_bs;
    const float* __restrict__ B = g.B + b * g.b_bs;
    float acc = 0.f;
    if (valid) {
#pragma unroll 4
      for (int64_t k = li; k < g.K; k += L) {
        const float av = a_kc ? A[m * g.lda + k] : A[k * g.lda + m];
        const float bv = b_kc ? B[n * g.ldb + k] : B[k * g.ldb + n];
        acc = fmaf(av, bv, acc);
      }
    }
    acc = group_sum<L>(acc);
    if (valid && li == 0) store_out(g, b, m, n, acc);
  }
}

int launch_gemm_tiny(const GemmArgs& g, int batch, bool a_kc, bool b_kc, hipStream_t stream) {
  const int64_t total = g.M * g.N * batch;
  // lanes per output: at most ~12 k per lane (the loop is load-latency bound), more while the
  // chip is short of lanes (< 2^16 busy), never more than K
  int64_t L = 1;
  while (L < 64 && L * 12 < g.K) L <<= 1;
  while (L < 64 && total * L < (1 << 16) && L < g.K) L <<= 1;
  const int64_t groups_per_block = 256 / L;
  const unsigned grid = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>(ceil_div(total, groups_per_block), 4096));
#define GATX_TINY(LL) \
  gemm_tiny_kernel<LL><<<grid, 256, 0, stream>>>(g, batch, (int)a_kc, (int)b_kc)
  switch (L) {
    case 1: GATX_TINY(1); break; case 2: GATX_TINY(2); break; case 4: GATX_TINY(4); break;
    case 8: GATX_TINY(8); break; case 16: GATX_TINY(16); break; case 32: GATX_TINY(32); break;
    default: GATX_TINY(64); break;
  }
#undef GATX_TINY
  GATX_LAUNCH_CHECK("gemm_tiny");
  return 0;
}

// Tail fix-up: the last tail_rem tiles, each the sum of tail_s K-slices in slice order.
__global__ void __launch_bounds__(256) tail_fixup_kernel(GemmArgs g) {
  const int64_t BN = g.bn, TS = (int64_t)g.bm * BN, total = g.tail_rem * TS;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ti = t / TS, rc = t - ti * TS, rl = rc / BN, cl = rc - rl * BN;
    const int64_t lin = g.dp_blocks + ti, tm = lin / g.tiles_n, tn = lin - tm * g.tiles_n;
    const int64_t row = tm * g.bm + rl, col = tn * BN + cl;
    if (row >= g.M || col >= g.N) continue;
    float v = 0.f;
    for (int z = 0; z < g.tail_s; ++z) v += g.tail_partial[((int64_t)z * g.tail_rem + ti) * TS + rc];
    store_out(g, 0, row, col, v);
  }
}

// Tail fix-up of a projection with fused scores (g.s_part): block (tail tile, 64-row chunk), a
// wave per row, lane l the four columns 4l..4l+3; the K-slices summed in slice order exactly as
// tail_fixup_kernel, stored, then the row's share of each score reduced over the wave in a fixed
// butterfly into s_part[tn][row][h]. The tile's A2 columns are staged in LDS once per block.
__global__ void __launch_bounds__(256) tail_fixup_scores_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float a2s[16 * 256];   // [H2][bn]
  const int BN = g.bn, H2 = g.s_h2, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t TS = (int64_t)g.bm * BN, chunks = g.bm / 64;
  const int64_t ti = blockIdx.x / chunks, ch = blockIdx.x - ti * chunks;
  const int64_t lin = g.dp_blocks + ti, tm = lin / g.tiles_n, tn = lin - tm * g.tiles_n;
  for (int t = threadIdx.x; t < H2 * BN; t += 256) {
    const int h = t / BN, c = t - h * BN;
    const int64_t col = tn * BN + c;
    a2s[t] = col < g.N ? score_weight(g.s_a, g.s_nh, g.s_f, g.s_fp, h, col) : 0.f;
  }
  __syncthreads();
  const int cl = 4 * lane;
  for (int r = wave; r < 64; r += 4) {
    const int64_t rl = ch * 64 + r, row = tm * g.bm + rl;
    if (row >= g.M) break;   // wave-uniform
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cl < BN) {
      for (int z = 0; z < g.tail_s; ++z) {
        const float4 p = *(const float4*)(g.tail_partial + ((int64_t)z * g.tail_rem + ti) * TS +
                                          rl * BN + cl);
        v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
      }
      const int64_t col = tn * BN + cl;
      if (col < g.N) store_out(g, 0, row, col, v.x);
      if (col + 1 < g.N) store_out(g, 0, row, col + 1, v.y);
      if (col + 2 < g.N) store_out(g, 0, row, col + 2, v.z);
      if (col + 3 < g.N) store_out(g, 0, row, col + 3, v.w);
    }
    for (int h = 0; h < H2; ++h) {
      float t = 0.f;
      if (cl < BN) {
        const float4 w = *(const float4*)(a2s + h * BN + cl);
        t = fmaf(v.x, w.x, t);
        t = fmaf(v.y, w.y, t);
        t = fmaf(v.z, w.z, t);
        t = fmaf(v.w, w.w, t);
      }
      for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
      if (lane == 0) g.s_part[(tn * g.M + row) * H2 + h] = t;
    }
  }
}

// S = sum over the column tiles of the fused-score partials, in tile order (deterministic).
__global__ void __launch_bounds__(256) score_combine_kernel(const float* __restrict__ part,
                                                            int64_t MH, int tiles,
                                                            float* __restrict__ S) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < MH;
       t += (int64_t)gridDim.x * blockDim.x) {
    float v = part[t];
    for (int k = 1; k < tiles; ++k) v += part[k * MH + t];
    S[t] = v;
  }
}

// A_KC: A is k-contiguous (sak == 1, ld = sam) else m-contiguous; B_KC: B is k-contiguous
// (sbk == 1, ld = sbn) else n-contiguous. TAG only separates the symbol names of the call sites
// in profiles (0 = forward projection, 1 = auxiliary products, 2 = split-K weight gradient).
// WGM x WGN waves per workgroup, each owning (BM/WGM) x (BN/WGN) = MB x NB MFMA blocks of 32x32.
template <bool A_KC, bool B_KC, bool VEC, int TAG, int BK, int MINB, int WGM, int WGN>
__global__ void __launch_bounds__(64 * WGM * WGN, MINB) gemm_f32_kernel(GemmArgs g) {
  constexpr int NT = 64 * WGM * WGN, MB = 4 / WGM, NB = 4 / WGN;
  using TA = Tile<A_KC, BM, BK, NT>;
  using TB = Tile<B_KC, BN, BK, NT>;
  constexpr int STAGE = TA::SIZE + TB::SIZE;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

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
  } else if (g.tail_s > 1) {   // data-parallel part of a tail-split launch: whole K
    tile_of(blockIdx.x, g.dp_blocks, g.tiles_n, tm, tn);
    kb = 0;
    K = g.K;
  } else {
    tile_of(blockIdx.x, T, g.tiles_n, tm, tn);
    // split-K: slice blockIdx.z covers k in [kb, ke) and writes its own partial slab
    kb = blockIdx.z * g.k_per_split;
    K = min(g.K, kb + g.k_per_split);
  }
  const int64_t m0 = tm * BM, n0 = tn * BN;
  const float* __restrict__ A = g.A + blockIdx.y * g.a_bs;
  const float* __restrict__ B = g.B + blockIdx.y * g.b_bs;
  const int64_t M = g.M, N = g.N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int il = lane & 31, h4 = 4 * (lane >> 5);

  floatx16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float4 va[TA::NV], vb[TB::NV];
  const int64_t nk = K > kb ? ceil_div(K - kb, BK) : 0;
  if (nk > 0) {
    TA::template load<VEC>(A, g.lda, m0, M, kb, K, va);
    TB::template load<VEC>(B, g.ldb, n0, N, kb, K, vb);
    TA::template store<VEC>(smem, va, m0, M, kb, K);
    TB::template store<VEC>(smem + TA::SIZE, vb, n0, N, kb, K);
  }
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    float* cur = smem + (kt & 1) * STAGE;
    float* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    const bool more = kt + 1 < nk;
    if (more) {
      TA::template load<VEC>(A, g.lda, m0, M, kb + (kt + 1) * BK, K, va);
      TB::template load<VEC>(B, g.ldb, n0, N, kb + (kt + 1) * BK, K, vb);
    }
    const float* ai = cur;
    const float* bi = cur + TA::SIZE;
    float4 fa[MB], fb[NB];
#pragma unroll
    for (int x = 0; x < MB; ++x) fa[x] = TA::frag(ai, wm * (MB * 32) + x * 32 + il, h4);
#pragma unroll
    for (int x = 0; x < NB; ++x) fb[x] = TB::frag(bi, wn * (NB * 32) + x * 32 + il, h4);
#pragma unroll
    for (int grp = 0; grp < BK / 8; ++grp) {
      float4 na[MB], nb[NB];
      if (grp + 1 < BK / 8) {
#pragma unroll
        for (int x = 0; x < MB; ++x)
          na[x] = TA::frag(ai, wm * (MB * 32) + x * 32 + il, 8 * (grp + 1) + h4);
#pragma unroll
        for (int x = 0; x < NB; ++x)
          nb[x] = TB::frag(bi, wn * (NB * 32) + x * 32 + il, 8 * (grp + 1) + h4);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MB; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(get4(fa[mi], j), get4(fb[ni], j),
                                                              acc[mi][ni], 0, 0, 0);
      if (grp + 1 < BK / 8) {
#pragma unroll
        for (int x = 0; x < MB; ++x) fa[x] = na[x];
#pragma unroll
        for (int x = 0; x < NB; ++x) fb[x] = nb[x];
      }
    }
    if (more) {
      TA::template store<VEC>(nxt, va, m0, M, kb + (kt + 1) * BK, K);
      TB::template store<VEC>(nxt + TA::SIZE, vb, n0, N, kb + (kt + 1) * BK, K);
    }
    __syncthreads();
  }

  write_tile<MB, NB, BM, BN, false>(g, acc, tail_z, tail_ti, m0, n0, wm, wn, lane);
}

// GEMM arithmetic, gatx_set_gemm_mode (never the environment): 2 "f16x3" (default) = the split-fp16
// kernel of gemm_x3.hip (3 fp16 MFMA products; tiles outside its operand range fall back to the
// bf16 split in-kernel), 1 "x3" = the split-bf16 kernel (6 bf16 products), 0 "f32" =
// v_mfma_f32_32x32x2_f32.
int g_gemm_mode = 2;
int gemm_mode() { return g_gemm_mode; }

// The f32-MFMA kernel's K-tile depth / occupancy: BK 16 at 4 workgroups per CU (LDS 4 x 40 KB,
// <= 128 VGPRs). Measured on the PPI shapes (round 1): BK 64 / 1 WG 93 TF, BK 32 / 2 WG 111, BK 16
// / 3 WG 115, BK 16 / 4 WG 118 (occupancy hides the barrier and LDS latency that one K-tile of
// MFMAs cannot); 8-wave workgroups with 32 x 64 wave tiles 113 TF. Only the last is built.

// The pre-split kernel, then the tail fix-up of its partial last wave (as launch_gemm).
int launch_f16p_and_fixups(const GemmArgs& g, int tag, hipStream_t stream) {
  GATX_CALL(launch_gemm_f16p(g, tag, stream));
  if (g.tail_s > 1 && g.s_part) {
    tail_fixup_scores_kernel<<<(unsigned)(g.tail_rem * (g.bm / 64)), 256, 0, stream>>>(g);
    GATX_LAUNCH_CHECK("tail_fixup_scores");
  } else if (g.tail_s > 1) {
    const int64_t total = g.tail_rem * g.bm * g.bn;
    tail_fixup_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 8192), 256, 0, stream>>>(g);
    GATX_LAUNCH_CHECK("tail_fixup");
  }
  return 0;
}

// The row-contiguous f16x3 weight-gradient kernel, then the split-K reduction of its slabs.
int launch_f16rc_and_reduce(const GemmArgs& g, hipStream_t stream) {
  GATX_CALL(launch_gemm_f16rc(g, stream));
  if (g.splits > 1) {
    launch_splitk_reduce(g, 1, stream);
    GATX_LAUNCH_CHECK("splitk_reduce");
  }
  return 0;
}

template <int TAG>
int launch_gemm(const GemmArgs& g0, bool a_kc, bool b_kc, int batch, hipStream_t stream) {
  GemmArgs g = g0;
  const int64_t tiles = g.tiles_m * g.tiles_n;
  GATX_REQUIRE(tiles < (1ll << 31) && batch < 65536, "gemm: too many tiles");
  const int64_t gx = g.tail_s > 1 ? g.dp_blocks + g.tail_rem * g.tail_s : tiles;
  dim3 grid((unsigned)gx, (unsigned)batch, (unsigned)g.splits);
  if (gemm_mode() >= 1) {
    GATX_CALL(launch_gemm_x3(g, a_kc, b_kc, batch, TAG, stream));
  } else {
#define GATX_GEMM_V(AK, BKC, V) gemm_f32_kernel<AK, BKC, V, TAG, 16, 4, 2, 2><<<grid, 256, 0, stream>>>(g)
#define GATX_GEMM_GO(AK, BKC)                                                                  \
  do {                                                                                        \
    if (g.a_vec && g.b_vec) GATX_GEMM_V(AK, BKC, true);                                       \
    else GATX_GEMM_V(AK, BKC, false);                                                         \
  } while (0)
  if (a_kc && b_kc) GATX_GEMM_GO(true, true);
  else if (a_kc) GATX_GEMM_GO(true, false);
  else if (b_kc) GATX_GEMM_GO(false, true);
  else GATX_GEMM_GO(false, false);
#undef GATX_GEMM_GO
#undef GATX_GEMM_V
    GATX_LAUNCH_CHECK("gemm_f32");
  }
  if (g.splits > 1) {
    launch_splitk_reduce(g, batch, stream);
    GATX_LAUNCH_CHECK("splitk_reduce");
  }
  if (g.tail_s > 1 && g.s_part) {
    tail_fixup_scores_kernel<<<(unsigned)(g.tail_rem * (g.bm / 64)), 256, 0, stream>>>(g);
    GATX_LAUNCH_CHECK("tail_fixup_scores");
  } else if (g.tail_s > 1) {
    const int64_t total = g.tail_rem * g.bm * g.bn;
    tail_fixup_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 8192), 256, 0, stream>>>(g);
    GATX_LAUNCH_CHECK("tail_fixup");
  }
  return 0;
}

// Kernel kind for an M x N output: 0 = f32 MFMA (128 x 128 tiles); 1 = x3, 128 x 128 tiles;
// 2 = x3, 256 x 256 tiles (one 8-wave workgroup per CU: half the LDS staging per MFMA) when the
// output is large and the bigger tiles cover it with at most 15% more padding (PPI L1's 1032 x 1024
// weight gradient: 11% more padding, still faster than 128 x 128 tiles; train step -0.03 ms).
struct Kind {
  int id, bm, bn;
};
Kind choose_kind(int64_t M, int64_t N) {
  if (gemm_mode() == 0) return {0, 128, 128};
  const int64_t small_area = round_up(M, 128) * round_up(N, 128);
  const int64_t big_area = round_up(M, 256) * round_up(N, 256);
  if (M >= 256 && N >= 256 && big_area * 100 <= small_area * 115) return {2, 256, 256};
  return {1, 128, 128};
}

// Workgroups of the chosen kernel resident on the whole device at once.
int64_t resident_blocks(const Kind& kd) {
  static int64_t cached[3] = {0, 0, 0};
  if (cached[kd.id]) return cached[kd.id];
  int dev = 0, cus = 0, per_cu = 0;
  int nt = kd.id == 2 ? 512 : 256;
  const void* fn = reinterpret_cast<const void*>(&gemm_f32_kernel<true, true, true, 0, 16, 4, 2, 2>);
  if (kd.id >= 1) fn = gemm_x3_occupancy_fn(kd.id == 2 ? 1 : 0);
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nt, 0) != hipSuccess ||
      cus <= 0 || per_cu <= 0) {
    (void)hipGetLastError();
    return cached[kd.id] = kd.id == 2 ? 256 : 512;
  }
  return cached[kd.id] = (int64_t)cus * per_cu;
}

// Split K when the output alone cannot fill the chip (g_W = G^T x: ~70 tiles, K = #nodes):
// the most slices (<= 64) with tiles * slices still within one resident wave, each slice
// >= 512 k, or >= 128 k (64 k for <= 4 tiles) when that leaves fewer than 16 slices. A lone
// workgroup walking a
// long K is latency-bound: PATTERN's weight gradients (one 128 x 128 tile, K = 951 nodes) took
// 60-74 us as one workgroup (~1 us per K-tile), 15 us in 6 slices of 160.
int choose_splits(int64_t tiles, int64_t K, int64_t slots) {
  int s = 1;
  while ((s + 1) * tiles <= slots && K / (s + 1) >= 512 && s < 64) ++s;
  if (s < 16) {
    const int64_t min_k = tiles <= 4 ? 64 : 128;
    int t = s;
    while ((t + 1) * tiles <= slots && K / (t + 1) >= min_k && t < 16) ++t;
    s = t;
  }
  return s;
}

// Tail split of a data-parallel GEMM: the last `rem` tiles (the partial wave) are each cut into
// s K-slices; s minimises the tail's length in waves, ceil(rem*s/slots)/s, plus the fix-up's
// partial-tile traffic (~5 TB/s) measured in waves of bm x bn x K tiles at the kernel's rate.
int choose_tail_split(int64_t tiles, int64_t K, int64_t slots, const Kind& kd, int64_t& rem) {
  rem = tiles % slots;
  if (rem == 0 || tiles < 1) return 1;
  const double peak = kd.id == 0 ? 120e12 : 200e12;   // sustained rates, f32 vs x3
  const double wave_s = 2.0 * kd.bm * kd.bn * (double)K / (peak / (double)slots);
  int best = 1;
  double best_c = 0.75 / 0.95;   // only clear wins: wave boundaries are soft in practice
  for (int s = 2; s <= 16; ++s) {
    if (ceil_div(K, s) < 2 * KSTEP) break;
    const double waves = (double)ceil_div(rem * s, slots) / s;
    const double fix = (double)rem * (s + 1) * kd.bm * kd.bn * 4.0 / 5e12 / wave_s;
    if (waves + fix < best_c * 0.95) { best = s; best_c = waves + fix; }
  }
  return best;
}


// dst[c][r] = src[r][c] through a 64 x 65 LDS tile (coalesced on both sides).
__global__ void __launch_bounds__(256) transpose_kernel(const float* __restrict__ src,
                                                        int64_t rows, int64_t cols, int64_t lds_,
                                                        float* __restrict__ dst, int64_t ldd) {
  __shared__ float t[64][65];
  const int64_t r0 = blockIdx.y * 64ll, c0 = blockIdx.x * 64ll;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < rows && c < cols) ? src[r * lds_ + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[c * ldd + r] = t[tx][i];
  }
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" int gatx_transpose_f32(int64_t rows, int64_t cols, const float* src, int64_t ld_src,
                                  float* dst, int64_t ld_dst, gatx_stream_t s) {
  GATX_REQUIRE(rows >= 0 && cols >= 0 && ld_src >= cols && ld_dst >= rows,
               "transpose: bad shape");
  if (rows == 0 || cols == 0) return 0;
  GATX_REQUIRE(ceil_div(rows, 64) < 65536, "transpose: too many rows");
  dim3 grid((unsigned)ceil_div(cols, 64), (unsigned)ceil_div(rows, 64));
  transpose_kernel<<<grid, 256, 0, (hipStream_t)s>>>(src, rows, cols, ld_src, dst, ld_dst);
  GATX_LAUNCH_CHECK("transpose");
  return 0;
}

// A node-score request riding on a projection (gatx_projection_gemm_scores).
struct ScoreReq {
  const float* a;
  int nh, f;
  float* S;
};
// Bytes of the per-column-tile score partials (0: one column tile writes S directly).
static size_t score_part_bytes(int64_t tiles_n, int64_t M, int nh) {
  return tiles_n > 1 ? (size_t)tiles_n * M * 2 * nh * sizeof(float) + 256 : 0;
}

static int gemm_impl(int64_t M, int64_t N, int64_t K, int batch, const float* A, int64_t sam,
                     int64_t sak, int64_t a_bs, const float* B, int64_t sbk, int64_t sbn,
                     int64_t b_bs, float* C0, int64_t ldc0, int64_t c0_bs, int64_t n_split,
                     float* C1, int64_t ldc1, int64_t c1_bs, int accumulate, const float* bias,
                     int64_t bias_bs, const float* resid, int64_t resid_ld, int64_t resid_bs,
                     int elu, void* workspace, size_t workspace_bytes, int tag,
                     hipStream_t stream, int64_t n_split2 = -1, float* C2 = nullptr,
                     int64_t ldc2 = 0, const ScoreReq* sc = nullptr, bool* fused = nullptr,
                     const void* b_planes = nullptr, const float* a_rowmax = nullptr) {
  if (fused) *fused = false;
  GATX_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "gemm: negative size");
  if (M == 0 || N == 0) return 0;
  GATX_REQUIRE(sak == 1 || sam == 1, "gemm: A needs a unit stride");
  GATX_REQUIRE(sbn == 1 || sbk == 1, "gemm: B needs a unit stride");
  GATX_REQUIRE(n_split >= N || C1 != nullptr, "gemm: split output needs C1");
  GATX_REQUIRE(n_split2 < 0 || (n_split2 >= n_split && (n_split2 >= N || C2 != nullptr)),
               "gemm: third output range needs n_split2 >= n_split and C2");
  GATX_REQUIRE(K > 0 || accumulate, "gemm: K == 0 needs accumulate (output would be zero)");
  if (K == 0) return 0;
  GemmArgs g;
  const bool a_kc = (sak == 1);
  const bool b_kc = (sbk == 1);
  g.M = M; g.N = N; g.K = K;
  g.A = A; g.lda = a_kc ? sam : sak; g.a_bs = a_bs;
  g.B = B; g.ldb = b_kc ? sbn : sbk; g.b_bs = b_bs;
  g.C0 = C0; g.ldc0 = ldc0; g.c0_bs = c0_bs; g.n_split = n_split;
  g.C1 = C1; g.ldc1 = ldc1; g.c1_bs = c1_bs;
  g.n_split2 = n_split2 < 0 ? INT64_MAX : n_split2;
  g.C2 = C2; g.ldc2 = ldc2;
  g.accumulate = accumulate;
  g.bias = bias; g.bias_bs = bias_bs;
  g.resid = resid; g.resid_ld = resid_ld; g.resid_bs = resid_bs;
  g.elu = elu;
  g.splits = 1; g.k_per_split = K; g.partial = nullptr;
  g.s_a = nullptr; g.s_nh = g.s_f = g.s_fp = g.s_h2 = 0; g.s_part = nullptr;
  g.b_planes = nullptr; g.b_prow = 0;
  g.a_rowmax = a_rowmax;
  auto aligned = [](const void* p, int64_t ld, int64_t bs) {
    return ((uintptr_t)p % 16 == 0) && (ld % 4 == 0) && (bs % 4 == 0);
  };
  g.a_vec = aligned(A, g.lda, a_bs);
  g.b_vec = aligned(B, g.ldb, b_bs);
  // (only short K and few rows: every output re-reads its A row and B column, so the VALU
  // kernel turns TA-bound — PATTERN's K = 952-node weight gradients ran 28 us vs 12 us tiled,
  // PPI's 44900 x 8 x 50 score product 26 us vs 11 us on the small-K MFMA kernel)
  if (K <= 64 && M <= 16384 && M * N * K * batch <= (int64_t(1) << 25)) {
    g.splits = 1; g.tail_s = 1; g.tiles_m = g.tiles_n = 1; g.dp_blocks = g.tail_rem = 0;
    g.bm = g.bn = 32; g.tail_partial = nullptr;
    return launch_gemm_tiny(g, batch, a_kc, b_kc, stream);
  }
  if (gemm_mode() >= 1 && n_split >= N &&
      gemm_smallk_fits(M, N, K, a_kc, b_kc, accumulate, resid != nullptr)) {
    g.splits = 1; g.tail_s = 1; g.tiles_m = g.tiles_n = 1; g.dp_blocks = g.tail_rem = 0;
    g.bm = g.bn = 32; g.tail_partial = nullptr;
    return launch_gemm_smallk(g, batch, stream);
  }
  if (gemm_mode() >= 1 && n_split >= N && !sc &&
      gemm_smalln_fits(M, N, K, a_kc, b_kc, accumulate, bias || resid || elu)) {
    g.splits = 1; g.tail_s = 1; g.tiles_m = g.tiles_n = 1; g.dp_blocks = g.tail_rem = 0;
    g.bm = g.bn = 32; g.tail_partial = nullptr;
    return launch_gemm_smalln(g, batch, stream);
  }
  const Kind kd = choose_kind(M, N);
  g.tiles_m = ceil_div(M, kd.bm);
  g.tiles_n = ceil_div(N, kd.bn);
  g.dp_blocks = 0; g.tail_rem = 0; g.tail_s = 1; g.bm = kd.bm; g.bn = kd.bn;
  g.tail_partial = nullptr;
  // the weight gradient G_aug^T x with G_aug's exact column maxima: the row-contiguous f16x3
  // kernel (gemm_f16p.hip), its 256-row tiles all full (a few rows past them: the thin kernel)
  const bool wgrad_f16 = a_rowmax && tag == 2 && gemm_mode() == 2 &&
                         kd.id == 2 && batch == 1 && !a_kc && !b_kc && !accumulate;
  if (wgrad_f16 && wgrad_thin_rows(M) && g.a_vec && g.b_vec && N % 4 == 0) g.tiles_m = M / kd.bm;
  const int64_t tiles = g.tiles_m * g.tiles_n * batch;
  const int64_t slots = resident_blocks(kd);
  // fused scores: x3 tiles, one batch entry, no split-K; the partials take the workspace's end
  float* s_part = nullptr;
  if (sc && kd.id >= 1 && batch == 1 && tag == 0 && !accumulate) {
    const size_t pb = score_part_bytes(g.tiles_n, M, sc->nh);
    if (pb == 0) {
      s_part = sc->S;
    } else if (workspace && workspace_bytes >= pb) {
      const size_t off = (workspace_bytes - pb) / 256 * 256;
      s_part = (float*)((char*)workspace + off);
      workspace_bytes = off;
    }
  }
  // skinny weight gradient (<= 8 output rows, row-contiguous operands, long K): the VALU kernel
  if (tag == 2 && batch == 1 && !a_kc && !b_kc && M <= kSkinnyRows && K >= 4096 && N <= 4096) {
    const int64_t chunks = ceil_div(N, (int64_t)64);
    int sp = (int)std::min<int64_t>(std::max<int64_t>(1, 256 / chunks), K / 256);
    while (sp > 1 && (!workspace || (size_t)sp * M * N * sizeof(float) > workspace_bytes)) --sp;
    g.splits = sp < 1 ? 1 : sp;
    g.k_per_split = ceil_div(K, (int64_t)g.splits);
    g.splits = (int)ceil_div(K, g.k_per_split);
    g.partial = g.splits > 1 ? (float*)workspace : nullptr;
    g.tiles_m = g.tiles_n = 1;
    gemm_skinny_rc_kernel<<<dim3((unsigned)chunks, (unsigned)g.splits), 1024, 0, stream>>>(g);
    GATX_LAUNCH_CHECK("gemm_skinny_rc");
    if (g.splits > 1) {
      splitk_reduce_lanes_kernel<<<(unsigned)ceil_div(M * N, (int64_t)4), 256, 0, stream>>>(g);
      GATX_LAUNCH_CHECK("splitk_reduce_lanes");
    }
    return 0;
  }
  // long-K weight gradient into <= 64 columns with row-contiguous operands (the reassociated
  // first layer's go_h^T Z_h): the row-streaming kernel of gemm_smallk.hip
  if (tag == 2 && gemm_mode() >= 1 && n_split >= N && !sc && gemm_tn_fits(M, N, K, a_kc, b_kc) &&
      launch_gemm_tn(g, batch, workspace, workspace_bytes, stream))
    return 0;
  if (workspace && tag == 2) {   // explicit split-K into [M][N] slabs
    int sp = choose_splits(tiles, K, slots);
    while (sp > 1 && (size_t)sp * batch * M * N * sizeof(float) > workspace_bytes) --sp;
    if (sp > 1) {
      g.k_per_split = round_up(ceil_div(K, sp), KSTEP);
      g.splits = (int)ceil_div(K, g.k_per_split);
      g.partial = (float*)workspace;
    }
  } else if (workspace && batch == 1) {   // tail split of the last partial wave
    int64_t rem = 0;
    int ts = choose_tail_split(tiles, K, slots, kd, rem);
    while (ts > 1 && (size_t)ts * rem * kd.bm * kd.bn * sizeof(float) > workspace_bytes) --ts;
    if (ts > 1) {
      g.k_per_split = round_up(ceil_div(K, ts), KSTEP);
      g.tail_s = (int)ceil_div(K, g.k_per_split);
      if (g.tail_s >= 2) {
        g.tail_rem = rem;
        g.dp_blocks = tiles - rem;
        g.tail_partial = (float*)workspace;
      } else {
        g.tail_s = 1;
        g.k_per_split = K;
      }
    }
  }
  if (s_part) {
    g.s_a = sc->a; g.s_nh = sc->nh; g.s_f = sc->f; g.s_fp = (int)round_up(sc->f, 4);
    g.s_h2 = 2 * sc->nh; g.s_part = s_part;
  }
  if (b_planes && gemm_mode() == 2 && kd.id == 2 && batch == 1 && a_kc &&
      b_kc && g.a_vec && g.b_vec && g.splits == 1 && tag != 2 && g.lda < (1 << 20) &&
      N <= 60 * 256) {   // (the planes' header holds 60 tile flags)
    g.b_planes = (const char*)b_planes + 256;   // past the planes' header (gemm_f16p.hip)
    g.b_prow = round_up(K, (int64_t)32) * 4;
  }
  if (g.b_planes) GATX_CALL(launch_f16p_and_fixups(g, tag, stream));
  else if (wgrad_f16) GATX_CALL(launch_f16rc_and_reduce(g, stream));
  else if (tag == 0) GATX_CALL(launch_gemm<0>(g, a_kc, b_kc, batch, stream));
  else if (tag == 2) GATX_CALL(launch_gemm<2>(g, a_kc, b_kc, batch, stream));
  else GATX_CALL(launch_gemm<1>(g, a_kc, b_kc, batch, stream));
  if (s_part) {
    if (s_part != sc->S) {
      const int64_t MH = M * g.s_h2;
      score_combine_kernel<<<(unsigned)std::min<int64_t>(ceil_div(MH, 256), 4096), 256, 0,
                             stream>>>(s_part, MH, (int)g.tiles_n, sc->S);
      GATX_LAUNCH_CHECK("score_combine");
    }
    if (fused) *fused = true;
  }
  return 0;
}

extern "C" void gatx_set_gemm_mode(int mode) { g_gemm_mode = mode <= 0 ? 0 : mode == 1 ? 1 : 2; }

extern "C" int gatx_get_gemm_mode(void) { return gemm_mode(); }

extern "C" int gatx_gemm_layout_mode(int a_kc, int b_kc) {
  // f16x3 runs on k-contiguous operand pairs (gemm_x3.hip f16_mainloop, gemm_f16p.hip) and on
  // the weight gradient's row-contiguous pair (gatx_gemm_wgrad with G_aug's column maxima,
  // gemm_f16p.hip f16rc); the mixed layouts run x3
  const int m = gemm_mode();
  if (m != 2) return m;
  if (a_kc && b_kc) return 2;
  return !a_kc && !b_kc ? 2 : 1;
}

extern "C" int gatx_gemm_fallback_read(uint64_t* dst, int reset, gatx_stream_t stream) {
  GATX_REQUIRE(dst != nullptr, "gatx_gemm_fallback_read: dst is NULL");
  int rc = read_f16_fallbacks((unsigned long long*)dst, reset, (hipStream_t)stream);
  if (rc) return rc;
  return read_f16p_fallbacks((unsigned long long*)dst, reset, (hipStream_t)stream);
}

extern "C" size_t gatx_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  int64_t rem = 0;
  const Kind kd = choose_kind(M, N);
  const int ts = choose_tail_split(ceil_div(M, kd.bm) * ceil_div(N, kd.bn), K,
                                   resident_blocks(kd), kd, rem);
  return ts > 1 ? (size_t)ts * rem * kd.bm * kd.bn * sizeof(float) : 0;
}

extern "C" int gatx_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                             int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C0,
                             int64_t ldc0, int64_t n_split, float* C1, int64_t ldc1,
                             int accumulate, void* workspace, size_t workspace_bytes,
                             gatx_stream_t s) {
  return gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C0, ldc0, 0, n_split, C1, ldc1, 0,
                   accumulate, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 1,
                   (hipStream_t)s);
}

extern "C" int gatx_projection_gemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                                    int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                                    float* C0, int64_t ldc0, int64_t n_split, float* C1,
                                    int64_t ldc1, void* workspace, size_t workspace_bytes,
                                    gatx_stream_t s) {
  return gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C0, ldc0, 0, n_split, C1, ldc1, 0,
                   0, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 0,
                   (hipStream_t)s);
}

extern "C" int gatx_projection_gemm3(int64_t M, int64_t N, int64_t K, const float* A,
                                     int64_t sam, int64_t sak, const float* B, int64_t sbk,
                                     int64_t sbn, float* C0, int64_t ldc0, int64_t n_split,
                                     float* C1, int64_t ldc1, int64_t n_split2, float* C2,
                                     int64_t ldc2, void* workspace, size_t workspace_bytes,
                                     gatx_stream_t s) {
  GATX_REQUIRE(n_split2 >= 0, "projection_gemm3: n_split2 must be >= 0");
  return gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C0, ldc0, 0, n_split, C1, ldc1, 0,
                   0, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 0,
                   (hipStream_t)s, n_split2, C2, ldc2);
}

extern "C" size_t gatx_projection_scores_workspace_bytes(int64_t M, int64_t N, int64_t K,
                                                         int NH) {
  const Kind kd = choose_kind(M, N);
  return gatx_gemm_workspace_bytes(M, N, K) + score_part_bytes(ceil_div(N, kd.bn), M, NH);
}

extern "C" int gatx_projection_gemm_scores(int64_t M, int64_t N, int64_t K, const float* A,
                                           int64_t sam, int64_t sak, const float* B, int64_t sbk,
                                           int64_t sbn, float* C0, int64_t ldc0, const float* a,
                                           int NH, int F, float* S, void* workspace,
                                           size_t workspace_bytes, gatx_stream_t s) {
  GATX_REQUIRE(NH >= 1 && F >= 1 && N == (int64_t)NH * round_up(F, 4) && ldc0 == N,
               "projection_gemm_scores: C0 must be the packed [M][NH * round4(F)] Wh");
  const ScoreReq sc{a, NH, F, S};
  bool fused = false;
  if (2 * NH <= 16 && M > 0) {
    GATX_CALL(gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C0, ldc0, 0, N, nullptr, 0,
                        0, 0, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 0,
                        (hipStream_t)s, -1, nullptr, 0, &sc, &fused));
  } else {
    GATX_CALL(gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C0, ldc0, 0, N, nullptr, 0,
                        0, 0, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 0,
                        (hipStream_t)s));
  }
  // shapes without the fused epilogue (f32 arithmetic, small-K / tiny kernels, > 8 heads): the
  // score pass over the stored Wh
  if (!fused) return gatx_node_scores(C0, M, NH, F, a, S, s);
  return 0;
}

extern "C" size_t gatx_weight_planes_bytes(int64_t rows, int64_t K) {
  return weight_planes_bytes(rows, K);
}

extern "C" int gatx_weight_planes(const float* W, int64_t rows, int64_t K, int64_t ld,
                                  void* planes, gatx_stream_t s) {
  GATX_REQUIRE(rows >= 1 && K >= 1 && ld >= K, "weight_planes: bad shape");
  GATX_REQUIRE((uintptr_t)planes % 256 == 0, "weight_planes: buffer must be 256-byte aligned");
  return build_weight_planes(W, rows, K, ld, planes, (hipStream_t)s);
}

extern "C" int gatx_gemm_planes(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                const float* B, int64_t ldb, const void* b_planes, float* C0,
                                int64_t ldc0, int64_t n_split, float* C1, int64_t ldc1,
                                int64_t n_split2, float* C2, int64_t ldc2, int accumulate,
                                const float* a, int NH, int F, float* S, int gradient,
                                const float* a_rowmax, void* workspace, size_t workspace_bytes,
                                gatx_stream_t s) {
  GATX_REQUIRE(b_planes == nullptr || (uintptr_t)b_planes % 256 == 0,
               "gemm_planes: planes must be 256-byte aligned");
  const int tag = gradient ? 1 : 0;
  if (a != nullptr) {   // the forward projection with the node scores fused (see _scores)
    GATX_REQUIRE(!gradient && !accumulate && n_split >= N && NH >= 1 && F >= 1 &&
                     N == (int64_t)NH * round_up(F, 4) && ldc0 == N,
                 "gemm_planes: scores need the packed [M][NH * round4(F)] Wh as the only output");
    const ScoreReq sc{a, NH, F, S};
    bool fused = false;
    if (2 * NH <= 16 && M > 0) {
      GATX_CALL(gemm_impl(M, N, K, 1, A, lda, 1, 0, B, 1, ldb, 0, C0, ldc0, 0, N, nullptr, 0, 0,
                          0, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 0,
                          (hipStream_t)s, -1, nullptr, 0, &sc, &fused, b_planes));
    } else {
      GATX_CALL(gemm_impl(M, N, K, 1, A, lda, 1, 0, B, 1, ldb, 0, C0, ldc0, 0, N, nullptr, 0, 0,
                          0, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 0,
                          (hipStream_t)s, -1, nullptr, 0, nullptr, nullptr, b_planes));
    }
    if (!fused) return gatx_node_scores(C0, M, NH, F, a, S, s);
    return 0;
  }
  return gemm_impl(M, N, K, 1, A, lda, 1, 0, B, 1, ldb, 0, C0, ldc0, 0, n_split, C1, ldc1, 0,
                   accumulate, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, tag,
                   (hipStream_t)s, n_split2, C2, ldc2, nullptr, nullptr, b_planes,
                   gradient ? a_rowmax : nullptr);
}

extern "C" int gatx_gemm_wgrad(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                               const float* B, int64_t ldb, const float* a_rowmax, float* C,
                               int64_t ldc, void* workspace, size_t workspace_bytes,
                               gatx_stream_t s) {
  return gemm_impl(M, N, K, 1, A, 1, lda, 0, B, ldb, 1, 0, C, ldc, 0, N, nullptr, 0, 0, 0,
                   nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 2, (hipStream_t)s,
                   -1, nullptr, 0, nullptr, nullptr, nullptr, a_rowmax);
}

extern "C" int gatx_absmax_rows_cols(const float* X, int64_t rows, int64_t cols, int64_t ld,
                                     float* rowmax, float* colmax, gatx_stream_t s) {
  GATX_REQUIRE(rows >= 0 && cols >= 1 && ld >= cols && rowmax != nullptr,
               "absmax_rows_cols: bad arguments");
  return absmax_rows_cols(X, rows, cols, ld, rowmax, colmax, (hipStream_t)s);
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
  const Kind kd = choose_kind(M, N);
  const int64_t tiles = ceil_div(M, kd.bm) * ceil_div(N, kd.bn);
  int sp = choose_splits(tiles, K, resident_blocks(kd));
  if (kd.id == 2 && wgrad_thin_rows(M))   // the f16x3 weight gradient tiles only full rows
    sp = std::max(sp, choose_splits((M / kd.bm) * ceil_div(N, kd.bn), K, resident_blocks(kd)));
  return sp > 1 ? (size_t)sp * M * N * sizeof(float) : 0;
}

extern "C" size_t gatx_gemm_splitk_batched_workspace_bytes(int64_t batch, int64_t M, int64_t N,
                                                           int64_t K) {
  const Kind kd = choose_kind(M, N);
  const int64_t tiles = ceil_div(M, kd.bm) * ceil_div(N, kd.bn) * batch;
  const int sp = choose_splits(tiles, K, resident_blocks(kd));
  return sp > 1 ? (size_t)sp * batch * M * N * sizeof(float) : 0;
}

extern "C" int gatx_gemm_f32_splitk_batched(int64_t batch, int64_t M, int64_t N, int64_t K,
                                            const float* A, int64_t sam, int64_t sak,
                                            int64_t a_bs, const float* B, int64_t sbk,
                                            int64_t sbn, int64_t b_bs, float* C, int64_t ldc,
                                            int64_t c_bs, int accumulate, void* workspace,
                                            size_t workspace_bytes, gatx_stream_t s) {
  return gemm_impl(M, N, K, (int)batch, A, sam, sak, a_bs, B, sbk, sbn, b_bs, C, ldc, c_bs, N,
                   nullptr, 0, 0, accumulate, nullptr, 0, nullptr, 0, 0, 0, workspace,
                   workspace_bytes, 2, (hipStream_t)s);
}

extern "C" int gatx_gemm_f32_splitk(int64_t M, int64_t N, int64_t K, const float* A, int64_t sam,
                                    int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                                    float* C, int64_t ldc, int accumulate, void* workspace,
                                    size_t workspace_bytes, gatx_stream_t s) {
  return gemm_impl(M, N, K, 1, A, sam, sak, 0, B, sbk, sbn, 0, C, ldc, 0, N, nullptr, 0, 0,
                   accumulate, nullptr, 0, nullptr, 0, 0, 0, workspace, workspace_bytes, 2,
                   (hipStream_t)s);
}
