// Shared pieces of the two GEMM kernels (gemm.hip: f32 MFMA; gemm_x3.hip: split-bf16):
// operand tile staging, launch arguments, tile order and the fused epilogue.
#pragma once

#include "gatx_common.h"

namespace gatx {
namespace gk {


typedef float floatx16 __attribute__((ext_vector_type(16)));

// Two floats -> packed bf16 pair, round to nearest even (v_cvt_pk_bf16_f32). The empty asm keeps
// the compiler from re-deriving each half from its own single-value conversion.
__device__ inline uint32_t cvt_pk_bf16(float a, float b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  bf2 v = {(__bf16)a, (__bf16)b};
  uint32_t u = __builtin_bit_cast(uint32_t, v);
  asm("" : "+v"(u));
  return u;
}

// (x, y) -> the three bf16 planes of both, packed as pairs (x in the low half).
__device__ inline void split_pair(float x, float y, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = cvt_pk_bf16(x, y);
  const float rx = x - __uint_as_float(h << 16), ry = y - __uint_as_float(h & 0xffff0000u);
  m = cvt_pk_bf16(rx, ry);
  l = cvt_pk_bf16(rx - __uint_as_float(m << 16), ry - __uint_as_float(m & 0xffff0000u));
}


constexpr int BM = 128, BN = 128;
constexpr int KSTEP = 32;   // split-K / tail slice granularity

// One operand tile of ROWS rows x BK k. KC: k-contiguous in memory (row stride ld).
template <bool KC, int ROWS, int BK, int NT>
struct Tile {
  static constexpr int LD = KC ? BK + 4 : ROWS + 4;
  static constexpr int SIZE = KC ? ROWS * LD : BK * LD;   // floats per stage
  static constexpr int NV = ROWS * BK / 4 / NT;           // float4 per thread
  // VEC (16-byte aligned rows, ld % 4 == 0): every thread issues NV float4 loads from clamped
  // in-bounds addresses and zeroes the components outside the matrix; otherwise scalar loads.
  template <bool VEC>
  static __device__ inline void load(const float* __restrict__ P, int64_t ld, int64_t r0,
                                     int64_t rmax, int64_t k0, int64_t kmax, float4 (&v)[NV]) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + NT * c;
      int64_t r, k;
      if (KC) { r = r0 + idx / (BK / 4); k = k0 + 4 * (idx % (BK / 4)); }
      else { k = k0 + idx / (ROWS / 4); r = r0 + 4 * (idx % (ROWS / 4)); }
      if (VEC) {
        // KC: lanes j run along k (valid while k + j < kmax); RC: along rows
        const bool rok = r < rmax, kok = k < kmax;
        const int64_t rc = rok ? r : (KC ? rmax - 1 : 0);
        const int64_t kc = kok ? k : (KC ? 0 : kmax - 1);
        v[c] = *(const float4*)(KC ? P + rc * ld + kc : P + kc * ld + rc);   // masked in store
      } else {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = KC ? (r < rmax && k + j < kmax) : (k < kmax && r + j < rmax);
          e[j] = ok ? (KC ? P[r * ld + k + j] : P[k * ld + r + j]) : 0.f;
        }
        v[c] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  }
  // Components outside the matrix are zeroed here, after the MFMAs of the current tile, so the
  // loads' latency stays hidden (a select right after the load would wait for it).
  template <bool VEC>
  static __device__ inline void store(float* img, float4 (&v)[NV], int64_t r0, int64_t rmax,
                                      int64_t k0, int64_t kmax) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + NT * c;
      const int row = KC ? idx / (BK / 4) : 4 * (idx % (ROWS / 4));
      const int kk = KC ? 4 * (idx % (BK / 4)) : idx / (ROWS / 4);
      if (VEC) {
        const int64_t r = r0 + row, k = k0 + kk;
        const bool ok = r < rmax && k < kmax;
        const int64_t lim = KC ? kmax - k : rmax - r;
        v[c].x = ok ? v[c].x : 0.f;
        v[c].y = ok && lim > 1 ? v[c].y : 0.f;
        v[c].z = ok && lim > 2 ? v[c].z : 0.f;
        v[c].w = ok && lim > 3 ? v[c].w : 0.f;
      }
      const int off = KC ? row * LD + kk : kk * LD + row;
      *(float4*)&img[off] = v[c];
    }
  }
  // k = kb .. kb+3 of row `row`
  static __device__ inline float4 frag(const float* img, int row, int kb) {
    if (KC) return *(const float4*)&img[row * LD + kb];
    return make_float4(img[kb * LD + row], img[(kb + 1) * LD + row], img[(kb + 2) * LD + row],
                       img[(kb + 3) * LD + row]);
  }
};

struct GemmArgs {
  int64_t M, N, K;
  const float* A; int64_t lda, a_bs;
  const float* B; int64_t ldb, b_bs;
  float* C0; int64_t ldc0, c0_bs;
  int64_t n_split;
  float* C1; int64_t ldc1, c1_bs;
  // third output range (the folded skip projection): columns >= n_split2 go to C2 raw
  int64_t n_split2;
  float* C2; int64_t ldc2;
  int accumulate, a_vec, b_vec;
  int64_t tiles_m, tiles_n;
  // epilogue on C0 columns: C = elu?(acc (+C) + bias[col] + resid[row][col])
  const float* bias; int64_t bias_bs;
  const float* resid; int64_t resid_ld, resid_bs;
  int elu;
  int64_t k_per_split; int splits; float* partial;
  // tail split (splits == 1): blocks >= dp_blocks each take K-slice z of one of the last
  // tail_rem tiles and write a BM x BN partial; tail_fixup_kernel sums the slices in z order
  int64_t dp_blocks, tail_rem; int tail_s, bm, bn; float* tail_partial;
  // node scores fused into the forward projection (x3 tiles, s_part != nullptr): every column
  // tile tn adds its columns' share of S = Wh . A2^T as s_part[tn][row][s_h2], A2 read from the
  // reference's attention vector s_a (heads s_nh, features s_f, padded s_fp per head of Wh)
  const float* s_a; int s_nh, s_f, s_fp, s_h2; float* s_part;
  // f16p (gemm_f16p.hip): B's pre-split fp16 planes (after their header; nullptr = none) with
  // b_prow bytes per row
  const void* b_planes; int64_t b_prow;
  // exact max |A row| per row (gatx_absmax_rows_cols; nullptr = none): the split kernels scale
  // each A row by it instead of by its first K-tile's max
  const float* a_rowmax;
};

// A2[h2][col] of the attention vector a (models/gat_layer.py:76-82 split per half): the weight of
// Wh column col = head k, feature f (Wh rows padded to fp per head) in score h2 (< nh: source
// half of head h2, else destination half of head h2 - nh); 0 on padding.
__device__ inline float score_weight(const float* a, int nh, int F, int fp, int h2, int64_t col) {
  const int k = (int)(col / fp), f = (int)(col - (int64_t)k * fp);
  if (f >= F || k >= nh) return 0.f;
  const int hh = h2 < nh ? h2 : h2 - nh;
  return a[(int64_t)hh * 2 * nh * F + k * 2 * F + (h2 < nh ? 0 : F) + f];
}

// C = elu?(v (+C) + bias + resid) for one output element (columns >= n_split go to C1 raw,
// columns >= n_split2 to C2 raw)
__device__ inline void store_out(const GemmArgs& g, int64_t b, int64_t row, int64_t col, float v) {
  float* Cb;
  int64_t ldc, c;
  const bool first = col < g.n_split;
  if (first) { Cb = g.C0 + b * g.c0_bs; ldc = g.ldc0; c = col; }
  else if (col < g.n_split2) { Cb = g.C1 + b * g.c1_bs; ldc = g.ldc1; c = col - g.n_split; }
  else { Cb = g.C2; ldc = g.ldc2; c = col - g.n_split2; }
  float* p = Cb + row * ldc + c;
  if (g.accumulate) v += *p;
  if (first) {
    if (g.bias) v += g.bias[b * g.bias_bs + c];
    if (g.resid) v += g.resid[b * g.resid_bs + row * g.resid_ld + c];
    if (g.elu) v = elu_act(v);
  }
  *p = v;
}

// One finished 32 x 32 MFMA block through the epilogue of store_out: this lane's column `col`
// and rows row0 + (r & 3) + 8 (r >> 2) (row0 includes the lane half's 4 (lane >> 5)). Column
// terms are resolved once per block instead of per element (the per-element 64-bit index
// arithmetic of store_out cost the projection GEMMs ~3% of their time), and the column's bias
// comes in from the caller, loaded before any store: on gfx9 loads and stores share the vmcnt
// counter, so a load issued after a block's stores waits for all of them to reach memory.
__device__ inline float block_bias(const GemmArgs& g, int64_t b, int64_t col) {
  return (g.bias && col < g.N && col < g.n_split) ? g.bias[b * g.bias_bs + col] : 0.f;
}
// PRE = false keeps the per-element form (no extra registers: the f32 kernel's 128-VGPR cap).
template <bool PRE = true>
__device__ inline void store_block(const GemmArgs& g, int64_t b, int64_t row0, int64_t col,
                                   const floatx16& acc, float bias) {
  if (col >= g.N) return;
  const bool first = col < g.n_split;
  float* base;
  int64_t ldc;
  if (first) { base = g.C0 + b * g.c0_bs + col; ldc = g.ldc0; }
  else if (col < g.n_split2) { base = g.C1 + b * g.c1_bs + (col - g.n_split); ldc = g.ldc1; }
  else { base = g.C2 + (col - g.n_split2); ldc = g.ldc2; }
  const bool has_bias = first && g.bias != nullptr;
  const float* rp = (first && g.resid) ? g.resid + b * g.resid_bs + col : nullptr;
  const bool elu = first && g.elu;
  const bool full = row0 + 27 < g.M;
  if (!PRE || (!g.accumulate && !rp)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t row = row0 + (r & 3) + 8 * (r >> 2);
      if (!full && row >= g.M) continue;
      float* p = base + row * ldc;
      float v = acc[r];
      if (!PRE && g.accumulate) v += *p;
      if (has_bias) v += bias;
      if (!PRE && rp) v += rp[row * g.resid_ld];
      if (elu) v = elu_act(v);
      *p = v;
    }
    return;
  }
  // accumulate / residual: each half-block's 8 loads are issued before its 8 stores, so a load
  // waits on at most one half-block of stores (per element it waited on every earlier store;
  // that doubled the PPI L1 g_x GEMM, whose epilogue accumulates the identity-skip gradient)
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    float cv[8], rv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = hb * 8 + i;
      const int64_t row = row0 + (r & 3) + 8 * (r >> 2);
      const bool ok = full || row < g.M;
      cv[i] = (g.accumulate && ok) ? base[row * ldc] : 0.f;
      rv[i] = (rp && ok) ? rp[row * g.resid_ld] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = hb * 8 + i;
      const int64_t row = row0 + (r & 3) + 8 * (r >> 2);
      if (!full && row >= g.M) continue;
      float v = acc[r];
      if (g.accumulate) v += cv[i];   // the order of store_out: ((acc + C) + bias) + resid
      if (has_bias) v += bias;
      if (rp) v += rv[i];
      if (elu) v = elu_act(v);
      base[row * ldc] = v;
    }
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

// Epilogue shared by both kernels. C/D map of a 32x32 f32 MFMA block: col = lane&31,
// row = (r&3) + 8*(r>>2) + 4*(lane>>5).
template <int MB, int NB, int TBM = BM, int TBN = BN, bool PRE = true>
__device__ inline void write_tile(const GemmArgs& g, floatx16 (&acc)[MB][NB], int tail_z,
                                  int64_t tail_ti, int64_t m0, int64_t n0, int wm, int wn,
                                  int lane) {
  const int64_t M = g.M, N = g.N;
  if (tail_z >= 0) {   // tail slice: tile-local partial, summed by tail_fixup_kernel
    float* P = g.tail_partial + ((int64_t)tail_z * g.tail_rem + tail_ti) * (TBM * TBN);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm * (MB * 32) + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          P[rl * TBN + wn * (NB * 32) + ni * 32 + (lane & 31)] = acc[mi][ni][r];
        }
    return;
  }
  float bias[NB];   // loaded before the first store (see store_block)
#pragma unroll
  for (int ni = 0; ni < NB; ++ni)
    bias[ni] = g.splits > 1 ? 0.f : block_bias(g, blockIdx.y, n0 + wn * (NB * 32) + ni * 32 + (lane & 31));
#pragma unroll
  for (int mi = 0; mi < MB; ++mi)
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
      const int64_t col = n0 + wn * (NB * 32) + ni * 32 + (lane & 31);
      if (col >= N) continue;
      if (g.splits > 1) {   // partial slab z: plain [M][N] store, reduced by splitk_reduce_kernel
        float* P = g.partial + ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * M * N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = m0 + wm * (MB * 32) + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < M) P[row * N + col] = acc[mi][ni][r];
        }
        continue;
      }
      store_block<PRE>(g, blockIdx.y, m0 + wm * (MB * 32) + mi * 32 + 4 * (lane >> 5), col,
                  acc[mi][ni], bias[ni]);
    }
}

}  // namespace gk

// gemm_x3.hip: launch the split-bf16 kernel for GemmArgs prepared by gemm_impl (gemm.hip).
int launch_gemm_x3(const gk::GemmArgs& g, bool a_kc, bool b_kc, int batch, int tag, hipStream_t stream);
// gemm_smallk.hip: K <= 64, N <= 256 products with the fused epilogue (x3 arithmetic)
bool gemm_smallk_fits(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc, int accumulate,
                      bool resid);
int launch_gemm_smallk(const gk::GemmArgs& g, int batch, hipStream_t stream);
// gemm_smallk.hip: 64 < K <= 256, N <= 64 products, B n-contiguous, no epilogue (x3 arithmetic)
bool gemm_smalln_fits(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc, int accumulate,
                      bool epilogue);
int launch_gemm_smalln(const gk::GemmArgs& g, int batch, hipStream_t stream);
// gemm_smallk.hip: C = A^T B, both row-contiguous, 8 < M <= 256, N <= 64, long K, split-K into
// the workspace + splitk_reduce (x3 arithmetic); returns 0 without launching when the
// workspace holds fewer than two slices
bool gemm_tn_fits(int64_t M, int64_t N, int64_t K, bool a_kc, bool b_kc);
int launch_gemm_tn(gk::GemmArgs g, int batch, void* workspace, size_t workspace_bytes,
                   hipStream_t stream);
// gemm.hip: sum the split-K slabs [z][b][M][N] into C through the epilogue
void launch_splitk_reduce(const gk::GemmArgs& g, int batch, hipStream_t stream);
// gemm_f16p.hip: the f16x3 kernel with B given as pre-split fp16 planes (tags 0 and 1)
int launch_gemm_f16p(const gk::GemmArgs& g, int tag, hipStream_t stream);
int launch_gemm_f16rc(const gk::GemmArgs& g, hipStream_t stream);
// rows past the last multiple of 256 of a weight gradient that the f16x3 kernel leaves to its
// VALU thin-row kernel (0: none)
int wgrad_thin_rows(int64_t M);
size_t weight_planes_bytes(int64_t rows, int64_t K);
int absmax_rows_cols(const float* X, int64_t rows, int64_t cols, int64_t ld, float* rowmax,
                     float* colmax, hipStream_t stream);
int build_weight_planes(const float* W, int64_t rows, int64_t K, int64_t ld, void* buf,
                        hipStream_t stream);
// gemm_x3.hip: the device address of the f16x3 -> x3 fallback tile counter
// gemm_x3.hip: copy (and optionally zero) the f16x3 -> x3 fallback tile counter
int read_f16_fallbacks(unsigned long long* dst, int reset, hipStream_t stream);
// adds gemm_f16p.hip's own count to dst[0] (after read_f16_fallbacks wrote it)
int read_f16p_fallbacks(unsigned long long* dst, int reset, hipStream_t stream);
// the x3 kernel instance whose occupancy sizes tail / split-K decisions
const void* gemm_x3_occupancy_fn(int cfg);   // cfg 0: 128 x 128 tiles, 1: 256 x 256

}  // namespace gatx
