// Device code shared by the split-arithmetic GEMM kernels (gemm_x3.hip: the x3 / f16x3
// kernel; gemm_f16p.hip: f16x3 with a pre-split weight operand): operand staging into
// fp16 / bf16 plane images, the x3 and f16x3 mainloops and the transposed-product epilogue.
#pragma once
#include "gemm_common.h"

namespace gatx {
namespace {
using namespace gk;

// ---------------------------------------------------------------------------------------------
// fp32 GEMM as a three-way bf16 split ("x3"): every fp32 operand element is written exactly as
// x = h + m + l with h = bf16_rn(x), m = bf16_rn(x - h), l = x - h - m (exactly a bf16: 24 =
// 8 + 8 + 8 significand bits), and the product as the six bf16 MFMA products whose magnitude
// reaches fp32 resolution: a_h b_h + a_h b_m + a_m b_h + a_h b_l + a_l b_h + a_m b_m. The dropped
// terms a_m b_l + a_l b_m + a_l b_l are below 2^-23 |a||b| — the size of one fp32 rounding — and
// bf16 products are exact in the f32 accumulator, so the result has the fp32 GEMM's accuracy
// (checked against fp64 beside the f32-MFMA kernel in tests/test_gpu_layer.py) at 6 x 32 cycles
// per 32x32x16 step instead of 8 x 64 for v_mfma_f32_32x32x2_f32: 2.7x fewer MFMA cycles.
//
// Two tile configurations (XCD-contiguous tile order, tail split and fused epilogue shared with
// gemm_f32_kernel): CFG 1 = 256 x 256 per 8-wave workgroup, 128 x 64 per wave (4 x 2 blocks of
// v_mfma_f32_32x32x16_bf16), 96 KB of LDS, one workgroup per CU — the large products; CFG 0 =
// 128 x 128 per 4-wave workgroup, 64 x 64 per wave, 48 KB, three per CU — small outputs.
// Measured on the PPI projection shape (44900 x 1024 x 1024), 128 x 128 tiles reach 148 TF:
// re-staging 6 bytes per element per 24 MFMAs keeps the LDS ~65% busy; 256 x 256 tiles halve
// the staging per MFMA.
// The fp32 tiles are split once per workgroup while they are staged into LDS (each element then
// feeds several waves), into three bf16 planes per operand:
//  * k-contiguous operand: [slot = k/8][row ^ (slot*64/BK)][8 k] — 16-byte fragment reads
//    (ds_read_b128) and 8-byte staging stores, both conflict-free;
//  * row-contiguous operand: [k][128 rows] with 256-byte rows whose 16-byte chunks are XOR'd by k
//    — the fragment is read transposed by two ds_read_b64_tr_b16 (4 k each), conflict-free.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// Two floats -> packed fp16 pair, round to nearest even (v_cvt_pk_f16_f32).
__device__ inline uint32_t cvt_pk_f16(float a, float b) {
  f16x2 v = {(_Float16)a, (_Float16)b};
  uint32_t u = __builtin_bit_cast(uint32_t, v);
  asm("" : "+v"(u));
  return u;
}

// (x, y) -> h = fp16_rn pair and l = fp16_rn(2^11 (x - h)) pair (x in the low halves). x - h is
// exact (Sterbenz), the scaling by 2^11 keeps l a normal fp16 down to |x - h| = 2^-25.
__device__ inline void split_pair_f16(float x, float y, uint32_t& h, uint32_t& l) {
  h = cvt_pk_f16(x, y);
  const f16x2 hv = __builtin_bit_cast(f16x2, h);
  l = cvt_pk_f16((x - (float)hv[0]) * 2048.f, (y - (float)hv[1]) * 2048.f);
}

// One bf16 plane image of a ROWS-row x BK-k operand tile (byte offsets).
template <bool KC, int ROWS, int BK>
struct PlaneImg {
  static constexpr int BYTES = ROWS * BK * 2;
  // offset of the 4 consecutive k (KC, k % 4 == 0) or 4 consecutive rows (RC, r % 4 == 0)
  // starting at (r, k)
  static __device__ inline int off(int r, int k) {
    if (KC) {
      // rows of the second 8-k slot XOR'd by 12: conflict-free ds_read_b128 fragment reads for
      // both MFMA shapes (32x32x16: lane -> (row l&31, slot l>>5); 16x16x32 plane pairs: lane ->
      // (row l&15, slot (l>>4)&1)) and conflict-free ds_write_b64 staging stores
      static_assert(BK == 16, "x3 images hold 16-k tiles");
      const int s = k >> 3;
      return s * (ROWS * 16) + ((r ^ (s * 12)) << 4) + ((k & 4) << 1);
    }
    const int c = (r >> 3) ^ (((k & 3) << 2) | ((k >> 2) & 3));
    return k * (ROWS * 2) + (c << 4) + ((r & 7) << 1);
  }
};

// Staging of one operand tile: NV float4 per thread, thread idx -> (row, k) as Tile<> maps it.
template <bool KC, int ROWS, int BK, int NT>
struct X3Tile {
  using T = Tile<KC, ROWS, BK, NT>;
  static constexpr int NV = T::NV;
  using Img = PlaneImg<KC, ROWS, BK>;
  static __device__ inline int row_of(int idx) { return KC ? idx / (BK / 4) : 4 * (idx % (ROWS / 4)); }
  static __device__ inline int k_of(int idx) { return KC ? 4 * (idx % (BK / 4)) : idx / (ROWS / 4); }
  // Fast path: per-thread pointers at K-tile 0 (rows past rmax clamped to a valid row: their
  // products only reach output rows/columns that are never stored) and the per-tile step.
  static __device__ inline void setup(const float* P, int64_t ld, int64_t r0, int64_t rmax,
                                      int64_t k0, const float* (&p)[NV], int64_t& step) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + NT * c;
      int64_t r = r0 + row_of(idx);
      if (r >= rmax) r = KC ? rmax - 1 : 0;
      const int64_t k = k0 + k_of(idx);
      p[c] = KC ? P + r * ld + k : P + k * ld + r;
    }
    step = KC ? BK : BK * ld;
  }
  // Split the staged float4s into the three planes at img. KTAIL: zero k >= kmax (the last,
  // partial K-tile); MASK: also rows >= rmax (generic path, Tile::load's clamped addresses).
  template <bool MASK, bool KTAIL>
  static __device__ inline void mask(float4 (&v)[NV], int64_t r0, int64_t rmax, int64_t k0,
                                     int64_t kmax) {
    if (!(MASK || KTAIL)) return;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + NT * c;
      const int64_t r = r0 + row_of(idx), k = k0 + k_of(idx);
      const bool ok = (!MASK || r < rmax) && k < kmax;
      const int64_t lim = (KC || !MASK) ? (KC ? kmax - k : 4) : rmax - r;
      v[c].x = ok ? v[c].x : 0.f;
      v[c].y = ok && lim > 1 ? v[c].y : 0.f;
      v[c].z = ok && lim > 2 ? v[c].z : 0.f;
      v[c].w = ok && lim > 3 ? v[c].w : 0.f;
    }
  }
  // Power-of-two scale per staged row from its max |x| in this (the first) K-tile: the row is
  // brought to max |x| in [2^(TGT-1), 2^TGT) (1 for an all-zero or non-finite max). KC only: a
  // row's 4 staging lanes are adjacent.
  template <int TGT>
  static __device__ inline void row_scales(const float4 (&v)[NV], float (&sc)[NV]) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      float m = fmaxf(fmaxf(fabsf(v[c].x), fabsf(v[c].y)), fmaxf(fabsf(v[c].z), fabsf(v[c].w)));
      m = fmaxf(m, __shfl_xor(m, 1));
      m = fmaxf(m, __shfl_xor(m, 2));
      int e = 0;
      (void)frexpf(m, &e);   // m = f 2^e, f in [0.5, 1)
      sc[c] = (m > 0.f && m <= 3.0e38f) ? ldexpf(1.f, TGT - e) : 1.f;
    }
  }
  // f16x3 staging (see f16_mainloop): plane 0 = h = fp16_rn(x), plane 1 = fp16_rn(2^11 (x - h));
  // amax tracks max |x| over the staged elements for the caller's range check.
  template <bool MASK, bool KTAIL, bool SCALED>
  static __device__ inline void store_f16(char* img, float4 (&v)[NV], int64_t r0, int64_t rmax,
                                          int64_t k0, int64_t kmax, float (&amax)[NV],
                                          const float (&sc)[NV]) {
    mask<MASK, KTAIL>(v, r0, rmax, k0, kmax);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + NT * c;
      if (SCALED) v[c] = v[c] * sc[c];   // the row's power-of-two scale (exact)
      amax[c] = fmaxf(amax[c], fmaxf(fmaxf(fabsf(v[c].x), fabsf(v[c].y)),
                                     fmaxf(fabsf(v[c].z), fabsf(v[c].w))));
      uint32_t h0, l0, h1, l1;
      split_pair_f16(v[c].x, v[c].y, h0, l0);
      split_pair_f16(v[c].z, v[c].w, h1, l1);
      const int o = Img::off(row_of(idx), k_of(idx));
      *(uint2*)(img + o) = make_uint2(h0, h1);
      *(uint2*)(img + Img::BYTES + o) = make_uint2(l0, l1);
    }
  }
  template <bool MASK, bool KTAIL>
  static __device__ inline void store(char* img, float4 (&v)[NV], int64_t r0, int64_t rmax,
                                      int64_t k0, int64_t kmax) {
    mask<MASK, KTAIL>(v, r0, rmax, k0, kmax);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int idx = threadIdx.x + NT * c;
      const int row = row_of(idx), kk = k_of(idx);
      uint32_t h0, m0, l0, h1, m1, l1;
      split_pair(v[c].x, v[c].y, h0, m0, l0);
      split_pair(v[c].z, v[c].w, h1, m1, l1);
      const int o = Img::off(row, kk);
      *(uint2*)(img + o) = make_uint2(h0, h1);
      *(uint2*)(img + Img::BYTES + o) = make_uint2(m0, m1);
      *(uint2*)(img + 2 * Img::BYTES + o) = make_uint2(l0, l1);
    }
  }
  // MFMA 32x32x16 operand fragment of rows rb..rb+31, k = k16..k16+15 from one plane.
  static __device__ inline bf16x8 frag(const char* plane, int rb, int k16, int lane) {
    if (KC) {
      return *(const bf16x8*)(plane + Img::off(rb + (lane & 31), k16 + 8 * (lane >> 5)));
    } else {
      const int g = lane >> 4, i = lane & 15;
      const int r = rb + 16 * (g & 1) + 4 * (i & 3), k = k16 + 8 * (g >> 1) + (i >> 2);
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4*)(__attribute__((address_space(3))) char*)(plane + Img::off(r, k)));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s16x4*)(__attribute__((address_space(3))) char*)(plane + Img::off(r, k + 4)));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  }
};

// Tile configurations: CFG 0 = 128 x 128, 2 x 2 waves; CFG 1 = 256 x 256, 2 x 4 waves.
template <int CFG>
struct X3Cfg {
  static constexpr int TBM = CFG ? 256 : 128, TBN = CFG ? 256 : 128;
  static constexpr int WGM = 2, WGN = CFG ? 4 : 2;
  static constexpr int NT = 64 * WGM * WGN;
  static constexpr int MB = TBM / WGM / 32, NB = TBN / WGN / 32;
  static constexpr int MINB = CFG ? 1 : 3;
  static constexpr int BK = 16;
};

// Main loop over nk K-tiles starting at kb. MASK (unaligned operands): every tile through
// Tile::load's clamped scalar/vector loads and full masking. Otherwise each thread streams its
// float4s from fixed per-thread pointers; only a partial last K-tile is masked (k >= K zeroed).
template <bool A_KC, bool B_KC, bool MASK, int CFG>
__device__ inline void x3_mainloop(const GemmArgs& g, const float* __restrict__ A,
                                   const float* __restrict__ B, int64_t m0, int64_t n0,
                                   int64_t kb, int64_t K, int64_t nk, char* smem, int wm, int wn,
                                   int lane, floatx16 (&acc)[X3Cfg<CFG>::MB][X3Cfg<CFG>::NB]) {
  using C = X3Cfg<CFG>;
  constexpr int NT = C::NT, BK = C::BK, MB = C::MB, NB = C::NB;
  using TA = X3Tile<A_KC, C::TBM, BK, NT>;
  using TB = X3Tile<B_KC, C::TBN, BK, NT>;
  constexpr int PA = TA::Img::BYTES, PBy = TB::Img::BYTES;   // bytes per plane
  constexpr int STAGE = 3 * (PA + PBy);                      // A planes h, m, l then B's
  const int64_t M = g.M, N = g.N;
  const bool ktail = (K - kb) % BK != 0;
  float4 va[TA::NV], vb[TB::NV];
  const float* pa[TA::NV];
  const float* pb[TB::NV];
  int64_t sa = 0, sb = 0;
  if (!MASK) {
    TA::setup(A, g.lda, m0, M, kb, pa, sa);
    TB::setup(B, g.ldb, n0, N, kb, pb, sb);
  }
  auto load = [&](int64_t k0) {
    if (MASK) {
      TA::T::template load<false>(A, g.lda, m0, M, k0, K, va);
      TB::T::template load<false>(B, g.ldb, n0, N, k0, K, vb);
    } else if (k0 + BK > K) {
      // partial last K-tile: a k >= K reads k = kb instead (always inside the matrix) and is
      // zeroed in store; k < K reads in place (KC: k % 4 == 0 and ld % 4 == 0 keep the float4
      // inside the row's ld)
#pragma unroll
      for (int c = 0; c < TA::NV; ++c) {
        const int64_t k = k0 + TA::k_of(threadIdx.x + NT * c);
        va[c] = *(const float4*)(k < K ? pa[c] : pa[c] - (k - kb) * (A_KC ? 1 : g.lda));
      }
#pragma unroll
      for (int c = 0; c < TB::NV; ++c) {
        const int64_t k = k0 + TB::k_of(threadIdx.x + NT * c);
        vb[c] = *(const float4*)(k < K ? pb[c] : pb[c] - (k - kb) * (B_KC ? 1 : g.ldb));
      }
    } else {
#pragma unroll
      for (int c = 0; c < TA::NV; ++c) { va[c] = *(const float4*)pa[c]; pa[c] += sa; }
#pragma unroll
      for (int c = 0; c < TB::NV; ++c) { vb[c] = *(const float4*)pb[c]; pb[c] += sb; }
    }
  };
  auto store = [&](char* st, int64_t k0) {
    if (MASK) {
      TA::template store<true, true>(st, va, m0, M, k0, K);
      TB::template store<true, true>(st + 3 * PA, vb, n0, N, k0, K);
    } else if (k0 + BK > K) {
      TA::template store<false, true>(st, va, m0, M, k0, K);
      TB::template store<false, true>(st + 3 * PA, vb, n0, N, k0, K);
    } else {
      TA::template store<false, false>(st, va, m0, M, k0, K);
      TB::template store<false, false>(st + 3 * PA, vb, n0, N, k0, K);
    }
  };
  (void)ktail;
  load(kb);
  store(smem, kb);
  __syncthreads();
  bf16x8 fa[MB][3], fb[NB][3];
  constexpr int PLA[6] = {2, 0, 1, 1, 0, 0};
  constexpr int PLB[6] = {0, 2, 1, 0, 1, 0};
  int64_t kt = 0;
  auto frags = [&](const char* cur) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int x = 0; x < MB; ++x) fa[x][p] = TA::frag(cur + p * PA, wm * (MB * 32) + x * 32, 0, lane);
#pragma unroll
      for (int x = 0; x < NB; ++x)
        fb[x][p] = TB::frag(cur + 3 * PA + p * PBy, wn * (NB * 32) + x * 32, 0, lane);
    }
  };
  auto mfmas = [&]() {
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
          // C^T = B^T A^T (operand roles swapped): lane = output row, registers = columns,
          // see write_tile_t
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[ni][PLB[t]], fa[mi][PLA[t]],
                                                                acc[mi][ni], 0, 0, 0);
  };
  auto load_full = [&]() {
#pragma unroll
    for (int c = 0; c < TA::NV; ++c) { va[c] = *(const float4*)pa[c]; pa[c] += sa; }
#pragma unroll
    for (int c = 0; c < TB::NV; ++c) { vb[c] = *(const float4*)pb[c]; pb[c] += sb; }
  };
  auto store_full = [&](char* st) {
    TA::template store<false, false>(st, va, m0, M, 0, K);
    TB::template store<false, false>(st + 3 * PA, vb, n0, N, 0, K);
  };
  if constexpr (!MASK && CFG == 1) {
    // Steady state (full K-tiles, no branches): operands one K-tile further ahead. Tile kt + 1
    // (loaded during iteration kt - 1) is split into the other stage right after this tile's
    // fragment reads, then tile kt + 2's loads go out, then the MFMAs: the LDS stores drain under
    // the MFMAs instead of just ahead of the barrier, and the global loads have a whole
    // iteration to land. -5 to -6% against load-at-top / store-at-bottom on the PPI projection
    // and 8192 x 4096 x 4096 shapes (round-2 interleaved A/B); forcing an interleave with
    // sched_group_barrier was slower than the compiler's schedule. A partial last tile and the
    // unaligned (MASK) path take the generic loop below, and so does CFG 0 (three workgroups per
    // CU: the extra live operands spill under its 168-VGPR cap).
    const int64_t nfull = (K - kb) / BK;
    if (nfull >= 2) {
      load_full();   // tile 1
      for (; kt + 2 < nfull; ++kt) {
        char* cur = smem + (kt & 1) * STAGE;
        char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
        frags(cur);
        store_full(nxt);
        load_full();
        mfmas();
        __syncthreads();
      }
      char* cur = smem + (kt & 1) * STAGE;
      char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
      frags(cur);
      store_full(nxt);
      mfmas();
      __syncthreads();
      ++kt;
    }
  }
  for (; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    const bool more = kt + 1 < nk;
    if (more) load(kb + (kt + 1) * BK);
    frags(cur);
    mfmas();   // small terms first: (l,h) (h,l) (m,m) (m,h) (h,m) (h,h)
    if (more) store(nxt, kb + (kt + 1) * BK);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// fp32 GEMM as a two-way fp16 split ("f16x3"): x = h + l 2^-11 with h = fp16_rn(x) and
// l = fp16_rn(2^11 (x - h)) (11 + 11 significand bits: |x - h| <= 2^-11 |x|, and rounding l to
// fp16 leaves |x - h - l 2^-11| <= 2^-22 |x|; the 2^11 keeps l a normal fp16 wherever x is), and
// the product as three fp16 MFMA products, all carrying the same factor 2^11:
//     2^11 a b ~= (64 a_h)(32 b_h) + a_h b_l + a_l b_h        (dropped: a_l b_l 2^-22 <= 2^-22 |ab|)
// So each product carries a relative error of a few 2^-22 — not one fp32 rounding (2^-24). What
// makes the result as accurate as an fp32 GEMM is the accumulation: the fp16 products are exact
// in the f32 accumulator, whose K-long summation error dominates the per-product terms;
// tests/test_gpu_layer.py::test_gemm_x3_split_accuracy holds the kernel to <= 1.25x the exact
// fp32-MFMA kernel's error against fp64 (tests/test_f16x3_numerics.py: the 2^-22 split bound).
// The 64 / 32 factors of the first product are applied to the hi fragments in registers
// (v_pk_mul_f16, exact) and the accumulator is scaled by 2^-11 (exact) at the end: 3 MFMA
// products per step instead of the bf16 split's 6, and two LDS planes per operand instead of 3.
// Row scaling: every A row (an output row: activations, or a gradient's ~1e-7 rows) is multiplied
// by a power of two chosen from its max |x| in the workgroup's first K-tile (to [2^7, 2^8)),
// exactly undone in the epilogue, so it lands in the fp16 range with 4-8x headroom for the rest
// of its K range. B (the weights in every caller) is not scaled (a per-column scale cost 14-19
// spilled VGPRs in the epilogue).
// Range: 64 a_h and 32 b_h must be finite fp16, i.e. |a| <= 1023 and |b| <= 2047; and below
// 2^-13 an element's pieces reach fp16 subnormals (absolute error up to 2^-36), harmless next to
// the row's larger elements but not for a row that is tiny throughout. Every thread tracks
// max |x| of its staged row slices; per operand row (an A row = an output row, a B row = an
// output column; k-contiguous operands: the row's 4 staging lanes are adjacent) the amax must
// be 0 or within [2^-13, limit]. A workgroup with any row outside (or holding inf) discards its
// accumulators and recomputes its tile with the bf16 split (x3_mainloop, fp32 exponent range),
// so accuracy never depends on the operands' magnitudes. Used for k-contiguous A and B (the
// forward projection's layout); the other layouts run x3.
constexpr float kF16LimA = 1023.f, kF16LimB = 2047.f, kF16Tiny = 0x1p-13f;

__device__ inline bool f16_row_bad(float m, float lim) {
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  return !(m <= lim) || (m > 0.f && m < kF16Tiny);
}

template <bool A_KC, bool B_KC, bool MASK, int CFG, bool SCALE>
__device__ inline bool f16_mainloop(const GemmArgs& g, const float* __restrict__ A,
                                    const float* __restrict__ B, int64_t m0, int64_t n0,
                                    int64_t kb, int64_t K, int64_t nk, char* smem, int wm, int wn,
                                    int lane, floatx16 (&acc)[X3Cfg<CFG>::MB][X3Cfg<CFG>::NB]) {
  using C = X3Cfg<CFG>;
  constexpr int NT = C::NT, BK = C::BK, MB = C::MB, NB = C::NB;
  using TA = X3Tile<A_KC, C::TBM, BK, NT>;
  using TB = X3Tile<B_KC, C::TBN, BK, NT>;
  constexpr int PA = TA::Img::BYTES, PBy = TB::Img::BYTES;   // bytes per plane
  constexpr int STAGE = 2 * (PA + PBy);                      // A planes h, l then B's
  const int64_t M = g.M, N = g.N;
  static_assert(A_KC && B_KC, "f16x3 staging needs k-contiguous operands (row amax lanes)");
  float amax_a[TA::NV], amax_b[TB::NV];
#pragma unroll
  for (int c = 0; c < TA::NV; ++c) amax_a[c] = 0.f;
#pragma unroll
  for (int c = 0; c < TB::NV; ++c) amax_b[c] = 0.f;
  float4 va[TA::NV], vb[TB::NV];
  float sca[TA::NV], scb[TB::NV];   // per staged row: power-of-two scale (see above)
  const float* pa[TA::NV];
  const float* pb[TB::NV];
  int64_t sa = 0, sb = 0;
  if (!MASK) {
    TA::setup(A, g.lda, m0, M, kb, pa, sa);
    TB::setup(B, g.ldb, n0, N, kb, pb, sb);
  }
  auto load = [&](int64_t k0) {
    if (MASK) {
      TA::T::template load<false>(A, g.lda, m0, M, k0, K, va);
      TB::T::template load<false>(B, g.ldb, n0, N, k0, K, vb);
    } else if (k0 + BK > K) {
#pragma unroll
      for (int c = 0; c < TA::NV; ++c) {
        const int64_t k = k0 + TA::k_of(threadIdx.x + NT * c);
        va[c] = *(const float4*)(k < K ? pa[c] : pa[c] - (k - kb) * (A_KC ? 1 : g.lda));
      }
#pragma unroll
      for (int c = 0; c < TB::NV; ++c) {
        const int64_t k = k0 + TB::k_of(threadIdx.x + NT * c);
        vb[c] = *(const float4*)(k < K ? pb[c] : pb[c] - (k - kb) * (B_KC ? 1 : g.ldb));
      }
    } else {
#pragma unroll
      for (int c = 0; c < TA::NV; ++c) { va[c] = *(const float4*)pa[c]; pa[c] += sa; }
#pragma unroll
      for (int c = 0; c < TB::NV; ++c) { vb[c] = *(const float4*)pb[c]; pb[c] += sb; }
    }
  };
  auto store = [&](char* st, int64_t k0) {
    if (MASK) {
      TA::template store_f16<true, true, SCALE>(st, va, m0, M, k0, K, amax_a, sca);
      TB::template store_f16<true, true, false>(st + 2 * PA, vb, n0, N, k0, K, amax_b, scb);
    } else if (k0 + BK > K) {
      TA::template store_f16<false, true, SCALE>(st, va, m0, M, k0, K, amax_a, sca);
      TB::template store_f16<false, true, false>(st + 2 * PA, vb, n0, N, k0, K, amax_b, scb);
    } else {
      TA::template store_f16<false, false, SCALE>(st, va, m0, M, k0, K, amax_a, sca);
      TB::template store_f16<false, false, false>(st + 2 * PA, vb, n0, N, k0, K, amax_b, scb);
    }
  };
  f16x8 fa[MB][2], fb[NB][2];
  auto frags = [&](const char* cur) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int x = 0; x < MB; ++x)
        fa[x][p] = __builtin_bit_cast(f16x8, TA::frag(cur + p * PA, wm * (MB * 32) + x * 32, 0, lane));
#pragma unroll
      for (int x = 0; x < NB; ++x)
        fb[x][p] = __builtin_bit_cast(f16x8, TB::frag(cur + 2 * PA + p * PBy, wn * (NB * 32) + x * 32, 0, lane));
    }
  };
  auto mfmas = [&]() {
    // small terms first: a_h b_l, a_l b_h, then (64 a_h)(32 b_h); C^T = B^T A^T as in x3
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
    f16x8 sa8[MB], sb8[NB];
#pragma unroll
    for (int mi = 0; mi < MB; ++mi) sa8[mi] = fa[mi][0] * (_Float16)64.0f;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) sb8[ni] = fb[ni][0] * (_Float16)32.0f;
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(sb8[ni], sa8[mi], acc[mi][ni], 0, 0, 0);
  };
  auto rows_bad = [&]() {
    bool bad = false;
#pragma unroll
    for (int c = 0; c < TA::NV; ++c) bad |= f16_row_bad(amax_a[c], kF16LimA);
#pragma unroll
    for (int c = 0; c < TB::NV; ++c) bad |= f16_row_bad(amax_b[c], kF16LimB);
    return bad;
  };
  int64_t kt = 0;
  load(kb);
#pragma unroll
  for (int c = 0; c < TB::NV; ++c) scb[c] = 1.f;   // B (the weights) is not scaled
#pragma unroll
  for (int c = 0; c < TA::NV; ++c) sca[c] = 1.f;
  if constexpr (SCALE) {
    TA::template row_scales<8>(va, sca);
    // the A rows' inverse scales, for the epilogue: [TBM] floats after the two stages
    float* inv = (float*)(smem + 2 * STAGE);
#pragma unroll
    for (int c = 0; c < TA::NV; ++c)
      if ((threadIdx.x & 3) == 0) inv[TA::row_of(threadIdx.x + NT * c)] = 1.f / sca[c];
  }
  store(smem, kb);
  // early exit: rows already out of range in the first K-tile (e.g. a gradient operand, whose
  // rows are tiny throughout) go to the x3 fallback before any MFMA work is spent on them
  if (__syncthreads_or(rows_bad())) return true;
  if constexpr (!MASK && CFG == 1) {
    // steady state as in x3_mainloop: tile kt + 1 staged into the other buffer right after this
    // tile's fragment reads, tile kt + 2's loads issued before the MFMAs
    const int64_t nfull = (K - kb) / BK;
    if (nfull >= 2) {
      load(kb + BK);
      for (; kt + 2 < nfull; ++kt) {
        char* cur = smem + (kt & 1) * STAGE;
        char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
        frags(cur);
        TA::template store_f16<false, false, SCALE>(nxt, va, m0, M, 0, K, amax_a, sca);
        TB::template store_f16<false, false, false>(nxt + 2 * PA, vb, n0, N, 0, K, amax_b, scb);
#pragma unroll
        for (int c = 0; c < TA::NV; ++c) { va[c] = *(const float4*)pa[c]; pa[c] += sa; }
#pragma unroll
        for (int c = 0; c < TB::NV; ++c) { vb[c] = *(const float4*)pb[c]; pb[c] += sb; }
        mfmas();
        __syncthreads();
      }
      char* cur = smem + (kt & 1) * STAGE;
      char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
      frags(cur);
      TA::template store_f16<false, false, SCALE>(nxt, va, m0, M, 0, K, amax_a, sca);
      TB::template store_f16<false, false, false>(nxt + 2 * PA, vb, n0, N, 0, K, amax_b, scb);
      mfmas();
      __syncthreads();
      ++kt;
    }
  }
  for (; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    const bool more = kt + 1 < nk;
    if (more) load(kb + (kt + 1) * BK);
    frags(cur);
    mfmas();
    if (more) store(nxt, kb + (kt + 1) * BK);
    __syncthreads();
  }
  // true: a row of this thread's operand slices out of range (see above)
  static_assert(BK / 4 == 4, "a k-contiguous row is staged by 4 adjacent lanes");
  return rows_bad();
}

// Epilogue of the transposed product. acc[mi][ni] is the C^T block of output rows
// rb = wm*MB*32 + mi*32 and columns cb = wn*NB*32 + ni*32: lane l holds row rb + (l & 31),
// registers 4j..4j+3 the four consecutive columns cb + 8j + 4(l >> 5) + 0..3. Every group of
// four is one 16-byte load / store where it lies inside one output range and is aligned (the
// C layout of the untransposed product stores a dword per lane), else per element (store_out's
// order of operations either way: ((acc + C) + bias) + resid, then ELU).
__device__ inline float4 f4_of(const floatx16& a, int j) {
  return make_float4(a[4 * j], a[4 * j + 1], a[4 * j + 2], a[4 * j + 3]);
}

// slab (split-K): the partial slab this block writes; -1 = blockIdx.z (x gridDim.y + y).
template <int MB, int NB, int TBM, int TBN>
__device__ inline void write_tile_t(const GemmArgs& g, floatx16 (&acc)[MB][NB], int tail_z,
                                    int64_t tail_ti, int64_t m0, int64_t n0, int wm, int wn,
                                    int lane, int64_t slab = -1) {
  const int lr = lane & 31, lc = 4 * (lane >> 5);
  const int64_t M = g.M, N = g.N;
  if (tail_z >= 0) {   // tail slice: tile-local partial [TBM][TBN], summed by tail_fixup_kernel
    float* P = g.tail_partial + ((int64_t)tail_z * g.tail_rem + tail_ti) * (TBM * TBN);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rl = wm * (MB * 32) + mi * 32 + lr, cl = wn * (NB * 32) + ni * 32 + 8 * j + lc;
          *(float4*)(P + rl * TBN + cl) = f4_of(acc[mi][ni], j);
        }
    return;
  }
  if (g.splits > 1) {   // partial slab z: plain [M][N], reduced by splitk_reduce_kernel
    const int64_t z = slab >= 0 ? slab : (int64_t)blockIdx.z * gridDim.y + blockIdx.y;
    float* P = g.partial + z * M * N;
    const bool v4 = (N & 3) == 0;   // (the slab base is 16-byte aligned: M N floats per slab)
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni) {
        const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t col = n0 + wn * (NB * 32) + ni * 32 + 8 * j + lc;
          if (v4 && col + 3 < N) {
            *(float4*)(P + row * N + col) = f4_of(acc[mi][ni], j);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (col + i < N) P[row * N + col + i] = acc[mi][ni][4 * j + i];
          }
        }
      }
    return;
  }
  const int64_t b = blockIdx.y;
#pragma unroll
  for (int ni = 0; ni < NB; ++ni) {
    // the block column's range, decided per 32 columns (wave-uniform): one output range,
    // inside N, 16-byte aligned rows -> float4 groups; otherwise store_out per element
    const int64_t cb = n0 + wn * (NB * 32) + ni * 32;
    const bool first = cb < g.n_split;
    float* base;
    int64_t ldc, cc;
    if (first) { base = g.C0 + b * g.c0_bs; ldc = g.ldc0; cc = cb; }
    else if (cb < g.n_split2) { base = g.C1 + b * g.c1_bs; ldc = g.ldc1; cc = cb - g.n_split; }
    else { base = g.C2; ldc = g.ldc2; cc = cb - g.n_split2; }
    const int64_t lim = first ? g.n_split : (cb < g.n_split2 ? g.n_split2 : INT64_MAX);
    const bool vec = cb + 32 <= N && cb + 32 <= lim && ldc % 4 == 0 &&
                     ((uintptr_t)(base + cc) % 16) == 0;
    if (!vec) {
#pragma unroll
      for (int mi = 0; mi < MB; ++mi) {
        const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 v = f4_of(acc[mi][ni], j);
          const int64_t col = cb + 8 * j + lc;
          if (col < N) store_out(g, b, row, col, v.x);
          if (col + 1 < N) store_out(g, b, row, col + 1, v.y);
          if (col + 2 < N) store_out(g, b, row, col + 2, v.z);
          if (col + 3 < N) store_out(g, b, row, col + 3, v.w);
        }
      }
      continue;
    }
    const bool epi = first && (g.bias || g.resid || g.elu);
    float4 bias[4];   // loaded before this block column's stores (loads and stores share vmcnt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bias[j] = (first && g.bias) ? *(const float4*)(g.bias + b * g.bias_bs + cc + 8 * j + lc)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
    const float* rbase = (first && g.resid) ? g.resid + b * g.resid_bs + cb + lc : nullptr;
    const bool rvec = rbase && g.resid_ld % 4 == 0 && ((uintptr_t)rbase % 16) == 0;
#pragma unroll
    for (int mi = 0; mi < MB; ++mi) {
      const int64_t row = m0 + wm * (MB * 32) + mi * 32 + lr;
      if (row >= M) continue;
      float* d = base + row * ldc + cc + lc;
      float4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = f4_of(acc[mi][ni], j);
      if (g.accumulate || rbase) {   // the block's loads before its stores
        float4 cv[4], rv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          cv[j] = g.accumulate ? *(const float4*)(d + 8 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
          const float* rp = rbase ? rbase + row * g.resid_ld + 8 * j : nullptr;
          rv[j] = !rp ? make_float4(0.f, 0.f, 0.f, 0.f)
                      : (rvec ? *(const float4*)rp : make_float4(rp[0], rp[1], rp[2], rp[3]));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // store_out's order: ((acc + C) + bias) + resid
          if (g.accumulate) v[j] = add4(v[j], cv[j]);
          if (first && g.bias) v[j] = add4(v[j], bias[j]);
          if (rbase) v[j] = add4(v[j], rv[j]);
        }
      } else if (first && g.bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = add4(v[j], bias[j]);
      }
      if (epi && g.elu) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = make_float4(elu_act(v[j].x), elu_act(v[j].y), elu_act(v[j].z), elu_act(v[j].w));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) *(float4*)(d + 8 * j) = v[j];
    }
  }
}

// Fused node scores of one finished output tile (the forward projection, g.s_part set): the
// tile's share of S[row][h] = sum_col Wh[row][col] A2[h][col] over its TBN columns, written as
// s_part[tn][row][h] (combined over the column tiles in a fixed order by score_combine_kernel).
// A lane holds 16 columns of one row per block (write_tile_t's layout), so a head's partial is
// a register dot product plus one exchange between the two lane halves; the WGN waves sharing
// the rows are summed in wave order through LDS. Runs after the tile's stores, acc still live.
template <int MB, int NB, int TBM, int TBN, int WGN>
__device__ inline void scores_tile(const GemmArgs& g, const floatx16 (&acc)[MB][NB], int64_t m0,
                                   int64_t n0, int64_t tn, int wm, int wn, int lane, char* smem) {
  const int H2 = g.s_h2, lr = lane & 31, lc = 4 * (lane >> 5);
  const int H2p = (H2 + 1) & ~1;          // scores in pairs (zero weights past H2)
  float* a2s = (float*)smem;              // [H2p][TBN]
  float* red = a2s + H2p * TBN;           // [WGN][TBM][H2]
  for (int t = threadIdx.x; t < H2p * TBN; t += 64 * WGN * (TBM / (MB * 32))) {
    const int h = t / TBN, c = t - h * TBN;
    const int64_t col = n0 + c;
    a2s[t] = (h < H2 && col < g.N) ? score_weight(g.s_a, g.s_nh, g.s_f, g.s_fp, h, col) : 0.f;
  }
  __syncthreads();
  // two scores per pass over the accumulators (each accumulator read H2p / 2 times, not H2;
  // four per pass spilled: the compiler hoists every column group's weights)
#pragma unroll 1
  for (int h0 = 0; h0 < H2p; h0 += 2) {
    float t[2][MB];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int mi = 0; mi < MB; ++mi) t[q][mi] = 0.f;
#pragma unroll
    for (int ni = 0; ni < NB; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cl = wn * (NB * 32) + ni * 32 + 8 * j + lc;
        float4 w[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) w[q] = *(const float4*)(a2s + (h0 + q) * TBN + cl);
#pragma unroll
        for (int mi = 0; mi < MB; ++mi) {
          const float x0 = acc[mi][ni][4 * j], x1 = acc[mi][ni][4 * j + 1];
          const float x2 = acc[mi][ni][4 * j + 2], x3 = acc[mi][ni][4 * j + 3];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            t[q][mi] = fmaf(x0, w[q].x, t[q][mi]);
            t[q][mi] = fmaf(x1, w[q].y, t[q][mi]);
            t[q][mi] = fmaf(x2, w[q].z, t[q][mi]);
            t[q][mi] = fmaf(x3, w[q].w, t[q][mi]);
          }
        }
      }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (h0 + q >= H2) break;
#pragma unroll
      for (int mi = 0; mi < MB; ++mi) {
        const float tot = t[q][mi] + __shfl_xor(t[q][mi], 32);   // the same sum in both halves
        if (lane < 32) red[(wn * TBM + wm * (MB * 32) + mi * 32 + lr) * H2 + h0 + q] = tot;
      }
    }
  }
  __syncthreads();
  float* P = g.s_part + tn * g.M * H2;
  for (int t = threadIdx.x; t < TBM * H2; t += 64 * WGN * (TBM / (MB * 32))) {
    const int rl = t / H2, h = t - rl * H2;
    const int64_t row = m0 + rl;
    if (row >= g.M) continue;
    float v = red[rl * H2 + h];
#pragma unroll
    for (int w = 1; w < WGN; ++w) v += red[(w * TBM + rl) * H2 + h];
    P[row * H2 + h] = v;
  }
}


}  // namespace
}  // namespace gatx
