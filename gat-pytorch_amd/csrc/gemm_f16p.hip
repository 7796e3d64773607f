// f16x3 GEMM with the weight operand pre-split ("f16p"): C = A . B^T for a k-contiguous fp32 A
// (activations, or a gradient G_aug) and a weight B (W_aug, W_aug^T) given as fp16 planes built
// once per weight version by gatx_weight_planes.
//
// Arithmetic: the f16x3 split of gemm_x3_impl.h (x = h + l 2^-11, three fp16 MFMA products), with
// the 2^11 of the main product carried by the planes themselves instead of register multiplies:
//     A planes  Ah = fp16(64 s_r a),       Al = fp16(64 s_r a - Ah)       (s_r: row scale, A)
//     B planes  Bh = fp16(32 s_B b),       Bl = fp16(32 s_B b - Bh)       (s_B: one scale, B)
//     Ah Bh + Ah Bl + Al Bh = 2^11 s_r s_B a b  (dropped: Al Bl, <= 2^-22 |2^11 s_r s_B a b|)
// so the MFMA phase is three plain v_mfma_f32_32x32x16_f16 per block (no v_pk_mul), and the split
// of A is four v_fma_mix per element pair (fp16 rounding of the exact product, then of the exact
// residual) instead of eight conversions and subtractions. B's planes come from memory (two
// 16-byte loads per thread per K-tile, no VALU). Per K-tile and wave the VALU work drops from ~113
// instructions (gemm_x3_impl.h f16_mainloop) to ~30, which is what kept the matrix pipe waiting
// there: with two waves per SIMD the split, the planes' LDS stores and the hi-fragment scaling
// filled most of the issue slots between MFMAs.
//
// Range: s_B puts max |B| at [2^9, 2^10) (32 s_B |b| < 2^15), so B never overflows; a B row whose
// max is below 2^-8 / s_B (its residual plane would lose precision) flags its 256-row tile, and
// workgroups reading a flagged tile recompute as x3 (the fp32 weight is still passed). A rows are
// scaled by their max over the first K-tile to [2^7, 2^8) (SCALE) or taken as they are; a row
// whose max leaves [2^-9, 1023] after scaling sends its workgroup to the x3 recomputation too, so
// accuracy never depends on the operands' magnitudes (tests/test_gpu_layer.py::
// test_gemm_f16p_accuracy). Loads go through buffer resources bounded to the tile's rows: rows
// past M or N read as zero.
#include <cstring>
#include <type_traits>

#include "gemm_x3_impl.h"

namespace gatx {
namespace {
using namespace gk;

// This file's f16x3 -> x3 fallback workgroups (gemm_x3.hip keeps its own count for the in-loop
// kernels): a __device__ symbol of this code object, so every launch counts on the device it
// runs on (a pointer cached from another translation unit would name one device's copy).
__device__ unsigned long long g_f16p_fallback_tiles = 0;

__global__ void f16p_fallback_add_kernel(unsigned long long* dst, int reset) {
  if (threadIdx.x == 0) {
    dst[0] += __hip_atomic_load(&g_f16p_fallback_tiles, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    if (reset)
      __hip_atomic_store(&g_f16p_fallback_tiles, 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

// h = fp16_rn(x c), l = fp16_rn(x c - h) for an element pair (x in the low halves): v_fma_mix
// rounds the exact product and then the exact residual (hipcc never selects fma_mix here).
__device__ inline void split_mix(float x, float y, float c, uint32_t& h, uint32_t& l) {
  asm volatile(
      "v_fma_mixlo_f16 %0, %2, %4, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h), "=&v"(l)
      : "v"(x), "v"(y), "v"(c));
}

__device__ inline __amdgpu_buffer_rsrc_t buffer_rsrc(const void* base, int64_t bytes) {
  const int nr = (int)(bytes > 0x7ffffff0 ? 0x7ffffff0 : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, nr, 0x00020000);
}

// One fp16 plane image of 256 rows x BK k (gemm_x3_impl.h PlaneImg extended to BK 32): 16-byte
// 8-k slots, slot-major; odd slots' rows XOR'd by 12 for conflict-free fragment reads.
template <int BK>
struct PImg {
  static constexpr int BYTES = 256 * BK * 2;
  static __device__ inline int off(int r, int k) {
    const int s = k >> 3;
    return s * (256 * 16) + ((r ^ ((s & 1) * 12)) << 4) + ((k & 4) << 1);
  }
};

constexpr int kPlanesHeader = 256;   // bytes before the planes: [0] 2^-11 / s_B, [1] s_B, [16..] tile flags
constexpr int64_t kPlanesMaxRows = 60 * 256;   // one header flag per 256-row tile: 60 fit

template <int BK>
struct F16pCfg {
  static constexpr int PB = PImg<BK>::BYTES;
  static constexpr int STAGE = 4 * PB;   // A_h A_l B_h B_l
  static constexpr int X3_STAGE = 3 * 2 * (256 + 256) * 16;
  static constexpr int SMEM = (2 * STAGE > 2 * X3_STAGE ? 2 * STAGE : 2 * X3_STAGE) + 256 * 4;
};

// Main loop over the K-tiles [kb, K) of one 256 x 256 tile. Returns true when a row of A left the
// fp16 range (the caller recomputes the tile as x3). inv[256] (LDS, after the stages) receives
// 1 / s_r per tile row.
// Ping-pong (16-deep K-tiles; the single-phase loop measured 2-3% slower in situ): the block's two wave groups (waves 0-3: tile rows 0-127, waves
// 4-7: rows 128-255; one wave of each per SIMD) run the loop one barrier apart, each K-tile as
// MEM (this tile's fragments, the next tile's split + LDS stores, the loads of the one after) |
// raw barrier | MATH (the 24 MFMAs, raised priority) | raw barrier, so one group's MFMAs overlap
// the other's memory phase instead of both groups stalling on the same phase (lab v6: -10 to -12%
// on the PPI projections and 8192^2 x 4096, tools/gemm_lab). Group 1 starts one barrier late and
// group 0 ends with one more, so every s_barrier pairs the groups' n-th calls. Buffer reuse: a
// wave's stores of tile i + 1 (buffer (i + 1) & 1) come after the barrier that follows every
// wave's reads of tile i - 1; reads of tile i + 1 come after both groups' stores (each wave waits
// for its LDS stores before every barrier). Global loads stay in flight across the barriers.
template <int BK, int SCALE>
__device__ inline bool f16p_mainloop(const GemmArgs& g, const float* __restrict__ A, int64_t m0,
                                     int64_t n0, int64_t kb, int64_t K, char* smem, int wm,
                                     int wn, int lane, floatx16 (&acc)[4][2]) {
  using I = PImg<BK>;
  using Cf = F16pCfg<BK>;
  constexpr int PB = Cf::PB, STAGE = Cf::STAGE, MB = 4, NB = 2, NT = 512;
  constexpr int NV = BK / 8;   // float4 (A) and 16-byte plane pieces (B) per thread per K-tile
  constexpr int TPR = BK / 4;  // staging threads per row
  float* inv = (float*)(smem + 2 * STAGE);
  const int tid = threadIdx.x;
  const int64_t arows = g.M - m0 < 256 ? g.M - m0 : 256;
  const int64_t brows = g.N - n0 < 256 ? g.N - n0 : 256;
  const auto ra = buffer_rsrc(A + m0 * g.lda, arows * g.lda * 4);
  const auto rb = buffer_rsrc((const char*)g.b_planes + n0 * g.b_prow, brows * g.b_prow);
  int voa[NV], vob[NV], oa[NV], ob[NV], ka[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int idx = tid + NT * c;
    const int r = idx / TPR, k = 4 * (idx % TPR), j = idx % TPR;
    voa[c] = (r * (int)g.lda + k) * 4;
    oa[c] = I::off(r, k);
    ka[c] = k;
    vob[c] = r * (int)g.b_prow + (j >> 1) * 32 + (j & 1) * 16;   // slot j >> 1, plane j & 1
    ob[c] = (2 + (j & 1)) * PB + I::off(r, 8 * (j >> 1));
  }
  float4 va[NV];
  uint4 vb[NV];
  const int nk = (int)ceil_div(K - kb, BK);
  auto load = [&](int kt) {
    const int so = (int)((kb + kt * BK) * 4);   // bytes: 4 per k in A and in the planes
#pragma unroll
    for (int c = 0; c < NV; ++c)
      va[c] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, voa[c], so, 0));
#pragma unroll
    for (int c = 0; c < NV; ++c)
      vb[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb, vob[c], so, 0));
  };
  // range check on the hi plane itself: max |Ah| per thread as packed fp16 bit patterns (|.| by
  // clearing the sign bits; non-negative fp16 order as unsigned integers), one AND and one
  // v_pk_max_u16 per element pair instead of four abs / max on the fp32 values
  float cs[NV];
  uint32_t hmax[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) { cs[c] = 64.f; hmax[c] = 0u; }
  auto pk_max_u16 = [](uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
  };
  // the last K-tile may run past K: A's k >= K would read the next row (B's planes are zero
  // there, but an inf / nan in A would still poison the sums) -> zeroed
  auto mask_tail = [&](int kt) {
    const int64_t k0 = kb + (int64_t)kt * BK;
    if (k0 + BK <= K) return;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int64_t lim = K - (k0 + ka[c]);
      va[c].x = lim > 0 ? va[c].x : 0.f;
      va[c].y = lim > 1 ? va[c].y : 0.f;
      va[c].z = lim > 2 ? va[c].z : 0.f;
      va[c].w = lim > 3 ? va[c].w : 0.f;
    }
  };
  auto store = [&](char* st) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const float4 v = va[c];
      uint32_t h0, l0, h1, l1;
      split_mix(v.x, v.y, cs[c], h0, l0);
      split_mix(v.z, v.w, cs[c], h1, l1);
      hmax[c] = pk_max_u16(hmax[c], pk_max_u16(h0 & 0x7fff7fffu, h1 & 0x7fff7fffu));
      *(uint2*)(st + oa[c]) = make_uint2(h0, h1);
      *(uint2*)(st + PB + oa[c]) = make_uint2(l0, l1);
    }
#pragma unroll
    for (int c = 0; c < NV; ++c) *(uint4*)(st + ob[c]) = vb[c];
  };
  load(0);
  mask_tail(0);
  if constexpr (SCALE > 0) {
    // power-of-two row scale bringing the row's max |a| to [2^7, 2^8): the exact max over the
    // whole row (SCALE 2: g.a_rowmax) or the first K-tile's (SCALE 1; a row's TPR staging lanes
    // are adjacent)
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      float m;
      if constexpr (SCALE == 2) {
        const int64_t row = m0 + (tid + NT * c) / TPR;
        m = row < g.M ? g.a_rowmax[row] : 0.f;
      } else {
        const float4 v = va[c];
        m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
#pragma unroll
        for (int o = 1; o < TPR; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
      }
      int e = 0;
      (void)frexpf(m, &e);
      const float sc = (m > 0.f && m <= 3.0e38f) ? ldexpf(1.f, 8 - e) : 1.f;
      cs[c] = 64.f * sc;
      if ((tid % TPR) == 0) inv[(tid + NT * c) / TPR] = 1.f / sc;
    }
  } else if (tid < 256) {
    inv[tid] = 1.f;
  }
  store(smem);
  if (nk > 1) {
    load(1);
    mask_tail(1);
  }
  static_assert(BK == 16, "the ping-pong loop takes one 16-deep MFMA step per K-tile");
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  barrier();               // tile 0 staged by every wave
  if (wm == 1) barrier();  // group 1 one barrier behind
  // one K-tile; the stage is a compile-time constant (the loop below is unrolled by two), so
  // the fragment reads and stores take immediate LDS offsets instead of per-tile address math
  auto step = [&](int kt, auto stage) {
    constexpr int CS = decltype(stage)::value;
    const char* cur = smem + CS * STAGE;
    char* nxt = smem + (CS ^ 1) * STAGE;
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
    if (kt + 2 < nk) {
      load(kt + 2);
      mask_tail(kt + 2);
    }
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
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    step(kt + 1, std::integral_constant<int, 1>{});
  }
  if (kt < nk) step(kt, std::integral_constant<int, 0>{});
  if (wm == 0) barrier();  // balances group 1's extra barrier
  // a row is out of range when its largest |Ah| = |fp16(64 s a)| is inf / nan (64 s |a| past the
  // fp16 range: |s a| > 1023) or, unless the row is zero, below 2^-3 (s |a| < 2^-9: the residual
  // plane would go subnormal)
  bool bad = false;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    uint32_t m = hmax[c];
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) m = pk_max_u16(m, (uint32_t)__shfl_xor((int)m, o));
    const uint32_t mh = (m & 0xffffu) > (m >> 16) ? (m & 0xffffu) : (m >> 16);
    bad |= mh >= 0x7c00u || (mh > 0u && mh < 0x3000u);
  }
  return bad;
}

template <int BK, int TAG>
__global__ void __launch_bounds__(512, 1) gemm_f16p_kernel(GemmArgs g) {
  using Cf = F16pCfg<BK>;
  using C = X3Cfg<1>;
  __shared__ __attribute__((aligned(16))) char smem[Cf::SMEM];
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
  const int64_t m0 = tm * 256, n0 = tn * 256;
  const float* __restrict__ A = g.A;
  // wave id through readfirstlane: known uniform, so the ping-pong's group branches stay scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / C::WGN, wn = wave % C::WGN;
  floatx16 acc[C::MB][C::NB];
#pragma unroll
  for (int i = 0; i < C::MB; ++i)
#pragma unroll
    for (int j = 0; j < C::NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const char* hdr = (const char*)g.b_planes - kPlanesHeader;
  if (K > kb) {
    // a flagged weight tile (a B row whose residual plane would lose precision) goes to x3
    const bool btile_bad = ((const uint32_t*)(hdr + 16))[tn] != 0;
    bool x3 = btile_bad;
    if (!btile_bad) {
      // gradients (TAG 1, rows ~1e-7): scaled by their exact row max when given, else by the
      // first K-tile's; activations (TAG 0) as they come
      const bool bad =
          TAG == 0 ? f16p_mainloop<BK, 0>(g, A, m0, n0, kb, K, smem, wm, wn, lane, acc)
          : g.a_rowmax ? f16p_mainloop<BK, 2>(g, A, m0, n0, kb, K, smem, wm, wn, lane, acc)
                       : f16p_mainloop<BK, 1>(g, A, m0, n0, kb, K, smem, wm, wn, lane, acc);
      x3 = __syncthreads_or(bad);
      const float* inv = (const float*)(smem + 2 * Cf::STAGE);
      const float binv = ((const float*)hdr)[0];
      const int lr = lane & 31;
#pragma unroll
      for (int i = 0; i < C::MB; ++i) {
        const float ra = inv[wm * (C::MB * 32) + i * 32 + lr] * binv;
#pragma unroll
        for (int j = 0; j < C::NB; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = x3 ? 0.f : acc[i][j][r] * ra;
      }
      __syncthreads();   // inv read before the fallback or the epilogue reuses the LDS
    }
    if (x3) {
      if (threadIdx.x == 0)
        __hip_atomic_fetch_add(&g_f16p_fallback_tiles, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      x3_mainloop<true, true, false, 1>(g, A, g.B, m0, n0, kb, K, ceil_div(K - kb, C::BK),
                                           smem, wm, wn, lane, acc);
    }
  }
  write_tile_t<C::MB, C::NB, C::TBM, C::TBN>(g, acc, tail_z, tail_ti, m0, n0, wm, wn, lane);
  if constexpr (TAG == 0)
    if (g.s_part && tail_z < 0)
      scores_tile<C::MB, C::NB, C::TBM, C::TBN, C::WGN>(g, acc, m0, n0, tn, wm, wn, lane, smem);
}

// ---- the weight gradient: g_W_aug = G_aug^T x (both operands row-contiguous, K = nodes) --------
// f16x3 with G_aug's columns (the A rows) scaled by their exact max (gatx_absmax_rows_cols) to
// [2^3, 2^4), which allows a third A plane carrying the main product's 2^11:
//     A planes  Ah = fp16(s_m a),  Ah' = 2^11 Ah (exact, <= 2^15),  Al = fp16(2^11 (s_m a - Ah))
//     B planes  Bh = fp16(b),      Bl = fp16(2^11 (b - Bh))          (x as it comes, any |x|)
//     Ah' Bh + Ah Bl + Al Bh = 2^11 s_m a b            (dropped: Al Bl 2^-11, <= 2^-22 of it)
// so B = x needs no scale (a column of x far below its peers keeps full precision down to
// 2^-13, as the in-loop kernel's unscaled operands), and no register multiply precedes the MFMAs.
// Staging as x3_mainloop's row-contiguous operands ([k][rows] plane images, fragments read
// transposed by ds_read_b64_tr_b16). Range: every B row (a column of x over this K-slice) must have
// max |b| <= 65504 and, unless zero, >= 2^-13; A rows (exactly scaled) only need to be finite. A
// workgroup with any row outside recomputes its tile as x3.

// (x, y) -> fp16_rn(x c) pair (one scale per element)
__device__ inline uint32_t mix_pair(float x, float y, float cx, float cy) {
  uint32_t h;
  asm volatile(
      "v_fma_mixlo_f16 %0, %1, %3, 0 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %2, %4, 0 op_sel_hi:[0,0,0]"
      : "=&v"(h)
      : "v"(x), "v"(y), "v"(cx), "v"(cy));
  return h;
}
// fp16_rn(x c - 2^11 h) pair, h the fp16 pair already in hp (2^11 h taken exactly inside the mix)
__device__ inline uint32_t mix_resid(float x, float y, float cx, float cy, uint32_t hp) {
  uint32_t l;
  float tx, ty;
  const float m2048 = -2048.f;   // not an inline constant: a register operand
  asm volatile(
      "v_fma_mix_f32 %1, %5, %8, 0 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %2, %5, %8, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixlo_f16 %0, %3, %6, %1 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %4, %7, %2 op_sel_hi:[0,0,0]"
      : "=&v"(l), "=&v"(tx), "=&v"(ty)
      : "v"(x), "v"(y), "v"(hp), "v"(cx), "v"(cy), "v"(m2048));
  return l;
}

template <bool MASK>
__device__ inline bool f16rc_mainloop(const GemmArgs& g, const float* __restrict__ A,
                                      const float* __restrict__ B, int64_t m0, int64_t n0,
                                      int64_t kb, int64_t K, int64_t nk, char* smem, int wm,
                                      int wn, int lane, floatx16 (&acc)[4][2]) {
  using C = X3Cfg<1>;
  constexpr int NT = C::NT, BK = C::BK, MB = C::MB, NB = C::NB;
  using TA = X3Tile<false, C::TBM, BK, NT>;
  using TB = X3Tile<false, C::TBN, BK, NT>;
  constexpr int PL = TA::Img::BYTES;   // bytes per plane (A and B images have the same size)
  constexpr int STAGE = 5 * PL;        // A: Ah, Ah', Al; B: Bh, Bl
  static_assert(TA::NV == 2 && TB::NV == 2, "256 x 16 row-contiguous tiles: 2 float4 per thread");
  const int64_t M = g.M, N = g.N;
  const int tid = threadIdx.x;
  // this thread's 4 A rows (fixed over K: NT is a multiple of ROWS / 4) and their scales
  const int ra = TA::row_of(tid);
  float4 sc;
  {
    float s4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t r = m0 + ra + j;
      const float m = r < M ? g.a_rowmax[r] : 0.f;
      int e = 0;
      (void)frexpf(m, &e);
      s4[j] = (m > 0.f && m <= 3.0e38f) ? ldexpf(1.f, 4 - e) : 1.f;   // max -> [2^3, 2^4)
    }
    sc = make_float4(s4[0], s4[1], s4[2], s4[3]);
  }
  float4 amax_a = make_float4(0.f, 0.f, 0.f, 0.f), amax_b = amax_a;
  float4 va[2], vb[2];
  const float* pa[2];
  const float* pb[2];
  int64_t sa = 0, sbs = 0;
  if (!MASK) {
    TA::setup(A, g.lda, m0, M, kb, pa, sa);
    TB::setup(B, g.ldb, n0, N, kb, pb, sbs);
  }
  auto load = [&](int64_t k0) {
    if (MASK) {
      TA::T::template load<false>(A, g.lda, m0, M, k0, K, va);
      TB::T::template load<false>(B, g.ldb, n0, N, k0, K, vb);
    } else {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int64_t k = k0 + TA::k_of(tid + NT * c);
        va[c] = *(const float4*)(k < K ? pa[c] : pa[c] - (k - kb) * g.lda);
        pa[c] += sa;
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int64_t k = k0 + TB::k_of(tid + NT * c);
        vb[c] = *(const float4*)(k < K ? pb[c] : pb[c] - (k - kb) * g.ldb);
        pb[c] += sbs;
      }
    }
  };
  auto absmax4 = [](float4 m, float4 v) {
    return make_float4(fmaxf(m.x, fabsf(v.x)), fmaxf(m.y, fabsf(v.y)), fmaxf(m.z, fabsf(v.z)),
                       fmaxf(m.w, fabsf(v.w)));
  };
  // zero what lies outside the matrices (rows past M / N, k past K): only edge tiles
  const bool edge_rows = MASK || m0 + C::TBM > M || n0 + C::TBN > N;
  auto store = [&](char* st, int64_t k0) {
    if (edge_rows || k0 + BK > K) {
      TA::template mask<true, true>(va, m0, M, k0, K);
      TB::template mask<true, true>(vb, n0, N, k0, K);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int idx = tid + NT * c;
      const int o = TA::Img::off(TA::row_of(idx), TA::k_of(idx));
      const float4 v = va[c], w = vb[c];
      amax_a = absmax4(amax_a, v);
      amax_b = absmax4(amax_b, w);
      // A: h = fp16(s a), h' = 2^11 h, l = fp16(2^11 (s a) - 2^11 h)
      const uint32_t h0 = mix_pair(v.x, v.y, sc.x, sc.y), h1 = mix_pair(v.z, v.w, sc.z, sc.w);
      const uint32_t l0 = mix_resid(v.x, v.y, 2048.f * sc.x, 2048.f * sc.y, h0);
      const uint32_t l1 = mix_resid(v.z, v.w, 2048.f * sc.z, 2048.f * sc.w, h1);
      const f16x2 k2048 = {(_Float16)2048.f, (_Float16)2048.f};
      const uint32_t g0 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, h0) * k2048);
      const uint32_t g1 = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, h1) * k2048);
      *(uint2*)(st + o) = make_uint2(h0, h1);
      *(uint2*)(st + PL + o) = make_uint2(g0, g1);
      *(uint2*)(st + 2 * PL + o) = make_uint2(l0, l1);
      // B: h = fp16(b), l = fp16(2^11 b - 2^11 h)
      const uint32_t b0 = mix_pair(w.x, w.y, 1.f, 1.f), b1 = mix_pair(w.z, w.w, 1.f, 1.f);
      const uint32_t e0 = mix_resid(w.x, w.y, 2048.f, 2048.f, b0);
      const uint32_t e1 = mix_resid(w.z, w.w, 2048.f, 2048.f, b1);
      *(uint2*)(st + 3 * PL + o) = make_uint2(b0, b1);
      *(uint2*)(st + 4 * PL + o) = make_uint2(e0, e1);
    }
  };
  load(kb);
  store(smem, kb);
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    const bool more = kt + 1 < nk;
    if (more) load(kb + (kt + 1) * BK);
    f16x8 fa[MB][3], fb[NB][2];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int x = 0; x < MB; ++x)
        fa[x][p] = __builtin_bit_cast(f16x8, TA::frag(cur + p * PL, wm * (MB * 32) + x * 32, 0, lane));
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int x = 0; x < NB; ++x)
        fb[x][p] = __builtin_bit_cast(f16x8, TB::frag(cur + (3 + p) * PL, wn * (NB * 32) + x * 32, 0, lane));
    // C^T = B^T A^T; small terms first: Ah Bl, Al Bh, then Ah' Bh
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][1], fa[mi][0], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][2], acc[mi][ni], 0, 0, 0);
#pragma unroll
    for (int mi = 0; mi < MB; ++mi)
#pragma unroll
      for (int ni = 0; ni < NB; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb[ni][0], fa[mi][1], acc[mi][ni], 0, 0, 0);
    if (more) store(nxt, kb + (kt + 1) * BK);
    __syncthreads();
  }
  // per-row range over this K-slice: a thread holds 4 rows at its k's; the 8 waves' lanes with the
  // same lane index share rows -> LDS reduction
  float* red = (float*)smem;   // [2][8][256]
  const int w8 = tid >> 6;
  *(float4*)&red[(0 * 8 + w8) * 256 + ra] = amax_a;
  *(float4*)&red[(1 * 8 + w8) * 256 + ra] = amax_b;
  __syncthreads();
  bool bad = false;
  if (tid < 256) {
    float ma = 0.f, mb = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      ma = fmaxf(ma, red[w * 256 + tid]);
      mb = fmaxf(mb, red[(8 + w) * 256 + tid]);
    }
    const float s = (m0 + tid < M) ? [&] {
      const float m = g.a_rowmax[m0 + tid];
      int e = 0;
      (void)frexpf(m, &e);
      return (m > 0.f && m <= 3.0e38f) ? ldexpf(1.f, 4 - e) : 1.f;
    }() : 1.f;
    bad = !(ma * s <= 31.f) || !(mb <= 65504.f) || (mb > 0.f && mb < 0x1p-13f);
  }
  bad = __syncthreads_or(bad);
  return bad;
}

template <bool VEC>
__global__ void __launch_bounds__(512, 1) gemm_f16rc_kernel(GemmArgs g) {
  using C = X3Cfg<1>;
  constexpr int SMEM = 2 * 5 * (256 * 16 * 2) > 2 * 3 * 2 * (256 + 256) * 16
                           ? 2 * 5 * (256 * 16 * 2) : 2 * 3 * 2 * (256 + 256) * 16;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  // 1-D grid over (split, tile), XCD-contiguous: the tiles of one K-split (which read the same
  // G_aug and x rows at about the same time) share an XCD and its L2 — round-robin placement put
  // them on different XCDs and fetched each operand slab ~3x
  const int64_t TT = g.tiles_m * g.tiles_n;
  int64_t z, tile, tm, tn;
  tile_of(blockIdx.x, TT * g.splits, TT, z, tile);
  tm = tile / g.tiles_n;
  tn = tile - tm * g.tiles_n;
  const int64_t kb = z * g.k_per_split;
  const int64_t K = min(g.K, kb + g.k_per_split);
  const int64_t m0 = tm * C::TBM, n0 = tn * C::TBN;
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
    const bool x3 = f16rc_mainloop<!VEC>(g, g.A, g.B, m0, n0, kb, K, nk, smem, wm, wn, lane, acc);
    // undo 2^11 and the A rows' scales (lane -> output row = A row, write_tile_t's layout)
    const int lr = lane & 31;
#pragma unroll
    for (int i = 0; i < C::MB; ++i) {
      const int64_t row = m0 + wm * (C::MB * 32) + i * 32 + lr;
      float f = 0x1p-11f;
      if (row < g.M) {
        const float m = g.a_rowmax[row];
        int e = 0;
        (void)frexpf(m, &e);
        f = (m > 0.f && m <= 3.0e38f) ? ldexpf(1.f, e - 4 - 11) : 0x1p-11f;
      }
#pragma unroll
      for (int j = 0; j < C::NB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = x3 ? 0.f : acc[i][j][r] * f;
    }
    if (x3) {
      if (threadIdx.x == 0)
        __hip_atomic_fetch_add(&g_f16p_fallback_tiles, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      x3_mainloop<false, false, !VEC, 1>(g, g.A, g.B, m0, n0, kb, K, nk, smem, wm, wn, lane,
                                            acc);
    }
  }
  write_tile_t<C::MB, C::NB, C::TBM, C::TBN>(g, acc, -1, 0, m0, n0, wm, wn, lane, z);
}

// ---- weight planes (gatx_weight_planes) ---------------------------------------------------------
// Header (kPlanesHeader bytes: [0] 2^-11 / s_B, [1] s_B, [16..] one flag per 256-row tile), then
// rows x prow bytes of planes: row n = K_pad / 8 slots of 32 bytes, each h[8] then l[8] (fp16),
// K_pad = round_up(K, 32), zero past K; then the scratch of the two build launches: rows row
// maxima and ceil(rows / 4) block maxima. Two launches, no memset and no atomics: every header
// word is written by the second launch (identical values from the blocks of one tile).

// One wave per row: the row's max |w| (nan -> inf) and, per block of 4 rows, their max.
__global__ void __launch_bounds__(256) planes_max_kernel(const float* __restrict__ W, int64_t rows,
                                                         int64_t K, int64_t ld,
                                                         float* __restrict__ rowmax,
                                                         float* __restrict__ blockmax) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = blockIdx.x * 4ll + wave;
  float m = 0.f;
  if (row < rows) {
    const float* w = W + row * ld;
    for (int64_t k = lane; k < K; k += 64) {
      const float v = fabsf(w[k]);
      m = (v > m || v != v) ? (v != v ? __int_as_float(0x7f800000) : v) : m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) rowmax[row] = m;
  }
  if (lane == 0) red[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) blockmax[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// One wave per row: the global max from the block maxima, s_B, the row's tile flag (from the
// tile's row maxima), the planes.
__global__ void __launch_bounds__(256) planes_split_kernel(const float* __restrict__ W,
                                                           int64_t rows, int64_t K, int64_t ld,
                                                           char* __restrict__ planes,
                                                           const float* __restrict__ rowmax,
                                                           const float* __restrict__ blockmax,
                                                           int64_t nblk) {
  char* hdr = planes - kPlanesHeader;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gm = 0.f;
  for (int64_t i = lane; i < nblk; i += 64) gm = fmaxf(gm, blockmax[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) gm = fmaxf(gm, __shfl_xor(gm, o));
  int e = 0;
  (void)frexpf(gm, &e);
  const bool finite = gm <= 3.0e38f;
  const float sB = (gm > 0.f && finite) ? ldexpf(1.f, 10 - e) : 1.f;
  const float c = 32.f * sB;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ((float*)hdr)[0] = 0x1p-11f / sB;
    ((float*)hdr)[1] = sB;
  }
  // the tile flag: a nonzero row whose residual plane would go subnormal (max s_B < 2^-8), or a
  // non-finite value anywhere (the global max is then inf): the tile recomputes as x3. Wave 0 of
  // the first block of each tile's rows (every block of a tile would write the same value).
  const int64_t row0 = blockIdx.x * 4ll;
  if (wave == 0 && row0 % 256 == 0) {
    bool bad = !finite;
    for (int64_t r = row0 + lane; r < rows && r < row0 + 256; r += 64) {
      const float m = rowmax[r];
      bad |= m > 0.f && m * sB < 0x1p-8f;
    }
    bad = __any(bad);
    if (lane == 0) ((uint32_t*)(hdr + 16))[row0 / 256] = bad ? 1u : 0u;
  }
  const int64_t row = row0 + wave;
  if (row >= rows) return;
  const int64_t kpad = round_up(K, (int64_t)32);
  const int64_t prow = kpad * 4;
  const float* w = W + row * ld;
  char* dst = planes + row * prow;
  for (int64_t s = lane; s < kpad / 8; s += 64) {   // one 8-k slot per lane
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t k = 8 * s + j;
      v[j] = k < K ? w[k] : 0.f;
    }
    uint32_t h[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split_mix(v[2 * j], v[2 * j + 1], finite ? c : 0.f, h[j], l[j]);
    uint4* d = (uint4*)(dst + s * 32);
    d[0] = make_uint4(h[0], h[1], h[2], h[3]);
    d[1] = make_uint4(l[0], l[1], l[2], l[3]);
  }
}

// Exact max |x| per row and per column of X (rows x cols, row stride ld): a wave takes two rows
// at a time, all their float4 loads issued before any is used, the row max by a wave reduction,
// every lane keeping its columns' running max over the block's rows; the block's kStatWaves
// waves combine in LDS, then one atomicMax per column (non-negative floats order as their bit
// patterns; nan counts as inf; 256-B wave-instructions at the memory side). The column atomics
// are the cost beyond the read (tools/absmax_lab.hip, PPI G_aug 44906 x 1032: 32-row blocks of
// 4 waves 46 us, the same without column maxima 31 us), so a block of kStatWaves waves takes
// ~rows / kStatBlocks rows: ~2 blocks per CU, a third of the atomics, the same waves in flight
// (33 us; the 128-row, 8-wave, 151-VGPR form of round 3 held one block per CU: ~2 TB/s).
// colmax must be zero on entry. Either output may be NULL.
// VEC (ld % 4 == 0, X 16-byte aligned): unconditional float4 loads (a column index past cols
// reads column 0 of the row and is zeroed; a partial last float4 stays inside the row stride).
constexpr int kStatWaves = 8;
constexpr int64_t kStatBlocks = 512;
template <int CH, bool VEC>     // CH: 256-column chunks per lane (cols <= 256 CH)
__global__ void __launch_bounds__(64 * kStatWaves)
absmax_rows_cols_kernel(const float* __restrict__ X, int64_t rows, int64_t cols, int64_t ld,
                        int64_t rpb, float* rowmax, uint32_t* colmax) {
  __shared__ float red[kStatWaves][CH * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4 cm[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) cm[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto absn = [](float v) { return v != v ? __int_as_float(0x7f800000) : fabsf(v); };
  auto load = [&](const float* x, int64_t c) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (VEC) {
      v = *(const float4*)(x + (c < cols ? c : 0));
      v.x = c < cols ? v.x : 0.f;
      v.y = c + 1 < cols ? v.y : 0.f;
      v.z = c + 2 < cols ? v.z : 0.f;
      v.w = c + 3 < cols ? v.w : 0.f;
    } else {
      if (c < cols) v.x = x[c];
      if (c + 1 < cols) v.y = x[c + 1];
      if (c + 2 < cols) v.z = x[c + 2];
      if (c + 3 < cols) v.w = x[c + 3];
    }
    return v;
  };
  const int64_t r0 = blockIdx.x * rpb, rend = min(rows, r0 + rpb);
  for (int64_t r = r0 + 2 * wave; r < rend; r += 2 * kStatWaves) {
    const bool two = r + 1 < rend;
    const float* x0 = X + r * ld;
    const float* x1 = X + (two ? r + 1 : r) * ld;
    float4 v0[CH], v1[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int64_t c = 256 * j + 4 * lane;
      v0[j] = load(x0, c);
      v1[j] = load(x1, c);
    }
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const float4 a = make_float4(absn(v0[j].x), absn(v0[j].y), absn(v0[j].z), absn(v0[j].w));
      float4 b = make_float4(absn(v1[j].x), absn(v1[j].y), absn(v1[j].z), absn(v1[j].w));
      if (!two) b = make_float4(0.f, 0.f, 0.f, 0.f);
      cm[j] = make_float4(fmaxf(cm[j].x, fmaxf(a.x, b.x)), fmaxf(cm[j].y, fmaxf(a.y, b.y)),
                          fmaxf(cm[j].z, fmaxf(a.z, b.z)), fmaxf(cm[j].w, fmaxf(a.w, b.w)));
      m0 = fmaxf(m0, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
      m1 = fmaxf(m1, fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w)));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      m0 = fmaxf(m0, __shfl_xor(m0, o));
      m1 = fmaxf(m1, __shfl_xor(m1, o));
    }
    if (lane == 0 && rowmax) {
      rowmax[r] = m0;
      if (two) rowmax[r + 1] = m1;
    }
  }
  if (!colmax) return;   // (uniform over the block: no barrier is skipped by part of it)
#pragma unroll
  for (int j = 0; j < CH; ++j) *(float4*)&red[wave][256 * j + 4 * lane] = cm[j];
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 64 * kStatWaves) {
    float v = red[0][c];
#pragma unroll
    for (int w = 1; w < kStatWaves; ++w) v = fmaxf(v, red[w][c]);
    atomicMax(colmax + c, __float_as_uint(v));
  }
}

template <int CH>
void launch_absmax(const float* X, int64_t rows, int64_t cols, int64_t ld, float* rowmax,
                   float* colmax, hipStream_t stream) {
  const int64_t rpb = ceil_div(rows, kStatBlocks);
  const unsigned nb = (unsigned)ceil_div(rows, rpb);
  if (ld % 4 == 0 && (uintptr_t)X % 16 == 0)
    absmax_rows_cols_kernel<CH, true><<<nb, 64 * kStatWaves, 0, stream>>>(X, rows, cols, ld, rpb,
                                                                          rowmax, (uint32_t*)colmax);
  else
    absmax_rows_cols_kernel<CH, false><<<nb, 64 * kStatWaves, 0, stream>>>(X, rows, cols, ld, rpb,
                                                                           rowmax, (uint32_t*)colmax);
}

}  // namespace

int read_f16p_fallbacks(unsigned long long* dst, int reset, hipStream_t stream) {
  f16p_fallback_add_kernel<<<1, 64, 0, stream>>>(dst, reset);
  GATX_LAUNCH_CHECK("gatx_gemm_fallback_read");
  return 0;
}

int absmax_rows_cols(const float* X, int64_t rows, int64_t cols, int64_t ld, float* rowmax,
                     float* colmax, hipStream_t stream) {
  GATX_REQUIRE(cols <= 2048, "absmax_rows_cols: at most 2048 columns");
  // zeroed by a kernel, not hipMemsetAsync: inside a captured hipGraph the memset node was not
  // ordered before the atomicMax kernel once a kernel had run outside the graph between replays
  // (PPI train step: the stale maxima of the previous replay sent every weight-gradient tile of
  // the second layer to the x3 fallback, 270 -> 570 us; the same failure as round 5's node-block
  // count)
  if (colmax) {
    zero_words_kernel<<<(unsigned)ceil_div(cols, (int64_t)256), 256, 0, stream>>>((uint32_t*)colmax, cols);
    GATX_LAUNCH_CHECK("absmax_rows_cols zero");
  }
  if (rows == 0) return 0;
  if (cols <= 512) launch_absmax<2>(X, rows, cols, ld, rowmax, colmax, stream);
  else if (cols <= 1024) launch_absmax<4>(X, rows, cols, ld, rowmax, colmax, stream);
  else if (cols <= 1280) launch_absmax<5>(X, rows, cols, ld, rowmax, colmax, stream);
  else launch_absmax<8>(X, rows, cols, ld, rowmax, colmax, stream);
  GATX_LAUNCH_CHECK("absmax_rows_cols");
  return 0;
}

size_t weight_planes_bytes(int64_t rows, int64_t K) {
  if (rows <= 0 || rows > kPlanesMaxRows || K <= 0) return 0;   // no planes for this shape
  return (size_t)kPlanesHeader + (size_t)rows * round_up(K, (int64_t)32) * 4 +
         4 * (size_t)(rows + ceil_div(rows, (int64_t)4));
}

int build_weight_planes(const float* W, int64_t rows, int64_t K, int64_t ld, void* buf,
                        hipStream_t stream) {
  GATX_REQUIRE(rows <= kPlanesMaxRows,
               "weight planes: at most 15360 rows (tile flags in the header)");
  char* planes = (char*)buf + kPlanesHeader;
  float* rowmax = (float*)(planes + rows * round_up(K, (int64_t)32) * 4);
  const int64_t nblk = ceil_div(rows, (int64_t)4);
  float* blockmax = rowmax + rows;
  planes_max_kernel<<<(unsigned)nblk, 256, 0, stream>>>(W, rows, K, ld, rowmax, blockmax);
  GATX_LAUNCH_CHECK("weight_planes max");
  planes_split_kernel<<<(unsigned)nblk, 256, 0, stream>>>(W, rows, K, ld, planes, rowmax,
                                                          blockmax, nblk);
  GATX_LAUNCH_CHECK("weight_planes split");
  return 0;
}

// The weight gradient's thin rows: C rows [256 tiles_m, M) (at most kThinRows: G_aug's score-
// gradient columns past a multiple of 256, e.g. PPI L1's 1024 + 8) in plain fp32 on the VALU, so
// the MFMA kernel's tiles are all full (a 256-row tile for 8 rows cost a fifth of PPI L1's weight
// gradient). C[m][n] = sum_k A[k][m] B[k][n] over this split's K range: 16 waves x 4 k-groups of
// lanes walk the rows (each lane 4 columns of a 64-column chunk, 256-B row segments), partials
// summed over the 64 (wave, group) slices in fixed order through LDS. Writes the split's slab (or
// C when there is no split), which splitk_reduce_kernel sums with the MFMA kernel's rows.
constexpr int kThinRows = 8;
__global__ void __launch_bounds__(1024) wgrad_thin_kernel(GemmArgs g) {
  constexpr int T = kThinRows, KG = 4, NW = 16, CW = 64;
  __shared__ float red[NW * KG][T][CW];   // 128 KB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int kg = lane >> 4, cq = lane & 15;
  const int64_t m0 = g.tiles_m * 256;
  const int64_t n = blockIdx.x * (int64_t)CW + 4 * cq;
  const int z = blockIdx.y;
  const int64_t kb = (int64_t)z * g.k_per_split, ke = min(g.K, kb + g.k_per_split);
  const bool nv = n < g.N;   // (N % 4 == 0: the vector path)
  const int64_t T_rows = g.M - m0;
  float acc[T][4];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t][0] = acc[t][1] = acc[t][2] = acc[t][3] = 0.f;
  const float* B = g.B + (nv ? n : 0);
  const float* A = g.A + m0;
  static_assert(T == 8, "two float4 loads per row");
  constexpr int U = 4, STEP = NW * KG;   // rows per slice per iteration; slices
  for (int64_t k0 = kb + wave * KG + kg; k0 < ke; k0 += (int64_t)STEP * U) {
    float4 b[U];
    float a[U][T];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = k0 + (int64_t)u * STEP;
      const bool ok = k < ke;
      const int64_t kk = ok ? k : kb;
      b[u] = *(const float4*)(B + kk * g.ldb);
      if (!ok || !nv) b[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      // the row's thin A values as 16-byte loads (a_vec: lda % 4 == 0 and A aligned; m0 % 256
      // == 0); columns past M are masked and stay inside the row stride (lda >= round4(M)), the
      // second load only when more than 4 rows remain
      const float4 a0 = *(const float4*)(A + kk * g.lda);
      const float4 a1 = T_rows > 4 ? *(const float4*)(A + kk * g.lda + 4)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
      a[u][0] = a0.x; a[u][1] = a0.y; a[u][2] = a0.z; a[u][3] = a0.w;
      a[u][4] = a1.x; a[u][5] = a1.y; a[u][6] = a1.z; a[u][7] = a1.w;
#pragma unroll
      for (int t = 0; t < T; ++t) a[u][t] = t < T_rows ? a[u][t] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < T; ++t) {
        acc[t][0] = fmaf(a[u][t], b[u].x, acc[t][0]);
        acc[t][1] = fmaf(a[u][t], b[u].y, acc[t][1]);
        acc[t][2] = fmaf(a[u][t], b[u].z, acc[t][2]);
        acc[t][3] = fmaf(a[u][t], b[u].w, acc[t][3]);
      }
  }
  const int slice = wave * KG + kg;
#pragma unroll
  for (int t = 0; t < T; ++t)
    *(float4*)&red[slice][t][4 * cq] = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
  __syncthreads();
  if (threadIdx.x < T * CW) {
    const int t = threadIdx.x / CW, c = threadIdx.x % CW;
    float v = 0.f;
    for (int s2 = 0; s2 < NW * KG; ++s2) v += red[s2][t][c];
    const int64_t row = m0 + t, col = blockIdx.x * (int64_t)CW + c;
    if (row < g.M && col < g.N) {
      if (g.splits > 1) g.partial[(int64_t)z * g.M * g.N + row * g.N + col] = v;
      else g.C0[row * g.ldc0 + col] = v;
    }
  }
}

int wgrad_thin_rows(int64_t M) {
  const int64_t r = M % 256;
  return (M > 256 && r > 0 && r <= kThinRows) ? (int)r : 0;
}

// The weight-gradient kernel (row-contiguous A and B, split-K slabs; g.a_rowmax = the exact
// max of every A row, i.e. of every G_aug column); rows past 256 tiles_m (< M: the thin rows,
// see wgrad_thin_rows) by wgrad_thin_kernel.
int launch_gemm_f16rc(const gk::GemmArgs& g, hipStream_t stream) {
  dim3 grid((unsigned)(g.tiles_m * g.tiles_n * g.splits), 1u, 1u);
  if (g.a_vec && g.b_vec) gemm_f16rc_kernel<true><<<grid, 512, 0, stream>>>(g);
  else gemm_f16rc_kernel<false><<<grid, 512, 0, stream>>>(g);
  GATX_LAUNCH_CHECK("gemm_f16rc");
  if (g.tiles_m * 256 < g.M) {
    GATX_REQUIRE(g.M - g.tiles_m * 256 <= kThinRows && g.a_vec && g.b_vec && g.N % 4 == 0,
                 "gemm_f16rc: thin rows out of range");
    wgrad_thin_kernel<<<dim3((unsigned)ceil_div(g.N, (int64_t)64), (unsigned)g.splits), 1024, 0,
                        stream>>>(g);
    GATX_LAUNCH_CHECK("wgrad_thin");
  }
  return 0;
}

// The pre-split kernel for GemmArgs prepared by gemm_impl; g.b_planes points at the planes (after
// the header), g.B at the fp32 weight (the x3 recomputation of flagged tiles).
int launch_gemm_f16p(const gk::GemmArgs& g, int tag, hipStream_t stream) {
  const int64_t tiles = g.tiles_m * g.tiles_n;
  const int64_t gx = g.tail_s > 1 ? g.dp_blocks + g.tail_rem * g.tail_s : tiles;
  dim3 grid((unsigned)gx, 1u, (unsigned)g.splits);
  // (32-deep K-tiles measured slower in the library: they spill beside the x3 fallback, bench
  // 1.43 -> 1.61 ms, gpurun_out/r05h; lab numbers in DESIGN.md §8)
  if (tag == 0) gemm_f16p_kernel<16, 0><<<grid, 512, 0, stream>>>(g);
  else gemm_f16p_kernel<16, 1><<<grid, 512, 0, stream>>>(g);
  GATX_LAUNCH_CHECK("gemm_f16p");
  return 0;
}

}  // namespace gatx
