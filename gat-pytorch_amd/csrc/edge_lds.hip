// LDS-staged edge forward (round 5) for graphs that split into node blocks of <= kLdsRows nodes
// with no edge between blocks (a PyG-style batch of graphs: gatx_graph_segments). Replaces the
// L2-gather aggregation of edge_fwd.hip (one wave per (node, head), one 1 KB row gathered per
// edge, bound by the L2 -> CU gather rate, ~15 TB/s) with two passes:
//
//   records   one wave per destination n, all NH heads: raw = s_src[src] + s_dst[n] (the
//             factorised logits), ex = exp(0.01 (raw - M)), den = sum ex (the same per-lane
//             partials and butterfly as edge_forward_kernel, so den and alpha are bitwise the
//             L2-gather pass's), alpha = ex / (den + 1e-8) written in edge_index' order (the
//             reference's returned attention, models/gat_layer.py:106-110, one NH-float row per
//             edge), max()'s tied argmax entries recorded as attention_alpha_ei does, and per
//             (head, CSR slot) the record {64 * src, alpha~} (the source row's byte offset in a
//             whole-graph image of 64-byte rows) (alpha~ = dropout(alpha), :112-115).
//   aggregate one 1024-thread workgroup per (node block, head, 16-float chunk of the head's row):
//             the chunk of every row of the block is staged in LDS (<= 2304 x 64 B = 144 KB), then
//             each wave takes 16 destinations at a time, a quad of lanes per destination walking
//             its CSR segment: per edge one 8-byte record load, one ds_read_b128 of the source's
//             16 B piece per lane, one float4 FMA — out[n, h, chunk] = sum_e alpha~ Wh[src, h,
//             chunk] (:117-127), then bias, the fused skip add, ELU and the next layer's input
//             dropout as edge_forward_kernel's epilogue.
// The staged bytes are read from LDS at up to 256 B/clk/CU (MI355X_MICROARCH.md §LDS) instead of
// from L2 at ~64 B/clk/CU.
#include "gatx_common.h"

namespace gatx {
namespace {

constexpr int kLdsRows = 2304;         // rows of one staged chunk image (2304 x 64 B = 144 KB)
constexpr int kChunk = 16;             // floats per chunk (64 B rows: 4 lanes x float4)

__device__ inline int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline int64_t xcd_contiguous(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, xcd = b % 8, j = b / 8;
  return (xcd < r) ? xcd * (q + 1) + j : r * (q + 1) + (xcd - r) * q + j;
}

struct RecArgs {
  const float* S;            // [N][2NH] = (s_src | s_dst)
  const uint32_t* M_ord;
  const int32_t* rowptr;
  const int32_t* col;
  const int32_t* perm;       // CSR slot -> edge_index' position
  int64_t N, E_bound;
  int NH, const_att;
  float p_drop;
  const uint64_t* seed;
  int2* rec;                 // [NH][E_bound]
  float* den;                // [N][NH]
  float* alpha;              // [E'][NH], edge_index' order (nullable)
  long long* argmax;         // tie records (nullable)
};

// NHC consecutive floats at p (a per-node row of NHC or 2 NHC floats, or its second half) as
// vector loads when the row allows it
template <int NHC>
__device__ inline void load_nh(const float* __restrict__ p, float (&v)[NHC]) {
  if constexpr (NHC % 4 == 0) {
#pragma unroll
    for (int h = 0; h < NHC; h += 4) {
      const float4 t = *(const float4*)(p + h);
      v[h] = t.x; v[h + 1] = t.y; v[h + 2] = t.z; v[h + 3] = t.w;
    }
  } else if constexpr (NHC % 2 == 0) {
#pragma unroll
    for (int h = 0; h < NHC; h += 2) {
      const float2 t = *(const float2*)(p + h);
      v[h] = t.x; v[h + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int h = 0; h < NHC; ++h) v[h] = p[h];
  }
}
// s_src[src, 0..NHC) of S's row
template <int NHC>
__device__ inline void load_ssrc(const float* __restrict__ S, int64_t src, float (&v)[NHC]) {
  load_nh<NHC>(S + src * (2 * NHC), v);
}

// one wave per destination; lane j <-> CSR slot beg + j of each 64-edge batch. A segment of at
// most 64 edges (nearly every PPI node) keeps its sources, logits and exponentials in registers
// between the denominator and the record sweeps (the second sweep divides the first's exp).
template <int NHC>
__global__ void __launch_bounds__(256) edge_records_kernel(RecArgs g) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= g.N) return;
  const int NH = NHC, S2 = 2 * NHC;
  const int beg = uni(g.rowptr[n]), end = uni(g.rowptr[n + 1]);
  const float M = g.const_att ? 0.f : ord_to_float(*g.M_ord);
  float sdst[NHC], dn[NHC];
#pragma unroll
  for (int h = 0; h < NHC; ++h) {
    sdst[h] = g.const_att ? 0.f : g.S[n * S2 + NH + h];
    dn[h] = 0.f;
  }
  const bool one = end - beg <= 64;
  // sweep 1: denominators (per-lane partials over the batches, then the butterfly, exactly as
  // edge_forward_kernel sums them)
  int src0 = 0;
  float raw0[NHC], ex0[NHC];
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    if (e < end) {
      const int src = g.col[e];
      float ss[NHC];
      if (!g.const_att) load_ssrc<NHC>(g.S, src, ss);
#pragma unroll
      for (int h = 0; h < NHC; ++h) {
        const float raw = g.const_att ? 0.f : ss[h] + sdst[h];
        const float ex = g.const_att ? 1.f : att_exp(raw, M);
        dn[h] += ex;
        raw0[h] = raw;
        ex0[h] = ex;
      }
      src0 = src;
    }
  }
#pragma unroll
  for (int h = 0; h < NHC; ++h) {
    float t = dn[h];
    for (int off = 1; off < 64; off <<= 1) t += __shfl_xor(t, off);
    dn[h] = t;
  }
  if (lane < NHC) {
    float d = 0.f;
#pragma unroll
    for (int h = 0; h < NHC; ++h)
      if (h == lane) d = dn[h];
    g.den[n * NH + lane] = d;
  }
  const bool drop = g.p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  const uint64_t seed = drop ? *g.seed : 0ull;
  // sweep 2: alpha, its records, ties
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    if (e >= end) continue;
    int src = src0;
    float raw[NHC], exv[NHC];
    if (one) {
#pragma unroll
      for (int h = 0; h < NHC; ++h) { raw[h] = raw0[h]; exv[h] = ex0[h]; }
    } else {
      src = g.col[e];
      float ss[NHC];
      if (!g.const_att) load_ssrc<NHC>(g.S, src, ss);
#pragma unroll
      for (int h = 0; h < NHC; ++h) {
        raw[h] = g.const_att ? 0.f : ss[h] + sdst[h];
        exv[h] = g.const_att ? 1.f : att_exp(raw[h], M);
      }
    }
    const int64_t p = g.perm[e];
    float a[NHC];
#pragma unroll
    for (int h = 0; h < NHC; ++h) {
      a[h] = exv[h] / (dn[h] + kSoftmaxEps);
      if (!g.const_att && raw[h] == M && g.argmax) {   // rare: every tied argmax (slot, head)
        unsigned long long k = atomicAdd((unsigned long long*)g.argmax, 1ull);
        if (k < GATX_ARGMAX_CAP) g.argmax[1 + k] = (long long)e * NH + h;
      }
      float w = a[h];
      if (drop) w = dropout_keep(seed, p * NH + h, g.p_drop) ? w * drop_scale : 0.f;
      g.rec[(int64_t)h * g.E_bound + e] = make_int2(src * (4 * kChunk), __float_as_int(w));
    }
    if (g.alpha) {
      float* o = g.alpha + p * NH;
      if constexpr (NHC % 4 == 0) {
#pragma unroll
        for (int h = 0; h < NHC; h += 4) *(float4*)(o + h) = make_float4(a[h], a[h + 1], a[h + 2], a[h + 3]);
      } else if constexpr (NHC % 2 == 0) {
#pragma unroll
        for (int h = 0; h < NHC; h += 2) *(float2*)(o + h) = make_float2(a[h], a[h + 1]);
      } else {
#pragma unroll
        for (int h = 0; h < NHC; ++h) o[h] = a[h];
      }
    }
  }
}

// ---- backward (round 6): the source pass of a concat layer as the same LDS walk.
// g_Wh[s, h, :] = sum over s's out-edges (s -> d) of alpha~[e, h] go[d, h, :] (autograd of
// models/gat_layer.py:117-127) is the forward aggregation on the transposed CSR with go's rows in
// place of Wh's: edge_records_src writes its records — per (head, transposed slot j) {64 d,
// alpha~} with d = scol[j], alpha~ recomputed from S / den exactly as edge_bwd_src_kernel does —
// plus that pass's other output, g_s_src[s, h] = sum of g_raw over s's out-edges (the same
// per-lane partials and butterfly, so the same bits), into G_aug[s, Dp + h]; then
// gatx_edge_lds_forward walks go with them into G_aug[s, 0 : Dp).
struct SrcRecArgs {
  const float* S;            // [N][2NH]
  const uint32_t* M_ord;
  const float* den;          // [N][NH]
  const int32_t* srowptr;    // transposed CSR (by source)
  const int32_t* scol;       // transposed slot -> destination
  const int32_t* seid;       // transposed slot -> CSR slot
  const int32_t* perm;       // CSR slot -> edge_index' position (dropout mask)
  int64_t N, E_bound;
  int NH, const_att;
  float p_drop;
  const uint64_t* seed;
  const float* g_raw;        // [NH][E_bound] per CSR slot (nullable)
  float* G_aug;
  int64_t ldg, Dp;
  int2* rec;                 // [NH][E_bound] per transposed slot
};

template <int NHC>
__global__ void __launch_bounds__(256) edge_records_src_kernel(SrcRecArgs g) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= g.N) return;
  const int NH = NHC, S2 = 2 * NHC;
  const int beg = uni(g.srowptr[s]), end = uni(g.srowptr[s + 1]);
  const float M = g.const_att ? 0.f : ord_to_float(*g.M_ord);
  const bool drop = g.p_drop > 0.f;
  const float drop_scale = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  const uint64_t seed = drop ? *g.seed : 0ull;
  float ssrc[NHC], gs[NHC];
#pragma unroll
  for (int h = 0; h < NHC; ++h) {
    ssrc[h] = g.const_att ? 0.f : g.S[s * S2 + h];
    gs[h] = 0.f;
  }
  for (int base = beg; base < end; base += 64) {
    const int j = base + lane;
    if (j >= end) continue;
    const int d = g.scol[j];
    const int e = g.seid[j];
    const int64_t ep = drop ? (int64_t)g.perm[e] : 0;
    float sd[NHC], dn[NHC], gr[NHC];
    if (!g.const_att) load_nh<NHC>(g.S + (int64_t)d * S2 + NH, sd);   // s_dst[d] row
    load_nh<NHC>(g.den + (int64_t)d * NH, dn);
#pragma unroll
    for (int h = 0; h < NHC; ++h) gr[h] = g.g_raw ? g.g_raw[(int64_t)h * g.E_bound + e] : 0.f;
#pragma unroll
    for (int h = 0; h < NHC; ++h) {
      const float ex = g.const_att ? 1.f : att_exp(ssrc[h] + sd[h], M);
      float w = ex / (dn[h] + kSoftmaxEps);
      if (drop) w = dropout_keep(seed, ep * NH + h, g.p_drop) ? w * drop_scale : 0.f;
      if (g.g_raw) gs[h] += gr[h];
      g.rec[(int64_t)h * g.E_bound + j] = make_int2(d * (4 * kChunk), __float_as_int(w));
    }
  }
  if (g.const_att) return;
#pragma unroll
  for (int h = 0; h < NHC; ++h) {
    const float t = group_sum<64>(gs[h]);
    if (lane == 0) g.G_aug[s * g.ldg + g.Dp + h] = t + 0.f;   // (as the src pass: + no g_corr)
  }
}

struct LdsArgs {
  const float* rows;         // Wh: row r, head h, feature f at rows[r * row_stride + h * Fp + f]
  int64_t row_stride;
  const int32_t* rowptr;
  const int2* rec;           // [NH][E_bound]
  int64_t E_bound;
  const int32_t* segs;       // block b = nodes [segs[b], segs[b + 1])
  const int32_t* seg_count;
  int64_t seg_bound;         // grid's block dimension (>= *seg_count)
  int64_t N;
  int NH, F, Fp, nchunks;
  const float* bias;         // [NH * F] or nullptr
  float* out;
  int64_t out_ld;
  const float* resid;
  int64_t resid_ld;
  int elu;
  float out_p;
  const uint64_t* out_seed;
  int vec_out;               // F % 4 == 0 and 16-byte aligned rows of out / resid
  int64_t ocols;             // output row width: NH F (concat) or F (head mean)
  int nranges;               // head-mean kernel: destination ranges per node block
};

template <bool DROP>
__device__ inline float lds_epilogue(float v, const LdsArgs& g, int64_t n, int64_t col) {
  if (g.bias) v += g.bias[col];
  if (g.resid) v += g.resid[n * g.resid_ld + col];
  if (g.elu) v = elu_act(v);
  if (DROP)
    v = dropout_keep(*g.out_seed, n * g.ocols + col, g.out_p) ? v * (1.f / (1.f - g.out_p))
                                                                          : 0.f;
  return v;
}

// every lane of a quad gets lane T's value: a legacy mov_dpp (undefined old value), which the
// compiler folds into the consuming address add (v_add_u32_dpp)
template <int T>
__device__ inline int quad_bcast(int v) {
  return __builtin_amdgcn_mov_dpp(v, T | (T << 2) | (T << 4) | (T << 6), 0xf, 0xf, true);
}

// the walk's epilogue for destination n, features [f0, f0 + 4) of column block cb = h F + f0
template <bool DROP>
__device__ inline void lds_store(const LdsArgs& g, int64_t n, int64_t cb, int f0, float4 acc) {
  float* orow = g.out + n * g.out_ld;
  if (g.vec_out) {
    float4 o = acc;
    if (g.bias) o = add4(o, *(const float4*)(g.bias + cb));
    if (g.resid) o = add4(o, *(const float4*)(g.resid + n * g.resid_ld + cb));
    if (g.elu) {
      o.x = elu_act(o.x); o.y = elu_act(o.y); o.z = elu_act(o.z); o.w = elu_act(o.w);
    }
    if (DROP) {
      const float sc = 1.f / (1.f - g.out_p);
      const int64_t base = n * g.ocols + cb;
      const uint64_t sd = *g.out_seed;
      o.x = dropout_keep(sd, base, g.out_p) ? o.x * sc : 0.f;
      o.y = dropout_keep(sd, base + 1, g.out_p) ? o.y * sc : 0.f;
      o.z = dropout_keep(sd, base + 2, g.out_p) ? o.z * sc : 0.f;
      o.w = dropout_keep(sd, base + 3, g.out_p) ? o.w * sc : 0.f;
    }
    *(float4*)(orow + cb) = o;
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (f0 + t < g.F) orow[cb + t] = lds_epilogue<DROP>(get4(acc, t), g, n, cb + t);
  }
}

// a value another kernel of the same step wrote, read past the scalar / vector L1 caches
__device__ inline int coherent_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Fallback walk when the graph no longer cuts into at most seg_bound blocks (a captured step
// replayed on edges whose node blocks differ from the ones its launch was sized for): the
// workgroups split the node range evenly and gather rows from global memory. Correct, slow, and
// never taken by a step whose edges kept their block structure.
template <bool DROP>
__device__ void lds_global_walk(const LdsArgs& g, int64_t k, int c, int h) {
  const int64_t per = ceil_div(g.N, g.seg_bound);
  const int64_t n0 = k * per;
  const int64_t R = min(per, g.N - n0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane & 3, j = lane >> 2;
  const int f0 = c * kChunk + q * 4;
  const int2* rh = g.rec + (int64_t)h * g.E_bound;
  const float* base = g.rows + (int64_t)h * g.Fp + f0;
  for (int64_t d0 = wave * 16; d0 < R; d0 += 256) {
    if (d0 + j >= R) continue;
    const int64_t n = n0 + d0 + j;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (f0 < g.Fp)
      for (int e = g.rowptr[n], end = g.rowptr[n + 1]; e < end; ++e) {
        const int2 r = rh[e];
        const float4 v = *(const float4*)(base + (int64_t)(r.x >> 6) * g.row_stride);
        acc = fma4(__int_as_float(r.y), v, acc);
      }
    if (f0 < g.F) lds_store<DROP>(g, n, (int64_t)h * g.F + f0, f0, acc);
  }
}

// RPL records per lane (4 RPL per quad per group), groups loaded unconditionally (clamped index,
// out-of-range records masked when consumed) in a counted ping-pong loop, so the next group's
// loads are in flight while this group's rows are read from LDS (tools/edge_lab: 245 vs 300 us
// for the PPI-L1 aggregation with the loads issued inside the walk)
// one record {64 src, alpha~} at byte offset off of a head's records (base: wave-uniform)
__device__ inline uint64_t load_rec(const int2* base, int off) {
  uint64_t v;
  asm volatile("global_load_dwordx2 %0, %1, %2" : "=v"(v) : "v"(off), "s"(base));
  return v;
}
// wait until at most N vector-memory operations of this wave are outstanding (loads return in
// issue order, so the N newest are the ones still allowed in flight)
template <int N, int RPL>
__device__ inline void wait_vm(uint64_t (&r)[RPL]) {
  if constexpr (RPL == 1)
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(r[0]) : "n"(N));
  else if constexpr (RPL == 2)
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(r[0]), "+v"(r[1]) : "n"(N));
  else
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]) : "n"(N));
}

constexpr int kRPL = 2;        // records per lane per group
constexpr int kDegBins = 64;   // degree buckets of the in-workgroup destination sort
static_assert(kLdsRows <= 3 * 1024, "the destination sort gives each thread <= 3 destinations");

template <int RPL, bool DROP>   // DROP: output dropout in the epilogue (its hoisted hash constants
__global__ void __launch_bounds__(1024) edge_lds_kernel(LdsArgs g) {   // spill at 128 VGPRs)
  __shared__ __attribute__((aligned(16))) float4 img[kLdsRows * 4];
  __shared__ unsigned short order[kLdsRows];   // the block's destinations, grouped by degree
  __shared__ int lrp[kLdsRows + 1];             // the block's row pointers (the walk's segment
  __shared__ int bins[kDegBins];                // bounds without a global-latency hop)
  const int64_t b = xcd_contiguous(blockIdx.x, gridDim.x);   // the chunks of one (block, head)
  const int c = (int)(b % g.nchunks);                           // run on one XCD: its records
  const int h = (int)((b / g.nchunks) % g.NH);                  // stay in that L2
  const int64_t k = b / ((int64_t)g.nchunks * g.NH);
  const int cnt = coherent_load(g.seg_count);
  if (cnt < 0 || cnt > g.seg_bound) {
    lds_global_walk<DROP>(g, k, c, h);
    return;
  }
  if (k >= cnt) return;
  const int n0 = coherent_load(g.segs + k), R = coherent_load(g.segs + k + 1) - n0;
  if (R <= 0) return;
  const int tid = threadIdx.x;
  const int F4 = g.Fp / 4;
  if (tid < kDegBins) bins[tid] = 0;
  // stage: 4 lanes per row (64 B); pieces past the head's padded row end stage zeros. Every
  // load of the prologue (the <= 9 row pieces of this thread and its <= 3 row-pointer pairs) is
  // issued before the first is waited on: with one workgroup per CU nothing else covers this
  // phase, and a load / wait / store loop paid one memory round trip per 256 rows.
  constexpr int kStage = kLdsRows / 256;
  float4 st[kStage];
  {
    // unconditional loads of clamped addresses (a guarded load made the compiler wait for it
    // before the next one went out), zeroed when consumed
    const int q = tid & 3;
    const int f4 = c * 4 + q;
    const float4* src = (const float4*)(g.rows + (int64_t)h * g.Fp) + min(f4, F4 - 1);
    const int64_t rs4 = g.row_stride / 4;
#pragma unroll
    for (int i = 0; i < kStage; ++i)
      st[i] = src[(int64_t)(n0 + min((tid >> 2) + 256 * i, R - 1)) * rs4];
  }
  int lo[3], hi[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int d = tid + 1024 * t;
    lo[t] = 0; hi[t] = 0;
    if (d <= R) lo[t] = g.rowptr[n0 + d];
    if (d < R) hi[t] = g.rowptr[n0 + d + 1];
  }
#pragma unroll
  for (int i = 0; i < kStage; ++i) {
    const int r = (tid >> 2) + 256 * i;
    if (r < R) img[r * 4 + (tid & 3)] = c * 4 + (tid & 3) < F4 ? st[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // destinations grouped by in-degree (a counting sort in LDS), so the 16 destinations a wave
  // walks together have similar trip counts: the walk's padding to the longest segment of the
  // 16 drops from ~1.7x (random degrees) to ~1.1-1.2x. The order inside a bucket is whatever
  // the LDS atomics give; every destination is still summed by one quad in CSR order, so the
  // result does not depend on it.
  int degs[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int d = tid + 1024 * t;
    if (d <= R) lrp[d] = lo[t];
    degs[t] = d < R ? min(hi[t] - lo[t], kDegBins - 1) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (degs[t] >= 0) atomicAdd(&bins[degs[t]], 1);
  __syncthreads();
  if (tid < 64) {   // exclusive scan of the 64 bucket counts (one wave)
    const int v = bins[tid];
    int x = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (tid >= off) x += y;
    }
    bins[tid] = x - v;
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (degs[t] >= 0) order[atomicAdd(&bins[degs[t]], 1)] = (unsigned short)(tid + 1024 * t);
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6, q = lane & 3, j = lane >> 2;
  const int2* rh = g.rec + (int64_t)h * g.E_bound;
  const int qb = 16 * q - 64 * n0;   // image byte of (source s, piece q) = 64 s + 16 q - 64 n0
  const char* imgb = (const char*)img;
  const int f0 = c * kChunk + q * 4;   // this lane's first feature in the head's row
  constexpr int G = 4 * RPL;           // records per quad per group
  // records as raw 64-bit loads issued from inline asm and retired by counted vmcnt waits: the
  // compiler sinks ordinary loads to just before their use (at the 128-VGPR cap it would rather
  // wait than keep a group in flight), which left every group's latency exposed. The wait asm
  // takes the loaded registers as in/out operands, so no use can be scheduled above it. Groups
  // go in pairs through a flattened loop over the wave's destination sets: step A consumes the
  // pair in (ra, rb) while the next pair loads into (rc, rd), step B the reverse, so every
  // register keeps one role and a pair is issued a whole pair ahead of its use (the next set's
  // first pair during a set's last one). Targets are selected, not branched on, so every path
  // issues the same loads (tools/check_asm_loads.py checks that no register is touched while
  // its load is in flight).
  uint64_t ra[RPL], rb[RPL], rc[RPL], rd[RPL];
  auto issue = [&](uint64_t (&r)[RPL], int e0, int lim) {
#pragma unroll
    for (int u = 0; u < RPL; ++u) r[u] = load_rec(rh, min((e0 + q * RPL + u) * 8, lim));
  };
  // this lane's destination of the set starting at d0 (segment [e, end); lim: its last record)
  // and the set's wave-uniform count of record pairs (at least 1)
  auto dest = [&](int d0, bool& live, int& dl, int& e, int& end, int& lim) {
    live = d0 + j < R;
    dl = live ? (int)order[d0 + j] : 0;
    e = live ? lrp[dl] : 0;
    end = live ? lrp[dl + 1] : 0;
    lim = (end > 0 ? end - 1 : 0) * 8;
  };
  auto pairs_of = [&](int e, int end) {
    int need = (end - e + 2 * G - 1) / (2 * G);
    for (int off = 4; off < 64; off <<= 1) need = max(need, __shfl_xor(need, off));
    return max(uni(need), 1);
  };
  int d0 = uni(wave * 16);
  if (d0 < R) {
    bool live, live1;
    int dl, e, end, lim, dl1, e1, end1, lim1;
    dest(d0, live, dl, e, end, lim);
    dest(d0 + 256, live1, dl1, e1, end1, lim1);
    int left = pairs_of(e, end);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    issue(ra, e, lim);
    issue(rb, e + G, lim);
    auto consume = [&](const uint64_t (&cur)[RPL], int e0) {
#pragma unroll
      for (int u = 0; u < RPL; ++u) {
        const bool ok = e0 + q * RPL + u < end;
        const int cx = ok ? (int)(uint32_t)cur[u] : 64 * n0;
        const int cy = ok ? (int)(uint32_t)(cur[u] >> 32) : 0;
#define GATX_LDS_STEP(T)                                                        \
        {                                                                       \
          const float4 v = *(const float4*)(imgb + (quad_bcast<T>(cx) + qb));   \
          acc = fma4(__int_as_float(quad_bcast<T>(cy)), v, acc);                \
        }
        GATX_LDS_STEP(0) GATX_LDS_STEP(1) GATX_LDS_STEP(2) GATX_LDS_STEP(3)
#undef GATX_LDS_STEP
      }
    };
    // one pair: consume (c0, c1), prefetch the pair after it into (p0, p1); true when the
    // wave's last set is done
    auto step = [&](uint64_t (&c0)[RPL], uint64_t (&c1)[RPL], uint64_t (&p0)[RPL],
                    uint64_t (&p1)[RPL]) {
      const bool more = left > 1;
      const int pe = more ? e + 2 * G : e1, pl = more ? lim : lim1;
      issue(p0, pe, pl);
      issue(p1, pe + G, pl);
      wait_vm<3 * RPL>(c0);   // c0 landed; c1, p0, p1 in flight
      consume(c0, e);
      wait_vm<2 * RPL>(c1);
      consume(c1, e + G);
      e += 2 * G;
      left = uni(left - 1);   // (kept provably uniform: the set loop stays scalar control flow)
      if (left > 0) return false;
      if (live && f0 < g.F) lds_store<DROP>(g, n0 + dl, (int64_t)h * g.F + f0, f0, acc);
      d0 = uni(d0 + 256);
      if (d0 >= R) return true;
      live = live1; dl = dl1; e = e1; end = end1; lim = lim1;
      dest(d0 + 256, live1, dl1, e1, end1, lim1);
      left = pairs_of(e, end);
      acc = make_float4(0.f, 0.f, 0.f, 0.f);
      return false;
    };
    for (;;) {
      if (step(ra, rb, rc, rd)) break;
      if (step(rc, rd, ra, rb)) break;
    }
  }
  wait_vm<0>(ra);   // nothing may still write these registers after the walk
  wait_vm<0>(rb);
  wait_vm<0>(rc);
  wait_vm<0>(rd);
}


// ---- head mean (round 6): PPI's last layer, out[n] = mean_h sum_e alpha~[e,h] Wh[src,h,:] + bias
// (models/gat_layer.py:117-135 with concat=False). One workgroup per (node block, 16-float chunk,
// destination range): the heads are staged one after another into the same image and every
// head's walk adds into the same registers, so the head mean is fused, with no per-head partials
// in memory and no cross-workgroup combine. 12 waves (768 threads: 168 VGPRs per lane) hold four
// float4 set accumulators per lane across the heads, so a range is at most 768 destinations and
// PPI's 2245-node blocks split into three: 20 blocks x 8 chunks x 3 ranges = 480 workgroups.
// Each head's first record pair is issued before that head's rows are staged, so the two memory
// round trips overlap.
constexpr int kMeanThreads = 768;
constexpr int kMeanWaves = kMeanThreads / 64;
constexpr int kMeanStride = 16 * kMeanWaves;              // destinations per sweep of the waves
constexpr int kMeanSets = 4;                              // sweeps (set accumulators per lane)
constexpr int kMeanRange = kMeanStride * kMeanSets;       // 768 destinations per workgroup
constexpr int kMeanStage = (kLdsRows + kMeanThreads / 4 - 1) / (kMeanThreads / 4);
static_assert(kMeanRange <= kMeanThreads, "the degree sort gives each thread one destination");

// fallback of the head-mean walk (see lds_global_walk): node range split evenly, rows from
// global memory, heads summed in order
template <bool DROP>
__device__ __attribute__((always_inline)) void lds_global_walk_mean(const LdsArgs& g,
                                                                    int64_t unit, int64_t units,
                                                                    int c) {
  const int64_t per = ceil_div(g.N, units);
  const int64_t n0 = unit * per;
  const int64_t R = min(per, g.N - n0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane & 3, j = lane >> 2;
  const int f0 = c * kChunk + q * 4;
  const float inv = 1.f / (float)g.NH;
  for (int64_t d0 = wave * 16; d0 < R; d0 += kMeanStride) {
    if (d0 + j >= R) continue;
    const int64_t n = n0 + d0 + j;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (f0 < g.Fp)
      for (int h = 0; h < g.NH; ++h) {
        const int2* rh = g.rec + (int64_t)h * g.E_bound;
        const float* base = g.rows + (int64_t)h * g.Fp + f0;
        float4 ah = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int e = g.rowptr[n], end = g.rowptr[n + 1]; e < end; ++e) {
          const int2 r = rh[e];
          const float4 v = *(const float4*)(base + (int64_t)(r.x >> 6) * g.row_stride);
          ah = fma4(__int_as_float(r.y), v, ah);
        }
        acc = add4(acc, ah);
      }
    if (f0 < g.F) lds_store<DROP>(g, n, f0, f0, acc * inv);
  }
}

template <int RPL, bool DROP>
__global__ void __launch_bounds__(kMeanThreads) edge_lds_mean_kernel(LdsArgs g) {
  __shared__ __attribute__((aligned(16))) float4 img[kLdsRows * 4];
  __shared__ unsigned short order[kMeanRange];   // the range's destinations, grouped by degree
  __shared__ int lrp[kMeanRange + 1];             // the range's row pointers
  __shared__ int bins[kDegBins];
  const int64_t b = xcd_contiguous(blockIdx.x, gridDim.x);   // the ranges and chunks of one
  const int nr = g.nranges;                                   // block run on one XCD: its
  const int rr = (int)(b % nr);                               // records stay in that L2
  const int c = (int)((b / nr) % g.nchunks);
  const int64_t k = b / ((int64_t)nr * g.nchunks);
  const int cnt = coherent_load(g.seg_count);
  if (cnt < 0 || cnt > g.seg_bound) {
    lds_global_walk_mean<DROP>(g, k * nr + rr, g.seg_bound * nr, c);
    return;
  }
  if (k >= cnt) return;
  const int n0 = coherent_load(g.segs + k), R = coherent_load(g.segs + k + 1) - n0;
  if (R <= 0) return;
  const int r0 = (int)((int64_t)R * rr / nr);
  const int Rr = (int)((int64_t)R * (rr + 1) / nr) - r0;   // <= ceil(kLdsRows / nr) <= kMeanRange
  if (Rr <= 0) return;
  const int tid = threadIdx.x;
  const int F4 = g.Fp / 4;
  if (tid < kDegBins) bins[tid] = 0;
  int deg = -1;
  if (tid < Rr) {
    const int lo = g.rowptr[n0 + r0 + tid], hi = g.rowptr[n0 + r0 + tid + 1];
    lrp[tid] = lo;
    if (tid == Rr - 1) lrp[Rr] = hi;
    deg = min(hi - lo, kDegBins - 1);
  }
  __syncthreads();
  if (deg >= 0) atomicAdd(&bins[deg], 1);
  __syncthreads();
  if (tid < 64) {
    const int v = bins[tid];
    int x = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (tid >= off) x += y;
    }
    bins[tid] = x - v;
  }
  __syncthreads();
  if (deg >= 0) order[atomicAdd(&bins[deg], 1)] = (unsigned short)tid;
  const int lane = tid & 63, wave = tid >> 6, q = lane & 3, j = lane >> 2;
  const int qb = 16 * q - 64 * n0;
  const char* imgb = (const char*)img;
  const int f0 = c * kChunk + q * 4;
  constexpr int G = 4 * RPL;
  const int64_t rs4 = g.row_stride / 4;
  const bool walker = wave * 16 < Rr;   // wave-uniform: this wave has destinations
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, a2 = a0, a3 = a0;
  uint64_t ra[RPL], rb[RPL], rc[RPL], rd[RPL];
  // records of head h at byte hoff = 8 E_bound h past g.rec (the asm loads' scalar base: a kernel
  // argument; 8 NH E_bound < 2^32, checked by the entry point)
  uint32_t hoff = 0;
  const int2* const rec0 = g.rec;
  auto issue = [&](uint64_t (&r)[RPL], int e0, int lim) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < RPL; ++u)
      r[u] = load_rec(rec0, (int)(hoff + (uint32_t)min((e0 + q * RPL + u) * 8, lim)));
  };
  auto dest = [&](int d0, int& e, int& end, int& lim) __attribute__((always_inline)) {
    const bool live = d0 + j < Rr;
    const int dl = live ? (int)order[d0 + j] : 0;
    e = live ? lrp[dl] : 0;
    end = live ? lrp[dl + 1] : 0;
    lim = (end > 0 ? end - 1 : 0) * 8;
  };
  auto pairs_of = [&](int e, int end) __attribute__((always_inline)) {
    int need = (end - e + 2 * G - 1) / (2 * G);
    for (int off = 4; off < 64; off <<= 1) need = max(need, __shfl_xor(need, off));
    return max(uni(need), 1);
  };
  for (int h = 0; h < g.NH; ++h) {
    __syncthreads();   // h = 0: order / lrp written; h > 0: every wave is done with head h - 1
    hoff = (uint32_t)uni((int)((uint32_t)h * (uint32_t)g.E_bound * 8u));
    // this head's first record pair, in flight while its rows are staged
    int e = 0, end = 0, lim = 0, e1 = 0, end1 = 0, lim1 = 0;
    int d0 = uni(wave * 16);
    if (walker) {
      dest(d0, e, end, lim);
      dest(d0 + kMeanStride, e1, end1, lim1);
      issue(ra, e, lim);
      issue(rb, e + G, lim);
    }
    {
      const int f4 = c * 4 + (tid & 3);
      const float4* src = (const float4*)(g.rows + (int64_t)h * g.Fp) + min(f4, F4 - 1);
      float4 st[kMeanStage];
#pragma unroll
      for (int i = 0; i < kMeanStage; ++i)
        st[i] = src[(int64_t)(n0 + min((tid >> 2) + kMeanThreads / 4 * i, R - 1)) * rs4];
#pragma unroll
      for (int i = 0; i < kMeanStage; ++i) {
        const int r = (tid >> 2) + kMeanThreads / 4 * i;
        if (r < R) img[r * 4 + (tid & 3)] = f4 < F4 ? st[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    __syncthreads();
    if (walker) {
      int left = pairs_of(e, end);
      int s = 0;   // the wave's set index (uniform)
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      auto consume = [&](const uint64_t (&cur)[RPL], int e0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
          const bool ok = e0 + q * RPL + u < end;
          const int cx = ok ? (int)(uint32_t)cur[u] : 64 * n0;
          const int cy = ok ? (int)(uint32_t)(cur[u] >> 32) : 0;
#define GATX_LDS_STEP(T)                                                        \
          {                                                                     \
            const float4 v = *(const float4*)(imgb + (quad_bcast<T>(cx) + qb)); \
            acc = fma4(__int_as_float(quad_bcast<T>(cy)), v, acc);              \
          }
          GATX_LDS_STEP(0) GATX_LDS_STEP(1) GATX_LDS_STEP(2) GATX_LDS_STEP(3)
#undef GATX_LDS_STEP
        }
      };
      auto step = [&](uint64_t (&c0)[RPL], uint64_t (&c1)[RPL], uint64_t (&p0)[RPL],
                      uint64_t (&p1)[RPL]) __attribute__((always_inline)) {
        const bool more = left > 1;
        const int pe = more ? e + 2 * G : e1, pl = more ? lim : lim1;
        issue(p0, pe, pl);
        issue(p1, pe + G, pl);
        wait_vm<3 * RPL>(c0);
        consume(c0, e);
        wait_vm<2 * RPL>(c1);
        consume(c1, e + G);
        e += 2 * G;
        left = uni(left - 1);
        if (left > 0) return false;
        // the set's sum into its accumulator (selects, not branches: static registers)
        a0 = s == 0 ? add4(a0, acc) : a0;
        a1 = s == 1 ? add4(a1, acc) : a1;
        a2 = s == 2 ? add4(a2, acc) : a2;
        a3 = s == 3 ? add4(a3, acc) : a3;
        s = uni(s + 1);
        d0 = uni(d0 + kMeanStride);
        if (d0 >= Rr) return true;
        e = e1; end = end1; lim = lim1;
        dest(d0 + kMeanStride, e1, end1, lim1);
        left = pairs_of(e, end);
        acc = make_float4(0.f, 0.f, 0.f, 0.f);
        return false;
      };
      for (;;) {
        if (step(ra, rb, rc, rd)) break;
        if (step(rc, rd, ra, rb)) break;
      }
      wait_vm<0>(ra);   // the pair prefetched past the last set lands before the next head
      wait_vm<0>(rb);
      wait_vm<0>(rc);
      wait_vm<0>(rd);
    }
  }
  if (!walker || f0 >= g.F) return;
  const float inv = 1.f / (float)g.NH;
#pragma unroll
  for (int s = 0; s < kMeanSets; ++s) {
    const int d = wave * 16 + kMeanStride * s + j;
    if (d < Rr) {
      const float4 a = s == 0 ? a0 : (s == 1 ? a1 : (s == 2 ? a2 : a3));
      lds_store<DROP>(g, n0 + r0 + (int)order[d], f0, f0, a * inv);
    }
  }
}
}  // namespace

extern "C" int gatx_edge_lds_rows(void) { return kLdsRows; }

extern "C" int gatx_edge_records(const float* S, const uint32_t* M_ord, const int32_t* rowptr,
                                 const int32_t* col, const int32_t* perm, int64_t N,
                                 int64_t E_bound, int NH, int const_att, float dropout_p,
                                 const uint64_t* seed, void* rec, float* den, float* alpha,
                                 long long* argmax, gatx_stream_t s) {
  GATX_REQUIRE(N >= 0 && E_bound >= 0 && NH >= 1 && NH <= 8, "edge_records: bad arguments");
  GATX_REQUIRE(dropout_p == 0.f || seed != nullptr, "edge_records: dropout needs its seed");
  if (N == 0) return 0;
  RecArgs g;
  g.S = S; g.M_ord = M_ord; g.rowptr = rowptr; g.col = col; g.perm = perm;
  g.N = N; g.E_bound = E_bound; g.NH = NH; g.const_att = const_att;
  g.p_drop = dropout_p; g.seed = seed; g.rec = (int2*)rec; g.den = den; g.alpha = alpha;
  g.argmax = argmax;
  const unsigned grid = (unsigned)ceil_div(N, (int64_t)4);
  hipStream_t st = (hipStream_t)s;
  switch (NH) {
    case 1: edge_records_kernel<1><<<grid, 256, 0, st>>>(g); break;
    case 2: edge_records_kernel<2><<<grid, 256, 0, st>>>(g); break;
    case 3: edge_records_kernel<3><<<grid, 256, 0, st>>>(g); break;
    case 4: edge_records_kernel<4><<<grid, 256, 0, st>>>(g); break;
    case 5: edge_records_kernel<5><<<grid, 256, 0, st>>>(g); break;
    case 6: edge_records_kernel<6><<<grid, 256, 0, st>>>(g); break;
    case 7: edge_records_kernel<7><<<grid, 256, 0, st>>>(g); break;
    default: edge_records_kernel<8><<<grid, 256, 0, st>>>(g); break;
  }
  GATX_LAUNCH_CHECK("edge_records");
  return 0;
}

extern "C" int gatx_edge_records_src(const float* S, const uint32_t* M_ord, const float* den,
                                     const int32_t* srowptr, const int32_t* scol,
                                     const int32_t* seid, const int32_t* perm, int64_t N,
                                     int64_t E_bound, int NH, int const_att, float dropout_p,
                                     const uint64_t* seed, const float* g_raw, float* G_aug,
                                     int64_t ldg, int64_t Dp, void* rec, gatx_stream_t s) {
  GATX_REQUIRE(N >= 0 && E_bound >= 0 && NH >= 1 && NH <= 8 && N < (1ll << 25),
               "edge_records_src: bad arguments");
  GATX_REQUIRE(dropout_p == 0.f || seed != nullptr, "edge_records_src: dropout needs its seed");
  if (N == 0) return 0;
  SrcRecArgs g;
  g.S = S; g.M_ord = M_ord; g.den = den; g.srowptr = srowptr; g.scol = scol; g.seid = seid;
  g.perm = perm; g.N = N; g.E_bound = E_bound; g.NH = NH; g.const_att = const_att;
  g.p_drop = dropout_p; g.seed = seed; g.g_raw = const_att ? nullptr : g_raw; g.G_aug = G_aug;
  g.ldg = ldg; g.Dp = Dp; g.rec = (int2*)rec;
  const unsigned grid = (unsigned)ceil_div(N, (int64_t)4);
  hipStream_t st = (hipStream_t)s;
  switch (NH) {
    case 1: edge_records_src_kernel<1><<<grid, 256, 0, st>>>(g); break;
    case 2: edge_records_src_kernel<2><<<grid, 256, 0, st>>>(g); break;
    case 3: edge_records_src_kernel<3><<<grid, 256, 0, st>>>(g); break;
    case 4: edge_records_src_kernel<4><<<grid, 256, 0, st>>>(g); break;
    case 5: edge_records_src_kernel<5><<<grid, 256, 0, st>>>(g); break;
    case 6: edge_records_src_kernel<6><<<grid, 256, 0, st>>>(g); break;
    case 7: edge_records_src_kernel<7><<<grid, 256, 0, st>>>(g); break;
    default: edge_records_src_kernel<8><<<grid, 256, 0, st>>>(g); break;
  }
  GATX_LAUNCH_CHECK("edge_records_src");
  return 0;
}

extern "C" int gatx_edge_lds_forward(const float* rows, int64_t row_stride,
                                     const int32_t* rowptr, int64_t N, const void* rec,
                                     int64_t E_bound, const int32_t* segs,
                                     const int32_t* seg_count, int64_t seg_bound, int NH, int F,
                                     const float* bias, float* out, int64_t out_ld,
                                     const float* resid, int64_t resid_ld, int elu,
                                     float out_p, const uint64_t* out_seed, gatx_stream_t s) {
  const int Fp = (int)round_up(F, 4);
  GATX_REQUIRE(NH >= 1 && F >= 1 && N >= 0 && seg_bound >= 0 && E_bound < (1ll << 28) &&
                   row_stride >= (int64_t)NH * Fp &&
                   row_stride % 4 == 0 && (uintptr_t)rows % 16 == 0,
               "edge_lds_forward: bad arguments");
  GATX_REQUIRE(out_p == 0.f || out_seed != nullptr, "edge_lds_forward: dropout needs its seed");
  if (seg_bound == 0) return 0;
  LdsArgs g;
  g.rows = rows; g.row_stride = row_stride; g.rowptr = rowptr; g.rec = (const int2*)rec;
  g.E_bound = E_bound; g.segs = segs; g.seg_count = seg_count; g.seg_bound = seg_bound;
  g.N = N;
  g.NH = NH; g.F = F; g.Fp = Fp; g.nchunks = (int)ceil_div(Fp, kChunk);
  g.bias = bias; g.out = out; g.out_ld = out_ld; g.resid = resid; g.resid_ld = resid_ld;
  g.elu = elu; g.out_p = out_p; g.out_seed = out_seed;
  g.ocols = (int64_t)NH * F; g.nranges = 1;
  auto al = [](const void* p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 16 == 0 && ld % 4 == 0); };
  g.vec_out = (F % 4 == 0) && al(out, out_ld) && al(resid, resid_ld) && al(bias, 0);
  const int64_t blocks = seg_bound * NH * g.nchunks;
  GATX_REQUIRE(blocks < (1ll << 31), "edge_lds_forward: too many workgroups");
  if (out_p > 0.f)
    edge_lds_kernel<kRPL, true><<<(unsigned)blocks, 1024, 0, (hipStream_t)s>>>(g);
  else
    edge_lds_kernel<kRPL, false><<<(unsigned)blocks, 1024, 0, (hipStream_t)s>>>(g);
  GATX_LAUNCH_CHECK("edge_lds_forward");
  return 0;
}

extern "C" int gatx_edge_lds_mean_forward(const float* rows, int64_t row_stride,
                                          const int32_t* rowptr, int64_t N, const void* rec,
                                          int64_t E_bound, const int32_t* segs,
                                          const int32_t* seg_count, int64_t seg_bound, int NH,
                                          int F, const float* bias, float* out, int64_t out_ld,
                                          const float* resid, int64_t resid_ld, int elu,
                                          float out_p, const uint64_t* out_seed,
                                          gatx_stream_t s) {
  const int Fp = (int)round_up(F, 4);
  GATX_REQUIRE(NH >= 1 && NH <= 8 && F >= 1 && N >= 0 && seg_bound >= 0 &&
                   E_bound < (1ll << 28) && row_stride >= (int64_t)NH * Fp &&
                   row_stride % 4 == 0 && (uintptr_t)rows % 16 == 0,
               "edge_lds_mean_forward: bad arguments");
  // (a head-mean layer feeding another layer's input dropout takes the L2-gather pass: the
  // dropout variant of this kernel ran out of scalar registers for the records' base)
  GATX_REQUIRE(out_p == 0.f, "edge_lds_mean_forward: no fused output dropout");
  GATX_REQUIRE((int64_t)NH * E_bound * 8 < (1ll << 32),
               "edge_lds_mean_forward: records past 32-bit offsets");
  if (seg_bound == 0) return 0;
  LdsArgs g;
  g.rows = rows; g.row_stride = row_stride; g.rowptr = rowptr; g.rec = (const int2*)rec;
  g.E_bound = E_bound; g.segs = segs; g.seg_count = seg_count; g.seg_bound = seg_bound;
  g.N = N;
  g.NH = NH; g.F = F; g.Fp = Fp; g.nchunks = (int)ceil_div(Fp, kChunk);
  g.bias = bias; g.out = out; g.out_ld = out_ld; g.resid = resid; g.resid_ld = resid_ld;
  g.elu = elu; g.out_p = out_p; g.out_seed = out_seed;
  g.ocols = F;
  g.nranges = (int)ceil_div(kLdsRows, kMeanRange);   // every block's range fits kMeanRange
  auto al = [](const void* p, int64_t ld) { return p == nullptr || ((uintptr_t)p % 16 == 0 && ld % 4 == 0); };
  g.vec_out = (F % 4 == 0) && al(out, out_ld) && al(resid, resid_ld) && al(bias, 0);
  const int64_t blocks = seg_bound * g.nranges * g.nchunks;
  GATX_REQUIRE(blocks < (1ll << 31), "edge_lds_mean_forward: too many workgroups");
  edge_lds_mean_kernel<kRPL, false><<<(unsigned)blocks, kMeanThreads, 0, (hipStream_t)s>>>(g);
  GATX_LAUNCH_CHECK("edge_lds_mean_forward");
  return 0;
}

}  // namespace gatx
