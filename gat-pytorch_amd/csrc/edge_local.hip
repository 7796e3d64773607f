// Graph-local edge pass: the attention + aggregation of models/gat_layer.py:66-127 for the
// destinations of self-contained node windows, with the gathered rows staged in LDS.
//
// A batch of graphs (PPI, PATTERN: models/GATModel.py:273-287 collates them into one disjoint
// union) is block-diagonal: every edge of a destination in graph g comes from a source in g. The
// edge pass of csrc/edge_fwd.hip gathers each edge's source row from L2 (~16 TB/s, the guide's
// L2-gather ceiling); here one workgroup owns (window, head, 16-float chunk of the head's row),
// loads that chunk of every source row of the window into LDS once (64 B per node), and every
// edge then reads its source chunk from LDS (~150 TB/s aggregate) — no per-edge L2 traffic but
// the CSR itself.
//
//  * gatx_graph_windows: cuts of the node order that no edge crosses (no destination left of the
//    cut has a source right of it, and vice versa) split the nodes into components; a component
//    of at most GATX_LOCAL_MAX_NODES nodes is a window (its nodes flagged in_window), larger ones
//    (Cora, R-MAT: one component) stay on the generic pass. Device-side, no host sync.
//  * edge_local_kernel: lanes 4j..4j+3 of a wave own destination slot j (16 per wave, 256 per
//    1024-thread workgroup); lane q holds float4 q of the chunk. Edges are taken 8 at a time:
//    each lane of the quad loads two edges' source ids and computes their attention weights
//    ex = exp(0.01 (s_src[src] + s_dst[n] - M)) (s_src from an LDS copy of the window's scores),
//    then the quad broadcasts (DPP) every edge's id and weight and accumulates the chunk
//    ex * Wh[src] from LDS. den = sum ex per destination; the normalisation 1/(den + 1e-8) and the
//    epilogue (bias, residual, ELU, next layer's dropout) run once per destination. Attention
//    dropout uses the same counter-based mask as the generic pass (edge id = position in
//    edge_index').
//  * head mean (concat = 0): every (window, head) writes its normalised head output to a
//    [NH][N][Fp] buffer; local_mean_combine_kernel sums the heads in order, / NH, + bias, epilogue.
#include "gatx_common.h"

namespace gatx {
namespace {

constexpr int kLocalMaxNodes = 2368;   // 64 B row chunk + 4 B score per node: 161,024 B of LDS
constexpr int kLocalThreads = 1024;    // 16 waves x 16 destination slots

// ------------------------------------------------------------------ window plan
// diff[lo + 1] += 1, diff[hi + 1] -= 1 for the node interval [lo, hi] each destination's edges span
__global__ void __launch_bounds__(256) window_span_kernel(const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col,
                                                          int64_t N, int32_t* __restrict__ diff) {
  const int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (d >= N) return;
  int lo = (int)d, hi = (int)d;
  const int beg = rowptr[d], end = rowptr[d + 1];
  for (int e = beg; e < end; ++e) {
    const int s = col[e];
    lo = min(lo, s);
    hi = max(hi, s);
  }
  if (hi > lo) {
    atomicAdd(&diff[lo + 1], 1);
    atomicAdd(&diff[hi + 1], -1);
  }
}

__global__ void __launch_bounds__(256) zero_i32_kernel(int32_t* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = 0;
}

// Block-wide inclusive scan of one int per thread (256 threads); *total = the block's sum.
__device__ inline int block_scan256(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  const int t0 = sh[0], t1 = sh[1], t2 = sh[2], t3 = sh[3];
  total = t0 + t1 + t2 + t3;
  const int base = (wave > 0 ? t0 : 0) + (wave > 1 ? t1 : 0) + (wave > 2 ? t2 : 0);
  __syncthreads();
  return base + x;
}

// sum of the first b entries of a per-block array (b <= a few hundred: a strided wave sum)
__device__ inline int prefix_of(const int32_t* __restrict__ v, int b, int* sh) {
  int s = 0;
  for (int i = threadIdx.x; i < b; i += 256) s += v[i];
  int tot;
  (void)block_scan256(s, sh, tot);
  return tot;
}

// per block of 256 nodes: the sum of diff
__global__ void __launch_bounds__(256) window_bsum_kernel(const int32_t* __restrict__ diff,
                                                          int64_t N, int32_t* __restrict__ bsum) {
  __shared__ int sh[4];
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int tot;
  (void)block_scan256(n < N ? diff[n] : 0, sh, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// cover[n] = sum_{i <= n} diff[i] (the edge spans crossing the boundary before node n);
// cut[n] = (n == 0 || cover[n] == 0); per block: the number of cuts
__global__ void __launch_bounds__(256) window_cut_kernel(const int32_t* __restrict__ diff,
                                                         const int32_t* __restrict__ bsum,
                                                         int64_t N, uint8_t* __restrict__ cut,
                                                         int32_t* __restrict__ csum) {
  __shared__ int sh[4];
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int base = prefix_of(bsum, blockIdx.x, sh);
  int tot;
  const int cover = base + block_scan256(n < N ? diff[n] : 0, sh, tot);
  const int c = (n < N && (n == 0 || cover == 0)) ? 1 : 0;
  if (n < N) cut[n] = (uint8_t)c;
  (void)block_scan256(c, sh, tot);
  if (threadIdx.x == 0) csum[blockIdx.x] = tot;
}

// component id of every node (cuts up to it - 1), the components' starts P[c] and P[C] = N,
// and the component count
__global__ void __launch_bounds__(256) window_cid_kernel(const uint8_t* __restrict__ cut,
                                                         const int32_t* __restrict__ csum,
                                                         int64_t N, int32_t* __restrict__ cid,
                                                         int32_t* __restrict__ P,
                                                         int32_t* __restrict__ count) {
  __shared__ int sh[4];
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int base = prefix_of(csum, blockIdx.x, sh);
  const int c = n < N ? cut[n] : 0;
  int tot;
  const int k = base + block_scan256(c, sh, tot) - 1;
  if (n < N) {
    cid[n] = k;
    if (c) P[k] = (int32_t)n;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    P[base + tot] = (int32_t)N;
    *count = base + tot;
  }
}

__global__ void __launch_bounds__(256) window_flag_kernel(const int32_t* __restrict__ cid,
                                                          const int32_t* __restrict__ P,
                                                          int64_t N, int T,
                                                          uint8_t* __restrict__ in_window) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int k = cid[n];
  in_window[n] = (P[k + 1] - P[k] <= T) ? 1 : 0;
}

// ------------------------------------------------------------------ local edge pass
struct LocalArgs {
  const float4* rows;      // Wh [N][row_stride4] float4s, head h at float4 h * Fp4
  int64_t row_stride4;
  int Fp4;                 // float4s per head (padded features / 4)
  int F, NH, nch;          // output features, heads, 16-float chunks per head
  const float* S;          // [N][2 NH]
  const uint32_t* M_ord;
  const int32_t* rowptr;
  const int32_t* col;
  const int32_t* perm;
  const int32_t* windows;  // [W][2] node ranges
  const int32_t* win_count;
  int64_t N;
  float p_drop;
  const uint64_t* seed;
  // concat epilogue: out[n][h F + f] = drop?(elu?(o + bias + resid))
  float* out;
  int64_t out_ld;
  const float* bias;
  const float* resid;
  int64_t resid_ld;
  int elu;
  float out_p;
  const uint64_t* out_seed;
  int64_t out_cols;
  int vec_out;
  float* den;              // [N][NH]
  float* part;             // head mean: [NH][N][Fp4 * 4] normalised head outputs
};

__device__ inline float local_out_drop(float v, const LocalArgs& g, int64_t n, int64_t col) {
  return dropout_keep(*g.out_seed, n * g.out_cols + col, g.out_p) ? v * (1.f / (1.f - g.out_p))
                                                                   : 0.f;
}

__device__ inline float local_epi(float v, const LocalArgs& g, int64_t n, int64_t col) {
  if (g.bias) v += g.bias[col];
  if (g.resid) v += g.resid[n * g.resid_ld + col];
  if (g.elu) v = elu_act(v);
  if (g.out_p > 0.f) v = local_out_drop(v, g, n, col);
  return v;
}

// broadcast lane u of each quad (DPP quad_perm)
template <int U>
__device__ inline int quad_bcast(int v) {
  return __builtin_amdgcn_mov_dpp(v, U | (U << 2) | (U << 4) | (U << 6), 0xf, 0xf, false);
}
template <int U>
__device__ inline float quad_bcastf(float v) {
  return __int_as_float(quad_bcast<U>(__float_as_int(v)));
}

// Per-destination prefetch of the software pipeline: the segment bounds, the destination score
// and the first batch of source ids (lane q: edges beg + q + 4j, j < kLocalB).
constexpr int kLocalB = 12;   // 48 edges per quad and batch: PPI's in-degrees are ~28 +- 5

struct LocalPrefetch {
  int beg, end;
  float sd;
  int src[kLocalB];
  int pos[kLocalB];
};

template <bool DROP, bool CONST_ATT>
__device__ inline void local_prefetch(const LocalArgs& g, int d, int b, int a, int h, int q,
                                      LocalPrefetch& f) {
  const bool dv = d < b;
  f.beg = dv ? g.rowptr[d] : 0;
  f.end = dv ? g.rowptr[d + 1] : 0;
  f.sd = (CONST_ATT || !dv) ? 0.f : g.S[(int64_t)d * 2 * g.NH + g.NH + h];
#pragma unroll
  for (int j = 0; j < kLocalB; ++j) {
    const int e = f.beg + q + 4 * j;
    const bool v = e < f.end;
    f.src[j] = v ? g.col[e] - a : 0;
    if (DROP) f.pos[j] = v ? g.perm[e] : 0;
  }
}

// ex * row chunk of kLocalB x 4 edges (lane q computed the weights of its own edges; the quad
// broadcasts every edge's source and weight)
template <bool DROP, bool CONST_ATT>
__device__ inline void local_batch(const int (&src)[kLocalB], const int (&pos)[kLocalB], int e0,
                                   int end, int q, float sd, float M, int NH, int h,
                                   uint64_t seed, float p, float drop_scale,
                                   const float* __restrict__ ssrc, const float4* __restrict__ tab,
                                   float4& acc, float& dl) {
  float w[kLocalB];
#pragma unroll
  for (int j = 0; j < kLocalB; ++j) {
    const bool v = e0 + q + 4 * j < end;
    float x = CONST_ATT ? 1.f : att_exp(ssrc[src[j]] + sd, M);
    x = v ? x : 0.f;
    dl += x;
    if (DROP) x = dropout_keep(seed, (int64_t)pos[j] * NH + h, p) ? x * drop_scale : 0.f;
    w[j] = x;
  }
#pragma unroll
  for (int j = 0; j < kLocalB; ++j) {
    if (e0 + 4 * j >= end) break;   // quad-uniform
    const int s0 = quad_bcast<0>(src[j]), s1 = quad_bcast<1>(src[j]),
              s2 = quad_bcast<2>(src[j]), s3 = quad_bcast<3>(src[j]);
    const float4 v0 = tab[s0 * 4 + q], v1 = tab[s1 * 4 + q], v2 = tab[s2 * 4 + q],
                 v3 = tab[s3 * 4 + q];
    acc = fma4(quad_bcastf<0>(w[j]), v0, acc);
    acc = fma4(quad_bcastf<1>(w[j]), v1, acc);
    acc = fma4(quad_bcastf<2>(w[j]), v2, acc);
    acc = fma4(quad_bcastf<3>(w[j]), v3, acc);
  }
}

template <bool DROP, bool CONST_ATT, bool MEAN>
__global__ void __launch_bounds__(kLocalThreads) edge_local_kernel(LocalArgs g) {
  __shared__ float4 tab[kLocalMaxNodes * 4];
  __shared__ float ssrc[kLocalMaxNodes];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slot = lane >> 2, q = lane & 3;
  const int NH = g.NH, nch = g.nch, S2 = 2 * NH;
  // items: (component, head, chunk) over every component of the plan; components larger than
  // kLocalMaxNodes are skipped (their nodes are on the generic pass)
  const int64_t items = (int64_t)(*g.win_count) * NH * nch;
  const float M = CONST_ATT ? 0.f : ord_to_float(*g.M_ord);
  const uint64_t seed = DROP ? *g.seed : 0ull;
  const float drop_scale = DROP ? 1.f / (1.f - g.p_drop) : 1.f;
  // chunk fastest, dealt so that each XCD (blocks b % 8) sweeps a contiguous range: the chunks of
  // one (component, head) share L2 lines of the rows
  const int64_t G = gridDim.x;
  const int64_t v0 = (G % 8 == 0) ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  for (int64_t it = v0; it < items; it += G) {
    const int64_t w = it / (NH * nch);
    const int rem = (int)(it - w * NH * nch);
    const int h = rem / nch, c = rem - h * nch;
    const int a = g.windows[w], b = g.windows[w + 1];
    const int nw = b - a;
    if (nw > kLocalMaxNodes) continue;   // block-uniform
    const int cq = c * 4 + q;          // this lane's float4 within the head's row
    const bool qv = cq < g.Fp4;
    // the first destination's prefetch goes out before the staging loads
    int d = a + wave * 16 + slot;
    LocalPrefetch cur;
    local_prefetch<DROP, CONST_ATT>(g, d, b, a, h, q, cur);
    // stage the window's chunk of every source row, and its source scores for head h
    {
      const float4* srcp = g.rows + (int64_t)h * g.Fp4 + (qv ? cq : 0);
      for (int i = tid >> 2; i < nw; i += kLocalThreads / 4) {
        float4 v = srcp[(int64_t)(a + i) * g.row_stride4];
        if (!qv) v = make_float4(0.f, 0.f, 0.f, 0.f);
        tab[i * 4 + q] = v;
      }
      if (!CONST_ATT)
        for (int i = tid; i < nw; i += kLocalThreads) ssrc[i] = g.S[(int64_t)(a + i) * S2 + h];
    }
    __syncthreads();
    // destinations d, d + 256, ... of this slot (the whole quad runs the loop together: DPP
    // broadcasts); the next destination's bounds, score and first source batch are loaded before
    // this one is computed
    for (; d - slot < b; d += kLocalThreads / 4) {
      LocalPrefetch nxt;
      local_prefetch<DROP, CONST_ATT>(g, d + kLocalThreads / 4, b, a, h, q, nxt);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      float dl = 0.f;
      local_batch<DROP, CONST_ATT>(cur.src, cur.pos, cur.beg, cur.end, q, cur.sd, M, NH, h, seed,
                                   g.p_drop, drop_scale, ssrc, tab, acc, dl);
      for (int e0 = cur.beg + 4 * kLocalB; e0 < cur.end; e0 += 4 * kLocalB) {   // long segments
        int sx[kLocalB], px[kLocalB];
#pragma unroll
        for (int j = 0; j < kLocalB; ++j) {
          const int e = e0 + q + 4 * j;
          const bool v = e < cur.end;
          sx[j] = v ? g.col[e] - a : 0;
          px[j] = (DROP && v) ? g.perm[e] : 0;
        }
        local_batch<DROP, CONST_ATT>(sx, px, e0, cur.end, q, cur.sd, M, NH, h, seed, g.p_drop,
                                     drop_scale, ssrc, tab, acc, dl);
      }
      // den: the quad's partial sums (each lane summed its own edges)
      dl += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(dl), 0xb1, 0xf, 0xf, false));
      dl += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(dl), 0x4e, 0xf, 0xf, false));
      const bool dv = d < b;
      if (dv) {
        if (c == 0 && q == 0) g.den[(int64_t)d * NH + h] = dl;
        const float inv = 1.f / (dl + kSoftmaxEps);
        const float4 o = acc * inv;
        const int f0 = cq * 4;           // feature index inside the head
        if (MEAN) {
          if (qv) *(float4*)(g.part + ((int64_t)h * g.N + d) * ((int64_t)g.Fp4 * 4) + f0) = o;
        } else if (f0 < g.F) {
          const int64_t cb = (int64_t)h * g.F + f0;
          float* orow = g.out + (int64_t)d * g.out_ld;
          if (g.vec_out) {
            float4 r = o;
            if (g.bias) r = add4(r, *(const float4*)(g.bias + cb));
            if (g.resid) r = add4(r, *(const float4*)(g.resid + (int64_t)d * g.resid_ld + cb));
            if (g.elu) r = make_float4(elu_act(r.x), elu_act(r.y), elu_act(r.z), elu_act(r.w));
            if (g.out_p > 0.f) {
              r.x = local_out_drop(r.x, g, d, cb);
              r.y = local_out_drop(r.y, g, d, cb + 1);
              r.z = local_out_drop(r.z, g, d, cb + 2);
              r.w = local_out_drop(r.w, g, d, cb + 3);
            }
            *(float4*)(orow + cb) = r;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (f0 + j < g.F) orow[cb + j] = local_epi(get4(o, j), g, d, cb + j);
          }
        }
      }
      cur = nxt;
    }
    __syncthreads();
  }
}

// Head mean of the windowed nodes: out[n][f] = epi(sum_h part[h][n][f] / NH + bias[f]) (heads
// summed in order; the generic pass's multi-pass order is also head order).
__global__ void __launch_bounds__(256) local_mean_combine_kernel(LocalArgs g,
                                                                 const uint8_t* __restrict__ in_window) {
  const int64_t Fpad = (int64_t)g.Fp4 * 4;
  const int64_t total = g.N * g.F;
  const float inv_nh = 1.f / (float)g.NH;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int64_t n = i / g.F, f = i - n * g.F;
    if (!in_window[n]) continue;
    float s = 0.f;
    for (int h = 0; h < g.NH; ++h) s += g.part[((int64_t)h * g.N + n) * Fpad + f];
    g.out[n * g.out_ld + f] = local_epi(s * inv_nh, g, n, f);
  }
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" int gatx_local_max_nodes(void) { return kLocalMaxNodes; }

extern "C" size_t gatx_graph_windows_workspace_bytes(int64_t N) {
  const int64_t nb = ceil_div(std::max<int64_t>(N, 1), 256);
  return (size_t)(2 * N + 2 * nb + 8) * sizeof(int32_t) + (size_t)round_up(N + 1, 16);
}

extern "C" int gatx_graph_windows(const int32_t* rowptr, const int32_t* col, int64_t N,
                                  int max_nodes, int32_t* windows, int32_t* win_count,
                                  uint8_t* in_window, void* workspace, size_t ws_bytes,
                                  gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  GATX_REQUIRE(N >= 0 && N < (1ll << 31), "graph_windows: bad node count");
  GATX_REQUIRE(max_nodes >= 1 && max_nodes <= kLocalMaxNodes,
               "graph_windows: max_nodes must be in [1, %d]", kLocalMaxNodes);
  GATX_REQUIRE(ws_bytes >= gatx_graph_windows_workspace_bytes(N), "graph_windows: workspace");
  // (zeroing by kernels: a hipMemsetAsync captured into a hipGraph was not re-run on replay —
  // the second replay saw the first one's span counts)
  if (N == 0) {
    zero_i32_kernel<<<1, 256, 0, st>>>(win_count, 1);
    GATX_LAUNCH_CHECK("graph_windows zero");
    return 0;
  }
  const int64_t nb = ceil_div(N, 256);
  GATX_REQUIRE(nb <= 4096, "graph_windows: more than 2^20 nodes");
  int32_t* diff = (int32_t*)workspace;   // N + 2
  int32_t* cid = diff + N + 2;           // N
  int32_t* bsum = cid + N;               // nb
  int32_t* csum = bsum + nb;             // nb
  uint8_t* cut = (uint8_t*)(csum + nb + 4);
  int32_t* P = windows;                  // the component starts, [N + 1] of the [N][2] buffer
  zero_i32_kernel<<<(unsigned)std::min<int64_t>(ceil_div(N + 2, 256), 1024), 256, 0, st>>>(diff,
                                                                                         N + 2);
  GATX_LAUNCH_CHECK("graph_windows zero");
  window_span_kernel<<<(unsigned)nb, 256, 0, st>>>(rowptr, col, N, diff);
  GATX_LAUNCH_CHECK("window_span");
  window_bsum_kernel<<<(unsigned)nb, 256, 0, st>>>(diff, N, bsum);
  GATX_LAUNCH_CHECK("window_bsum");
  window_cut_kernel<<<(unsigned)nb, 256, 0, st>>>(diff, bsum, N, cut, csum);
  GATX_LAUNCH_CHECK("window_cut");
  window_cid_kernel<<<(unsigned)nb, 256, 0, st>>>(cut, csum, N, cid, P, win_count);
  GATX_LAUNCH_CHECK("window_cid");
  window_flag_kernel<<<(unsigned)nb, 256, 0, st>>>(cid, P, N, max_nodes, in_window);
  GATX_LAUNCH_CHECK("window_flag");
  return 0;
}

extern "C" size_t gatx_edge_forward_local_part_bytes(int64_t N, int NH, int F, int concat) {
  return concat ? 0 : (size_t)NH * N * round_up(F, 4) * sizeof(float);
}

extern "C" int gatx_edge_forward_local(
    const float* rows, int64_t row_stride, const float* S, const uint32_t* M_ord,
    const int32_t* rowptr, const int32_t* col, const int32_t* perm, int64_t N, int NH, int F,
    int concat, int const_att, const float* bias, float p, const uint64_t* seed, float* out,
    int64_t out_ld, const float* resid, int64_t resid_ld, int elu, float* den, float out_p,
    const uint64_t* out_seed, const int32_t* windows, const int32_t* win_count,
    const uint8_t* in_window, int64_t max_items, float* part, gatx_stream_t s) {
  hipStream_t st = (hipStream_t)s;
  GATX_REQUIRE(NH >= 1 && F >= 1, "edge_forward_local: bad sizes");
  GATX_REQUIRE(row_stride % 4 == 0 && ((uintptr_t)rows % 16) == 0,
               "edge_forward_local: source rows must be float4-aligned");
  GATX_REQUIRE(row_stride >= (int64_t)NH * round_up(F, 4), "edge_forward_local: row stride");
  GATX_REQUIRE(p >= 0.f && p < 1.f && (p == 0.f || seed), "edge_forward_local: dropout");
  GATX_REQUIRE(out_p >= 0.f && out_p < 1.f && (out_p == 0.f || out_seed),
               "edge_forward_local: output dropout");
  GATX_REQUIRE(concat || bias == nullptr || NH == 1,
               "edge_forward_local: bias with head-mean needs num_heads == 1");
  GATX_REQUIRE(concat || (part && in_window), "edge_forward_local: head mean needs its buffer");
  if (N == 0 || max_items <= 0) return 0;
  LocalArgs g;
  g.rows = (const float4*)rows; g.row_stride4 = row_stride / 4;
  g.Fp4 = (int)(round_up(F, 4) / 4); g.F = F; g.NH = NH; g.nch = (int)ceil_div(g.Fp4, 4);
  g.S = S; g.M_ord = M_ord; g.rowptr = rowptr; g.col = col; g.perm = perm;
  g.windows = windows; g.win_count = win_count; g.N = N;
  g.p_drop = p; g.seed = seed;
  g.out = out; g.out_ld = out_ld; g.bias = bias; g.resid = resid; g.resid_ld = resid_ld;
  g.elu = elu; g.out_p = out_p; g.out_seed = out_seed; g.out_cols = concat ? (int64_t)NH * F : F;
  g.vec_out = concat && (F & 3) == 0 && out_ld % 4 == 0 && ((uintptr_t)out % 16) == 0 &&
              (!resid || (resid_ld % 4 == 0 && ((uintptr_t)resid % 16) == 0)) &&
              (!bias || ((uintptr_t)bias % 16) == 0);
  g.den = den; g.part = part;
  // one workgroup per CU (the LDS table), persistent over the (window, head, chunk) items
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const int64_t items_bound = max_items * NH * g.nch;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(items_bound, cus));
  const bool drop = p > 0.f, mean = !concat;
#define GATX_LOC(D, C, Mn) edge_local_kernel<D, C, Mn><<<grid, kLocalThreads, 0, st>>>(g)
  if (const_att) {
    if (drop) { if (mean) GATX_LOC(true, true, true); else GATX_LOC(true, true, false); }
    else { if (mean) GATX_LOC(false, true, true); else GATX_LOC(false, true, false); }
  } else {
    if (drop) { if (mean) GATX_LOC(true, false, true); else GATX_LOC(true, false, false); }
    else { if (mean) GATX_LOC(false, false, true); else GATX_LOC(false, false, false); }
  }
#undef GATX_LOC
  GATX_LAUNCH_CHECK("edge_local");
  if (mean) {
    const int64_t total = N * F;
    local_mean_combine_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0,
                                st>>>(g, in_window);
    GATX_LAUNCH_CHECK("local_mean_combine");
  }
  return 0;
}
