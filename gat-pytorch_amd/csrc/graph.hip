// Graph preprocessing on device: the self-loop rewrite of models/utils.py:47-67 and the
// destination-/source-ordered CSR the fused edge kernels stream.
//
// Everything is integer work (HBM-bound, no MFMA): a stats reduction, a stable compaction
// (prefix sum over the keep flags), a stable LSD radix sort by destination (rocPRIM), and
// boundary detection for rowptr. All orders are deterministic, so CSR segments list their
// edges in edge_index' order and per-segment float sums are bitwise reproducible.
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "gatx_common.h"

namespace gatx {
namespace {

template <typename I>
__device__ inline int64_t ld_idx(const void* p, int64_t i) {
  return (int64_t)((const I*)p)[i];
}

constexpr int kStatsBlocks = 1024;

// Per-block {min, max, self-loops} partials (no 64-bit atomics), reduced by stats_final_kernel.
template <typename I>
__global__ void __launch_bounds__(256) edge_stats_kernel(const void* ei, int64_t E, int64_t ld,
                                                         long long* part) {
  long long mn = LLONG_MAX, mx = LLONG_MIN, loops = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    long long s = ld_idx<I>(ei, i), d = ld_idx<I>(ei, ld + i);
    mn = min(mn, min(s, d));
    mx = max(mx, max(s, d));
    loops += (s == d);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (long long)__shfl_xor(mn, o));
    mx = max(mx, (long long)__shfl_xor(mx, o));
    loops += __shfl_xor(loops, o);
  }
  __shared__ long long red[3][4];
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { red[0][w] = mn; red[1][w] = mx; red[2][w] = loops; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      mn = min(mn, red[0][k]); mx = max(mx, red[1][k]); loops += red[2][k];
    }
    part[3 * blockIdx.x + 0] = mn;
    part[3 * blockIdx.x + 1] = mx;
    part[3 * blockIdx.x + 2] = loops;
  }
}

__global__ void __launch_bounds__(256) stats_final_kernel(const long long* part, int nb,
                                                          long long* stats) {
  long long mn = LLONG_MAX, mx = LLONG_MIN, loops = 0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    mn = min(mn, part[3 * b]); mx = max(mx, part[3 * b + 1]); loops += part[3 * b + 2];
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (long long)__shfl_xor(mn, o));
    mx = max(mx, (long long)__shfl_xor(mx, o));
    loops += __shfl_xor(loops, o);
  }
  __shared__ long long red[3][4];
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { red[0][w] = mn; red[1][w] = mx; red[2][w] = loops; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      mn = min(mn, red[0][k]); mx = max(mx, red[1][k]); loops += red[2][k];
    }
    stats[0] = mn; stats[1] = mx; stats[2] = loops;
  }
}

// keep flag of input edge i (1 = survives the self-loop rewrite)
template <typename I>
struct KeepFlag {
  const void* ei;
  int64_t ld;
  int drop_loops;
  __device__ int operator()(int64_t i) const {
    return drop_loops ? (ld_idx<I>(ei, i) != ld_idx<I>(ei, ld + i)) : 1;
  }
};

// Scatter kept edges to their compacted slot, append the loops (i, i), i < num_loops.
template <typename I>
__global__ void __launch_bounds__(256) compact_kernel(const void* ei, int64_t E, int64_t ld,
                                                       int drop_loops, const int32_t* pos,
                                                       int64_t num_loops, int64_t E2,
                                                       int64_t* ei_out, int32_t* src32,
                                                       int32_t* dst32, int32_t* iota) {
  const int64_t total = E + num_loops;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s, d, p;
    if (i < E) {
      s = ld_idx<I>(ei, i);
      d = ld_idx<I>(ei, ld + i);
      if (drop_loops && s == d) continue;
      p = pos[i];
    } else {
      s = d = i - E;
      p = E2 - num_loops + (i - E);
    }
    if (ei_out) { ei_out[p] = s; ei_out[E2 + p] = d; }
    src32[p] = (int32_t)s;
    dst32[p] = (int32_t)d;
    iota[p] = (int32_t)p;
  }
}

// rowptr from a sorted key array: rows (key[e-1], key[e]] start at e.
__global__ void __launch_bounds__(256) rowptr_kernel(const int32_t* keys, int64_t E2,
                                                      int64_t num_rows, int32_t* rowptr) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e <= E2;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = (e < E2) ? keys[e] : num_rows;
    int64_t kp = (e > 0) ? keys[e - 1] : -1;
    for (int64_t r = kp + 1; r <= k; ++r) rowptr[r] = (int32_t)e;
  }
}

__global__ void __launch_bounds__(256) gather_kernel(const int32_t* src, const int32_t* idx,
                                                      int64_t n, int32_t* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = src[idx[i]];
}

__global__ void __launch_bounds__(256) iota_kernel(int64_t n, int32_t* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)i;
}

inline unsigned grid_for(int64_t n, int block = 256, int64_t cap = 16384) {
  int64_t g = ceil_div(n > 0 ? n : 1, block);
  return (unsigned)(g < cap ? g : cap);
}

inline unsigned bits_for(int64_t n) {  // bits to represent values in [0, n)
  unsigned b = 1;
  while (b < 31 && ((int64_t)1 << b) < n) ++b;
  return b;
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t scan_bytes(int64_t E) {
  size_t bytes = 0;
  KeepFlag<int64_t> f{nullptr, 0, 1};
  auto it = rocprim::make_transform_iterator(rocprim::make_counting_iterator<int64_t>(0), f);
  (void)rocprim::exclusive_scan(nullptr, bytes, it, (int32_t*)nullptr, 0, (size_t)(E > 0 ? E : 1),
                          rocprim::plus<int32_t>(), (hipStream_t)0);
  return bytes;
}

size_t sort_bytes(int64_t n, unsigned bits) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (int32_t*)nullptr, (int32_t*)nullptr,
                            (int32_t*)nullptr, (int32_t*)nullptr, (unsigned)(n > 0 ? n : 1), 0,
                            bits, (hipStream_t)0);
  return bytes;
}

template <typename I>
int graph_build_impl(const void* ei, int64_t E, int64_t ld, int add_loops, int64_t num_loops,
                     int64_t N, int64_t E2, int64_t* ei_out, int32_t* rowptr, int32_t* col,
                     int32_t* rowidx, int32_t* perm, void* ws, size_t ws_bytes,
                     hipStream_t stream) {
  // workspace carve: pos [E] | src32 [E2] | dst32 [E2] | iota [E2] | rocprim temp
  char* p = (char*)ws;
  int32_t* pos = (int32_t*)p;   p += align256(sizeof(int32_t) * (E > 0 ? E : 1));
  int32_t* src32 = (int32_t*)p; p += align256(sizeof(int32_t) * (E2 > 0 ? E2 : 1));
  int32_t* dst32 = (int32_t*)p; p += align256(sizeof(int32_t) * (E2 > 0 ? E2 : 1));
  int32_t* iota = (int32_t*)p;  p += align256(sizeof(int32_t) * (E2 > 0 ? E2 : 1));
  size_t used = (size_t)(p - (char*)ws);
  GATX_REQUIRE(used <= ws_bytes, "graph_build: workspace too small");
  void* tmp = p;
  size_t tmp_bytes = ws_bytes - used;

  if (add_loops && E > 0) {
    KeepFlag<I> f{ei, ld, 1};
    auto it = rocprim::make_transform_iterator(rocprim::make_counting_iterator<int64_t>(0), f);
    size_t b = tmp_bytes;
    hipError_t r = rocprim::exclusive_scan(tmp, b, it, pos, 0, (size_t)E,
                                           rocprim::plus<int32_t>(), stream);
    if (r != hipSuccess) { set_error("exclusive_scan: %s", hipGetErrorString(r)); return (int)r; }
  } else if (E > 0) {
    iota_kernel<<<grid_for(E), 256, 0, stream>>>(E, pos);
    GATX_LAUNCH_CHECK("iota");
  }
  if (E + (add_loops ? num_loops : 0) > 0) {
    compact_kernel<I><<<grid_for(E + num_loops), 256, 0, stream>>>(
        ei, E, ld, add_loops, pos, add_loops ? num_loops : 0, E2, ei_out, src32, dst32, iota);
    GATX_LAUNCH_CHECK("compact");
  }
  if (E2 > 0) {
    size_t b = tmp_bytes;
    hipError_t r = rocprim::radix_sort_pairs(tmp, b, dst32, rowidx, iota, perm, (unsigned)E2, 0,
                                             bits_for(N), stream);
    if (r != hipSuccess) { set_error("radix_sort: %s", hipGetErrorString(r)); return (int)r; }
    gather_kernel<<<grid_for(E2), 256, 0, stream>>>(src32, perm, E2, col);
    GATX_LAUNCH_CHECK("gather col");
  }
  rowptr_kernel<<<grid_for(E2 + 1), 256, 0, stream>>>(rowidx, E2, N, rowptr);
  GATX_LAUNCH_CHECK("rowptr");
  return 0;
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" int gatx_edge_stats(const void* edge_index, int is64, int64_t E, int64_t ld,
                               int64_t* stats, void* workspace, gatx_stream_t s) {
  hipStream_t stream = (hipStream_t)s;
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(E, 256), kStatsBlocks));
  long long* part = (long long*)workspace;
  if (is64)
    edge_stats_kernel<int64_t><<<nb, 256, 0, stream>>>(edge_index, E, ld, part);
  else
    edge_stats_kernel<int32_t><<<nb, 256, 0, stream>>>(edge_index, E, ld, part);
  GATX_LAUNCH_CHECK("edge_stats");
  stats_final_kernel<<<1, 256, 0, stream>>>(part, nb, (long long*)stats);
  GATX_LAUNCH_CHECK("edge_stats_final");
  return 0;
}

extern "C" size_t gatx_edge_stats_workspace_bytes(void) {
  return (size_t)3 * sizeof(long long) * kStatsBlocks;
}

extern "C" size_t gatx_graph_build_workspace_bytes(int64_t E, int64_t E2, int64_t N) {
  size_t b = align256(sizeof(int32_t) * (E > 0 ? E : 1)) +
             3 * align256(sizeof(int32_t) * (E2 > 0 ? E2 : 1));
  size_t t = std::max(scan_bytes(E), sort_bytes(E2, bits_for(N)));
  return b + align256(t) + 256;
}

extern "C" int gatx_graph_build(const void* edge_index, int is64, int64_t E, int64_t ld,
                                int add_self_loops, int64_t num_loops, int64_t num_nodes,
                                int64_t E2, int64_t* edge_index_out, int32_t* rowptr,
                                int32_t* col, int32_t* rowidx, int32_t* perm, void* ws,
                                size_t ws_bytes, gatx_stream_t s) {
  GATX_REQUIRE(num_nodes >= 0 && num_nodes < INT32_MAX && E2 < INT32_MAX && E >= 0,
               "graph_build: sizes out of int32 range");
  GATX_REQUIRE(add_self_loops || E2 == E,
               "graph_build: E2 must equal E without self-loop rewrite");
  if (is64)
    return graph_build_impl<int64_t>(edge_index, E, ld, add_self_loops, num_loops, num_nodes, E2,
                                     edge_index_out, rowptr, col, rowidx, perm, ws, ws_bytes,
                                     (hipStream_t)s);
  return graph_build_impl<int32_t>(edge_index, E, ld, add_self_loops, num_loops, num_nodes, E2,
                                   edge_index_out, rowptr, col, rowidx, perm, ws, ws_bytes,
                                   (hipStream_t)s);
}

extern "C" size_t gatx_graph_transpose_workspace_bytes(int64_t E2, int64_t N) {
  return 2 * align256(sizeof(int32_t) * (E2 > 0 ? E2 : 1)) + align256(sort_bytes(E2, bits_for(N))) +
         256;
}

extern "C" int gatx_graph_transpose(const int32_t* col, const int32_t* rowidx, int64_t N,
                                    int64_t E2, int32_t* srowptr, int32_t* scol, int32_t* seid,
                                    void* ws, size_t ws_bytes, gatx_stream_t s) {
  hipStream_t stream = (hipStream_t)s;
  char* p = (char*)ws;
  int32_t* iota = (int32_t*)p;  p += align256(sizeof(int32_t) * (E2 > 0 ? E2 : 1));
  int32_t* skeys = (int32_t*)p; p += align256(sizeof(int32_t) * (E2 > 0 ? E2 : 1));
  size_t used = (size_t)(p - (char*)ws);
  GATX_REQUIRE(used <= ws_bytes, "graph_transpose: workspace too small");
  if (E2 > 0) {
    iota_kernel<<<grid_for(E2), 256, 0, stream>>>(E2, iota);
    GATX_LAUNCH_CHECK("iota");
    size_t b = ws_bytes - used;
    hipError_t r = rocprim::radix_sort_pairs((void*)p, b, col, skeys, iota, seid, (unsigned)E2, 0,
                                             bits_for(N), stream);
    if (r != hipSuccess) { set_error("radix_sort: %s", hipGetErrorString(r)); return (int)r; }
    gather_kernel<<<grid_for(E2), 256, 0, stream>>>(rowidx, seid, E2, scol);
    GATX_LAUNCH_CHECK("gather scol");
  }
  rowptr_kernel<<<grid_for(E2 + 1), 256, 0, stream>>>(skeys, E2, N, srowptr);
  GATX_LAUNCH_CHECK("srowptr");
  return 0;
}
