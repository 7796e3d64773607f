// Graph preprocessing on device: the self-loop rewrite of models/utils.py:47-67 and the
// destination-/source-ordered CSR the fused edge kernels stream.
//
// Everything is integer work (HBM-bound, no MFMA): a stats reduction, a stable compaction
// (prefix sum over the keep flags), a stable LSD radix sort by destination (rocPRIM), and
// boundary detection for rowptr. All orders are deterministic, so CSR segments list their
// edges in edge_index' order and per-segment float sums are bitwise reproducible.
//
// No host sync: |edge_index'| = E - #self-loops + max id + 1 is only known on the device, so
// the host allocates for the bound E + num_nodes and the kernels take the exact size from the
// device-side meta record (gatx_graph_meta). Padding slots past E' sort after every real slot
// (key = num_nodes) and rowptr[num_nodes] = E', so nothing that walks the CSR ever sees them.
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
// stats / compaction block ranges: >= 256 blocks' worth of input when there is enough, at most
// kStatsBlocks, each a multiple of 256 edges
inline int64_t stats_chunk(int64_t E) {
  return std::max<int64_t>(256, round_up(ceil_div(E > 0 ? E : 1, kStatsBlocks), 256));
}
inline int stats_blocks(int64_t E) { return (int)ceil_div(E > 0 ? E : 1, stats_chunk(E)); }

// Per-block {min, max, self-loops, kept edges} partials (no 64-bit atomics), reduced by
// graph_meta_kernel. Block b covers the contiguous input range [b chunk, (b+1) chunk) so that
// its kept-edge count is the block's share of the compaction (graph_meta_kernel scans them).
template <typename I>
__global__ void __launch_bounds__(256) edge_stats_kernel(const void* ei, int64_t E, int64_t ld,
                                                         int64_t chunk, long long* part) {
  long long mn = LLONG_MAX, mx = LLONG_MIN, loops = 0;
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(E, lo + chunk);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
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
    part[4 * blockIdx.x + 0] = mn;
    part[4 * blockIdx.x + 1] = mx;
    part[4 * blockIdx.x + 2] = loops;
    part[4 * blockIdx.x + 3] = hi > lo ? hi - lo : 0;   // the block's input edges
  }
}

// Device-side sizing of the rewrite from the stats partials: meta = {E2, num_loops, status, min,
// max, n_selfloops, nb, chunk} followed by the exclusive scan of the blocks' kept-edge counts
// (int32, meta + 8: the compaction's block offsets). status 1 / 2 (a negative id / an id >=
// num_nodes) zeroes E2 and num_loops, so every later kernel sees an empty graph and nothing
// indexes out of bounds; the host raises when it reads the meta (the reference raises in
// index_select / scatter_add_).
__global__ void __launch_bounds__(256) graph_meta_kernel(const long long* part, int nb, int64_t E,
                                                         int64_t chunk, int add_loops,
                                                         int64_t num_nodes, long long* meta) {
  long long mn = LLONG_MAX, mx = LLONG_MIN, loops = 0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    mn = min(mn, part[4 * b]); mx = max(mx, part[4 * b + 1]); loops += part[4 * b + 2];
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (long long)__shfl_xor(mn, o));
    mx = max(mx, (long long)__shfl_xor(mx, o));
    loops += __shfl_xor(loops, o);
  }
  __shared__ long long red[3][4];
  __shared__ int wsum[4];
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { red[0][w] = mn; red[1][w] = mx; red[2][w] = loops; }
  // block offsets of the compaction: thread t scans blocks [4t, 4t+4) (nb <= 1024); a block
  // keeps all its edges without the rewrite, all but its self-loops with it
  int c[4], tot = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = 4 * threadIdx.x + j;
    c[j] = b < nb ? (int)(part[4 * b + 3] - (add_loops ? part[4 * b + 2] : 0)) : 0;
    tot += c[j];
  }
  int x = tot;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (l >= o) x += y;
  }
  if (l == 63) wsum[w] = x;
  __syncthreads();
  int run = x - tot;
  for (int k = 0; k < w; ++k) run += wsum[k];
  int32_t* boff = (int32_t*)(meta + 8);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int b = 4 * threadIdx.x + j;
    if (b < nb) boff[b] = run;
    run += c[j];
  }
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      mn = min(mn, red[0][k]); mx = max(mx, red[1][k]); loops += red[2][k];
    }
    long long status = 0;
    if (E > 0 && mn < 0) status = 1;
    else if (E > 0 && mx >= num_nodes) status = 2;
    long long num_loops = (add_loops && E > 0) ? mx + 1 : 0;
    long long e2 = add_loops ? E - loops + num_loops : E;
    if (status) { e2 = 0; num_loops = 0; }
    meta[0] = e2; meta[1] = num_loops; meta[2] = status;
    meta[3] = E > 0 ? mn : 0; meta[4] = E > 0 ? mx : -1; meta[5] = loops;
    meta[6] = nb; meta[7] = chunk;
  }
}

// The self-loop rewrite's compaction, stable, with no separate scan: blocks [0, nb) walk their
// stats block's contiguous input range 256 edges at a time and place each surviving edge at
// boff[b] + (kept edges before it in the range) (wave ballots + per-round wave totals in LDS);
// the blocks after them fill slot q in [E2 - num_loops, E2) with the loop (i, i),
// i = q - (E2 - num_loops), and the padding slots q >= E2 (src = dst = N: sorts after every real
// key, in the destination sort and in the backward's source sort alike, so col's padding slots
// hold N and serve as the transpose's keys as they are).
// edge_index' is written flat with its exact size: sources at [p], destinations at [E2 + p],
// so edge_index'[:2*E2].view(2, E2) is the reference's contiguous (2, E') tensor.
template <typename I>
__global__ void __launch_bounds__(256) compact_kernel(const void* ei, int64_t E, int64_t ld,
                                                       int drop_loops, const long long* meta,
                                                       int64_t E_bound, int64_t num_nodes,
                                                       int64_t* ei_out, int32_t* src32,
                                                       int32_t* dst32) {
  const int64_t E2 = meta[0], num_loops = meta[1];
  const bool ok = meta[2] == 0;
  const int nb = (int)meta[6];
  const int64_t chunk = meta[7];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((int)blockIdx.x < nb) {
    if (!ok) return;
    __shared__ int wtot[4];
    int64_t run = ((const int32_t*)(meta + 8))[blockIdx.x];
    const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(E, lo + chunk);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int64_t base = lo; base < hi; base += 256) {
      const int64_t t = base + tid;
      int64_t s = 0, d = 0;
      bool keep = false;
      if (t < hi) {
        s = ld_idx<I>(ei, t);
        d = ld_idx<I>(ei, ld + t);
        keep = !drop_loops || s != d;
      }
      const uint64_t bal = __ballot(keep);
      if (lane == 0) wtot[wave] = __popcll(bal);
      __syncthreads();
      int64_t p = run + __popcll(bal & lt);
      for (int k = 0; k < wave; ++k) p += wtot[k];
      if (keep) {
        if (ei_out) { ei_out[p] = s; ei_out[E2 + p] = d; }
        src32[p] = (int32_t)s;
        dst32[p] = (int32_t)d;
      }
      run += wtot[0] + wtot[1] + wtot[2] + wtot[3];
      __syncthreads();
    }
    return;
  }
  const int64_t first = E2 - num_loops;   // loop and padding slots
  for (int64_t q = first + ((int64_t)blockIdx.x - nb) * blockDim.x + tid; q < E_bound;
       q += ((int64_t)gridDim.x - nb) * blockDim.x) {
    if (q < 0) continue;
    if (q >= E2) {   // padding slot
      src32[q] = (int32_t)num_nodes;
      dst32[q] = (int32_t)num_nodes;
      continue;
    }
    const int64_t v = q - first;
    if (ei_out) { ei_out[q] = v; ei_out[E2 + q] = v; }
    src32[q] = (int32_t)v;
    dst32[q] = (int32_t)v;
  }
}

// rowptr from a sorted key array: rows (key[e-1], key[e]] start at e.
__global__ void __launch_bounds__(256) rowptr_kernel(const int32_t* keys, int64_t E2,
                                                      int64_t num_rows, int32_t* rowptr) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e <= E2;
       e += (int64_t)gridDim.x * blockDim.x) {
    // clamped: a key outside [0, num_rows] (never produced by the builders) cannot write
    // outside rowptr
    int64_t k = (e < E2) ? min<int64_t>(max<int64_t>(keys[e], 0), num_rows) : num_rows;
    int64_t kp = (e > 0) ? min<int64_t>(max<int64_t>(keys[e - 1], -1), num_rows) : -1;
    for (int64_t r = kp + 1; r <= k; ++r) rowptr[r] = (int32_t)e;
  }
}

__global__ void __launch_bounds__(256) iota_kernel(int64_t n, int32_t* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)i;
}

// ------------------------------------------------------------------ stable LSD radix sort
// (key, value) int32 pairs, keys in [0, 2^bits), 8-bit digits, stable: equal keys keep their
// input order. Capturable into a hipGraph: no host-side memset or sync anywhere (rocPRIM's
// onesweep radix sort resets its atomic block-id counter with a synchronous hipMemset on
// gfx942/gfx950, which a captured graph never replays). Per pass:
//  * radix_hist: block b counts the digits of its tile of 256 * items keys (LDS atomics) into
//    hist[digit * nblocks + b] (digit-major, so one exclusive scan gives every (digit, block)
//    its output base);
//  * rocPRIM exclusive_scan (lookback scan, capture-safe) over the 256 * nblocks counts;
//  * radix_scatter: block b walks its tile in input order, 256 keys per round (4 waves x 64):
//    a wave ranks lanes with equal digits by 8 ballots (stable: lower lanes first), waves are
//    ordered through per-(wave, digit) counts in LDS, rounds through running per-digit bases.
constexpr int kRadixBits = 8, kRadix = 1 << kRadixBits;
constexpr int kMaxSortItems = 16;
// small sorts (keys < 2^12: graphs of up to 4095 nodes, PATTERN-size batches) take ONE pass of
// 12-bit digits instead of two 8-bit passes: 4 launches fewer per graph build, on steps that are
// launch-bound
constexpr int kWideBits = 12;

// keys per thread per block: up to 16, but at least ~256 blocks — a block walks its tile in
// serial rounds, so small sorts (PATTERN: 50 k keys) need short tiles to fill the chip
inline int sort_items(int64_t n) {
  int it = kMaxSortItems;
  while (it > 1 && ceil_div(n, 256 * it) < 256) it >>= 1;
  return it;
}

// (digit bits, keys per thread) of each pass for keys in [0, 2^bits)
inline bool wide_pass(unsigned bits, int64_t n) { return bits > kRadixBits && bits <= kWideBits && n <= (1 << 20); }
// the wide pass keeps ~48 blocks: its histogram (nblocks x 4096 counts) stays small to scan,
// and each block walks few serial rounds
inline int pass_items(unsigned bits, int64_t n) {
  if (!wide_pass(bits, n)) return sort_items(n);
  return (int)std::max<int64_t>(1, std::min<int64_t>(kMaxSortItems, ceil_div(n, 256 * 48)));
}

template <int BITS>
__global__ void __launch_bounds__(256) radix_hist_kernel(const int32_t* __restrict__ keys,
                                                         int64_t n, int shift, int items,
                                                         int64_t nblocks,
                                                         uint32_t* __restrict__ hist) {
  constexpr int R = 1 << BITS, PER = R / 256;
  __shared__ uint32_t h[R];
#pragma unroll
  for (int j = 0; j < PER; ++j) h[threadIdx.x + 256 * j] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * 256 * items;
  for (int i = 0; i < items; ++i) {
    const int64_t idx = base + i * 256 + threadIdx.x;
    if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & (R - 1)], 1u);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j)
    hist[(int64_t)(threadIdx.x + 256 * j) * nblocks + blockIdx.x] = h[threadIdx.x + 256 * j];
}

// DS (digit scan, one-pass sorts): offs holds each digit's exclusive prefix over the blocks and
// dtot (R) the digit totals (radix_digit_scan_kernel); the digit bases come from a scan of dtot
// here. They are also the row pointers of the sorted keys (row d starts after every key < d), so
// block 0 writes rowptr[0 .. num_rows] when rowptr is given: no separate pass over the keys.
template <int BITS, bool V2 = false, bool DS = false>
__global__ void __launch_bounds__(256) radix_scatter_kernel(
    const int32_t* __restrict__ keys, const int32_t* __restrict__ vals, int64_t n, int shift,
    int items, int64_t nblocks, const uint32_t* __restrict__ offs, int32_t* __restrict__ keys_out,
    int32_t* __restrict__ vals_out, const int32_t* __restrict__ vals2 = nullptr,
    int32_t* __restrict__ vals2_out = nullptr, const uint32_t* __restrict__ dtot = nullptr,
    int32_t* __restrict__ rowptr = nullptr, int64_t num_rows = 0) {
  constexpr int R = 1 << BITS, PER = R / 256;
  __shared__ uint32_t base[R];
  __shared__ uint32_t cnt[4][R];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if constexpr (DS) {
    __shared__ uint32_t wsum[4];
    uint32_t v[PER], sum = 0;   // thread t: digits [PER t, PER t + PER)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      v[j] = dtot[PER * tid + j];
      sum += v[j];
    }
    uint32_t x = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t run = x - sum;
    for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int d = PER * tid + j;
      base[d] = run;
      if (rowptr && blockIdx.x == 0 && d <= num_rows) rowptr[d] = (int32_t)run;
      run += v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) base[tid + 256 * j] += offs[(int64_t)(tid + 256 * j) * nblocks + blockIdx.x];
  } else {
#pragma unroll
    for (int j = 0; j < PER; ++j) base[tid + 256 * j] = offs[(int64_t)(tid + 256 * j) * nblocks + blockIdx.x];
  }
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int j = 0; j < PER; ++j) cnt[w][tid + 256 * j] = 0;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile = (int64_t)blockIdx.x * 256 * items;
  for (int r = 0; r < items; ++r) {
    const int64_t idx = tile + r * 256 + tid;
    const bool valid = idx < n;
    const int32_t key = valid ? keys[idx] : 0;
    const int32_t val = valid ? (vals ? vals[idx] : (int32_t)idx) : 0;
    const int32_t val2 = (V2 && valid) ? vals2[idx] : 0;
    const int d = (key >> shift) & (R - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(peers & lt);
    const bool lead = valid && rank == 0;   // one lane per (wave, digit present in it)
    __syncthreads();   // the previous round's base / cnt updates are complete
    if (lead) cnt[wave][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = base[d] + rank;
      for (int w = 0; w < wave; ++w) pos += cnt[w][d];
      keys_out[pos] = key;
      vals_out[pos] = val;
      if (V2) vals2_out[pos] = val2;
    }
    __syncthreads();
    // only the digits of this round are touched: every wave's leader adds its count to the
    // digit's base (commutative) and clears its own count, so no round walks all 2^BITS bins
    if (lead) {
      atomicAdd(&base[d], cnt[wave][d]);
      cnt[wave][d] = 0;
    }
  }
}

// The same pass with the block's tile staged in LDS: every key is first placed at its stable
// position within the tile's digit-sorted order (the round ranking above, against the tile's own
// per-digit exclusive prefix), then the tile is written out in that order, so consecutive
// threads store consecutive positions of one digit's run (runs of ~tile/2^BITS keys) instead of
// one scattered 4-byte store per key.
template <int BITS, bool V2 = false>
__global__ void __launch_bounds__(256) radix_scatter_lds_kernel(
    const int32_t* __restrict__ keys, const int32_t* __restrict__ vals, int64_t n, int shift,
    int items, int64_t nblocks, const uint32_t* __restrict__ offs,
    const uint32_t* __restrict__ hist, int32_t* __restrict__ keys_out,
    int32_t* __restrict__ vals_out, const int32_t* __restrict__ vals2 = nullptr,
    int32_t* __restrict__ vals2_out = nullptr) {
  constexpr int R = 1 << BITS, PER = R / 256;
  __shared__ uint32_t gbase[R];    // the digit's first global position for this block
  __shared__ uint32_t lstart[R];   // the digit's first position within the tile
  __shared__ uint32_t lrun[R];     // running position within the tile
  __shared__ uint32_t cnt[4][R];
  __shared__ int32_t tk[kMaxSortItems * 256];
  __shared__ int32_t tv[kMaxSortItems * 256];
  __shared__ int32_t tv2[V2 ? kMaxSortItems * 256 : 1];   // a second carried value (V2)
  __shared__ uint32_t wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // this block's digit counts -> exclusive prefix over the digits (PER consecutive per thread)
  uint32_t c[PER], tot = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int d = tid * PER + j;
    c[j] = hist[(int64_t)d * nblocks + blockIdx.x];
    tot += c[j];
    gbase[d] = offs[(int64_t)d * nblocks + blockIdx.x];
  }
  uint32_t x = tot;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int j = 0; j < PER; ++j) cnt[w][tid + 256 * j] = 0;
  __syncthreads();
  uint32_t run = x - tot;
  for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    lstart[tid * PER + j] = run;
    lrun[tid * PER + j] = run;
    run += c[j];
  }
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile = (int64_t)blockIdx.x * 256 * items;
  for (int r = 0; r < items; ++r) {
    const int64_t idx = tile + r * 256 + tid;
    const bool valid = idx < n;
    const int32_t key = valid ? keys[idx] : 0;
    const int32_t val = valid ? (vals ? vals[idx] : (int32_t)idx) : 0;
    const int32_t val2 = (V2 && valid) ? vals2[idx] : 0;
    const int d = (key >> shift) & (R - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(peers & lt);
    const bool lead = valid && rank == 0;
    __syncthreads();   // lstart/lrun ready (first round) / previous round's updates complete
    if (lead) cnt[wave][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = lrun[d] + rank;
      for (int w = 0; w < wave; ++w) pos += cnt[w][d];
      tk[pos] = key;
      tv[pos] = val;
      if (V2) tv2[pos] = val2;
    }
    __syncthreads();
    if (lead) {
      atomicAdd(&lrun[d], cnt[wave][d]);
      cnt[wave][d] = 0;
    }
  }
  __syncthreads();
  const int64_t count = min((int64_t)items * 256, n - tile);
  for (int j = tid; j < count; j += 256) {
    const int32_t key = tk[j];
    const int d = (key >> shift) & (R - 1);
    const uint32_t gpos = gbase[d] + ((uint32_t)j - lstart[d]);
    keys_out[gpos] = key;
    vals_out[gpos] = tv[j];
    if (V2) vals2_out[gpos] = tv2[j];
  }
}

// radix_scatter_lds_kernel<8> with 16 waves per tile instead of 4: a tile of 256 * items keys
// is ranked in items / 4 rounds of 1024 keys instead of items rounds of 256, and four times as
// many waves per CU overlap the rounds' LDS and barrier latency (the PPI pass kept ~1.2
// four-wave blocks per CU busy). Same stable order: ranks within a wave by ballots, across
// waves through the per-(wave, digit) counts, across rounds through the running digit bases.
// DS (digit scan): offs holds each digit's exclusive prefix over the blocks and dtot (256) the
// digit totals (radix_digit_scan_kernel); the digit bases come from a scan of dtot here.
template <bool V2, bool DS = false>
__global__ void __launch_bounds__(1024) radix_scatter_lds16_kernel(
    const int32_t* __restrict__ keys, const int32_t* __restrict__ vals, int64_t n, int shift,
    int items, int64_t nblocks, const uint32_t* __restrict__ offs,
    const uint32_t* __restrict__ hist, int32_t* __restrict__ keys_out,
    int32_t* __restrict__ vals_out, const int32_t* __restrict__ vals2 = nullptr,
    int32_t* __restrict__ vals2_out = nullptr, const uint32_t* __restrict__ dtot = nullptr) {
  constexpr int BITS = 8, R = 256, NW = 16, NT = 1024;
  __shared__ uint32_t gbase[R];
  __shared__ uint32_t lstart[R];
  __shared__ uint32_t lrun[R];
  __shared__ uint32_t cnt[NW][R];
  __shared__ int32_t tk[kMaxSortItems * 256];
  __shared__ int32_t tv[kMaxSortItems * 256];
  __shared__ int32_t tv2[V2 ? kMaxSortItems * 256 : 1];
  __shared__ uint32_t wsum[4], tsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t c = 0, x = 0, dt = 0, xt = 0;
  if (tid < R) {   // this block's digit counts -> exclusive prefix over the digits
    c = hist[(int64_t)tid * nblocks + blockIdx.x];
    gbase[tid] = offs[(int64_t)tid * nblocks + blockIdx.x];
    x = c;
    if (DS) xt = dt = dtot[tid];
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
      if (DS) {
        const uint32_t yt = __shfl_up(xt, o);
        if (lane >= o) xt += yt;
      }
    }
    if (lane == 63) {
      wsum[wave] = x;
      if (DS) tsum[wave] = xt;
    }
  }
  for (int i = tid; i < NW * R; i += NT) (&cnt[0][0])[i] = 0;
  __syncthreads();
  if (tid < R) {
    uint32_t run = x - c;
    for (int w = 0; w < wave; ++w) run += wsum[w];
    lstart[tid] = run;
    lrun[tid] = run;
    if (DS) {   // digit base = exclusive scan of the digit totals
      uint32_t base = xt - dt;
      for (int w = 0; w < wave; ++w) base += tsum[w];
      gbase[tid] += base;
    }
  }
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile = (int64_t)blockIdx.x * 256 * items;
  const int tile_keys = 256 * items, rounds = (tile_keys + NT - 1) / NT;
  for (int r = 0; r < rounds; ++r) {
    const int li = r * NT + tid;
    const int64_t idx = tile + li;
    const bool valid = li < tile_keys && idx < n;
    const int32_t key = valid ? keys[idx] : 0;
    const int32_t val = valid ? (vals ? vals[idx] : (int32_t)idx) : 0;
    const int32_t val2 = (V2 && valid) ? vals2[idx] : 0;
    const int d = (key >> shift) & (R - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(peers & lt);
    const bool lead = valid && rank == 0;
    __syncthreads();
    if (lead) cnt[wave][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = lrun[d] + rank;
      for (int w = 0; w < wave; ++w) pos += cnt[w][d];
      tk[pos] = key;
      tv[pos] = val;
      if (V2) tv2[pos] = val2;
    }
    __syncthreads();
    if (lead) {
      atomicAdd(&lrun[d], cnt[wave][d]);
      cnt[wave][d] = 0;
    }
  }
  __syncthreads();
  const int64_t count = min((int64_t)tile_keys, n - tile);
  for (int j = tid; j < count; j += NT) {
    const int32_t key = tk[j];
    const int d = (key >> shift) & (R - 1);
    const uint32_t gpos = gbase[d] + ((uint32_t)j - lstart[d]);
    keys_out[gpos] = key;
    vals_out[gpos] = tv[j];
    if (V2) vals2_out[gpos] = tv2[j];
  }
}

// Per-digit scan of the block counts (block d = digit d): P[d][b] = sum_{b' < b} hist[d][b'],
// T[d] = the digit's total; radix_scatter_lds16_kernel<DS> adds the scan of T itself. One
// launch instead of rocPRIM's two (lookback-state init + scan) over all 256 * nb counts; for
// nb <= 4096 (each thread sums at most 16 consecutive counts, all loads issued first).
__global__ void __launch_bounds__(256) radix_digit_scan_kernel(const uint32_t* __restrict__ hist,
                                                               int64_t nb,
                                                               uint32_t* __restrict__ P,
                                                               uint32_t* __restrict__ T) {
  __shared__ uint32_t wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k = (int)((nb + 255) / 256);   // <= 16
  const uint32_t* h = hist + (int64_t)blockIdx.x * nb;
  uint32_t v[16];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t b = (int64_t)tid * k + i;
    v[i] = (i < k && b < nb) ? h[b] : 0u;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) sum += v[i];
  uint32_t x = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  uint32_t run = x - sum;
  for (int w = 0; w < wave; ++w) run += wsum[w];
  uint32_t* p = P + (int64_t)blockIdx.x * nb;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t b = (int64_t)tid * k + i;
    if (i < k && b < nb) p[b] = run;
    run += v[i];
  }
  if (tid == 255) T[blockIdx.x] = run;
}

// radix_hist_kernel<8> for 1024-thread blocks (the tiles of radix_scatter_lds16_kernel).
__global__ void __launch_bounds__(1024) radix_hist16_kernel(const int32_t* __restrict__ keys,
                                                            int64_t n, int shift, int items,
                                                            int64_t nblocks,
                                                            uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  if (threadIdx.x < 256) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * 256 * items;
  const int tile_keys = 256 * items;
  for (int i = threadIdx.x; i < tile_keys; i += 1024) {
    const int64_t idx = base + i;
    if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & 255], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 256) hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
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

// ---- the radix sort's host side (workspace layout and passes)
struct SortWs {
  uint32_t* hist;
  uint32_t* offs;
  int32_t* tk;
  int32_t* tv;
  int32_t* tv2;
  void* scan_tmp;
  size_t scan_bytes;
};

size_t radix_scan_bytes(int64_t m) {
  size_t bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                0u, (size_t)(m > 0 ? m : 1), rocprim::plus<uint32_t>(),
                                (hipStream_t)0);
  return bytes;
}

inline int64_t hist_entries(int64_t n, unsigned bits) {
  const int64_t nb = ceil_div(n > 0 ? n : 1, 256 * pass_items(bits, n));
  return nb * (wide_pass(bits, n) ? (1 << kWideBits) : kRadix);
}

size_t sort_bytes(int64_t n, unsigned bits, bool v2 = false) {  // keys in [0, 2^bits)
  const int64_t m = hist_entries(n, bits);
  return 2 * align256(sizeof(uint32_t) * (m + (1 << kWideBits))) + (v2 ? 3 : 2) * align256(sizeof(int32_t) * (n > 0 ? n : 1)) +
         align256(radix_scan_bytes(m)) + 256;
}

SortWs carve_sort(void* ws, int64_t n, unsigned bits, bool v2 = false) {
  const int64_t m = hist_entries(n, bits);
  char* p = (char*)ws;
  SortWs w;
  w.hist = (uint32_t*)p; p += align256(sizeof(uint32_t) * (m + (1 << kWideBits)));
  w.offs = (uint32_t*)p; p += align256(sizeof(uint32_t) * (m + (1 << kWideBits)));   // + digit totals
  w.tk = (int32_t*)p; p += align256(sizeof(int32_t) * (n > 0 ? n : 1));
  w.tv = (int32_t*)p; p += align256(sizeof(int32_t) * (n > 0 ? n : 1));
  w.tv2 = nullptr;
  if (v2) { w.tv2 = (int32_t*)p; p += align256(sizeof(int32_t) * (n > 0 ? n : 1)); }
  w.scan_tmp = p;
  w.scan_bytes = radix_scan_bytes(m);
  return w;
}

// keys_in -> (keys_out, vals_out) sorted stably by key; vals_in NULL = the identity (input
// positions). Passes alternate between the output and the workspace pair so the last one lands
// in the output.
// vals2_in / vals2_out (nullable): a second value carried along (the graph build's source ids,
// so the CSR's col needs no gather through perm afterwards).
// rowptr (nullable, keys in [0, num_rows]): the one-pass (12-bit) sort with a second value also
// writes the row pointers of the sorted keys and sets *rowptr_done; otherwise the caller runs
// rowptr_kernel.
int sort_pairs(const int32_t* keys_in, const int32_t* vals_in, int32_t* keys_out,
               int32_t* vals_out, int64_t n, unsigned bits, void* ws, hipStream_t stream,
               const int32_t* vals2_in = nullptr, int32_t* vals2_out = nullptr,
               int32_t* rowptr = nullptr, int64_t num_rows = 0, bool* rowptr_done = nullptr) {
  if (rowptr_done) *rowptr_done = false;
  if (n <= 0) return 0;
  GATX_REQUIRE(n < (1ll << 31), "sort: too many keys");
  const bool v2 = vals2_in != nullptr;
  const SortWs w = carve_sort(ws, n, bits, v2);
  const bool wide = wide_pass(bits, n);
  const int items = pass_items(bits, n);
  const int64_t nb = ceil_div(n, 256 * items), m = hist_entries(n, bits);
  const int passes = wide ? 1 : (int)ceil_div((int64_t)(bits > 0 ? bits : 1), kRadixBits);
  const int32_t* ck = keys_in;
  const int32_t* cv = vals_in;
  const int32_t* cv2 = vals2_in;
  for (int ps = 0; ps < passes; ++ps) {
    const bool to_out = ((passes - 1 - ps) % 2) == 0;
    int32_t* ok = to_out ? keys_out : w.tk;
    int32_t* ov = to_out ? vals_out : w.tv;
    int32_t* ov2 = v2 ? (to_out ? vals2_out : w.tv2) : nullptr;
    const int shift = ps * kRadixBits;
    // 16-wave tiles for the 8-bit passes of sorts of at least 4 items per thread
    const bool big = !wide && items >= 4;
    if (wide) radix_hist_kernel<kWideBits><<<(unsigned)nb, 256, 0, stream>>>(ck, n, 0, items, nb, w.hist);
    else if (big) radix_hist16_kernel<<<(unsigned)nb, 1024, 0, stream>>>(ck, n, shift, items, nb, w.hist);
    else radix_hist_kernel<kRadixBits><<<(unsigned)nb, 256, 0, stream>>>(ck, n, shift, items, nb, w.hist);
    GATX_LAUNCH_CHECK("radix_hist");
    // per-digit scans of the block counts (one launch) up to 4096 tiles; rocPRIM's scan beyond
    const bool dscan = big && nb <= 4096;
    // the one-pass sort: per-digit scans (4096 digits) + the digit-total scan in the scatter,
    // which also writes rowptr — three launches for the whole sort instead of five
    const bool wscan = wide && v2 && nb <= 4096 && num_rows < (1 << kWideBits);
    if (dscan || wscan) {
      radix_digit_scan_kernel<<<wscan ? (1u << kWideBits) : (unsigned)kRadix, 256, 0, stream>>>(
          w.hist, nb, w.offs, w.offs + m);
      GATX_LAUNCH_CHECK("radix_digit_scan");
    } else {
      // (a single-workgroup LDS scan over all 256 * nb counts measured 35 us on PPI's 80 K
      // counts; rocPRIM's lookback scan over the whole chip for the general case)
      size_t b = w.scan_bytes;
      hipError_t r = rocprim::exclusive_scan(w.scan_tmp, b, w.hist, w.offs, 0u, (size_t)m,
                                             rocprim::plus<uint32_t>(), stream);
      if (r != hipSuccess) { set_error("radix scan: %s", hipGetErrorString(r)); return (int)r; }
    }
    if (dscan) {
      if (v2)
        radix_scatter_lds16_kernel<true, true><<<(unsigned)nb, 1024, 0, stream>>>(
            ck, cv, n, shift, items, nb, w.offs, w.hist, ok, ov, cv2, ov2, w.offs + m);
      else
        radix_scatter_lds16_kernel<false, true><<<(unsigned)nb, 1024, 0, stream>>>(
            ck, cv, n, shift, items, nb, w.offs, w.hist, ok, ov, nullptr, nullptr, w.offs + m);
    } else if (big) {
      if (v2)
        radix_scatter_lds16_kernel<true><<<(unsigned)nb, 1024, 0, stream>>>(
            ck, cv, n, shift, items, nb, w.offs, w.hist, ok, ov, cv2, ov2);
      else
        radix_scatter_lds16_kernel<false><<<(unsigned)nb, 1024, 0, stream>>>(
            ck, cv, n, shift, items, nb, w.offs, w.hist, ok, ov);
    } else if (wscan) {
      radix_scatter_kernel<kWideBits, true, true><<<(unsigned)nb, 256, 0, stream>>>(
          ck, cv, n, 0, items, nb, w.offs, ok, ov, cv2, ov2, w.offs + m, rowptr, num_rows);
      if (rowptr_done) *rowptr_done = rowptr != nullptr;
    } else if (v2 && wide)   // (the wide LDS tile has no room for a second value)
      radix_scatter_kernel<kWideBits, true><<<(unsigned)nb, 256, 0, stream>>>(
          ck, cv, n, 0, items, nb, w.offs, ok, ov, cv2, ov2);
    else if (v2)
      radix_scatter_lds_kernel<kRadixBits, true><<<(unsigned)nb, 256, 0, stream>>>(
          ck, cv, n, shift, items, nb, w.offs, w.hist, ok, ov, cv2, ov2);
    else if (wide)
      radix_scatter_lds_kernel<kWideBits><<<(unsigned)nb, 256, 0, stream>>>(
          ck, cv, n, 0, items, nb, w.offs, w.hist, ok, ov);
    else
      radix_scatter_lds_kernel<kRadixBits><<<(unsigned)nb, 256, 0, stream>>>(
          ck, cv, n, shift, items, nb, w.offs, w.hist, ok, ov);
    GATX_LAUNCH_CHECK("radix_scatter");
    ck = ok;
    cv = ov;
    cv2 = ov2;
  }
  return 0;
}

template <typename I>
int graph_build_impl(const void* ei, int64_t E, int64_t ld, int add_loops, int64_t N,
                     int64_t E_bound, const long long* meta, int64_t* ei_out, int32_t* rowptr,
                     int32_t* col, int32_t* rowidx, int32_t* perm, void* ws, size_t ws_bytes,
                     hipStream_t stream) {
  // workspace carve: src32 [Eb] | dst32 [Eb] | sort workspace (perm: the sort's identity values)
  char* p = (char*)ws;
  int32_t* src32 = (int32_t*)p; p += align256(sizeof(int32_t) * (E_bound > 0 ? E_bound : 1));
  int32_t* dst32 = (int32_t*)p; p += align256(sizeof(int32_t) * (E_bound > 0 ? E_bound : 1));
  size_t used = (size_t)(p - (char*)ws);
  GATX_REQUIRE(used <= ws_bytes, "graph_build: workspace too small");
  void* tmp = p;
  bool done = false;
  if (E_bound > 0) {
    // the stats launch's block count (meta[6]) is <= kStatsBlocks: that many range blocks, then
    // the loop / padding slot blocks
    const int64_t slot_blocks = std::max<int64_t>(1, std::min<int64_t>(ceil_div(E_bound, 256), 4096));
    compact_kernel<I><<<(unsigned)(stats_blocks(E) + slot_blocks), 256, 0, stream>>>(
        ei, E, ld, add_loops, meta, E_bound, N, ei_out, src32, dst32);
    GATX_LAUNCH_CHECK("compact");
    // src ids ride along as a second value: col comes out of the sort (no gather through perm)
    GATX_CALL(sort_pairs(dst32, nullptr, rowidx, perm, E_bound, bits_for(N + 1), tmp, stream, src32,
                         col, rowptr, N, &done));
  }
  if (!done) {
    rowptr_kernel<<<grid_for(E_bound + 1), 256, 0, stream>>>(rowidx, E_bound, N, rowptr);
    GATX_LAUNCH_CHECK("rowptr");
  }
  return 0;
}

// Hub plan: every destination segment of more than T edges becomes ceil(deg / T) pieces, listed
// as (node, piece, pieces, first slot) with the pieces of one node in consecutive slots. The
// slot ranges are claimed with one atomic per hub (their order varies from run to run; every
// consumer reads a hub's slots in piece order, so results do not).
__global__ void __launch_bounds__(256) hub_plan_kernel(const int32_t* __restrict__ rowptr,
                                                       int64_t N, int T, int32_t* __restrict__ hubs,
                                                       int64_t bound, int32_t* __restrict__ count) {
  for (int64_t n = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; n < N;
       n += (int64_t)gridDim.x * blockDim.x) {
    const int deg = rowptr[n + 1] - rowptr[n];
    if (deg <= T) continue;
    const int pieces = (int)ceil_div((int64_t)deg, T);
    const int first = atomicAdd(count, pieces);
    for (int p = 0; p < pieces && first + p < bound; ++p) {
      int32_t* h = hubs + 4 * (int64_t)(first + p);
      h[0] = (int32_t)n; h[1] = p; h[2] = pieces; h[3] = first;
    }
  }
}

}  // namespace
}  // namespace gatx

using namespace gatx;

extern "C" size_t gatx_graph_meta_workspace_bytes(void) {
  return (size_t)4 * sizeof(long long) * kStatsBlocks;
}

extern "C" int gatx_graph_meta(const void* edge_index, int is64, int64_t E, int64_t ld,
                               int add_self_loops, int64_t num_nodes, int64_t* meta,
                               void* workspace, gatx_stream_t s) {
  GATX_REQUIRE(E >= 0 && num_nodes >= 0, "graph_meta: negative size");
  hipStream_t stream = (hipStream_t)s;
  const int nb = stats_blocks(E);
  const int64_t chunk = stats_chunk(E);
  long long* part = (long long*)workspace;
  if (is64)
    edge_stats_kernel<int64_t><<<nb, 256, 0, stream>>>(edge_index, E, ld, chunk, part);
  else
    edge_stats_kernel<int32_t><<<nb, 256, 0, stream>>>(edge_index, E, ld, chunk, part);
  GATX_LAUNCH_CHECK("edge_stats");
  graph_meta_kernel<<<1, 256, 0, stream>>>(part, nb, E, chunk, add_self_loops, num_nodes,
                                           (long long*)meta);
  GATX_LAUNCH_CHECK("graph_meta");
  return 0;
}

extern "C" size_t gatx_graph_build_workspace_bytes(int64_t E, int64_t E_bound, int64_t N) {
  (void)E;
  size_t b = 2 * align256(sizeof(int32_t) * (E_bound > 0 ? E_bound : 1));
  return b + align256(sort_bytes(E_bound, bits_for(N + 1), true)) + 256;
}

extern "C" int gatx_graph_build(const void* edge_index, int is64, int64_t E, int64_t ld,
                                int add_self_loops, int64_t num_nodes, int64_t E_bound,
                                const int64_t* meta, int64_t* edge_index_out, int32_t* rowptr,
                                int32_t* col, int32_t* rowidx, int32_t* perm, void* ws,
                                size_t ws_bytes, gatx_stream_t s) {
  GATX_REQUIRE(num_nodes >= 0 && num_nodes < INT32_MAX && E_bound < INT32_MAX && E >= 0,
               "graph_build: sizes out of int32 range");
  GATX_REQUIRE(E_bound >= (add_self_loops ? E + num_nodes : E),
               "graph_build: E_bound below E (+ num_nodes with self-loops)");
  if (is64)
    return graph_build_impl<int64_t>(edge_index, E, ld, add_self_loops, num_nodes, E_bound,
                                     (const long long*)meta, edge_index_out, rowptr, col, rowidx,
                                     perm, ws, ws_bytes, (hipStream_t)s);
  return graph_build_impl<int32_t>(edge_index, E, ld, add_self_loops, num_nodes, E_bound,
                                   (const long long*)meta, edge_index_out, rowptr, col, rowidx,
                                   perm, ws, ws_bytes, (hipStream_t)s);
}

extern "C" size_t gatx_graph_transpose_workspace_bytes(int64_t E_bound, int64_t N) {
  return align256(sizeof(int32_t) * (E_bound > 0 ? E_bound : 1)) +
         align256(sort_bytes(E_bound, bits_for(N + 1), true)) + 256;
}

extern "C" int gatx_graph_transpose(const int32_t* col, const int32_t* rowidx, int64_t N,
                                    int64_t E_bound, const int64_t* e2, int32_t* srowptr,
                                    int32_t* scol, int32_t* seid, void* ws, size_t ws_bytes,
                                    gatx_stream_t s) {
  hipStream_t stream = (hipStream_t)s;
  (void)e2;   // (col's padding slots hold N: gatx_graph_build)
  char* p = (char*)ws;
  int32_t* skeys = (int32_t*)p; p += align256(sizeof(int32_t) * (E_bound > 0 ? E_bound : 1));
  size_t used = (size_t)(p - (char*)ws);
  GATX_REQUIRE(used <= ws_bytes, "graph_transpose: workspace too small");
  bool done = false;
  if (E_bound > 0) {
    // the keys are col itself (N in the padding slots, which sort last); seid = the slots (the
    // sort's identity values); each slot's destination rides through the sort as a second
    // value: scol comes out sorted
    GATX_CALL(sort_pairs(col, nullptr, skeys, seid, E_bound, bits_for(N + 1), (void*)p, stream,
                         rowidx, scol, srowptr, N, &done));
  }
  if (!done) {
    rowptr_kernel<<<grid_for(E_bound + 1), 256, 0, stream>>>(skeys, E_bound, N, srowptr);
    GATX_LAUNCH_CHECK("srowptr");
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Node blocks (round 5): the node range cut into contiguous blocks that no edge crosses, each at
// most max_rows nodes — the graphs of a PyG-style batch, packed greedily — found from the CSR
// alone. A boundary b (0 < b < N) is free when max_{d<b} hi[d] < b and min_{d>=b} lo[d] >= b,
// with lo / hi[d] the smallest / largest node among d and its in-neighbours (an edge s -> d
// covers every boundary in (min(s,d), max(s,d)]). The LDS-staged edge passes stage one block's
// rows per workgroup; the count is -1 when some gap-free run exceeds max_rows, when there are more
// than kSegMax runs, or N > kSegMaxNodes (those graphs keep the L2-gather passes).
constexpr int kSegMax = 4096;
constexpr int64_t kSegMaxNodes = int64_t(1) << 17;

// 16 lanes per destination (four per wave): lo / hi over its in-neighbours, lanes striding the
// segment (PPI's ~28-edge segments: a whole wave per destination left 3/4 of its lanes idle)
__global__ void __launch_bounds__(256) seg_hilo_kernel(const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ col, int64_t N,
                                                       int32_t* __restrict__ lo,
                                                       int32_t* __restrict__ hi) {
  const int sub = threadIdx.x & 15;
  const int64_t d = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const bool live = d < N;
  const int beg = live ? rowptr[d] : 0, end = live ? rowptr[d + 1] : 0;
  int mn = (int)d, mx = (int)d;
  for (int e = beg + sub; e < end; e += 16) {
    const int s = col[e];
    mn = min(mn, s);
    mx = max(mx, s);
  }
  for (int off = 8; off > 0; off >>= 1) {
    mn = min(mn, __shfl_xor(mn, off));
    mx = max(mx, __shfl_xor(mx, off));
  }
  if (live && sub == 0) {
    lo[d] = mn;
    hi[d] = mx;
  }
}

// The free boundaries of one 1024-boundary tile [T0, T0 + 1024) from a window of halo H =
// min(max_rows, kSegHalo) nodes on each side. Blocks of at most max_rows nodes can only exist if
// every interval [lo[d], hi[d]] spans at most H nodes (its two ends share a block); under that
// condition an interval that covers a boundary b has its destination within H of b, so the
// prefix max of hi over [T0 - H, b) and the suffix min of lo over [b, T0 + 1024 + H) decide b
// exactly as the whole-range scans would. A tile holding a longer interval sets its flag word and
// the pack reports no blocks. Tiles run in parallel (no whole-range scan, no atomics); every bit
// word and flag is rewritten on every call, so a captured step's replays recompute them.
constexpr int kSegHalo = 4096;
__global__ void __launch_bounds__(1024) seg_window_kernel(const int32_t* __restrict__ lo,
                                                          const int32_t* __restrict__ hi,
                                                          int64_t N, int H,
                                                          uint32_t* __restrict__ bits,
                                                          uint32_t* __restrict__ tflag) {
  constexpr int kW = kSegHalo + 1024;
  __shared__ int A[kW], B[kW];    // hi over [T0 - H, T0 + 1024), lo over [T0, T0 + 1024 + H)
  __shared__ int carry_a[1024], carry_b[1024];
  const int t = threadIdx.x, n = (int)N;
  const int T0 = blockIdx.x * 1024, W = H + 1024;
  for (int i = t; i < W; i += 1024) {
    const int da = T0 - H + i, db = T0 + i;
    A[i] = (da >= 0 && da < n) ? hi[da] : -1;
    B[i] = db < n ? lo[db] : n;
  }
  const int d = T0 + t;
  const bool lng = d < n && hi[d] - lo[d] > H;
  __syncthreads();
  // thread t scans A / B over [t C, t C + C) (C = ceil(W / 1024)): inclusive prefix max of A,
  // inclusive suffix min of B; the thread aggregates are scanned across the block
  const int C = (W + 1023) / 1024, c0 = t * C;
  int ma = -1, mb = n;
  for (int i = 0; i < C; ++i)
    if (c0 + i < W) {
      ma = max(ma, A[c0 + i]);
      A[c0 + i] = ma;
    }
  for (int i = C - 1; i >= 0; --i)
    if (c0 + i < W) {
      mb = min(mb, B[c0 + i]);
      B[c0 + i] = mb;
    }
  carry_a[t] = ma;
  carry_b[t] = mb;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int x = t >= off ? carry_a[t - off] : -1;
    const int y = t + off < 1024 ? carry_b[t + off] : n;
    __syncthreads();
    carry_a[t] = max(carry_a[t], x);
    carry_b[t] = min(carry_b[t], y);
    __syncthreads();
  }
  {
    const int pa = t > 0 ? carry_a[t - 1] : -1, pb = t < 1023 ? carry_b[t + 1] : n;
    for (int i = 0; i < C; ++i)
      if (c0 + i < W) {
        A[c0 + i] = max(A[c0 + i], pa);
        B[c0 + i] = min(B[c0 + i], pb);
      }
  }
  __syncthreads();
  // boundary b = T0 + t: max hi over d < b is A[H + t - 1], min lo over d >= b is B[t]
  bool fr = false;
  if (d > 0 && d < n) {
    const int before = H + t >= 1 ? A[H + t - 1] : -1;
    fr = before < d && B[t] >= d;
  }
  const uint64_t m = __ballot(fr);
  const int lane = t & 63;
  const int64_t w = (int64_t)d >> 5;
  if ((lane & 31) == 0 && w < ceil_div(N, (int64_t)64) * 2)
    bits[w] = (uint32_t)(lane == 0 ? m : m >> 32);
  if (__syncthreads_or(lng) && t == 0) tflag[blockIdx.x] = 1u;
  else if (t == 0) tflag[blockIdx.x] = 0u;
}

// pack: no blocks if a tile flagged a long interval; else the free boundaries in order (a
// block-wide scan of the words' popcounts), then the gap-free runs packed greedily into blocks of
// <= max_rows nodes (thread 0)
__global__ void __launch_bounds__(1024) seg_pack_kernel(const uint32_t* __restrict__ bits,
                                                        const uint32_t* __restrict__ tflag,
                                                        int ntiles, int64_t N, int max_rows,
                                                        int32_t* __restrict__ segs,
                                                        int32_t* __restrict__ seg_count) {
  __shared__ int bnd[kSegMax + 2];
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, n = (int)N;
  if (__syncthreads_or(t < ntiles && tflag[t] != 0u)) {
    if (t == 0) *seg_count = -1;
    return;
  }
  const int64_t nw = ceil_div(N, (int64_t)64) * 2;   // words (<= 2^17 / 32 = 4096)
  int base = 0;
  for (int64_t w0 = 0; w0 < nw; w0 += 1024) {
    const int64_t w = w0 + t;
    const uint32_t word = w < nw ? bits[w] : 0u;
    const int c = __popc(word);
    int x = c;   // inclusive wave scan
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int before = 0, total = 0;
    for (int i = 0; i < 16; ++i) {
      const int v = wsum[i];
      before += i < wave ? v : 0;
      total += v;
    }
    int pos = base + before + x - c;
    for (uint32_t m = word; m != 0u; m &= m - 1u, ++pos)
      if (pos < kSegMax) bnd[1 + pos] = (int)(w * 32 + __ffs(m) - 1);
    base += total;
    __syncthreads();   // wsum reused
  }
  if (t != 0) return;
  const int nb = base;
  if (nb > kSegMax) {
    *seg_count = -1;
    return;
  }
  bnd[0] = 0;
  bnd[nb + 1] = n;
  int count = 0, start = 0;
  segs[0] = 0;
  if (n > 0) {
    for (int i = 1; i <= nb + 1 && count >= 0; ++i) {
      const int b = bnd[i], prev = bnd[i - 1];
      if (b - prev > max_rows) {
        count = -1;
      } else if (b - start > max_rows) {
        segs[++count] = prev;
        start = prev;
      }
    }
    if (count >= 0) segs[++count] = n;
  }
  *seg_count = count;
}

__global__ void seg_none_kernel(int32_t* seg_count) {
  if (threadIdx.x == 0) *seg_count = -1;
}

extern "C" size_t gatx_graph_segments_workspace_bytes(int64_t N) {
  const size_t n1 = (size_t)(N > 0 ? N : 1);
  return 2 * align256(sizeof(int32_t) * n1) + align256(sizeof(uint32_t) * 2 * ceil_div(n1, 64)) +
         align256(sizeof(uint32_t) * ceil_div(n1, 1024));
}

extern "C" int gatx_graph_segments(const int32_t* rowptr, const int32_t* col, int64_t N,
                                   int max_rows, int32_t* segs, int32_t* seg_count, void* ws,
                                   size_t ws_bytes, gatx_stream_t s) {
  GATX_REQUIRE(N >= 0 && max_rows > 0, "graph_segments: bad arguments");
  hipStream_t st = (hipStream_t)s;
  if (N > kSegMaxNodes) {   // no blocks: the caller keeps the L2-gather passes
    seg_none_kernel<<<1, 64, 0, st>>>(seg_count);
    GATX_LAUNCH_CHECK("graph_segments none");
    return 0;
  }
  GATX_REQUIRE(ws_bytes >= gatx_graph_segments_workspace_bytes(N), "graph_segments: workspace");
  const size_t n1 = (size_t)(N > 0 ? N : 1);
  char* p = (char*)ws;
  int32_t* lo = (int32_t*)p; p += align256(sizeof(int32_t) * n1);
  int32_t* hi = (int32_t*)p; p += align256(sizeof(int32_t) * n1);
  uint32_t* bits = (uint32_t*)p; p += align256(sizeof(uint32_t) * 2 * ceil_div(n1, 64));
  uint32_t* tflag = (uint32_t*)p;
  const int ntiles = (int)ceil_div(n1, 1024);   // <= 128
  if (N > 0) {
    seg_hilo_kernel<<<(unsigned)ceil_div(N, (int64_t)16), 256, 0, st>>>(rowptr, col, N, lo, hi);
    GATX_LAUNCH_CHECK("graph_segments hilo");
    seg_window_kernel<<<(unsigned)ntiles, 1024, 0, st>>>(lo, hi, N, std::min(max_rows, kSegHalo),
                                                         bits, tflag);
    GATX_LAUNCH_CHECK("graph_segments window");
  }
  seg_pack_kernel<<<1, 1024, 0, st>>>(bits, tflag, N > 0 ? ntiles : 0, N, max_rows, segs,
                                      seg_count);
  GATX_LAUNCH_CHECK("graph_segments pack");
  return 0;
}

extern "C" int gatx_graph_segments_max(void) { return kSegMax; }

extern "C" int64_t gatx_graph_hub_bound(int64_t E_bound, int hub_edges) {
  // sum over hubs of ceil(deg / T) <= E'/T + #hubs <= 2 E'/T
  return hub_edges > 0 ? 2 * ceil_div(E_bound, hub_edges) + 1 : 0;
}

extern "C" int gatx_graph_hub_plan(const int32_t* rowptr, int64_t N, int hub_edges,
                                   int32_t* hubs, int64_t hub_bound, int32_t* hub_count,
                                   gatx_stream_t s) {
  GATX_REQUIRE(hub_edges > 0 && N >= 0, "graph_hub_plan: bad arguments");
  hipStream_t st = (hipStream_t)s;
  // a kernel, not hipMemsetAsync (memset nodes of a captured step were not ordered before the
  // next kernel once a kernel had run outside the graph: gemm_f16p.hip absmax_rows_cols)
  zero_words_kernel<<<1, 64, 0, st>>>((uint32_t*)hub_count, 1);
  GATX_LAUNCH_CHECK("graph_hub_plan zero");
  if (N == 0) return 0;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(N, 256), 8192);
  hub_plan_kernel<<<grid, 256, 0, st>>>(rowptr, N, hub_edges, hubs, hub_bound, hub_count);
  GATX_LAUNCH_CHECK("graph_hub_plan");
  return 0;
}
