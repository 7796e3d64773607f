// Walk lab (round 6): the LDS-staged aggregation of the PPI-L1 layer, out[d,h,:] = sum_e w[e,h]
// Wh[src_e,h,:] over a 20-graph PPI-shaped batch, the library kernel (edge_lds.hip, included
// as is) against walk variants, timed in isolation with the caches clobbered and Wh rewritten
// before every launch (in situ the projection GEMM has just written Wh), each checked against a
// host fp64 sum on sampled rows.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o walk_lab walk_lab.hip && ./walk_lab
#include "../../gat-pytorch_amd/csrc/edge_lds.hip"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace gatx {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fprintf(stderr, "\n");
}
}  // namespace gatx

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace lab {
using namespace gatx;

constexpr int kRows = 2304;

__device__ inline int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline int64_t xcd_map(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, xcd = b % 8, j = b / 8;
  return (xcd < r) ? xcd * (q + 1) + j : r * (q + 1) + (xcd - r) * q + j;
}

struct Args {
  const float* rows;      // [N][NH*F]
  int64_t row_stride;
  const int* rowptr;
  const int2* rec;        // [NH][E] {64 src, w}
  int64_t E;
  const int* segs;        // [G+1]
  int NH, F, nchunks;
  float* out;             // [N][NH*F]
};

// prologue shared by the variants: stage chunk c of head h of every row of the block, the block's
// row pointers, and the destinations sorted by in-degree (DESC: descending order)
template <bool DESC>
__device__ inline void prologue(const Args& g, int n0, int R, int h, int c, float4* img,
                                unsigned short* order, int* lrp, int* bins) {
  const int tid = threadIdx.x;
  if (tid < 64) bins[tid] = 0;
  constexpr int kStage = kRows / 256;
  float4 st[kStage];
  const float4* src = (const float4*)(g.rows + (int64_t)h * g.F) + c * 4 + (tid & 3);
  const int64_t rs4 = g.row_stride / 4;
#pragma unroll
  for (int i = 0; i < kStage; ++i) st[i] = src[(int64_t)(n0 + min((tid >> 2) + 256 * i, R - 1)) * rs4];
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
    if (r < R) img[r * 4 + (tid & 3)] = st[i];
  }
  int degs[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int d = tid + 1024 * t;
    if (d <= R) lrp[d] = lo[t];
    int dg = min(hi[t] - lo[t], 63);
    if (DESC) dg = 63 - dg;
    degs[t] = d < R ? dg : -1;
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (degs[t] >= 0) atomicAdd(&bins[degs[t]], 1);
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
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (degs[t] >= 0) order[atomicAdd(&bins[degs[t]], 1)] = (unsigned short)(tid + 1024 * t);
  __syncthreads();
}

// B: one lane per destination (64 per wave), the whole 64-B row per record as four
// ds_read_b128 in a lane-rotated piece order (lane class c reads piece (k + c) & 3 at step k,
// so the four lanes of a class are the only ones that can collide), U records per step, sets of
// 64 destinations dealt to the waves in snake order over the degree-descending list.
template <int U>
__global__ void __launch_bounds__(1024) walkB(Args g) {
  __shared__ __attribute__((aligned(16))) float4 img[kRows * 4];
  __shared__ unsigned short order[kRows];
  __shared__ int lrp[kRows + 1];
  __shared__ int bins[64];
  const int64_t b = xcd_map(blockIdx.x, gridDim.x);
  const int c = (int)(b % g.nchunks);
  const int h = (int)((b / g.nchunks) % g.NH);
  const int k = (int)(b / ((int64_t)g.nchunks * g.NH));
  const int n0 = g.segs[k], R = g.segs[k + 1] - n0;
  prologue<true>(g, n0, R, h, c, img, order, lrp, bins);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, cls = lane & 3;
  const int2* rh = g.rec + (int64_t)h * g.E;
  const char* imgb = (const char*)img;
  int rk[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) rk[t] = ((t + cls) & 3) * 16;
  const int nsets = (R + 63) / 64;
  for (int i = 0;; ++i) {
    const int s = (i & 1) ? (i + 1) * 16 - 1 - wave : i * 16 + wave;   // snake
    if (i * 16 >= nsets) break;
    if (s >= nsets) continue;
    const int d = s * 64 + lane;
    const bool live = d < R;
    const int dl = live ? (int)order[d] : 0;
    const int e = lrp[dl];
    const int end = live ? lrp[dl + 1] : e;
    int need = end - e;
    for (int off = 1; off < 64; off <<= 1) need = max(need, __shfl_xor(need, off));
    const int trips = uni(need);
    const int last = max(end - 1, 0);
    float4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t0 = 0; t0 < trips; t0 += U) {
      int2 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = rh[min(e + t0 + u, last)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = e + t0 + u < end;
        const int off = ok ? r[u].x - 64 * n0 : 0;
        const float w = ok ? __int_as_float(r[u].y) : 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float4 v = *(const float4*)(imgb + (off | rk[t]));
          acc[t] = fma4(w, v, acc[t]);
        }
      }
    }
    if (live) {
      float4* o = (float4*)(g.out + (int64_t)(n0 + dl) * g.row_stride + (int64_t)h * g.F + c * 16);
#pragma unroll
      for (int t = 0; t < 4; ++t) o[(t + cls) & 3] = acc[t];
    }
  }
}

// Q: one quad per destination (16 per wave) as the library, but every lane loads the records
// itself (the quad's four lanes the same address) instead of DPP broadcasts; U records per step.
template <int U>
__global__ void __launch_bounds__(1024) walkQ(Args g) {
  __shared__ __attribute__((aligned(16))) float4 img[kRows * 4];
  __shared__ unsigned short order[kRows];
  __shared__ int lrp[kRows + 1];
  __shared__ int bins[64];
  const int64_t b = xcd_map(blockIdx.x, gridDim.x);
  const int c = (int)(b % g.nchunks);
  const int h = (int)((b / g.nchunks) % g.NH);
  const int k = (int)(b / ((int64_t)g.nchunks * g.NH));
  const int n0 = g.segs[k], R = g.segs[k + 1] - n0;
  prologue<false>(g, n0, R, h, c, img, order, lrp, bins);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane & 3, j = lane >> 2;
  const int2* rh = g.rec + (int64_t)h * g.E;
  const char* imgb = (const char*)img + 16 * q - 64 * n0;
  for (int d0 = wave * 16; d0 < R; d0 += 256) {
    const int d = d0 + j;
    const bool live = d < R;
    const int dl = live ? (int)order[d] : 0;
    const int e = lrp[dl];
    const int end = live ? lrp[dl + 1] : e;
    int need = end - e;
    for (int off = 4; off < 64; off <<= 1) need = max(need, __shfl_xor(need, off));
    const int trips = uni(need);
    const int last = max(end - 1, 0);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t0 = 0; t0 < trips; t0 += U) {
      int2 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = rh[min(e + t0 + u, last)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = e + t0 + u < end;
        const int off = ok ? r[u].x : 64 * n0;
        const float w = ok ? __int_as_float(r[u].y) : 0.f;
        acc = fma4(w, *(const float4*)(imgb + off), acc);
      }
    }
    if (live)
      *(float4*)(g.out + (int64_t)(n0 + dl) * g.row_stride + (int64_t)h * g.F + c * 16 + 4 * q) = acc;
  }
}

__global__ void clobber(float4* p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = make_float4(1.f, (float)i, 0.f, 0.f);
}

}  // namespace lab

static uint64_t s_ = 88172645463325252ull;
static uint32_t rnd() { s_ ^= s_ << 13; s_ ^= s_ >> 7; s_ ^= s_ << 17; return (uint32_t)s_; }

int main(int argc, char** argv) {
  const int G = 20, NPG = 2245, EPG = 61318;
  const int NH = argc > 1 ? atoi(argv[1]) : 4, F = argc > 2 ? atoi(argv[2]) : 256;
  const int N = G * NPG, D = NH * F, nch = F / 16;
  std::vector<std::vector<int>> in(N);
  for (int gi = 0; gi < G; ++gi) {
    for (int k = 0; k < EPG; ++k) {
      int s = gi * NPG + rnd() % NPG, d = gi * NPG + rnd() % NPG;
      if (s != d) in[d].push_back(s);
    }
    for (int i = 0; i < NPG; ++i) in[gi * NPG + i].push_back(gi * NPG + i);
  }
  std::vector<int> rowptr(N + 1, 0), col;
  for (int d = 0; d < N; ++d) { rowptr[d + 1] = rowptr[d] + (int)in[d].size(); for (int s : in[d]) col.push_back(s); }
  const int E = rowptr[N];
  std::vector<float> wt((size_t)NH * E);
  for (auto& x : wt) x = (rnd() % 1000) / 1000.f;
  std::vector<int2> rec((size_t)NH * E);
  for (int h = 0; h < NH; ++h)
    for (int e = 0; e < E; ++e) rec[(size_t)h * E + e] = make_int2(col[e] * 64, *(int*)&wt[(size_t)h * E + e]);
  std::vector<int> seg(G + 1);
  for (int gi = 0; gi <= G; ++gi) seg[gi] = gi * NPG;
  int cnt = G;
  std::vector<float> Wh((size_t)N * D);
  for (auto& x : Wh) x = ((int)(rnd() % 2001) - 1000) / 1000.f;
  printf("N=%d E'=%d NH=%d F=%d\n", N, E, NH, F);

  float *dWh, *dpristine, *dout; int *drp, *dseg, *dcnt; int2* drec; float4* junk;
  const int64_t JN = 320ll << 20 >> 4;
  CK(hipMalloc(&dWh, Wh.size() * 4)); CK(hipMalloc(&dpristine, Wh.size() * 4));
  CK(hipMalloc(&dout, (size_t)N * D * 4));
  CK(hipMalloc(&drp, rowptr.size() * 4)); CK(hipMalloc(&drec, rec.size() * 8));
  CK(hipMalloc(&dseg, seg.size() * 4)); CK(hipMalloc(&dcnt, 4)); CK(hipMalloc(&junk, JN * 16));
  CK(hipMemcpy(dWh, Wh.data(), Wh.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpristine, Wh.data(), Wh.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drp, rowptr.data(), rowptr.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dseg, seg.data(), seg.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcnt, &cnt, 4, hipMemcpyHostToDevice));
  hipEvent_t a, bb; CK(hipEventCreate(&a)); CK(hipEventCreate(&bb));
  const int ITERS = 10;
  auto run = [&](const char* name, auto launch) {
    CK(hipMemset(dout, 0, (size_t)N * D * 4));
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int i = 0; i < ITERS; ++i) {
      lab::clobber<<<2048, 256>>>(junk, JN);
      CK(hipMemcpyAsync(dWh, dpristine, Wh.size() * 4, hipMemcpyDeviceToDevice));
      CK(hipEventRecord(a)); launch(); CK(hipEventRecord(bb)); CK(hipEventSynchronize(bb));
      float ms; CK(hipEventElapsedTime(&ms, a, bb)); t.push_back(ms * 1000.f);
    }
    std::sort(t.begin(), t.end());
    std::vector<float> got((size_t)N * D);
    CK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
    double maxd = 0;
    for (int k = 0; k < 300; ++k) {
      int d = rnd() % N, h = rnd() % NH;
      for (int f = 0; f < F; ++f) {
        double s = 0;
        for (int e = rowptr[d]; e < rowptr[d + 1]; ++e) s += (double)wt[(size_t)h * E + e] * Wh[(size_t)col[e] * D + h * F + f];
        maxd = std::max(maxd, std::fabs(s - got[(size_t)d * D + h * F + f]));
      }
    }
    printf("%-28s median %7.1f us  min %7.1f us   max|d| %.2e\n", name, t[ITERS / 2], t[0], maxd);
  };
  gatx::LdsArgs la{};
  la.rows = dWh; la.row_stride = D; la.rowptr = drp; la.rec = drec; la.E_bound = E; la.segs = dseg;
  la.seg_count = dcnt; la.seg_bound = G; la.N = N; la.NH = NH; la.F = F; la.Fp = F; la.nchunks = nch;
  la.out = dout; la.out_ld = D; la.vec_out = 1;
  lab::Args ga{dWh, D, drp, drec, E, dseg, NH, F, nch, dout};
  const unsigned blocks = G * NH * nch;
  auto lib = [&] { gatx::edge_lds_kernel<2, false><<<blocks, 1024>>>(la); };
  auto b4 = [&] { lab::walkB<4><<<blocks, 1024>>>(ga); };
  auto q8 = [&] { lab::walkQ<8><<<blocks, 1024>>>(ga); };
  auto b8 = [&] { lab::walkB<8><<<blocks, 1024>>>(ga); };
  auto b16 = [&] { lab::walkB<16><<<blocks, 1024>>>(ga); };
  auto q16 = [&] { lab::walkQ<16><<<blocks, 1024>>>(ga); };
  for (int rep = 0; rep < 2; ++rep) {
    run("lib edge_lds<2>", lib);
    run("B lane/dest U=4", b4);
    run("B lane/dest U=8", b8);
    run("B lane/dest U=16", b16);
    run("Q quad/dest own loads U=8", q8);
    run("Q quad/dest own loads U=16", q16);
  }
  return 0;
}
