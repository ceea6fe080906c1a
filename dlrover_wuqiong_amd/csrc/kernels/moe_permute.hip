// Expert-parallel MoE regroup in ONE launch (parallel/moe.py).
//
// After the token all-to-all, the rows a rank received are ordered
// (source rank, local expert): segment (s, e) holds counts[s][e] rows.  The
// grouped expert GEMM wants them (local expert, source rank)-ordered.  The
// permutation depends only on the [ep, L] count matrix, which stays on the
// device: every workgroup rebuilds both exclusive prefix sums in LDS (ep * L
// is at most a few hundred), each wave then maps its rows
//   i -> segment (s, e) (binary search in the source-major prefix)
//     -> dst = expert_major_off[e][s] + (i - src_major_off[s][e])
// and moves the row with 16-byte vector loads / stores.  dir = 0 scatters
// received -> grouped (out[dst(i)] = x[i]); dir = 1 gathers back
// (out[i] = x[dst(i)]) for the return trip / the backward.
//
// Replaces a host loop of ep * L torch.arange launches plus a host read of
// the counts for the regroup (the all-to-all split sizes still need one).
#include "dw_common.h"

constexpr int MAXSEG = 1024;  // ep * local experts

__global__ void __launch_bounds__(256) moe_regroup_kernel(const char* __restrict__ x, char* __restrict__ out,
                                                         const long long* __restrict__ counts, int ep, int L,
                                                         long long N, int row_bytes, int dir) {
  __shared__ long long src_off[MAXSEG + 1];  // source-major exclusive prefix, + total
  __shared__ long long exp_off[MAXSEG];      // expert-major exclusive prefix, indexed [s * L + e]
  const int nseg = ep * L;
  if (threadIdx.x == 0) {
    long long acc = 0;
    for (int i = 0; i < nseg; ++i) {
      src_off[i] = acc;
      acc += counts[i];
    }
    src_off[nseg] = acc;
    acc = 0;
    for (int e = 0; e < L; ++e)
      for (int s = 0; s < ep; ++s) {
        exp_off[s * L + e] = acc;
        acc += counts[s * L + e];
      }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long nwaves = (long long)gridDim.x * (blockDim.x >> 6);
  const int nvec = row_bytes >> 4;
  for (long long i = wave; i < N; i += nwaves) {
    // segment of row i: the last seg with src_off[seg] <= i (skips empty ones)
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (src_off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const long long dst = exp_off[lo] + (i - src_off[lo]);
    const long long from = dir == 0 ? i : dst, to = dir == 0 ? dst : i;
    const u32x4* src = (const u32x4*)(x + from * row_bytes);
    u32x4* d = (u32x4*)(out + to * row_bytes);
    for (int v = lane; v < nvec; v += 64) d[v] = src[v];
  }
}

// x / out: [N, row_bytes] (row_bytes % 16 == 0, 16-B aligned); counts int64
// [ep, L] on the device with sum == N.
extern "C" int dw_moe_regroup(const void* x, void* out, const void* counts, int ep, int L, long long N,
                              int row_bytes, int dir, void* stream) {
  if (ep * L > MAXSEG || (row_bytes & 15) || N < 0) return (int)hipErrorInvalidValue;
  if (N == 0) return 0;
  const int grid = dw_grid_for(N, 4, 4096);  // 4 waves (rows in flight) per block
  hipLaunchKernelGGL(moe_regroup_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const char*)x,
                     (char*)out, (const long long*)counts, ep, L, N, row_bytes, dir);
  DW_LAUNCH_RET;
}

DW_PRELOAD(moe_regroup_kernel);
