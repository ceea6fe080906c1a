// Fused softmax cross-entropy over a large vocabulary.
//
// fwd: one block (4 waves) per token row, single pass over the bf16 logits
//      with an online (max, sum-exp) per lane, combined across the block;
//      writes loss[t] and lse[t] (fp32).  The [T, V] probabilities are never
//      materialised.
// bwd: dlogits = (exp(x - lse) - onehot(target)) * dloss * valid, written
//      bf16 (may alias the logits buffer: each element is read before it is
//      written by the same thread).
//
// Parity: reference atorch/atorch/modules/transformer/cross_entropy.py
// (Triton fused CE, AtorchCrossEntropyLoss) and
// modules/distributed_modules/cross_entropy.py (vocab-parallel variant: this
// kernel also accepts a vocab offset so a TP rank can own a vocab slice; the
// cross-rank max/sum are combined by the caller with all-reduce).
#include "dw_common.h"

__global__ void __launch_bounds__(256) xent_fwd_kernel(const bf16_t* __restrict__ logits, const int64_t* __restrict__ target,
                                                       float* __restrict__ loss, float* __restrict__ lse_out,
                                                       float* __restrict__ rowmax_out, float* __restrict__ rowsum_out,
                                                       int64_t T, int V, int64_t ignore_index, int64_t vocab_start,
                                                       float smoothing) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const bf16_t* x = logits + row * (int64_t)V;
  const int nv = V >> 3;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  for (int c = threadIdx.x; c < nv; c += 256) {
    float f[8];
    unpack8(*(const u32x4*)(x + c * 8), f);
    float vm = f[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) vm = fmaxf(vm, f[k]);
    const float mn = fmaxf(m, vm);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) { acc += __expf(f[k] - mn); sx += f[k]; }
    s = s * __expf(m - mn) + acc;
    m = mn;
  }
  for (int c = nv * 8 + threadIdx.x; c < V; c += 256) {  // tail
    const float f = bf2f(x[c]);
    const float mn = fmaxf(m, f);
    s = s * __expf(m - mn) + __expf(f - mn);
    m = mn;
    sx += f;
  }
  const float M = block_max<256>(m, red);
  const float S = block_sum<256>(m == -INFINITY ? 0.f : s * __expf(m - M), red);
  const float SX = block_sum<256>(sx, red);
  if (threadIdx.x == 0) {
    const int64_t t = target[row];
    const float lse = M + __logf(S);
    if (lse_out) lse_out[row] = lse;
    if (rowmax_out) rowmax_out[row] = M;
    if (rowsum_out) rowsum_out[row] = S;
    float l = 0.f;
    if (t != ignore_index) {
      const int64_t lt = t - vocab_start;
      const float xt = (lt >= 0 && lt < V) ? bf2f(x[lt]) : 0.f;
      l = lse - xt;
      if (smoothing > 0.f) l = (1.f - smoothing) * l + smoothing * (lse - SX / (float)V);
    }
    loss[row] = l;
  }
}

__global__ void __launch_bounds__(256) xent_bwd_kernel(const bf16_t* logits, const int64_t* __restrict__ target,
                                                       const float* __restrict__ lse, const float* __restrict__ dloss,
                                                       int dloss_per_row, bf16_t* dlogits, int64_t T, int V,
                                                       int64_t ignore_index, int64_t vocab_start, float smoothing) {
  const int64_t row = blockIdx.x;
  const int64_t t = target[row];
  const float g = (t == ignore_index) ? 0.f : (dloss_per_row ? dloss[row] : dloss[0]);
  const float L = lse[row];
  const bf16_t* x = logits + row * (int64_t)V;
  bf16_t* dx = dlogits + row * (int64_t)V;
  const int64_t lt = t - vocab_start;
  const float off = smoothing / (float)V;
  const int nv = V >> 3;
  for (int c = threadIdx.x; c < nv; c += 256) {
    float f[8];
    unpack8(*(const u32x4*)(x + c * 8), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t j = (int64_t)c * 8 + k;
      const float p = __expf(f[k] - L);
      const float y = (j == lt) ? (1.f - smoothing) : 0.f;
      f[k] = (p - y - off) * g;
    }
    *(u32x4*)(dx + c * 8) = pack8(f);
  }
  for (int c = nv * 8 + threadIdx.x; c < V; c += 256) {
    const float p = __expf(bf2f(x[c]) - L);
    const float y = (c == lt) ? (1.f - smoothing) : 0.f;
    dx[c] = f2bf((p - y - off) * g);
  }
}

extern "C" int dw_xent_fwd(const void* logits, const void* target, void* loss, void* lse, void* rowmax,
                           void* rowsum, int64_t T, int V, int64_t ignore_index, int64_t vocab_start,
                           float smoothing, void* stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(xent_fwd_kernel, dim3((unsigned)T), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)logits, (const int64_t*)target, (float*)loss, (float*)lse,
                     (float*)rowmax, (float*)rowsum, T, V, ignore_index, vocab_start, smoothing);
  DW_LAUNCH_RET;
}

extern "C" int dw_xent_bwd(const void* logits, const void* target, const void* lse, const void* dloss,
                           int dloss_per_row, void* dlogits, int64_t T, int V, int64_t ignore_index,
                           int64_t vocab_start, float smoothing, void* stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(xent_bwd_kernel, dim3((unsigned)T), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)logits, (const int64_t*)target, (const float*)lse, (const float*)dloss,
                     dloss_per_row, (bf16_t*)dlogits, T, V, ignore_index, vocab_start, smoothing);
  DW_LAUNCH_RET;
}

DW_PRELOAD(xent_fwd_kernel);
