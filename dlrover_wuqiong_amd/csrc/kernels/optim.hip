// Fused optimizer kernels over *flat* parameter/gradient/state buffers.
//
// The training engine keeps every parameter, gradient and optimizer state as
// a view into one contiguous buffer per role (bf16 params, bf16 grads, fp32
// master/exp_avg/exp_avg_sq).  An optimizer step is then one HBM-streaming
// launch over N elements (28 B/elem for mixed-precision AdamW) instead of a
// python loop over ~600 tensors, and a flash checkpoint of the optimizer is a
// handful of large contiguous copies.
//
// Parity: reference ATorch optimizers (atorch/atorch/optimizers/agd.py,
// adam_offload.py, bf16_optimizer.py) and the apex/DeepSpeed FusedAdam it
// depends on.  Grad clipping needs no host sync: the global-norm kernel writes
// a device scalar that the update kernel reads.
#include "dw_common.h"

template <typename T> __device__ __forceinline__ float ld(const T* p, int64_t i);
template <> __device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <> __device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
template <typename T> __device__ __forceinline__ void st(T* p, int64_t i, float v);
template <> __device__ __forceinline__ void st<float>(float* p, int64_t i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void st<bf16_t>(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

// load 8 consecutive elements (i multiple of 8) as floats
template <typename T> __device__ __forceinline__ void ld8(const T* p, int64_t i, float* f);
template <> __device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, int64_t i, float* f) {
  u32x4 v = *(const u32x4*)(p + i);
  unpack8(v, f);
}
template <> __device__ __forceinline__ void ld8<float>(const float* p, int64_t i, float* f) {
  f32x4 a = *(const f32x4*)(p + i), b = *(const f32x4*)(p + i + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}
template <typename T> __device__ __forceinline__ void st8(T* p, int64_t i, const float* f);
template <> __device__ __forceinline__ void st8<bf16_t>(bf16_t* p, int64_t i, const float* f) {
  *(u32x4*)(p + i) = pack8(f);
}
template <> __device__ __forceinline__ void st8<float>(float* p, int64_t i, const float* f) {
  f32x4 a = {f[0], f[1], f[2], f[3]}, b = {f[4], f[5], f[6], f[7]};
  *(f32x4*)(p + i) = a;
  *(f32x4*)(p + i + 4) = b;
}

// Weight-decay selection: decay_mask (one byte per 64-element block; flat
// buffers align every parameter to 64 elements) when non-null, else the
// prefix [0, n_decay).
struct AdamArgs {
  float lr, beta1, beta2, eps, wd, bc1, bc2;  // bc = 1 - beta^t
  int64_t n, n_decay;
  int adamw;  // 1: decoupled weight decay, 0: L2 added to the gradient
  const unsigned char* decay_mask;
};

__device__ __forceinline__ bool decays(const unsigned char* mask, int64_t n_decay, int64_t i) {
  return mask ? (mask[i >> 6] != 0) : (i < n_decay);
}

// One AdamW / Adam-L2 update of one element -- shared by the flat update and
// the deferred-state replay below, so both produce bit-identical results.
__device__ __forceinline__ void adam_elem(float g, float gs, bool decay, const AdamArgs& a, float step_size,
                                          float rbc2, float& w, float& mm, float& vv) {
  // Every multiply-add is an explicit fma and no product feeds an add: the
  // library builds with -ffp-contract=fast, and the backend contracts the
  // packed-fp32 code of the vectorised flat update differently from the
  // scalar replay loop (1-ulp master differences on GPU).  With nothing left
  // to contract both kernels round identically.
  float gk = g * gs;
  if (!a.adamw && decay) gk = __builtin_fmaf(a.wd, w, gk);
  mm = __builtin_fmaf(a.beta1, mm, (1.f - a.beta1) * gk);
  vv = __builtin_fmaf(a.beta2, vv, (1.f - a.beta2) * gk * gk);
  const float denom = __builtin_fmaf(sqrtf(vv), rbc2, a.eps);
  if (a.adamw && decay) w = __builtin_fmaf(-(a.lr * a.wd), w, w);
  w = w - (step_size * mm) / denom;
}

// master == nullptr: the param itself is the fp32 master (P must be float)
template <typename G, typename P>
__global__ void __launch_bounds__(256) adam_flat_kernel(P* __restrict__ param, float* __restrict__ master,
                                                        const G* __restrict__ grad, float* __restrict__ m,
                                                        float* __restrict__ v, const float* __restrict__ gscale,
                                                        AdamArgs a) {
  const float gs = gscale ? *gscale : 1.f;
  const float step_size = a.lr / a.bc1;
  const float rbc2 = rsqrtf(a.bc2);
  const int64_t nvec = a.n >> 3;
  for (int64_t vi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; vi < nvec;
       vi += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = vi << 3;
    float g[8], w[8], mm[8], vv[8];
    ld8<G>(grad, i, g);
    if (master) ld8<float>(master, i, w); else ld8<P>(param, i, w);
    ld8<float>(m, i, mm);
    ld8<float>(v, i, vv);
    const bool dblk = decays(a.decay_mask, a.n_decay, i);  // 8-vector never straddles a 64-block
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool decay = a.decay_mask ? dblk : (i + k) < a.n_decay;
      adam_elem(g[k], gs, decay, a, step_size, rbc2, w[k], mm[k], vv[k]);
    }
    st8<float>(m, i, mm);
    st8<float>(v, i, vv);
    if (master) st8<float>(master, i, w);
    st8<P>(param, i, w);
  }
  // scalar tail
  for (int64_t i = (nvec << 3) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const bool decay = decays(a.decay_mask, a.n_decay, i);
    float w = master ? master[i] : ld<P>(param, i);
    float mk = m[i], vk = v[i];
    adam_elem(ld<G>(grad, i), gs, decay, a, step_size, rbc2, w, mk, vk);
    m[i] = mk; v[i] = vk;
    if (master) master[i] = w;
    st<P>(param, i, w);
  }
}

// Deferred optimizer-state write-back (flash-checkpoint ring snapshots,
// optimizers/fused.py): K consecutive updates of [0, n) from K saved
// gradients.  write_state = 0: only the parameters are written (the update
// of an element whose OLD master / exp_avg / exp_avg_sq a pending snapshot
// has not copied yet -- they stay untouched); write_state = 1: the replay
// once the snapshot has them -- master, moments and (identical) parameters.
constexpr int REPLAY_MAX = 8;
struct AdamReplay {
  AdamArgs a[REPLAY_MAX];        // per step: lr, bc1, bc2 (+ the shared betas / eps / wd)
  const void* grad[REPLAY_MAX];  // saved gradients, element 0 = element lo of the flat buffer
  const float* gscale[REPLAY_MAX];
  int K, write_state;
};

template <typename G, typename P>
__global__ void __launch_bounds__(256) adam_replay_kernel(P* __restrict__ param, float* __restrict__ master,
                                                          float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                          AdamReplay r) {
  float gs[REPLAY_MAX], ss[REPLAY_MAX], rb[REPLAY_MAX];
#pragma unroll
  for (int k = 0; k < REPLAY_MAX; ++k) {
    if (k < r.K) {
      gs[k] = r.gscale[k] ? *r.gscale[k] : 1.f;
      ss[k] = r.a[k].lr / r.a[k].bc1;
      rb[k] = rsqrtf(r.a[k].bc2);
    }
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float w = master ? master[i] : ld<P>(param, i);
    float mk = m[i], vk = v[i];
    const bool decay = decays(r.a[0].decay_mask, r.a[0].n_decay, i);
    for (int k = 0; k < r.K; ++k)
      adam_elem(ld<G>((const G*)r.grad[k], i), gs[k], decay, r.a[k], ss[k], rb[k], w, mk, vk);
    if (r.write_state) {
      m[i] = mk;
      v[i] = vk;
      if (master) master[i] = w;
    }
    st<P>(param, i, w);
  }
}

// lrs / bc1s / bc2s / grads / gscales: host arrays of K (<= 8) entries.
extern "C" int dw_adam_replay(void* param, int param_dtype, void* master, void* m, void* v, int64_t n, int K,
                              const void* const* grads, int grad_dtype, const void* const* gscales, const float* lrs,
                              const float* bc1s, const float* bc2s, float beta1, float beta2, float eps, float wd,
                              int adamw, const void* decay_mask, int write_state, void* stream) {
  if (K < 1 || K > REPLAY_MAX || n < 0) return (int)hipErrorInvalidValue;
  AdamReplay r{};
  r.K = K;
  r.write_state = write_state;
  for (int k = 0; k < K; ++k) {
    r.a[k] = AdamArgs{lrs[k], beta1, beta2, eps, wd, bc1s[k], bc2s[k], n, 0, adamw,
                      (const unsigned char*)decay_mask};
    r.grad[k] = grads[k];
    r.gscale[k] = (const float*)gscales[k];
  }
  if (n == 0) return 0;
  const int grid = dw_grid_for(n, 256, 8192);
  hipStream_t s = (hipStream_t)stream;
  if (param_dtype == 1 && grad_dtype == 1)
    hipLaunchKernelGGL((adam_replay_kernel<bf16_t, bf16_t>), dim3(grid), dim3(256), 0, s, (bf16_t*)param,
                       (float*)master, (float*)m, (float*)v, n, r);
  else if (param_dtype == 1 && grad_dtype == 0)
    hipLaunchKernelGGL((adam_replay_kernel<float, bf16_t>), dim3(grid), dim3(256), 0, s, (bf16_t*)param,
                       (float*)master, (float*)m, (float*)v, n, r);
  else if (param_dtype == 0 && grad_dtype == 0)
    hipLaunchKernelGGL((adam_replay_kernel<float, float>), dim3(grid), dim3(256), 0, s, (float*)param,
                       (float*)master, (float*)m, (float*)v, n, r);
  else
    hipLaunchKernelGGL((adam_replay_kernel<bf16_t, float>), dim3(grid), dim3(256), 0, s, (float*)param,
                       (float*)master, (float*)m, (float*)v, n, r);
  DW_LAUNCH_RET;
}

// dtype codes: 0 fp32, 1 bf16
extern "C" int dw_adam_flat(void* param, int param_dtype, void* master, const void* grad,
                            int grad_dtype, void* m, void* v, const void* gscale, int64_t n,
                            int64_t n_decay, float lr, float beta1, float beta2, float eps,
                            float wd, float bc1, float bc2, int adamw, const void* decay_mask,
                            void* stream) {
  AdamArgs a{lr, beta1, beta2, eps, wd, bc1, bc2, n, n_decay, adamw, (const unsigned char*)decay_mask};
  // up to 8192 blocks: 8.60 -> 8.30 ms at GPT2-1.5B size, where a pure
  // 28 B/element copy takes 8.24 ms -- the update runs at the HBM ceiling;
  // a contiguous-per-instruction layout and non-temporal accesses measured
  // within +-2 % (profiles/r4/adam_layout_probe.jsonl, scripts/probe/adam_probe.hip)
  int grid = dw_grid_for((n + 7) / 8, 256, 8192);
  hipStream_t s = (hipStream_t)stream;
  if (param_dtype == 1 && grad_dtype == 1) {
    hipLaunchKernelGGL((adam_flat_kernel<bf16_t, bf16_t>), dim3(grid), dim3(256), 0, s,
                       (bf16_t*)param, (float*)master, (const bf16_t*)grad, (float*)m, (float*)v,
                       (const float*)gscale, a);
  } else if (param_dtype == 1 && grad_dtype == 0) {
    hipLaunchKernelGGL((adam_flat_kernel<float, bf16_t>), dim3(grid), dim3(256), 0, s,
                       (bf16_t*)param, (float*)master, (const float*)grad, (float*)m, (float*)v,
                       (const float*)gscale, a);
  } else if (param_dtype == 0 && grad_dtype == 0) {
    hipLaunchKernelGGL((adam_flat_kernel<float, float>), dim3(grid), dim3(256), 0, s,
                       (float*)param, (float*)master, (const float*)grad, (float*)m, (float*)v,
                       (const float*)gscale, a);
  } else {
    hipLaunchKernelGGL((adam_flat_kernel<bf16_t, float>), dim3(grid), dim3(256), 0, s,
                       (float*)param, (float*)master, (const bf16_t*)grad, (float*)m, (float*)v,
                       (const float*)gscale, a);
  }
  DW_LAUNCH_RET;
}

// --------------------------------------------------------------------------
// AGD (Auto-switchable optimizer with stepwise Gradient Difference, NeurIPS'23).
// Bit-for-bit the update of reference atorch/atorch/optimizers/agd.py:84-150
// (decoupled, non-fixed decay; no amsgrad/win - those run the python path):
//   w   *= 1 - lr*wd                                   (decay params only)
//   m_t  = b1 m + (1-b1) g
//   s    = m_t/bc1_t - m_{t-1}/bc1_{t-1}   (s = m_t/bc1_t at t == 1)
//   v_t  = b2 v + (1-b2) s^2
//   upd  = m_t / max(sqrt(v_t), delta*sqrt(bc2_t)) ; clip to [-clip, clip]
//   w   -= lr*sqrt(bc2_t)/bc1_t * upd
struct AgdArgs {
  float lr, beta1, beta2, delta, wd, bc1, bc1_prev, bc2, clip;
  int64_t n, n_decay;
  const unsigned char* decay_mask;
};

template <typename G, typename P>
__global__ void __launch_bounds__(256) agd_flat_kernel(P* __restrict__ param, float* __restrict__ master,
                                                       const G* __restrict__ grad, float* __restrict__ m,
                                                       float* __restrict__ v, const float* __restrict__ gscale,
                                                       AgdArgs a) {
  const float gs = gscale ? *gscale : 1.f;
  const float sqbc2 = sqrtf(a.bc2);
  const float delta_adj = a.delta * sqbc2;
  const float lr_adj = a.lr * sqbc2 / a.bc1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float w = master ? master[i] : ld<P>(param, i);
    if (decays(a.decay_mask, a.n_decay, i)) w *= 1.f - a.lr * a.wd;
    const float gk = ld<G>(grad, i) * gs;
    const float mprev = m[i];
    const float mk = a.beta1 * mprev + (1.f - a.beta1) * gk;
    const float s = (a.bc1_prev > 0.f) ? (mk / a.bc1 - mprev / a.bc1_prev) : mk / a.bc1;
    const float vk = a.beta2 * v[i] + (1.f - a.beta2) * s * s;
    float upd = mk / fmaxf(sqrtf(vk), delta_adj);
    if (a.clip > 0.f) upd = fminf(fmaxf(upd, -a.clip), a.clip);
    w -= lr_adj * upd;
    m[i] = mk;
    v[i] = vk;
    if (master) master[i] = w;
    st<P>(param, i, w);
  }
}

extern "C" int dw_agd_flat(void* param, int param_dtype, void* master, const void* grad,
                           int grad_dtype, void* m, void* v, const void* gscale, int64_t n,
                           int64_t n_decay, float lr, float beta1, float beta2, float delta,
                           float wd, float bc1, float bc1_prev, float bc2, float clip,
                           const void* decay_mask, void* stream) {
  AgdArgs a{lr, beta1, beta2, delta, wd, bc1, bc1_prev, bc2, clip, n, n_decay,
            (const unsigned char*)decay_mask};
  int grid = dw_grid_for(n, 256, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (param_dtype == 1 && grad_dtype == 1)
    hipLaunchKernelGGL((agd_flat_kernel<bf16_t, bf16_t>), dim3(grid), dim3(256), 0, s, (bf16_t*)param,
                       (float*)master, (const bf16_t*)grad, (float*)m, (float*)v, (const float*)gscale, a);
  else if (param_dtype == 0 && grad_dtype == 0)
    hipLaunchKernelGGL((agd_flat_kernel<float, float>), dim3(grid), dim3(256), 0, s, (float*)param,
                       (float*)master, (const float*)grad, (float*)m, (float*)v, (const float*)gscale, a);
  else if (param_dtype == 1 && grad_dtype == 0)
    hipLaunchKernelGGL((agd_flat_kernel<float, bf16_t>), dim3(grid), dim3(256), 0, s, (bf16_t*)param,
                       (float*)master, (const float*)grad, (float*)m, (float*)v, (const float*)gscale, a);
  else
    hipLaunchKernelGGL((agd_flat_kernel<bf16_t, float>), dim3(grid), dim3(256), 0, s, (float*)param,
                       (float*)master, (const bf16_t*)grad, (float*)m, (float*)v, (const float*)gscale, a);
  DW_LAUNCH_RET;
}

// --------------------------------------------------------------------------
// Global L2 norm of a flat buffer: block partial sums, then a deterministic
// fixed-order grid sum (grid_sum_finish) added to *out (zeroed by the caller).
template <typename G>
__global__ void __launch_bounds__(256) sumsq_kernel(const G* __restrict__ x, int64_t n, float* out, float* ws) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t nvec = n >> 3;
  for (int64_t vi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; vi < nvec;
       vi += (int64_t)gridDim.x * blockDim.x) {
    float f[8];
    ld8<G>(x, vi << 3, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += f[k] * f[k];
  }
  for (int64_t i = (nvec << 3) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float f = ld<G>(x, i);
    acc += f * f;
  }
  acc = block_sum<256>(acc, red);
  __syncthreads();  // red is reused by the finish
  grid_sum_finish<256>(acc, ws, out, red);
}

// ws: float[GRID_SUM_MAX + 1] (see grid_sum_finish)
extern "C" int dw_sumsq_flat(const void* x, int dtype, int64_t n, void* out, void* ws, void* stream) {
  int grid = dw_grid_for((n + 7) / 8, 256, 1024);
  if (dtype == 1)
    hipLaunchKernelGGL(sumsq_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, n, (float*)out, (float*)ws);
  else
    hipLaunchKernelGGL(sumsq_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, n, (float*)out, (float*)ws);
  DW_LAUNCH_RET;
}

// coef = pre_scale * min(1, max_norm / (sqrt(sumsq)*pre_scale + 1e-6))
// writes coef and the (scaled) norm.
__global__ void clip_coef_kernel(const float* sumsq, float max_norm, float pre_scale, float* coef,
                                 float* norm_out) {
  float nrm = sqrtf(*sumsq) * pre_scale;
  float c = max_norm > 0.f ? fminf(1.f, max_norm / (nrm + 1e-6f)) : 1.f;
  *coef = c * pre_scale;
  if (norm_out) *norm_out = nrm;
}
extern "C" int dw_clip_coef(const void* sumsq, float max_norm, float pre_scale, void* coef,
                            void* norm_out, void* stream) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream,
                     (const float*)sumsq, max_norm, pre_scale, (float*)coef, (float*)norm_out);
  DW_LAUNCH_RET;
}

// y = x * (*scale)  (in place allowed), bf16 or fp32
template <typename T>
__global__ void scale_kernel(T* x, int64_t n, const float* scale) {
  const float s = *scale;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    st<T>(x, i, ld<T>(x, i) * s);
}
extern "C" int dw_scale_flat(void* x, int dtype, int64_t n, const void* scale, void* stream) {
  int grid = dw_grid_for(n, 256, 2048);
  if (dtype == 1)
    hipLaunchKernelGGL(scale_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (bf16_t*)x, n, (const float*)scale);
  else
    hipLaunchKernelGGL(scale_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (float*)x, n, (const float*)scale);
  DW_LAUNCH_RET;
}

DW_PRELOAD((adam_flat_kernel<float, bf16_t>));
