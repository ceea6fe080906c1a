// Fused element-wise ops: bias+GeLU(tanh), SwiGLU, RoPE — fwd and bwd.
// All HBM-bound: 16-byte vector loads/stores, grid-stride, fp32 math.
//
// Parity: reference ATorch fused ops used by auto_accelerate's module
// replacement (atorch/atorch/modules/transformer/layers.py: fused bias-gelu,
// rotary embedding; llama SwiGLU MLP).
#include "dw_common.h"

// y = gelu(x + bias); x:[R, C] bf16, bias [C] bf16 (nullable). Optionally
// writes the biased pre-activation (pre) for the backward.  The bias-free
// GPT2-1.5B pass (8192 x 6400) runs at 6.3 TB/s; 2 / 4 vectors per thread per
// trip measured the same (profiles/r4/norm_fwd_gelu_ab.jsonl).
__global__ void __launch_bounds__(256) bias_gelu_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ bias,
                                                            bf16_t* __restrict__ y, bf16_t* __restrict__ pre,
                                                            int64_t n, int C) {
  const int64_t nv = n >> 3;
  for (int64_t vi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; vi < nv;
       vi += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = vi << 3;
    float a[8], b[8], o[8];
    unpack8(*(const u32x4*)(x + i), a);
    if (bias) {
      unpack8(*(const u32x4*)(bias + (i % C)), b);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += b[k];
      if (pre) *(u32x4*)(pre + i) = pack8(a);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = gelu_tanh(a[k]);
    *(u32x4*)(y + i) = pack8(o);
  }
}

// dx = dy * gelu'(pre). (dbias is reduced by the caller from dx.)
__global__ void __launch_bounds__(256) gelu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ pre,
                                                       bf16_t* __restrict__ dx, int64_t n) {
  const int64_t nv = n >> 3;
  for (int64_t vi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; vi < nv;
       vi += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = vi << 3;
    float g[8], a[8], o[8];
    unpack8(*(const u32x4*)(dy + i), g);
    unpack8(*(const u32x4*)(pre + i), a);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] * gelu_tanh_grad(a[k]);
    *(u32x4*)(dx + i) = pack8(o);
  }
}

extern "C" int dw_bias_gelu_fwd(const void* x, const void* bias, void* y, void* pre, int64_t n, int C,
                                void* stream) {
  if (n % 8 || C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3(dw_grid_for(n / 8, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)x, (const bf16_t*)bias, (bf16_t*)y,
                     (bf16_t*)pre, n, C);
  DW_LAUNCH_RET;
}
extern "C" int dw_gelu_bwd(const void* dy, const void* pre, void* dx, int64_t n, void* stream) {
  if (n % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(dw_grid_for(n / 8, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)dy, (const bf16_t*)pre, (bf16_t*)dx, n);
  DW_LAUNCH_RET;
}

// Column sums of a [R, C] bf16 matrix -> fp32/bf16 [C] (bias gradients).
// Block = 256 threads covering 8*32 = 256 columns? -> each thread owns one
// 8-column vector and strides over rows; partial rows per blockIdx.y.
__global__ void __launch_bounds__(256) colsum_partial_kernel(const bf16_t* __restrict__ x, int64_t R, int C,
                                                             float* __restrict__ partial) {
  const int cv = blockIdx.x * 256 + threadIdx.x;  // vector column
  const int nvc = C >> 3;
  if (cv >= nvc) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = blockIdx.y; r < R; r += gridDim.y) {
    float f[8];
    unpack8(*(const u32x4*)(x + r * C + cv * 8), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += f[k];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) partial[(int64_t)blockIdx.y * C + cv * 8 + k] = acc[k];
}
__global__ void colsum_final_kernel(const float* __restrict__ partial, int P, int C, bf16_t* out_bf,
                                    float* out_f) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += partial[(int64_t)p * C + c];
  if (out_bf) out_bf[c] = f2bf(s);
  if (out_f) out_f[c] = s;
}
extern "C" int dw_colsum_parts(int64_t R) { return R < 256 ? (int)R : 256; }
extern "C" int dw_colsum(const void* x, int64_t R, int C, void* partial, void* out, int out_fp32,
                         void* stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int P = dw_colsum_parts(R);
  hipStream_t s = (hipStream_t)stream;
  dim3 g1((C / 8 + 255) / 256, P);
  hipLaunchKernelGGL(colsum_partial_kernel, g1, dim3(256), 0, s, (const bf16_t*)x, R, C, (float*)partial);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 255) / 256), dim3(256), 0, s, (const float*)partial, P, C,
                     out_fp32 ? nullptr : (bf16_t*)out, out_fp32 ? (float*)out : nullptr);
  DW_LAUNCH_RET;
}

// SwiGLU: y = silu(a) * b with a,b halves of x:[R, 2C] (gate|up) -> y:[R, C]
__device__ __forceinline__ float silu(float a) { return a / (1.f + __expf(-a)); }
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         int64_t R, int C) {
  const int64_t nv = R * (C >> 3);
  const int cvs = C >> 3;
  for (int64_t vi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; vi < nv;
       vi += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = vi / cvs;
    const int cv = (int)(vi % cvs);
    float a[8], b[8], o[8];
    unpack8(*(const u32x4*)(x + r * 2 * C + cv * 8), a);
    unpack8(*(const u32x4*)(x + r * 2 * C + C + cv * 8), b);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = silu(a[k]) * b[k];
    *(u32x4*)(y + r * C + cv * 8) = pack8(o);
  }
}
__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                         bf16_t* __restrict__ dx, int64_t R, int C) {
  const int64_t nv = R * (C >> 3);
  const int cvs = C >> 3;
  for (int64_t vi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; vi < nv;
       vi += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = vi / cvs;
    const int cv = (int)(vi % cvs);
    float a[8], b[8], g[8], da[8], dbv[8];
    unpack8(*(const u32x4*)(x + r * 2 * C + cv * 8), a);
    unpack8(*(const u32x4*)(x + r * 2 * C + C + cv * 8), b);
    unpack8(*(const u32x4*)(dy + r * C + cv * 8), g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float sg = 1.f / (1.f + __expf(-a[k]));
      const float sa = a[k] * sg;
      dbv[k] = g[k] * sa;
      da[k] = g[k] * b[k] * sg * (1.f + a[k] * (1.f - sg));
    }
    *(u32x4*)(dx + r * 2 * C + cv * 8) = pack8(da);
    *(u32x4*)(dx + r * 2 * C + C + cv * 8) = pack8(dbv);
  }
}
extern "C" int dw_swiglu_fwd(const void* x, void* y, int64_t R, int C, void* stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(dw_grid_for(R * C / 8, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, R, C);
  DW_LAUNCH_RET;
}
extern "C" int dw_swiglu_bwd(const void* dy, const void* x, void* dx, int64_t R, int C, void* stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(dw_grid_for(R * C / 8, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)dy, (const bf16_t*)x, (bf16_t*)dx, R, C);
  DW_LAUNCH_RET;
}

// RoPE (non-interleaved / "rotate_half" convention, as HF Llama):
// x:[B, S, NH, D] bf16 (contiguous), cos/sin:[S, D/2] fp32 table computed on
// the host (guide App. B: trig tables, not on-device sinf/cosf).
// out[..., i]       = x[i] * c - x[i + D/2] * s
// out[..., i + D/2] = x[i + D/2] * c + x[i] * s          (i < D/2)
// backward = same rotation with -sin (sign = -1).
__global__ void __launch_bounds__(256) rope_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                   const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                   int64_t BS, int S, int NH, int D, float sign,
                                                   const int* __restrict__ pos_ids, int rows) {
  const int half = D >> 1;
  const int hv = half >> 3;  // 8-wide vectors per half
  const int64_t total = BS * NH * hv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int v = (int)(t % hv);
    const int64_t rh = t / hv;  // (b*S + s)*NH + h
    const int64_t bs = rh / NH;
    // positions outside the table clamp to its range (never read past it)
    const int s = pos_ids ? min(max(pos_ids[bs], 0), rows - 1) : (int)(bs % S);
    const bf16_t* xr = x + rh * D;
    bf16_t* yr = y + rh * D;
    float a[8], b[8], o1[8], o2[8];
    unpack8(*(const u32x4*)(xr + v * 8), a);
    unpack8(*(const u32x4*)(xr + half + v * 8), b);
    const float* cr = cosb + (int64_t)s * half + v * 8;
    const float* sr = sinb + (int64_t)s * half + v * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float c = cr[k], sn = sign * sr[k];
      o1[k] = a[k] * c - b[k] * sn;
      o2[k] = b[k] * c + a[k] * sn;
    }
    *(u32x4*)(yr + v * 8) = pack8(o1);
    *(u32x4*)(yr + half + v * 8) = pack8(o2);
  }
}
extern "C" int dw_rope(const void* x, void* y, const void* cosb, const void* sinb, int64_t B, int S,
                       int NH, int D, int backward, const void* pos_ids, int rows, void* stream) {
  if (D % 16 || rows < 1 || (!pos_ids && rows < S)) return (int)hipErrorInvalidValue;
  const int64_t total = B * S * NH * (D / 16);
  hipLaunchKernelGGL(rope_kernel, dim3(dw_grid_for(total, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, (bf16_t*)y, (const float*)cosb, (const float*)sinb, B * S, S, NH, D,
                     backward ? -1.f : 1.f, (const int*)pos_ids, rows);
  DW_LAUNCH_RET;
}

// Fused QKV split + RoPE (Llama attention prologue).  The QKV projection's
// output [B, S, NH + 2 NKV, D] is read ONCE: query / key heads are rotated
// (rotate-half) and written to contiguous q [B, S, NH, D] / k [B, S, NKV, D],
// value heads copied to v [B, S, NKV, D] -- instead of three .contiguous()
// copies of the split views and two rope passes over q and k.  BACKWARD: the
// inverse -- dq / dk rotated back (sin negated) and dq | dk | dv written
// interleaved into dqkv [B, S, NH + 2 NKV, D] (the split's gradient), one
// pass.  One thread per (row, head, 8-wide vector of the first half): loads
// the 8 elements and their rotate-half partners 16 bytes at a time.
template <bool BWD>
__global__ void __launch_bounds__(256) qkv_rope_kernel(bf16_t* __restrict__ qkv, bf16_t* __restrict__ q,
                                                       bf16_t* __restrict__ k, bf16_t* __restrict__ v,
                                                       const float* __restrict__ cosb,
                                                       const float* __restrict__ sinb, int64_t BS, int S, int NH,
                                                       int NKV, int D, const int* __restrict__ pos_ids, int rows) {
  const int half = D >> 1;
  const int hv = half >> 3;
  const int NT = NH + 2 * NKV;
  const int64_t total = BS * NT * hv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int vi = (int)(t % hv);
    const int64_t rh = t / hv;  // (b*S + s) * NT + head
    const int head = (int)(rh % NT);
    const int64_t bs = rh / NT;
    bf16_t* packed = qkv + rh * D;
    bf16_t* sep;
    if (head < NH)
      sep = q + (bs * NH + head) * D;
    else if (head < NH + NKV)
      sep = k + (bs * NKV + head - NH) * D;
    else
      sep = v + (bs * NKV + head - NH - NKV) * D;
    const bf16_t* src = BWD ? sep : packed;
    bf16_t* dst = BWD ? packed : sep;
    const u32x4 a4 = *(const u32x4*)(src + vi * 8), b4 = *(const u32x4*)(src + half + vi * 8);
    if (head >= NH + NKV) {  // value head: a plain copy
      *(u32x4*)(dst + vi * 8) = a4;
      *(u32x4*)(dst + half + vi * 8) = b4;
      continue;
    }
    const int sp = pos_ids ? min(max(pos_ids[bs], 0), rows - 1) : (int)(bs % S);
    const float* cr = cosb + (int64_t)sp * half + vi * 8;
    const float* sr = sinb + (int64_t)sp * half + vi * 8;
    const f32x4 c0 = *(const f32x4*)cr, c1 = *(const f32x4*)(cr + 4);
    const f32x4 s0 = *(const f32x4*)sr, s1 = *(const f32x4*)(sr + 4);
    float a[8], b[8], o1[8], o2[8];
    unpack8(a4, a);
    unpack8(b4, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? c0[j] : c1[j - 4];
      const float sn = (BWD ? -1.f : 1.f) * (j < 4 ? s0[j] : s1[j - 4]);
      o1[j] = a[j] * c - b[j] * sn;
      o2[j] = b[j] * c + a[j] * sn;
    }
    *(u32x4*)(dst + vi * 8) = pack8(o1);
    *(u32x4*)(dst + half + vi * 8) = pack8(o2);
  }
}

// backward = 0: qkv -> (q, k, v) rotated; 1: (dq, dk, dv) -> dqkv, inverse
// rotation.  cos / sin: fp32 [rows, D/2]; pos_ids (nullable) int32 [B*S].
extern "C" int dw_qkv_rope(void* qkv, void* q, void* k, void* v, const void* cosb, const void* sinb, int64_t B,
                           int S, int NH, int NKV, int D, int backward, const void* pos_ids, int rows,
                           void* stream) {
  if (D % 16 || rows < 1 || (!pos_ids && rows < S) || NH < 1 || NKV < 1) return (int)hipErrorInvalidValue;
  const int64_t total = B * S * (NH + 2 * NKV) * (D / 16);
  const dim3 g(dw_grid_for(total, 256, 8192));
  if (backward)
    hipLaunchKernelGGL(qkv_rope_kernel<true>, g, dim3(256), 0, (hipStream_t)stream, (bf16_t*)qkv, (bf16_t*)q,
                       (bf16_t*)k, (bf16_t*)v, (const float*)cosb, (const float*)sinb, B * S, S, NH, NKV, D,
                       (const int*)pos_ids, rows);
  else
    hipLaunchKernelGGL(qkv_rope_kernel<false>, g, dim3(256), 0, (hipStream_t)stream, (bf16_t*)qkv, (bf16_t*)q,
                       (bf16_t*)k, (bf16_t*)v, (const float*)cosb, (const float*)sinb, B * S, S, NH, NKV, D,
                       (const int*)pos_ids, rows);
  DW_LAUNCH_RET;
}

DW_PRELOAD(gelu_bwd_kernel);
