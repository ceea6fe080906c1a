// Fused AdamW with 4-bit (or 8-bit) block-quantized optimizer states.
//
// One pass per element: dequantize m and v, AdamW update in fp32, write the
// parameter, re-quantize m and v with fresh per-group scales.  Memory per
// parameter element and step: param r/w (2x2 B bf16) + grad 2 B + states
// 2 x 0.5 B (4-bit) + scales -> ~7 B instead of ~18 B for fp32 states, and
// the state memory itself shrinks 8x (16 GB -> 2 GB for a 1B-param model).
//
// Quantization (groups of 128 consecutive elements, one fp32 scale each):
//  * first moment m (signed): scale = absmax; 4-bit code -> nonlinear signed
//    map {0, +-1/64, +-1/16, +-1/8, +-1/4, +-1/2, +-3/4, +-1} (dense near 0,
//    where most of m lives); 8-bit: linear in [-1, 1] (127 levels).
//  * second moment v (>= 0): scale = max; code k -> ((k+1)/L)^2 * scale
//    (quadratic map with NO zero level: a tiny v is rounded UP, never to 0,
//    so m / sqrt(v) cannot blow up -- the zero-point problem of 4-bit
//    second moments).
// A 16-lane group of a wave owns one 128-element group (8 elements per lane);
// group max / absmax come from 4 xor-shuffles, no LDS.
//
// Parity: ATorch ``atorch/optimizers/low_bit`` (Q_AdamW: group-wise 4-bit
// first moment, zero-point-free second moment; the reference implements it
// in Python + CUDA quant kernels, here one fused HIP kernel).
#include "dw_common.h"

__constant__ float kM4[16] = {0.f, 0.015625f, 0.0625f, 0.125f, 0.25f, 0.5f, 0.75f, 1.f,
                              0.f, -0.015625f, -0.0625f, -0.125f, -0.25f, -0.5f, -0.75f, -1.f};

__device__ __forceinline__ float group16_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  v = fmaxf(v, __shfl_xor(v, 8, 64));
  return v;
}

__device__ __forceinline__ int quant_m4(float x) {  // x in [-1, 1] -> nearest code
  const float a = fabsf(x);
  // thresholds = midpoints of {0, 1/64, 1/16, 1/8, 1/4, 1/2, 3/4, 1}
  int k = (a > 0.0078125f) + (a > 0.0390625f) + (a > 0.09375f) + (a > 0.1875f) + (a > 0.375f) + (a > 0.625f) +
          (a > 0.875f);
  return (x < 0.f && k > 0) ? (k | 8) : k;
}

template <int BITS>
__device__ __forceinline__ float deq_m(int code, float scale) {
  if constexpr (BITS == 4) return kM4[code] * scale;
  else return (float)((signed char)code) * (scale / 127.f);
}
template <int BITS>
__device__ __forceinline__ int q_m(float x, float inv_scale) {
  if constexpr (BITS == 4) return quant_m4(x * inv_scale);
  else {
    int q = __float2int_rn(x * inv_scale * 127.f);
    return (q < -127 ? -127 : (q > 127 ? 127 : q)) & 0xff;
  }
}
template <int BITS>
__device__ __forceinline__ float deq_v(int code, float scale) {
  constexpr float L = (BITS == 4) ? 16.f : 256.f;
  const float r = (float)(code + 1) / L;
  return r * r * scale;
}
template <int BITS>
__device__ __forceinline__ int q_v(float v, float scale) {  // smallest level >= (v rounded in sqrt space)
  constexpr int L = (BITS == 4) ? 16 : 256;
  if (scale <= 0.f) return 0;
  int k = __float2int_rn(sqrtf(v / scale) * (float)L) - 1;
  return k < 0 ? 0 : (k > L - 1 ? L - 1 : k);
}

// P: bf16 or fp32 parameter; G: bf16 or fp32 gradient.  n % 128 == 0 for the
// state arrays (callers pad); elements >= n_real are skipped for p/g.
template <int BITS, typename P, typename G>
__global__ void __launch_bounds__(256) qadamw_kernel(P* __restrict__ p, const G* __restrict__ g,
                                                     unsigned char* __restrict__ mq, unsigned char* __restrict__ vq,
                                                     float* __restrict__ ms, float* __restrict__ vs, int64_t n_real,
                                                     int64_t n_groups, float lr, float beta1, float beta2, float eps,
                                                     float wd, float bc1, float bc2, float grad_scale) {
  const int lane = threadIdx.x & 63;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t grp = tid >> 4;  // 16 lanes per 128-element group
  if (grp >= n_groups) return;
  const int64_t base = grp * 128 + (lane & 15) * 8;
  float m[8], v[8];
  const float msc = ms[grp], vsc = vs[grp];
  if constexpr (BITS == 4) {
    const unsigned int mw = *(const unsigned int*)(mq + base / 2);
    const unsigned int vw = *(const unsigned int*)(vq + base / 2);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m[k] = deq_m<4>((mw >> (4 * k)) & 15, msc);
      v[k] = deq_v<4>((vw >> (4 * k)) & 15, vsc);
    }
  } else {
    const uint2 mw = *(const uint2*)(mq + base);
    const uint2 vw = *(const uint2*)(vq + base);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned int wm = k < 4 ? mw.x : mw.y, wv = k < 4 ? vw.x : vw.y;
      m[k] = deq_m<8>((wm >> (8 * (k & 3))) & 255, msc);
      v[k] = deq_v<8>((wv >> (8 * (k & 3))) & 255, vsc);
    }
  }
  // fresh states never seen a step: scale 0 -> dequantized v = 0 handled by eps
  float amax = 0.f, vmax = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t i = base + k;
    if (i < n_real) {
      float gk;
      if constexpr (sizeof(G) == 2) gk = bf2f(((const bf16_t*)g)[i]) * grad_scale;
      else gk = ((const float*)g)[i] * grad_scale;
      if (vsc <= 0.f) v[k] = 0.f;
      if (msc <= 0.f) m[k] = 0.f;
      m[k] = beta1 * m[k] + (1.f - beta1) * gk;
      v[k] = beta2 * v[k] + (1.f - beta2) * gk * gk;
      float pk;
      if constexpr (sizeof(P) == 2) pk = bf2f(((bf16_t*)p)[i]);
      else pk = ((float*)p)[i];
      pk = pk * (1.f - lr * wd) - lr * (m[k] / bc1) / (sqrtf(v[k] / bc2) + eps);
      if constexpr (sizeof(P) == 2) ((bf16_t*)p)[i] = f2bf(pk);
      else ((float*)p)[i] = pk;
    } else {
      m[k] = 0.f;
      v[k] = 0.f;
    }
    amax = fmaxf(amax, fabsf(m[k]));
    vmax = fmaxf(vmax, v[k]);
  }
  amax = group16_max(amax);
  vmax = group16_max(vmax);
  const float inv = amax > 0.f ? 1.f / amax : 0.f;
  if constexpr (BITS == 4) {
    unsigned int mw = 0, vw = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mw |= (unsigned int)q_m<4>(m[k], inv) << (4 * k);
      vw |= (unsigned int)q_v<4>(v[k], vmax) << (4 * k);
    }
    *(unsigned int*)(mq + base / 2) = mw;
    *(unsigned int*)(vq + base / 2) = vw;
  } else {
    uint2 mw = {0, 0}, vw = {0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned int cm = (unsigned int)q_m<8>(m[k], inv), cv = (unsigned int)q_v<8>(v[k], vmax);
      if (k < 4) { mw.x |= cm << (8 * k); vw.x |= cv << (8 * k); }
      else { mw.y |= cm << (8 * (k - 4)); vw.y |= cv << (8 * (k - 4)); }
    }
    *(uint2*)(mq + base) = mw;
    *(uint2*)(vq + base) = vw;
  }
  if ((lane & 15) == 0) {
    ms[grp] = amax;
    vs[grp] = vmax;
  }
}

// pdtype/gdtype: 0 = bf16, 1 = fp32
extern "C" int dw_qadamw(void* p, const void* g, void* mq, void* vq, void* ms, void* vs, int64_t n_real,
                         int64_t n_groups, int bits, int pdtype, int gdtype, float lr, float beta1, float beta2,
                         float eps, float wd, float bc1, float bc2, float grad_scale, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int64_t threads = n_groups * 16;
  dim3 grid((unsigned)((threads + 255) / 256)), block(256);
#define QL(B, PT, GT)                                                                                          \
  hipLaunchKernelGGL((qadamw_kernel<B, PT, GT>), grid, block, 0, s, (PT*)p, (const GT*)g, (unsigned char*)mq,   \
                     (unsigned char*)vq, (float*)ms, (float*)vs, n_real, n_groups, lr, beta1, beta2, eps, wd,  \
                     bc1, bc2, grad_scale)
  if (bits == 4) {
    if (pdtype == 0 && gdtype == 0) QL(4, bf16_t, bf16_t);
    else if (pdtype == 1 && gdtype == 1) QL(4, float, float);
    else if (pdtype == 1 && gdtype == 0) QL(4, float, bf16_t);
    else QL(4, bf16_t, float);
  } else if (bits == 8) {
    if (pdtype == 0 && gdtype == 0) QL(8, bf16_t, bf16_t);
    else if (pdtype == 1 && gdtype == 1) QL(8, float, float);
    else if (pdtype == 1 && gdtype == 0) QL(8, float, bf16_t);
    else QL(8, bf16_t, float);
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef QL
  DW_LAUNCH_RET;
}

DW_PRELOAD((qadamw_kernel<8, float, float>));
