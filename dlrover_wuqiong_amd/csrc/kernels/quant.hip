// Group-wise int8 / int4 quantization for quantized collectives (ZeRO++-style
// qwZ weight all-gather and qgZ gradient reduce-scatter) and compressed
// checkpoints.  gfx950, wave64.
//
// Format (parity with ATorch's quantizer, atorch/ops/csrc/quantization and
// atorch/tests/common_tests/test_quantize.py):
//   * the tensor is split into `groups` contiguous groups of gs elements;
//   * symmetric:  scale = 2^bits / (2 absmax)   q = clamp(rint(x scale))
//     asymmetric: scale = 2^bits / (max - min)  q = clamp(rint(x scale + zp)),
//                 zp = qmin - min scale
//     (a constant group uses scale 1);
//   * params[g] = {1 / scale, zp} (fp32), dequantize x = (q - zp) / scale;
//   * int4 packs two values per byte, the first in the HIGH nibble.
//
// Design: one 256-thread block per group; pass 1 reduces absmax / min / max
// over 8-element vectors (16-byte bf16 / 32-byte fp32 loads), pass 2
// re-reads the group (<= a few hundred KB: L2-resident) and writes 8 codes
// per thread-step as one 8-byte (int8) or 4-byte (int4) store.  The
// dequantize-reduce kernel is the receive side of a quantized
// reduce-scatter: it sums N ranks' quantized chunks in fp32 registers and
// writes the reduced shard once (bf16 / fp32), so the wire carries 1 byte
// (or half a byte) per element instead of 2.
#include "dw_common.h"

namespace {

constexpr int QT = 256;

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* f);
template <>
__device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float* f) {
  unpack8(*(const u32x4*)p, f);
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* f) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[i] = a[i];
    f[4 + i] = b[i];
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float* f);
template <>
__device__ __forceinline__ void store8<bf16_t>(bf16_t* p, const float* f) {
  *(u32x4*)p = pack8(f);
}
template <>
__device__ __forceinline__ void store8<float>(float* p, const float* f) {
  *(f32x4*)p = (f32x4){f[0], f[1], f[2], f[3]};
  *(f32x4*)(p + 4) = (f32x4){f[4], f[5], f[6], f[7]};
}

template <int BITS>
__device__ __forceinline__ void unpack_codes(const int8_t* q, int64_t e, float* c) {
  if constexpr (BITS == 8) {
    const uint64_t w = *(const uint64_t*)(q + e);
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = (float)(int8_t)(w >> (8 * i));
  } else {
    const uint32_t w = *(const uint32_t*)(q + e / 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int byte = (int)(int8_t)(w >> (8 * i));
      c[2 * i] = (float)(byte >> 4);                        // high nibble first (arithmetic shift)
      c[2 * i + 1] = (float)((int)((unsigned)byte << 28) >> 28);  // sign-extended low nibble
    }
  }
}

template <typename T, int BITS, bool SYM>
__global__ void __launch_bounds__(QT) quant_kernel(const T* __restrict__ x, int8_t* __restrict__ q,
                                                   float* __restrict__ params, int64_t gs) {
  __shared__ float red[QT / 64];
  const int64_t g = blockIdx.x;
  const T* xg = x + g * gs;
  float mx = -INFINITY, mn = INFINITY;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < gs; e += QT * 8) {
    float f[8];
    load8<T>(xg + e, f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (SYM) {
        mx = fmaxf(mx, fabsf(f[i]));
      } else {
        mx = fmaxf(mx, f[i]);
        mn = fminf(mn, f[i]);
      }
    }
  }
  mx = block_max<QT>(mx, red);
  if constexpr (!SYM) mn = -block_max<QT>(-mn, red);
  constexpr float qrange = (float)(1 << BITS), qmin = -(float)(1 << (BITS - 1)), qmax = (float)((1 << (BITS - 1)) - 1);
  float scale, zp = 0.f;
  if constexpr (SYM) {
    scale = mx == 0.f ? 1.f : qrange / (2.f * mx);
  } else {
    scale = mx == mn ? 1.f : qrange / (mx - mn);
    zp = __fsub_rn(qmin, __fmul_rn(mn, scale));
  }
  if (threadIdx.x == 0) {
    params[2 * g] = 1.f / scale;
    params[2 * g + 1] = zp;
  }
  int8_t* qg = q + (BITS == 8 ? g * gs : g * gs / 2);
  for (int64_t e = (int64_t)threadIdx.x * 8; e < gs; e += QT * 8) {
    float f[8];
    load8<T>(xg + e, f);
    int c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = __fmul_rn(f[i], scale);
      if constexpr (!SYM) v = __fadd_rn(v, zp);
      c[i] = (int)fminf(fmaxf(__builtin_rintf(v), qmin), qmax);
    }
    if constexpr (BITS == 8) {
      uint64_t w = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) w |= (uint64_t)(uint8_t)c[i] << (8 * i);
      *(uint64_t*)(qg + e) = w;
    } else {
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) w |= (uint32_t)(((c[2 * i] & 0xF) << 4) | (c[2 * i + 1] & 0xF)) << (8 * i);
      *(uint32_t*)(qg + e / 2) = w;
    }
  }
}

// out[e] (+)= sum_n dequant(q_n[e]) over n_src quantized chunks of `elems`
// each (chunk n at q + n * chunk_bytes, params at params + n * 2 * gpc).
template <typename TO, int BITS>
__global__ void __launch_bounds__(QT) dequant_reduce_kernel(const int8_t* __restrict__ q,
                                                            const float* __restrict__ params, TO* __restrict__ out,
                                                            int n_src, int64_t elems, int64_t gs, int64_t chunk_bytes,
                                                            int64_t gpc, int accumulate) {
  const int64_t nv = elems / 8;
  for (int64_t v = blockIdx.x * (int64_t)QT + threadIdx.x; v < nv; v += (int64_t)gridDim.x * QT) {
    const int64_t e = v * 8;
    const int64_t g = e / gs;
    float acc[8];
    if (accumulate) {
      load8<TO>(out + e, acc);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    }
    for (int n = 0; n < n_src; ++n) {
      const float* pr = params + 2 * ((int64_t)n * gpc + g);
      const float inv = pr[0], zp = pr[1];
      float c[8];
      unpack_codes<BITS>(q + n * chunk_bytes, e, c);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += (c[i] - zp) * inv;
    }
    store8<TO>(out + e, acc);
  }
}

template <typename T, int BITS, bool SYM>
int launch_quant(const void* x, void* q, void* params, int64_t groups, int64_t gs, hipStream_t s) {
  hipLaunchKernelGGL((quant_kernel<T, BITS, SYM>), dim3((unsigned)groups), dim3(QT), 0, s, (const T*)x, (int8_t*)q,
                     (float*)params, gs);
  DW_LAUNCH_RET;
}

template <typename TO, int BITS>
int launch_dqr(const void* q, const void* params, void* out, int n_src, int64_t elems, int64_t gs,
               int64_t chunk_bytes, int64_t gpc, int accumulate, hipStream_t s) {
  const int grid = dw_grid_for(elems / 8, QT, 4096);
  hipLaunchKernelGGL((dequant_reduce_kernel<TO, BITS>), dim3(grid), dim3(QT), 0, s, (const int8_t*)q,
                     (const float*)params, (TO*)out, n_src, elems, gs, chunk_bytes, gpc, accumulate);
  DW_LAUNCH_RET;
}

}  // namespace

// x: `groups` groups of gs elements (gs % 8 == 0), dtype 0 = fp32, 1 = bf16.
// q: groups * gs bytes (int8) or groups * gs / 2 (int4); params: [groups, 2] fp32.
extern "C" int dw_quantize(const void* x, int dtype, void* q, void* params, int64_t groups, int64_t gs, int bits,
                           int symmetric, void* stream) {
  if (gs <= 0 || gs % 8 != 0 || groups <= 0 || groups > 0x7fffffff || (bits != 8 && bits != 4))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
#define DW_Q(T)                                                                               \
  if (bits == 8) return symmetric ? launch_quant<T, 8, true>(x, q, params, groups, gs, s)     \
                                  : launch_quant<T, 8, false>(x, q, params, groups, gs, s);   \
  return symmetric ? launch_quant<T, 4, true>(x, q, params, groups, gs, s)                    \
                   : launch_quant<T, 4, false>(x, q, params, groups, gs, s);
  if (dtype == 1) {
    DW_Q(bf16_t)
  }
  DW_Q(float)
#undef DW_Q
}

// out (+)= sum over n_src chunks of dequantized codes; dequantize is n_src = 1.
// Every chunk holds `elems` codes (elems % 8 == 0, gs % 8 == 0, elems % gs == 0)
// with gpc = elems / gs groups; out dtype 0 = fp32, 1 = bf16.
extern "C" int dw_dequant_reduce(const void* q, const void* params, void* out, int out_dtype, int n_src,
                                 int64_t elems, int64_t gs, int bits, int accumulate, void* stream) {
  if (gs <= 0 || gs % 8 != 0 || elems % 8 != 0 || elems % gs != 0 || n_src <= 0 || (bits != 8 && bits != 4))
    return (int)hipErrorInvalidValue;
  if (elems == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int64_t chunk_bytes = bits == 8 ? elems : elems / 2, gpc = elems / gs;
  if (out_dtype == 1)
    return bits == 8 ? launch_dqr<bf16_t, 8>(q, params, out, n_src, elems, gs, chunk_bytes, gpc, accumulate, s)
                     : launch_dqr<bf16_t, 4>(q, params, out, n_src, elems, gs, chunk_bytes, gpc, accumulate, s);
  return bits == 8 ? launch_dqr<float, 8>(q, params, out, n_src, elems, gs, chunk_bytes, gpc, accumulate, s)
                   : launch_dqr<float, 4>(q, params, out, n_src, elems, gs, chunk_bytes, gpc, accumulate, s);
}

DW_PRELOAD((quant_kernel<float, 8, true>));
