// FP8 training support for gfx950 (OCP e4m3 / e5m2, the formats the CDNA4
// MFMA consumes natively; ops/fp8.py).
//
//  * dw_fp8_cast_amax: one pass over a bf16 / fp32 tensor that (a) scales
//    it by the tensor's current delayed-scaling factor, saturates to the
//    format's range and converts 8 values per lane with v_cvt_pk_fp8_f32 /
//    v_cvt_pk_bf8_f32 (16-byte loads, 8-byte stores), and (b) records the
//    tensor's amax of THIS pass (block max, one vector atomic per block on
//    the float bits -- non-negative floats order like their bit patterns)
//    for the next iteration's scale.
//  * dw_fp8_update_scales: after an iteration, for every registered tensor
//    at once: push the recorded amax into its history, scale = fmax /
//    (max(history) * 2^margin) (unchanged while the history is all zero),
//    inv_scale = 1 / scale for the GEMM, and clear the recorded amax.  One
//    launch per training step for the whole model (delayed scaling, as
//    Transformer Engine's DelayedScaling recipe).
//
// The GEMMs themselves are hipBLASLt's FP8 kernels (torch._scaled_mm).
#include "dw_common.h"

template <bool E5M2>
__device__ __forceinline__ unsigned cvt4(float a, float b, float c, float d) {
  unsigned w = 0;
  if (E5M2) {
    w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, w, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
  } else {
    w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  }
  return w;
}

// Saturate to the format's finite range but let NaN through (fminf / fmaxf
// would turn it into -LIM): the converter then writes the format's NaN
// encoding, as torch's float8 cast does, so a NaN activation stays visible.
__device__ __forceinline__ float sat(float v, float lim) { return v != v ? v : fminf(fmaxf(v, -lim), lim); }

template <bool BF16_IN, bool E5M2>
__global__ void __launch_bounds__(256) fp8_cast_amax_kernel(const void* __restrict__ x, const float* __restrict__ scale,
                                                            unsigned char* __restrict__ out,
                                                            unsigned* __restrict__ amax, long long n) {
  constexpr float LIM = E5M2 ? 57344.f : 448.f;
  const float s = *scale;
  float m = 0.f;
  bool nan = false;  // fmaxf drops NaN: track it explicitly
  const long long nvec = n >> 3;
  for (long long v = blockIdx.x * 256ll + threadIdx.x; v < nvec; v += (long long)gridDim.x * 256) {
    float f[8];
    if (BF16_IN) {
      unpack8(((const u32x4*)x)[v], f);
    } else {
      const f32x4 a = ((const f32x4*)x)[2 * v], b = ((const f32x4*)x)[2 * v + 1];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[i] = a[i];
        f[4 + i] = b[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      nan |= f[i] != f[i];
      m = fmaxf(m, fabsf(f[i]));
      f[i] = sat(f[i] * s, LIM);
    }
    uint2 w;
    w.x = cvt4<E5M2>(f[0], f[1], f[2], f[3]);
    w.y = cvt4<E5M2>(f[4], f[5], f[6], f[7]);
    ((uint2*)out)[v] = w;
  }
  // tail (n % 8 elements): one value per thread of the first block
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const long long i = (nvec << 3) + threadIdx.x;
    const float f = BF16_IN ? bf2f(((const bf16_t*)x)[i]) : ((const float*)x)[i];
    nan |= f != f;
    m = fmaxf(m, fabsf(f));
    const float c = sat(f * s, LIM);
    out[i] = (unsigned char)(cvt4<E5M2>(c, 0.f, 0.f, 0.f) & 0xff);
  }
  __shared__ float red[4];
  if (nan) m = INFINITY;  // NaN input: record +inf so the next scale backs off
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (bm > 0.f) atomicMax(amax, __float_as_uint(bm));  // +inf bits = 0x7f800000 for NaN / inf
  }
}

// x: fp32 (in_bf16 = 0) or bf16 (1), 16-byte aligned; out: n bytes; scale /
// amax: device float / uint (float bits) of this tensor.
extern "C" int dw_fp8_cast_amax(const void* x, int in_bf16, const float* scale, void* out, unsigned* amax,
                                long long n, int e5m2, void* stream) {
  if (n <= 0) return 0;
  const int grid = dw_grid_for((n >> 3) > 0 ? (n >> 3) : 1, 256, 4096);
  hipStream_t s = (hipStream_t)stream;
#define L(B, E)                                                                                                 \
  hipLaunchKernelGGL((fp8_cast_amax_kernel<B, E>), dim3(grid), dim3(256), 0, s, x, scale, (unsigned char*)out, \
                     amax, n)
  if (in_bf16) {
    if (e5m2) L(true, true); else L(true, false);
  } else {
    if (e5m2) L(false, true); else L(false, false);
  }
#undef L
  DW_LAUNCH_RET;
}

// meta arrays of m tensors: amax_bits [m] (cleared here), history [m, h] as
// a RING (slot ``head`` receives this step's amax -- no shifting), fmax [m]
// (448 or 57344), scale / inv_scale [m].  One wave per tensor: the 64 lanes
// stride the history (coalesced) and reduce its max in registers.  (The
// first form -- one thread per tensor shifting h = 1024 entries serially --
// took 121 us per step for three tensors.)
__global__ void __launch_bounds__(256) fp8_update_scales_kernel(unsigned* __restrict__ amax_bits,
                                                                float* __restrict__ hist,
                                                                const float* __restrict__ fmax_,
                                                                float* __restrict__ scale,
                                                                float* __restrict__ inv_scale, int m, int h,
                                                                int head, float margin_pow2) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= m) return;
  float* hh = hist + (long long)t * h;
  const float cur = __uint_as_float(amax_bits[t]);
  float best = cur;
  for (int j = lane; j < h; j += 64)
    if (j != head) best = fmaxf(best, hh[j]);
  best = wave_max(best);
  if (lane == 0) {
    hh[head] = cur;
    amax_bits[t] = 0u;
    if (best > 0.f && best < INFINITY) {
      const float sc = fmax_[t] / (best * margin_pow2);
      scale[t] = sc;
      inv_scale[t] = 1.f / sc;
    } else if (best == INFINITY) {  // overflowed: shrink hard
      scale[t] *= 0.5f;
      inv_scale[t] = 1.f / scale[t];
    }
  }
}

extern "C" int dw_fp8_update_scales(unsigned* amax_bits, float* hist, const float* fmax_, float* scale,
                                    float* inv_scale, int m, int h, int head, float margin_pow2, void* stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(fp8_update_scales_kernel, dim3((m + 3) / 4), dim3(256), 0, (hipStream_t)stream, amax_bits,
                     hist, fmax_, scale, inv_scale, m, h, head, margin_pow2);
  DW_LAUNCH_RET;
}

// Cast + transpose in one pass: x [R, C] (bf16 / fp32, row-major) -> out
// [R, C] fp8 and/or out_t [C, R] fp8, scaled / saturated / amax-recorded as
// dw_fp8_cast_amax.  The FP8 GEMMs want every operand K-contiguous (A
// row-major, B column-major), and the backward contracts over different
// dims than the forward: the weight gradient needs x and the output
// gradient with the TOKEN dim contiguous, dgrad needs W^T.  Writing both
// layouts from one read replaces a separate transposed copy (torch's
// byte-wise transpose of a float8 tensor ran at ~0.25 TB/s:
// profiles/r3/fp8_linear_kernels.md).
// 128x128 tiles, 256 threads, every output row segment a whole 128-byte
// line in both layouts (a 64-wide tile wrote half lines and ran at ~1.4
// TB/s): phase 1 converts 8 x 8 contiguous elements per thread (16 threads
// per 256-byte input row; 8-byte row-major stores) and parks the bytes in
// LDS; phase 2 gives each thread a 16-row x 4-column block: 16 4-byte LDS
// reads, a byte transpose in registers, four 16-byte stores (8 threads per
// 128-byte transposed row).
template <bool BF16_IN, bool E5M2>
__global__ void __launch_bounds__(256) fp8_cast_t_kernel(const void* __restrict__ x, const float* __restrict__ scale,
                                                         unsigned char* __restrict__ out,
                                                         unsigned char* __restrict__ out_t,
                                                         unsigned* __restrict__ amax, int R, int C) {
  constexpr float LIM = E5M2 ? 57344.f : 448.f;
  constexpr int T = 128, P = T + 4;  // LDS row pitch (bytes)
  __shared__ __attribute__((aligned(16))) unsigned char tile[T * P];
  __shared__ float red[4];
  const float s = *scale;
  const int r0 = blockIdx.y * T, c0 = blockIdx.x * T;
  const int tid = threadIdx.x;
  float m = 0.f;
  bool nan = false;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int v = tid + 256 * k;  // 2048 vectors of 8 per tile
    const int rr = v >> 4, cc = (v & 15) * 8;
    const int r = r0 + rr, c = c0 + cc;
    uint2 w = {0u, 0u};
    if (r < R && c < C) {  // C is a multiple of 8: whole vectors
      float f[8];
      const long long off = (long long)r * C + c;
      if (BF16_IN) {
        unpack8(*(const u32x4*)((const bf16_t*)x + off), f);
      } else {
        const f32x4 a = *(const f32x4*)((const float*)x + off), b = *(const f32x4*)((const float*)x + off + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f[i] = a[i];
          f[4 + i] = b[i];
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        nan |= f[i] != f[i];
        m = fmaxf(m, fabsf(f[i]));
        f[i] = sat(f[i] * s, LIM);
      }
      w.x = cvt4<E5M2>(f[0], f[1], f[2], f[3]);
      w.y = cvt4<E5M2>(f[4], f[5], f[6], f[7]);
      if (out) *(uint2*)(out + off) = w;
    }
    if (out_t) *(uint2*)(tile + rr * P + cc) = w;
  }
  if (out_t) {
    __syncthreads();
    const int cg = tid >> 3, rg = tid & 7;  // columns 4cg .. 4cg+3, rows 16rg .. 16rg+15
    const int c = c0 + 4 * cg, r = r0 + 16 * rg;
    if (c < C && r < R) {  // C % 8 == 0 and R % 16 == 0: whole groups
      unsigned w[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = *(const unsigned*)(tile + (16 * rg + i) * P + 4 * cg);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        unsigned q[4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          q[g] = ((w[4 * g] >> (8 * j)) & 0xffu) | (((w[4 * g + 1] >> (8 * j)) & 0xffu) << 8) |
                 (((w[4 * g + 2] >> (8 * j)) & 0xffu) << 16) | (((w[4 * g + 3] >> (8 * j)) & 0xffu) << 24);
        *(u32x4*)(out_t + (long long)(c + j) * R + r) = (u32x4){q[0], q[1], q[2], q[3]};
      }
    }
  }
  if (nan) m = INFINITY;
  m = wave_max(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (bm > 0.f) atomicMax(amax, __float_as_uint(bm));
  }
}

// x [R, C] (C % 8 == 0, 16-byte aligned rows), out [R, C] and / or out_t
// [C, R] (either may be null; out_t rows 16-byte aligned: R % 16 == 0).
extern "C" int dw_fp8_cast_t(const void* x, int in_bf16, const float* scale, void* out, void* out_t,
                             unsigned* amax, int R, int C, int e5m2, void* stream) {
  if (R <= 0 || C <= 0) return 0;
  if (C % 8 || (out_t && R % 16)) return (int)hipErrorInvalidValue;
  dim3 grid((C + 127) / 128, (R + 127) / 128);
  hipStream_t s = (hipStream_t)stream;
#define L(B, E)                                                                                                \
  hipLaunchKernelGGL((fp8_cast_t_kernel<B, E>), grid, dim3(256), 0, s, x, scale, (unsigned char*)out,          \
                     (unsigned char*)out_t, amax, R, C)
  if (in_bf16) {
    if (e5m2) L(true, true); else L(true, false);
  } else {
    if (e5m2) L(false, true); else L(false, false);
  }
#undef L
  DW_LAUNCH_RET;
}

DW_PRELOAD(fp8_update_scales_kernel);
