// LayerNorm / RMSNorm forward + backward, bf16 I/O, fp32 math.
//
// One wave64 owns one row; the row lives in registers (VPL 16-byte vectors
// per lane), so x is read once in the forward and once in the backward.
// Row statistics use wave shuffles only (no LDS, no __syncthreads in the
// row path).  dgamma/dbeta are accumulated per lane across the rows a wave
// visits (grid-stride), reduced across the block's 4 waves through LDS into
// one fp32 partial row per block, and a second tiny kernel sums the partial
// rows -> no float atomics (guide G12: atomics would be bound at ~1.3 TB/s
// and non-deterministic).
//
// Parity: reference atorch/atorch/normalization/layernorm.py (Triton/apex
// fused LayerNorm) and the RMSNorm used by its Llama modules.
#include "dw_common.h"

// ADD: fused residual add -- h = x + res is formed in registers, rounded to
// bf16 (exactly what a separate bf16 add would store), written to h_out and
// normalized; the residual stream is read once instead of three times.
template <int VPL, bool RMS, bool ADD = false>
__global__ void __launch_bounds__(256) norm_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ gamma,
                                                       const bf16_t* __restrict__ beta, bf16_t* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int64_t rows, int H, float eps,
                                                       const bf16_t* __restrict__ res = nullptr,
                                                       bf16_t* __restrict__ h_out = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = H >> 3;
  const bf16_t* xr = x + row * H;
  float v[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nv) {
      unpack8(*(const u32x4*)(xr + c * 8), v[j]);
      if constexpr (ADD) {
        float r[8];
        unpack8(*(const u32x4*)(res + row * H + c * 8), r);
        u32x4 hv;
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += v[j][k];
        hv = pack8(r);
        *(u32x4*)(h_out + row * H + c * 8) = hv;
        unpack8(hv, v[j]);  // normalize the bf16-rounded sum
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[j][k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[j][k] = 0.f;
    }
  }
  float mu = 0.f;
  if (!RMS) mu = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[j][k] - mu;
        ss += d * d;
      }
    }
  }
  const float var = wave_sum(ss) / (float)H;
  const float rstd = rsqrtf(var + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mu;
    rstd_out[row] = rstd;
  }
  bf16_t* yr = y + row * H;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nv) {
      float g[8], b[8], o[8];
      unpack8(*(const u32x4*)(gamma + c * 8), g);
      if (!RMS) unpack8(*(const u32x4*)(beta + c * 8), b);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (v[j][k] - mu) * rstd * g[k] + (RMS ? 0.f : b[k]);
      *(u32x4*)(yr + c * 8) = pack8(o);
    }
  }
}

// (A grid-stride form that prefetches the next row and loads gamma / beta
// once per wave measured the same: 25.1 vs 24.9 us for the GPT2-1.5B add+norm,
// 8192 x 1600 -- profiles/r4/norm_fwd_gelu_ab.jsonl; one row per wave stays.)

// Backward. partial: [gridDim.x, 2, H] fp32 (dgamma, dbeta) per block.
// Two passes over each row (the second hits L1/L2): pass 1 forms the row
// sums and accumulates dgamma/dbeta into LDS (ds_add_f32), pass 2 writes dx.
// Register use is independent of H (no spills up to H = 8192).
template <int VPL, bool RMS>
__global__ void __launch_bounds__(256) norm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ gamma,
                                                       const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in, bf16_t* __restrict__ dx,
                                                       float* __restrict__ partial, int64_t rows, int H) {
  extern __shared__ __attribute__((aligned(16))) char nsm[];
  float* acc_g = (float*)nsm;      // [H]
  float* acc_b = acc_g + H;        // [H]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nv = H >> 3;
  // lane-owned column vectors c = lane + 64 j are the same for every row:
  // accumulate dgamma/dbeta in registers when they fit (H <= 2048)
  constexpr bool REG = VPL <= 4;
  float rg[REG ? VPL : 1][8], rb[REG ? VPL : 1][8];
  if constexpr (REG) {
#pragma unroll
    for (int j = 0; j < VPL; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) rg[j][k] = rb[j][k] = 0.f;
  }
  for (int c = threadIdx.x; c < 2 * H; c += 256) acc_g[c] = 0.f;
  __syncthreads();
  for (int64_t row = (int64_t)blockIdx.x * 4 + wid; row < rows; row += (int64_t)gridDim.x * 4) {
    const float mu = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    const bf16_t* xr = x + row * H;
    const bf16_t* dr = dy + row * H;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c >= nv) break;
      float xv[8], dv[8], gm[8];
      unpack8(*(const u32x4*)(xr + c * 8), xv);
      unpack8(*(const u32x4*)(dr + c * 8), dv);
      unpack8(*(const u32x4*)(gamma + c * 8), gm);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[k] - mu) * rstd;
        const float g = dv[k] * gm[k];
        s1 += g;
        s2 += g * xh;
        if constexpr (REG) {
          rg[j][k] += dv[k] * xh;
          rb[j][k] += dv[k];
        } else {
          atomicAdd(&acc_g[c * 8 + k], dv[k] * xh);
          if (!RMS) atomicAdd(&acc_b[c * 8 + k], dv[k]);
        }
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) / (float)H;
    const float m2 = wave_sum(s2) / (float)H;
    for (int c = lane; c < nv; c += 64) {
      float xv[8], dv[8], gm[8], o[8];
      unpack8(*(const u32x4*)(xr + c * 8), xv);
      unpack8(*(const u32x4*)(dr + c * 8), dv);
      unpack8(*(const u32x4*)(gamma + c * 8), gm);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[k] - mu) * rstd;
        o[k] = rstd * (dv[k] * gm[k] - m1 - xh * m2);
      }
      *(u32x4*)(dx + row * H + c * 8) = pack8(o);
    }
  }
  if constexpr (REG) {
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c >= nv) break;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        atomicAdd(&acc_g[c * 8 + k], rg[j][k]);  // 4 waves per column: cheap
        if (!RMS) atomicAdd(&acc_b[c * 8 + k], rb[j][k]);
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256) {
    partial[((int64_t)blockIdx.x * 2) * H + c] = acc_g[c];
    partial[((int64_t)blockIdx.x * 2 + 1) * H + c] = acc_b[c];
  }
}

// Sum partial rows -> dgamma/dbeta (bf16 or fp32 out).  Block = 64 columns x
// 4 row groups (each strides over the partial rows), combined through LDS.
template <typename TO>
__global__ void __launch_bounds__(256) norm_bwd_reduce_kernel(const float* __restrict__ partial, int nblk, int H,
                                                              TO* __restrict__ dgamma, TO* __restrict__ dbeta) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  const int which = blockIdx.y;
  float s = 0.f;
  if (col < H)
    for (int b = rg; b < nblk; b += 4) s += partial[((int64_t)b * 2 + which) * H + col];
  red[rg][cl] = s;
  __syncthreads();
  if (rg != 0 || col >= H) return;
  s = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
  TO* out = which == 0 ? dgamma : dbeta;
  if (!out) return;
  if constexpr (sizeof(TO) == 2) out[col] = f2bf(s); else out[col] = s;
}

#define DISPATCH_VPL(H, ...)                          \
  do {                                                \
    int nv_ = (H) / 8;                                \
    if (nv_ <= 64) { constexpr int VPL = 1; __VA_ARGS__; } \
    else if (nv_ <= 128) { constexpr int VPL = 2; __VA_ARGS__; } \
    else if (nv_ <= 256) { constexpr int VPL = 4; __VA_ARGS__; } \
    else if (nv_ <= 512) { constexpr int VPL = 8; __VA_ARGS__; } \
    else { constexpr int VPL = 16; __VA_ARGS__; }    \
  } while (0)

extern "C" int dw_norm_fwd(const void* x, const void* gamma, const void* beta, void* y, void* mean,
                           void* rstd, int64_t rows, int H, float eps, int rms, void* stream) {
  if (H % 8 != 0 || H > 8 * 64 * 16) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_VPL(H, {
    if (rms)
      hipLaunchKernelGGL((norm_fwd_kernel<VPL, true>), grid, block, 0, s, (const bf16_t*)x,
                         (const bf16_t*)gamma, nullptr, (bf16_t*)y, nullptr, (float*)rstd, rows, H, eps);
    else
      hipLaunchKernelGGL((norm_fwd_kernel<VPL, false>), grid, block, 0, s, (const bf16_t*)x,
                         (const bf16_t*)gamma, (const bf16_t*)beta, (bf16_t*)y, (float*)mean,
                         (float*)rstd, rows, H, eps);
  });
  DW_LAUNCH_RET;
}

// y = norm(x + res), h_out = x + res (bf16).  Fused pre-norm residual add.
extern "C" int dw_add_norm_fwd(const void* x, const void* res, const void* gamma, const void* beta, void* y,
                               void* h_out, void* mean, void* rstd, int64_t rows, int H, float eps, int rms,
                               void* stream) {
  if (H % 8 != 0 || H > 8 * 64 * 16) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_VPL(H, {
    if (rms)
      hipLaunchKernelGGL((norm_fwd_kernel<VPL, true, true>), grid, block, 0, s, (const bf16_t*)x,
                         (const bf16_t*)gamma, nullptr, (bf16_t*)y, nullptr, (float*)rstd, rows, H, eps,
                         (const bf16_t*)res, (bf16_t*)h_out);
    else
      hipLaunchKernelGGL((norm_fwd_kernel<VPL, false, true>), grid, block, 0, s, (const bf16_t*)x,
                         (const bf16_t*)gamma, (const bf16_t*)beta, (bf16_t*)y, (float*)mean, (float*)rstd, rows,
                         H, eps, (const bf16_t*)res, (bf16_t*)h_out);
  });
  DW_LAUNCH_RET;
}

// partial must hold nblk*2*H floats; returns nblk used through *nblk_out.
extern "C" int dw_norm_bwd_blocks(int64_t rows) {
  int64_t b = (rows + 3) / 4;
  return (int)(b < 512 ? b : 512);
}

extern "C" int dw_norm_bwd(const void* dy, const void* x, const void* gamma, const void* mean,
                           const void* rstd, void* dx, void* dgamma, void* dbeta, void* partial,
                           int64_t rows, int H, int rms, int out_fp32, void* stream) {
  if (H % 8 != 0 || H > 8 * 64 * 16) return (int)hipErrorInvalidValue;
  const int nblk = dw_norm_bwd_blocks(rows);
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_VPL(H, {
    if (rms)
      hipLaunchKernelGGL((norm_bwd_kernel<VPL, true>), dim3(nblk), dim3(256), 2 * H * sizeof(float), s, (const bf16_t*)dy,
                         (const bf16_t*)x, (const bf16_t*)gamma, nullptr, (const float*)rstd,
                         (bf16_t*)dx, (float*)partial, rows, H);
    else
      hipLaunchKernelGGL((norm_bwd_kernel<VPL, false>), dim3(nblk), dim3(256), 2 * H * sizeof(float), s, (const bf16_t*)dy,
                         (const bf16_t*)x, (const bf16_t*)gamma, (const float*)mean, (const float*)rstd,
                         (bf16_t*)dx, (float*)partial, rows, H);
  });
  dim3 rg((H + 63) / 64, rms ? 1 : 2);
  if (out_fp32)
    hipLaunchKernelGGL(norm_bwd_reduce_kernel<float>, rg, dim3(256), 0, s, (const float*)partial, nblk,
                       H, (float*)dgamma, (float*)dbeta);
  else
    hipLaunchKernelGGL(norm_bwd_reduce_kernel<bf16_t>, rg, dim3(256), 0, s, (const float*)partial, nblk,
                       H, (bf16_t*)dgamma, (bf16_t*)dbeta);
  DW_LAUNCH_RET;
}

DW_PRELOAD(norm_bwd_reduce_kernel<float>);
