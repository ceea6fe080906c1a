// Column reductions (bias / norm-weight gradients) and the row-wise norm dx.
//
// Bias grads db = sum_rows dy and norm weight grads dgamma = sum_rows dy*xhat,
// dbeta = sum_rows dy are column sums over [rows, C] -- tall and skinny
// (rows = tokens = 8K..64K, C = hidden).  One kernel per reduction:
//   * block = 4 waves; a wave covers 512 consecutive columns (64 lanes x one
//     16-byte vector of 8 bf16) of its rows, a block a [rows/RS] x 512 tile;
//   * per-lane fp32 accumulation in registers over the block's rows, one LDS
//     combine of the 4 waves, then ONE fp32 atomicAdd per column per block
//     into a workspace -> grid = (C/512) x RS blocks fills the chip without
//     any partial-row buffer or second pass over the data;
//   * a tiny finish kernel converts the fp32 workspace into the gradient
//     (bf16 or fp32), optionally ACCUMULATING into it (grad += sum), so the
//     result lands directly in the flat gradient buffer.
// The norm dx is a separate row kernel (one wave per row, everything in
// registers), so the backward is 2 streaming passes + 1 tiny kernel instead
// of a row pass with per-block partial rows and a serial reduce.
#include "dw_common.h"

// MODE 0: acc0 += dy ;  MODE 1: acc0 += dy * xhat, acc1 += dy (LayerNorm) ;
// MODE 2: acc0 += dy * xhat (RMSNorm)
template <int MODE>
__global__ void __launch_bounds__(256) colred_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     float* __restrict__ ws, int64_t rows, int C, int rows_per_blk) {
  __shared__ float red[2][4][512 + 4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int64_t r_beg = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t r_end = min(rows, r_beg + rows_per_blk);
  float a0[8], a1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a0[k] = a1[k] = 0.f;
  if (c0 < C) {
    for (int64_t r = r_beg + wid; r < r_end; r += 4) {
      float d[8];
      unpack8(*(const u32x4*)(dy + r * C + c0), d);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a0[k] += d[k];
      } else {
        float xv[8];
        unpack8(*(const u32x4*)(x + r * C + c0), xv);
        const float mu = (MODE == 1) ? mean[r] : 0.f, rs = rstd[r];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          a0[k] += d[k] * (xv[k] - mu) * rs;
          if constexpr (MODE == 1) a1[k] += d[k];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][wid][lane * 8 + k] = a0[k];
    if constexpr (MODE == 1) red[1][wid][lane * 8 + k] = a1[k];
  }
  __syncthreads();
  // 256 threads combine 512 columns (2 each) x 4 waves, one atomic per column
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = threadIdx.x + 256 * j;
    const int c = blockIdx.x * 512 + cl;
    if (c >= C) continue;
    const float s0 = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    atomicAdd(ws + c, s0);
    if constexpr (MODE == 1) {
      const float s1 = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
      atomicAdd(ws + C + c, s1);
    }
  }
}

// out[c] (+)= ws[c]; out dtype bf16 (is_fp32=0) or fp32.  The workspace is
// SELF-CLEANING: every reader zeroes the words it consumed, so ws is all-zero
// between calls and no per-call hipMemsetAsync (a 5 us fill launch, ~340 per
// GPT2-1.5B step) is needed.  out == nullptr only clears.
__global__ void colred_finish_kernel(float* __restrict__ ws, void* __restrict__ out, int C, int is_fp32,
                                     int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float v = ws[c];
  ws[c] = 0.f;
  if (!out) return;
  if (is_fp32) {
    float* o = (float*)out;
    o[c] = accumulate ? o[c] + v : v;
  } else {
    bf16_t* o = (bf16_t*)out;
    o[c] = f2bf(accumulate ? bf2f(o[c]) + v : v);
  }
}

// dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)) [+ dres]; one wave per row
template <int VPL, bool RMS>
__global__ void __launch_bounds__(256) norm_dx_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ gamma,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in,
                                                      const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                      int64_t rows, int H) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = H >> 3;
  const float mu = RMS ? 0.f : mean_in[row];
  const float rstd = rstd_in[row];
  const bf16_t* xr = x + row * H;
  const bf16_t* dr = dy + row * H;
  constexpr bool KEEP = VPL <= 8;  // keep xhat, dy*g in registers; else recompute (H > 4096)
  float xh[KEEP ? VPL : 1][8], g[KEEP ? VPL : 1][8];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nv) {
      float xv[8], dv[8], gm[8];
      unpack8(*(const u32x4*)(xr + c * 8), xv);
      unpack8(*(const u32x4*)(dr + c * 8), dv);
      unpack8(*(const u32x4*)(gamma + c * 8), gm);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float a = (xv[k] - mu) * rstd, b = dv[k] * gm[k];
        if constexpr (KEEP) { xh[j][k] = a; g[j][k] = b; }
        s1 += b;
        s2 += b * a;
      }
    }
  }
  const float m1 = RMS ? 0.f : wave_sum(s1) / (float)H;
  const float m2 = wave_sum(s2) / (float)H;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int c = lane + 64 * j;
    if (c < nv) {
      float o[8];
      if constexpr (KEEP) {
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (g[j][k] - m1 - xh[j][k] * m2);
      } else {
        float xv[8], dv[8], gm[8];
        unpack8(*(const u32x4*)(xr + c * 8), xv);
        unpack8(*(const u32x4*)(dr + c * 8), dv);
        unpack8(*(const u32x4*)(gamma + c * 8), gm);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (dv[k] * gm[k] - m1 - (xv[k] - mu) * rstd * m2);
      }
      if (dres) {  // fused residual-branch gradient (uniform branch)
        float r[8];
        unpack8(*(const u32x4*)(dres + row * H + c * 8), r);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] += r[k];
      }
      *(u32x4*)(dx + row * H + c * 8) = pack8(o);
    }
  }
}

static int colred_rows_per_blk(int64_t rows, int C) {
  // aim for ~4 blocks per CU over 256 CUs
  const int64_t col_blks = (C + 511) / 512;
  int64_t rs = (1024 + col_blks - 1) / col_blks;
  if (rs < 1) rs = 1;
  int64_t per = (rows + rs - 1) / rs;
  per = (per + 3) / 4 * 4;
  return (int)(per < 4 ? 4 : per);
}

// ws: fp32 [C], all-zero on entry, left all-zero.  out (+)= column sums of dy [rows, C].
extern "C" int dw_colsum_acc(const void* dy, int64_t rows, int C, void* ws, void* out, int out_fp32, int accumulate,
                             void* stream) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int per = colred_rows_per_blk(rows, C);
  dim3 grid((C + 511) / 512, (unsigned)((rows + per - 1) / per));
  hipLaunchKernelGGL(colred_kernel<0>, grid, dim3(256), 0, s, (const bf16_t*)dy, nullptr, nullptr, nullptr,
                     (float*)ws, rows, C, per);
  hipLaunchKernelGGL(colred_finish_kernel, dim3((C + 255) / 256), dim3(256), 0, s, (float*)ws, out, C, out_fp32,
                     accumulate);
  DW_LAUNCH_RET;
}

#define DISPATCH_VPL2(H, ...)                          \
  do {                                                 \
    int nv_ = (H) / 8;                                 \
    if (nv_ <= 64) { constexpr int VPL = 1; __VA_ARGS__; } \
    else if (nv_ <= 128) { constexpr int VPL = 2; __VA_ARGS__; } \
    else if (nv_ <= 256) { constexpr int VPL = 4; __VA_ARGS__; } \
    else if (nv_ <= 512) { constexpr int VPL = 8; __VA_ARGS__; } \
    else { constexpr int VPL = 16; __VA_ARGS__; }     \
  } while (0)

// Norm backward v2.  ws: fp32 [2H], all-zero on entry, left all-zero.
// dgamma/dbeta (+)= (accumulate flag).  dres (nullable): gradient of the
// residual sum that this norm's input also feeds (fused add+norm) -> dx += dres.
extern "C" int dw_norm_bwd2(const void* dy, const void* x, const void* gamma, const void* mean, const void* rstd,
                            const void* dres, void* dx, void* dgamma, void* dbeta, void* ws, int64_t rows, int H,
                            int rms, int out_fp32, int accumulate, void* stream) {
  if (H % 8 != 0 || H > 8 * 64 * 16) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  DISPATCH_VPL2(H, {
    if (rms)
      hipLaunchKernelGGL((norm_dx_kernel<VPL, true>), grid, block, 0, s, (const bf16_t*)dy, (const bf16_t*)x,
                         (const bf16_t*)gamma, nullptr, (const float*)rstd, (const bf16_t*)dres, (bf16_t*)dx, rows,
                         H);
    else
      hipLaunchKernelGGL((norm_dx_kernel<VPL, false>), grid, block, 0, s, (const bf16_t*)dy, (const bf16_t*)x,
                         (const bf16_t*)gamma, (const float*)mean, (const float*)rstd, (const bf16_t*)dres,
                         (bf16_t*)dx, rows, H);
  });
  if (!dgamma && !dbeta) { DW_LAUNCH_RET; }
  const int per = colred_rows_per_blk(rows, H);
  dim3 cg((H + 511) / 512, (unsigned)((rows + per - 1) / per));
  if (rms)
    hipLaunchKernelGGL(colred_kernel<2>, cg, dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)x, nullptr,
                       (const float*)rstd, (float*)ws, rows, H, per);
  else
    hipLaunchKernelGGL(colred_kernel<1>, cg, dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)x,
                       (const float*)mean, (const float*)rstd, (float*)ws, rows, H, per);
  // both halves are consumed (and cleared) even if one output is absent
  hipLaunchKernelGGL(colred_finish_kernel, dim3((H + 255) / 256), dim3(256), 0, s, (float*)ws, dgamma, H, out_fp32,
                     accumulate);
  if (!rms)
    hipLaunchKernelGGL(colred_finish_kernel, dim3((H + 255) / 256), dim3(256), 0, s, (float*)ws + H, dbeta, H,
                       out_fp32, accumulate);
  DW_LAUNCH_RET;
}
