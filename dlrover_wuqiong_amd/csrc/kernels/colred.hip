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
//   * the last block to finish in each 512-column strip (per-strip
//     completion counters after the sums) converts the strip's fp32 sums
//     into the gradient (bf16 or fp32), optionally
//     ACCUMULATING into it (grad += sum), so the result lands directly in the
//     flat gradient buffer with no second launch.  The workspace (sums +
//     counter) is SELF-CLEANING: the finishing block zeroes what it consumed,
//     so it is all-zero between calls and needs no per-call memset.
// The norm dx is a separate row kernel (one wave per row, everything in
// registers), so the backward is 2 streaming passes + 1 tiny kernel instead
// of a row pass with per-block partial rows and a serial reduce.
#include "dw_common.h"

#include <algorithm>
#include <cstdlib>

static bool getenv_flag(const char* name) {
  const char* v = std::getenv(name);
  return v && v[0] == '1';
}

__device__ __forceinline__ void colred_store(void* out, int c, float v, int is_fp32, int accumulate) {
  if (!out) return;
  if (is_fp32) {
    float* o = (float*)out;
    o[c] = accumulate ? o[c] + v : v;
  } else {
    bf16_t* o = (bf16_t*)out;
    o[c] = f2bf(accumulate ? bf2f(o[c]) + v : v);
  }
}

// Deterministic mode (``part`` != nullptr; DWAMD_DETERMINISTIC=1 or
// torch.use_deterministic_algorithms(True) on the Python side): every block
// stores its partial column sums instead of adding them atomically, and the
// finishing block adds the partials in block order -- bit-identical results
// from run to run at the cost of the partial buffer and the finishing
// block's serial sum.  Loads are issued 8 at a time, the adds stay in order.
__device__ __forceinline__ float ordered_sum(const float* p, int64_t stride, int n) {
  float a = 0.f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = __hip_atomic_load(p + (int64_t)(i + u) * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  for (; i < n; ++i) a += __hip_atomic_load(p + (int64_t)i * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return a;
}

// MODE 0: acc0 += dy ;  MODE 1: acc0 += dy * xhat, acc1 += dy (LayerNorm) ;
// MODE 2: acc0 += dy * xhat (RMSNorm) ;
// MODE 3: dxo = dy * gelu'(x), acc0 += dxo (GELU backward fused with the
//         gradient of the bias added before it: one pass instead of two)
template <int MODE>
__global__ void __launch_bounds__(256) colred_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     float* __restrict__ ws, int64_t rows, int C, int rows_per_blk,
                                                     void* __restrict__ out0, void* __restrict__ out1, int is_fp32,
                                                     int accumulate, bf16_t* __restrict__ dxo = nullptr,
                                                     float* __restrict__ part = nullptr) {
  __shared__ float red[2][4][512 + 4];
  constexpr int NS = MODE == 1 ? 2 : 1;  // sums per column
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int64_t r_beg = (int64_t)blockIdx.y * rows_per_blk;
  const int64_t r_end = min(rows, r_beg + rows_per_blk);
  float a0[8], a1[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a0[k] = a1[k] = 0.f;
  if (c0 < C) {
    // U rows per wave per iteration, every load issued before any math
    constexpr int U = 4;
    for (int64_t r0 = r_beg + wid; r0 < r_end; r0 += 4 * U) {
      u32x4 dv[U], xw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + 4 * u;
        if (r < r_end) {
          dv[u] = *(const u32x4*)(dy + r * C + c0);
          if constexpr (MODE != 0) xw[u] = *(const u32x4*)(x + r * C + c0);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + 4 * u;
        if (r >= r_end) break;
        float d[8];
        unpack8(dv[u], d);
        if constexpr (MODE == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) a0[k] += d[k];
        } else if constexpr (MODE == 3) {
          float xv[8];
          unpack8(xw[u], xv);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            d[k] *= gelu_tanh_grad(xv[k]);
            a0[k] += d[k];
          }
          *(u32x4*)(dxo + r * C + c0) = pack8(d);
        } else {
          float xv[8];
          unpack8(xw[u], xv);
          const float mu = (MODE == 1) ? mean[r] : 0.f, rs = rstd[r];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            a0[k] += d[k] * (xv[k] - mu) * rs;
            if constexpr (MODE == 1) a1[k] += d[k];
          }
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
    if (part) {
      // deterministic mode: this block's partial sums, combined in a fixed
      // order by the finishing block (agent-scope stores: performed at the
      // coherent level, like the atomics of the default mode)
      __hip_atomic_store(part + (int64_t)blockIdx.y * NS * C + c, s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      atomicAdd(ws + c, s0);
    }
    if constexpr (MODE == 1) {
      const float s1 = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
      if (part)
        __hip_atomic_store(part + ((int64_t)blockIdx.y * NS + 1) * C + c, s1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      else
        atomicAdd(ws + C + c, s1);
    }
  }
  // The last block of each 512-column strip converts the strip's fp32 sums
  // into the output(s) -- no second launch (a ~5 us kernel per reduction,
  // ~450 per GPT2-1.5B step), and the finish is spread over the strips.
  //
  // Ordering without a device-scope fence: a __threadfence() here is an L2
  // write-back + invalidate on gfx950 (per-XCD L2s), in every block -- it
  // made this kernel 5x slower.  All the data the finishing block reads was
  // produced by agent-scope atomics, so it is enough that this block's
  // atomics have COMPLETED (vmcnt drained: performed at the coherent level)
  // before its counter increment is issued, and that the finishing block
  // reads the sums with atomics too.
  __shared__ int is_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* cnt = (unsigned*)(ws + (MODE == 1 ? 2 * C : C)) + blockIdx.x;
  if (threadIdx.x == 0)
    is_last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.y - 1;
  __syncthreads();
  if (!is_last) return;
  float v0[2], v1[2];
  if (part) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = blockIdx.x * 512 + threadIdx.x + 256 * j;
      if (c < C) {
        v0[j] = ordered_sum(part + c, (int64_t)NS * C, gridDim.y);
        if constexpr (MODE == 1) v1[j] = ordered_sum(part + C + c, (int64_t)NS * C, gridDim.y);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      // read + clear (self-cleaning) with the same atomics that built the sums:
      // single-location atomicity, no cache maintenance; all in flight at once
      const int c = blockIdx.x * 512 + threadIdx.x + 256 * j;
      if (c < C) {
        v0[j] = __hip_atomic_exchange(ws + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (MODE == 1)
          v1[j] = __hip_atomic_exchange(ws + C + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = blockIdx.x * 512 + threadIdx.x + 256 * j;
    if (c < C) {
      colred_store(out0, c, v0[j], is_fp32, accumulate);
      if constexpr (MODE == 1) colred_store(out1, c, v1[j], is_fp32, accumulate);
    }
  }
  if (threadIdx.x == 0) __hip_atomic_exchange(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// Norm backward in ONE pass for H <= 4096: dx as norm_dx_kernel, and the
// weight gradients dgamma = sum dy*xhat, dbeta = sum dy accumulated per lane
// over the rows each wave visits (grid-stride over rows), reduced over the
// block's 4 waves through LDS, one atomic per column per block into ws; the
// last block converts ws into dgamma / dbeta (same completion protocol as
// colred_kernel).  Saves the second read of dy and x (colred_kernel<1>).
template <int VPL, bool RMS>
__global__ void __launch_bounds__(256) norm_bwd_fused_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, const bf16_t* __restrict__ dres,
    bf16_t* __restrict__ dx, float* __restrict__ ws, void* __restrict__ dgamma, void* __restrict__ dbeta,
    int is_fp32, int accumulate, int64_t rows, int H) {
  static_assert(VPL <= 8, "fused norm backward keeps xhat / dy*g in registers");
  __shared__ float red[2][4][512 + 4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nv = H >> 3;
  float ag[VPL][8], ab[VPL][8], ad[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) ag[j][k] = ab[j][k] = ad[j][k] = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wid; row < rows; row += (int64_t)gridDim.x * 4) {
    const float mu = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    const bf16_t* xr = x + row * H;
    const bf16_t* dr = dy + row * H;
    float xh[VPL][8], g[VPL][8];
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
          xh[j][k] = a;
          g[j][k] = b;
          ag[j][k] += dv[k] * a;
          if constexpr (!RMS) ab[j][k] += dv[k];
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
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (g[j][k] - m1 - xh[j][k] * m2);
        if (dres) {
          float r[8];
          unpack8(*(const u32x4*)(dres + row * H + c * 8), r);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += r[k];
        }
        *(u32x4*)(dx + row * H + c * 8) = pack8(o);
      }
    }
  }
  // block reduce, 512 columns (one j) at a time, one atomic per column
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[0][wid][lane * 8 + k] = ag[j][k];
      if constexpr (!RMS) red[1][wid][lane * 8 + k] = ab[j][k];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cl = threadIdx.x + 256 * h;
      const int c = 512 * j + cl;
      if (c < H) {
        atomicAdd(ws + c, red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl]);
        if constexpr (!RMS) atomicAdd(ws + H + c, red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl]);
      }
    }
    __syncthreads();
  }
  __shared__ int is_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's atomics performed (see colred_kernel)
  __syncthreads();
  unsigned* cnt = (unsigned*)(ws + 2 * H);
  if (threadIdx.x == 0)
    is_last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!is_last) return;
  for (int c0 = threadIdx.x; c0 < H; c0 += 256 * 4) {
    float v0[4], v1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + 256 * u;
      if (c < H) {
        v0[u] = __hip_atomic_exchange(ws + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (!RMS) v1[u] = __hip_atomic_exchange(ws + H + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + 256 * u;
      if (c < H) {
        colred_store(dgamma, c, v0[u], is_fp32, accumulate);
        if constexpr (!RMS) colred_store(dbeta, c, v1[u], is_fp32, accumulate);
      }
    }
  }
  if (threadIdx.x == 0) __hip_atomic_exchange(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Norm backward for SMALL H (< 2048, VPL <= 4), one pass over dy / x (/ dres):
// every wave strides over rows (grid = the resident workgroups), loading the
// next row before computing the current one, writes dx like norm_dx_kernel
// and keeps per-lane dgamma / dbeta sums; at the end the block's 4 waves
// combine them in LDS and store ONE fp32 partial row per block -- plain
// stores, no atomics (the atomic-combined fused kernel above, 512 blocks of
// 4-row waves, was latency-bound at H = 1600).  The [blocks, 2H] partials
// are summed by colsum_f32_kernel.
// DS: also the column sums of dx itself (the bias gradient of the Linear
// whose output is this add-norm's residual input): partial rows [3H].
#ifndef DWAMD_NORM_BWD_LDSACC
// A/B: the block's dgamma / dbeta (/ dx column) sums in LDS (ds_add_f32, the
// lane-contiguous layout [k][vector]) instead of 2-3 x 32 per-lane registers:
// the VPL = 4 instance (H 1025..2047, GPT2-1.5B's 1600) then fits more than
// one wave per SIMD (256 VGPRs + 82-114 AGPRs otherwise).  Sums in LDS are
// added in arrival order; DWAMD_DETERMINISTIC takes the two-pass path anyway.
// Measured: GPT2-1.5B step 108.4 -> 124.7 ms (the LDS float atomics cost more
// than the occupancy gains; profiles/r5/norm_bwd_ldsacc_ab.jsonl) -- off
#define DWAMD_NORM_BWD_LDSACC 0
#endif
#ifndef DWAMD_NORM_BWD_PF
// A/B: rows prefetched per wave (register sets); 2 = load the next row before
// computing the current one
#define DWAMD_NORM_BWD_PF 2
#endif
#ifndef DWAMD_NORM_BWD_W2
// A/B: the VPL = 4 instance (H 1025..2047) with ONE row register set and the
// per-lane column sums kept in registers, compiled for two waves per SIMD
// (<= 256 registers; gamma re-read per row, the residual gradient loaded
// where it is added): the second wave hides the row loads the prefetch set
// hid before, and twice the workgroups are resident (512).  GPT2-1.5B's call
// (H = 1600, dres + dx column sums) alone: 39.0 -> 36.9 us at 8192 rows, 62.0
// -> 56.1 us at 16384 (profiles/r6/norm_bwd_w2_ab.jsonl); inside the step the
// kernel goes 35.6 -> 34.5 us but the column-sum pass over twice the block
// partials 7.6 -> 10.4 us (profiles/r6/gpt2_1.5b_step_kernels.md): off
#define DWAMD_NORM_BWD_W2 0
#endif

template <int VPL, bool RMS, bool DS = false>
__global__ void __launch_bounds__(256, ((DWAMD_NORM_BWD_LDSACC || DWAMD_NORM_BWD_W2) && VPL == 4) ? 2 : 1)
norm_bwd_part_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, const bf16_t* __restrict__ dres,
    bf16_t* __restrict__ dx, float* __restrict__ part, int64_t rows, int H) {
  static_assert(VPL <= 4, "small-H norm backward");
  constexpr bool LA = DWAMD_NORM_BWD_LDSACC != 0;
  // two waves per SIMD: gamma re-read per row (L1-resident) and the residual
  // gradient loaded where it is added, not held across the row reductions
  constexpr bool W2 = DWAMD_NORM_BWD_W2 && VPL == 4 && !LA;
  constexpr int NVP = 64 * VPL;  // vectors per row, padded
  __shared__ float red[LA ? 1 : 2][LA ? 1 : 4][LA ? 1 : 512 + 4];
  __shared__ float lacc[LA ? (DS ? 3 : 2) : 1][LA ? 8 * NVP : 1];  // [array][k * NVP + vector]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nv = H >> 3;
  float ag[LA ? 1 : VPL][8], ab[LA ? 1 : VPL][8], ad[LA ? 1 : VPL][8];
  if constexpr (LA) {
    for (int i = threadIdx.x; i < (DS ? 3 : 2) * 8 * NVP; i += 256) (&lacc[0][0])[i] = 0.f;
    __syncthreads();
  } else {
#pragma unroll
    for (int j = 0; j < VPL; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) ag[j][k] = ab[j][k] = ad[j][k] = 0.f;
  }
  u32x4 gv[W2 ? 1 : VPL];
  if constexpr (!W2) {
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nv) gv[j] = *(const u32x4*)(gamma + c * 8);
    }
  }
  auto gam = [&](int j, int c) -> u32x4 {
    if constexpr (W2) return *(const u32x4*)(gamma + c * 8);
    else return gv[j];
  };
  // grid-stride over rows, one row per wave per step, the next row's x / dy
  // / dres (and mean / rstd) loaded before the current one is computed: two
  // named register sets, the loop unrolled by two so nothing is copied
  const int64_t stride = (int64_t)gridDim.x * 4;
  struct Row {
    u32x4 x[VPL], d[VPL], r[W2 ? 1 : VPL];
    float mu, rs;
  };
  auto load = [&](Row& b, int64_t row) {
    if (row >= rows) return;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nv) {
        b.x[j] = *(const u32x4*)(x + row * H + c * 8);
        b.d[j] = *(const u32x4*)(dy + row * H + c * 8);
        if constexpr (!W2)
          if (dres) b.r[j] = *(const u32x4*)(dres + row * H + c * 8);
      }
    }
    b.mu = RMS ? 0.f : mean_in[row];
    b.rs = rstd_in[row];
  };
  auto process = [&](const Row& b, int64_t row) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nv) {
        float xf[8], df[8], gm[8];
        unpack8(b.x[j], xf);
        unpack8(b.d[j], df);
        unpack8(gam(j, c), gm);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float a = (xf[k] - b.mu) * b.rs, g = df[k] * gm[k];
          if constexpr (LA) {
            atomicAdd(&lacc[0][k * NVP + c], df[k] * a);
            if constexpr (!RMS) atomicAdd(&lacc[1][k * NVP + c], df[k]);
          } else {
            ag[j][k] += df[k] * a;
            if constexpr (!RMS) ab[j][k] += df[k];
          }
          s1 += g;
          s2 += g * a;
        }
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) / (float)H;
    const float m2 = wave_sum(s2) / (float)H;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nv) {
        float xf[8], df[8], gm[8], o[8];
        u32x4 rv;
        if constexpr (W2)
          if (dres) rv = *(const u32x4*)(dres + row * H + c * 8);
        unpack8(b.x[j], xf);  // recomputed: cheaper than 64 more live registers
        unpack8(b.d[j], df);
        unpack8(gam(j, c), gm);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = b.rs * (df[k] * gm[k] - m1 - (xf[k] - b.mu) * b.rs * m2);
        if (dres) {
          float r[8];
          if constexpr (W2) unpack8(rv, r);
          else unpack8(b.r[W2 ? 0 : j], r);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += r[k];
        }
        if constexpr (DS) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if constexpr (LA)
              atomicAdd(&lacc[DS ? 2 : 0][k * NVP + c], o[k]);
            else
              ad[j][k] += o[k];
          }
        }
        *(u32x4*)(dx + row * H + c * 8) = pack8(o);
      }
    }
  };
  int64_t row = (int64_t)blockIdx.x * 4 + wid;
  if constexpr (LA || (DWAMD_NORM_BWD_W2 && VPL == 4)) {
    // more waves per SIMD instead of a second register set: one row in flight per wave
    Row A;
    for (; row < rows; row += stride) {
      load(A, row);
      process(A, row);
    }
  } else if constexpr (DWAMD_NORM_BWD_PF > 2) {
    // PF register sets: PF - 1 rows in flight while one is computed (a wave
    // owns ~rows / 1024 rows, 8 at GPT2's B*S = 8192, so the ramp matters)
    constexpr int PF = DWAMD_NORM_BWD_PF;
    Row R[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) load(R[p], row + p * stride);
    for (; row < rows; row += PF * stride) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const int64_t rr = row + p * stride;
        if (rr < rows) {
          process(R[p], rr);
          load(R[p], rr + PF * stride);
        }
      }
    }
  } else {
    Row A, B;
    load(A, row);
    while (row < rows) {
      load(B, row + stride);
      process(A, row);
      row += stride;
      if (row >= rows) break;
      load(A, row + stride);
      process(B, row);
      row += stride;
    }
  }
  float* prow = part + (int64_t)blockIdx.x * (DS ? 3 : 2) * H;
  if constexpr (LA) {
    __syncthreads();
    for (int col = threadIdx.x; col < H; col += 256) {
      const int cv = col >> 3, k = col & 7;
      prow[col] = lacc[0][k * NVP + cv];
      prow[H + col] = RMS ? 0.f : lacc[1][k * NVP + cv];
      if constexpr (DS) prow[2 * H + col] = lacc[DS ? 2 : 0][k * NVP + cv];
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[0][wid][lane * 8 + k] = ag[j][k];
      if constexpr (!RMS) red[1][wid][lane * 8 + k] = ab[j][k];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cl = threadIdx.x + 256 * h;
      const int c = 512 * j + cl;
      if (c < H) {
        prow[c] = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
        prow[H + c] = RMS ? 0.f : red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
      }
    }
    __syncthreads();
    if constexpr (DS) {
#pragma unroll
      for (int k = 0; k < 8; ++k) red[0][wid][lane * 8 + k] = ad[j][k];
      __syncthreads();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int cl = threadIdx.x + 256 * h;
        const int c = 512 * j + cl;
        if (c < H) prow[2 * H + c] = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
      }
      __syncthreads();
    }
  }
}

// Norm backward for 1024 < H < 2048 with TWO waves per row.  The one-wave
// form (VPL = 4 above) holds 4 vectors x 3 arrays of a row per lane plus 96
// per-lane column accumulators: ~310 VGPRs, one wave per SIMD, latency-bound
// at ~3 TB/s (GPT2-1.5B's H = 1600: 34.5 us per call in the step).  Here a
// row is split between a wave pair (each wave 2 vectors per lane = half the
// columns): 48 accumulators, 180-242 VGPRs, two waves per SIMD; the row
// reductions (sum g, sum g a) combine through LDS with one barrier per row
// step (parity double-buffered).  One 8-wave workgroup per CU (4 rows in
// flight, the next row of each pair prefetched) keeps ONE partial row per
// workgroup, as many as the one-wave form: the column-sum pass is unchanged.
// Deterministic: a fixed row order per pair and a fixed half-0 + half-1
// order for the row sums.
#ifndef DWAMD_NORM_BWD_PAIR_WAVES
#define DWAMD_NORM_BWD_PAIR_WAVES 8
#endif
// G = 4 (2048 <= H <= 4096, Llama's 4096): the same with a row split over a
// wave QUAD -- each wave still 2 vectors per lane (1024 columns), two rows
// in flight per workgroup.  The one-pass kernel it replaces there
// (norm_bwd_fused_kernel, 8 vectors per lane, float atomics per block)
// moved ~2.4 TB/s: Llama-3-8B's call (RMSNorm, 4096 x 4096, residual
// gradient fused) 43.1 -> 32.5 us, 8192 rows 66.7 -> 56.6 us
// (profiles/r6/norm_bwd_quad_ab.jsonl); 0: the atomic one-pass kernel
#ifndef DWAMD_NORM_BWD_QUAD
#define DWAMD_NORM_BWD_QUAD 1
#endif
template <bool RMS, bool DS, int G = 2>
__global__ void __launch_bounds__(64 * DWAMD_NORM_BWD_PAIR_WAVES, 1)
norm_bwd_pair_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ gamma,
                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                     const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ part,
                     int64_t rows, int H) {
  constexpr int NW = DWAMD_NORM_BWD_PAIR_WAVES, NP = NW / G;
  __shared__ float xch[2][NP][G][2];  // [parity][row group][part][sum g, sum g a]
  __shared__ float red[NW][1024];     // per-wave column partials of one array (final reduction)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int pair = wid / G, half = wid % G;  // row group, column part
  const int nv = H >> 3;
  float ag[2][8], ab[2][8], ad[2][8];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) ag[j][k] = ab[j][k] = ad[j][k] = 0.f;
  // this lane's vectors: half * 128 + lane + 64 j (j < 2) cover 0 .. 255
  int vc[2];
  bool vok[2];
  u32x4 gv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    vc[j] = 128 * half + lane + 64 * j;
    vok[j] = vc[j] < nv;
    gv[j] = vok[j] ? *(const u32x4*)(gamma + vc[j] * 8) : (u32x4){0, 0, 0, 0};
  }
  struct Row {
    u32x4 x[2], d[2], r[2];
    float mu, rs;
  };
  auto load = [&](Row& b, int64_t row) {
    if (row >= rows) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (vok[j]) {
        b.x[j] = *(const u32x4*)(x + row * H + vc[j] * 8);
        b.d[j] = *(const u32x4*)(dy + row * H + vc[j] * 8);
        if (dres) b.r[j] = *(const u32x4*)(dres + row * H + vc[j] * 8);
      }
    }
    b.mu = RMS ? 0.f : mean_in[row];
    b.rs = rstd_in[row];
  };
  auto process = [&](const Row& b, int64_t row, int it) {
    const bool ok = row < rows;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (ok && vok[j]) {
        float xf[8], df[8], gm[8];
        unpack8(b.x[j], xf);
        unpack8(b.d[j], df);
        unpack8(gv[j], gm);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float a = (xf[k] - b.mu) * b.rs, g = df[k] * gm[k];
          ag[j][k] += df[k] * a;
          if constexpr (!RMS) ab[j][k] += df[k];
          s1 += g;
          s2 += g * a;
        }
      }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    float(*xc)[G][2] = xch[it & 1];
    if (lane == 0) {
      xc[pair][half][0] = s1;
      xc[pair][half][1] = s2;
    }
    __syncthreads();  // the only barrier of the row step (the slot of step it-1 stays untouched)
    float t1 = 0.f, t2 = 0.f;  // fixed part order
#pragma unroll
    for (int q = 0; q < G; ++q) {
      t1 += xc[pair][q][0];
      t2 += xc[pair][q][1];
    }
    const float m1 = RMS ? 0.f : t1 / (float)H;
    const float m2 = t2 / (float)H;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (ok && vok[j]) {
        float xf[8], df[8], gm[8], o[8];
        unpack8(b.x[j], xf);
        unpack8(b.d[j], df);
        unpack8(gv[j], gm);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = b.rs * (df[k] * gm[k] - m1 - (xf[k] - b.mu) * b.rs * m2);
        if (dres) {
          float r[8];
          unpack8(b.r[j], r);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += r[k];
        }
        if constexpr (DS) {
#pragma unroll
          for (int k = 0; k < 8; ++k) ad[j][k] += o[k];
        }
        *(u32x4*)(dx + row * H + vc[j] * 8) = pack8(o);
      }
    }
  };
  // every wave of the workgroup runs the same number of row steps (barriers)
  const int64_t stride = (int64_t)gridDim.x * NP;
  const int64_t first = (int64_t)blockIdx.x * NP;
  const int n_it = first < rows ? (int)((rows - first + stride - 1) / stride) : 0;
  int64_t row = first + pair;
  Row A, B;
  load(A, row);
  for (int it = 0; it < n_it; ++it) {
    if (it & 1) {
      load(A, row + stride);
      process(B, row, it);
    } else {
      load(B, row + stride);
      process(A, row, it);
    }
    row += stride;
  }
  // column partials of the workgroup: the 6 waves of each half summed in a fixed order
  float* prow = part + (int64_t)blockIdx.x * (DS ? 3 : 2) * H;
  auto reduce = [&](const float (*acc)[8], int off) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[wid][8 * (lane + 64 * j) + k] = acc[j][k];
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += 64 * NW) {
      const int h = c >> 10, lc = c & 1023;
      float sum = 0.f;
#pragma unroll
      for (int p2 = 0; p2 < NP; ++p2) sum += red[G * p2 + h][lc];
      prow[off + c] = sum;
    }
    __syncthreads();
  };
  reduce(ag, 0);
  if constexpr (!RMS) reduce(ab, H);
  else
    for (int c = threadIdx.x; c < H; c += 64 * NW) prow[H + c] = 0.f;
  if constexpr (DS) reduce(ad, 2 * H);
}

// Column sums of fp32 partials [R, 2H] into out0 (columns 0..H-1) and out1
// (H..2H-1, may be null): thread = column, grid.y splits the rows; one
// atomic per (column, row-split) into ws, the last row-split block of each
// 256-column strip converts (+ accumulates) and clears -- colred_kernel's
// completion protocol.  ws: fp32 [2H + ceil(2H/256)], zero on entry and exit.
__global__ void __launch_bounds__(256) colsum_f32_kernel(const float* __restrict__ part, int R, int H2,
                                                         int rows_per_blk, float* __restrict__ ws,
                                                         void* __restrict__ out0, void* __restrict__ out1,
                                                         int is_fp32, int accumulate, int H,
                                                         void* __restrict__ out2, int accumulate2,
                                                         float* __restrict__ detp) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r0 = blockIdx.y * rows_per_blk, r1 = min(R, r0 + rows_per_blk);
  if (c < H2) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int r = r0;
    for (; r + 4 <= r1; r += 4) {
      a0 += part[(int64_t)r * H2 + c];
      a1 += part[(int64_t)(r + 1) * H2 + c];
      a2 += part[(int64_t)(r + 2) * H2 + c];
      a3 += part[(int64_t)(r + 3) * H2 + c];
    }
    for (; r < r1; ++r) a0 += part[(int64_t)r * H2 + c];
    if (detp)
      __hip_atomic_store(detp + (int64_t)blockIdx.y * H2 + c, (a0 + a1) + (a2 + a3), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    else
      atomicAdd(ws + c, (a0 + a1) + (a2 + a3));
  }
  __shared__ int is_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* cnt = (unsigned*)(ws + H2) + blockIdx.x;
  if (threadIdx.x == 0)
    is_last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.y - 1;
  __syncthreads();
  if (!is_last) return;
  if (c < H2) {
    const float v = detp ? ordered_sum(detp + c, H2, gridDim.y)
                         : __hip_atomic_exchange(ws + c, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c < H)
      colred_store(out0, c, v, is_fp32, accumulate);
    else if (c < 2 * H)
      colred_store(out1, c - H, v, is_fp32, accumulate);
    else
      colred_store(out2, c - 2 * H, v, is_fp32, accumulate2);  // the folded bias gradient
  }
  if (threadIdx.x == 0) __hip_atomic_exchange(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int colred_rows_per_blk(int64_t rows, int C, int dflt_blocks) {
  // Grid-size target per kernel flavour (DWAMD_COLRED_BLOCKS overrides all,
  // for A/B).  Fewer row blocks = fewer same-address atomics per column; the
  // plain column sum is atomic-bound and wants ~1 block per CU, the fused
  // GELU backward (3 streams of HBM traffic) wants more memory parallelism.
  // Measured on GPT2-1.5B shapes (scripts/bench_colred.py, profiles/r2/
  // bench_colred.jsonl): colsum 8192x1600 16.5 -> 10.9 us at 256 blocks,
  // gelu_bwd_dbias 8192x6400 60.9 -> 56.9 us at 2048.
  static const int env_target = [] {
    const char* e = getenv("DWAMD_COLRED_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  const int target = env_target > 0 ? env_target : dflt_blocks;
  const int64_t col_blks = (C + 511) / 512;
  int64_t rs = (target + col_blks - 1) / col_blks;
  if (rs < 1) rs = 1;
  int64_t per = (rows + rs - 1) / rs;
  per = (per + 3) / 4 * 4;
  return (int)(per < 4 ? 4 : per);
}

// ws: fp32 [C + ceil(C/512)] (sums + per-strip completion counters), all-zero on entry, left all-zero.  out (+)= column sums of dy [rows, C].
// det: nullptr (atomic combine) or fp32 scratch of dw_colred_det_floats(rows, C, 0) floats (any content).
extern "C" int dw_colsum_acc(const void* dy, int64_t rows, int C, void* ws, void* out, int out_fp32, int accumulate,
                             void* stream, void* det) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int per = colred_rows_per_blk(rows, C, 256);
  dim3 grid((C + 511) / 512, (unsigned)((rows + per - 1) / per));
  hipLaunchKernelGGL(colred_kernel<0>, grid, dim3(256), 0, s, (const bf16_t*)dy, nullptr, nullptr, nullptr,
                     (float*)ws, rows, C, per, out, nullptr, out_fp32, accumulate, nullptr, (float*)det);
  DW_LAUNCH_RET;
}

// dx = dy * gelu'(pre) [rows, C]; dbias (+)= column sums of dx.  ws as above.
// det: as dw_colsum_acc (dw_colred_det_floats(rows, C, 1) floats).
extern "C" int dw_gelu_bwd_dbias(const void* dy, const void* pre, void* dx, int64_t rows, int C, void* ws,
                                 void* dbias, int out_fp32, int accumulate, void* stream, void* det) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int per = colred_rows_per_blk(rows, C, 2048);
  dim3 grid((C + 511) / 512, (unsigned)((rows + per - 1) / per));
  hipLaunchKernelGGL(colred_kernel<3>, grid, dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)pre, nullptr,
                     nullptr, (float*)ws, rows, C, per, dbias, nullptr, out_fp32, accumulate, (bf16_t*)dx,
                     (float*)det);
  DW_LAUNCH_RET;
}

static int norm_colred_blocks() {
  static const int norm_blocks = [] {
    const char* e = getenv("DWAMD_COLRED_NORM_BLOCKS");
    return e && atoi(e) > 0 ? atoi(e) : 1024;
  }();
  return norm_blocks;
}

static int64_t colsum_f32_splits(int64_t nb) { return std::max<int64_t>(1, std::min<int64_t>(64, nb / 16)); }

// fp32 scratch the deterministic mode needs (kind 0: dw_colsum_acc, 1:
// dw_gelu_bwd_dbias, 2: dw_norm_bwd3): one partial row per row-block.
extern "C" int64_t dw_colred_det_floats(int64_t rows, int C, int kind) {
  auto grid_y = [&](int target) {
    const int per = colred_rows_per_blk(rows, C, target);
    return (rows + per - 1) / per;
  };
  if (kind == 0) return grid_y(256) * C;
  if (kind == 1) return grid_y(2048) * C;
  // norm: the two-pass path (colred_kernel<1>, 2 sums per column) or the
  // small-H partial-rows path (colsum_f32_kernel over <= 3H columns)
  const int64_t nb = std::min<int64_t>((rows + 3) / 4, (C > 1024 && !DWAMD_NORM_BWD_LDSACC) ? 256 : 512);
  return std::max<int64_t>(grid_y(norm_colred_blocks()) * 2 * C, colsum_f32_splits(nb) * 3 * C);
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

// Norm backward v2.  ws: fp32 [2H + ceil(H/512)], all-zero on entry, left all-zero.
// dgamma/dbeta (+)= (accumulate flag).  dres (nullable): gradient of the
// residual sum that this norm's input also feeds (fused add+norm) -> dx += dres.
// det: nullptr, or fp32 scratch of dw_colred_det_floats(rows, H, 2) floats:
// deterministic weight gradients (the two-pass path with ordered partials).
extern "C" int dw_norm_bwd2(const void* dy, const void* x, const void* gamma, const void* mean, const void* rstd,
                            const void* dres, void* dx, void* dgamma, void* dbeta, void* ws, int64_t rows, int H,
                            int rms, int out_fp32, int accumulate, void* stream, void* det) {
  if (H % 8 != 0 || H > 8 * 64 * 16) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  static const bool two_pass = getenv_flag("DWAMD_NORM_BWD_2PASS");  // A/B switch
  if ((dgamma || dbeta) && H >= 2048 && H <= 8 * 64 * 8 && !two_pass && !det) {
    // one pass: dx + weight gradients (2 blocks per CU of 4 row-striding
    // waves).  Measured (scripts/bench_norm.py): RMSNorm 16k x 4096 141 ->
    // 118 us; at H = 1600 the two passes are as fast (the row pass alone
    // fills the chip better), so small H keeps them.
    const unsigned nb = (unsigned)std::min<int64_t>((rows + 3) / 4, 512);
    DISPATCH_VPL2(H, {
      if constexpr (VPL <= 8) {
        if (rms)
          hipLaunchKernelGGL((norm_bwd_fused_kernel<VPL, true>), dim3(nb), block, 0, s, (const bf16_t*)dy,
                             (const bf16_t*)x, (const bf16_t*)gamma, nullptr, (const float*)rstd,
                             (const bf16_t*)dres, (bf16_t*)dx, (float*)ws, dgamma, nullptr, out_fp32, accumulate,
                             rows, H);
        else
          hipLaunchKernelGGL((norm_bwd_fused_kernel<VPL, false>), dim3(nb), block, 0, s, (const bf16_t*)dy,
                             (const bf16_t*)x, (const bf16_t*)gamma, (const float*)mean, (const float*)rstd,
                             (const bf16_t*)dres, (bf16_t*)dx, (float*)ws, dgamma, dbeta, out_fp32, accumulate,
                             rows, H);
      }
    });
    DW_LAUNCH_RET;
  }
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
  const int per = colred_rows_per_blk(rows, H, norm_colred_blocks());
  dim3 cg((H + 511) / 512, (unsigned)((rows + per - 1) / per));
  // both halves are consumed (and cleared) even if one output is absent
  if (rms)
    hipLaunchKernelGGL(colred_kernel<2>, cg, dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)x, nullptr,
                       (const float*)rstd, (float*)ws, rows, H, per, dgamma, nullptr, out_fp32, accumulate, nullptr,
                       (float*)det);
  else
    hipLaunchKernelGGL(colred_kernel<1>, cg, dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)x,
                       (const float*)mean, (const float*)rstd, (float*)ws, rows, H, per, dgamma, dbeta, out_fp32,
                       accumulate, nullptr, (float*)det);
  DW_LAUNCH_RET;
}

// Norm backward v3: v2, plus the small-H one-pass path (H < 2048) when the
// caller provides fp32 scratch ``part`` of at least part_floats =
// ceil(rows / 8) * 2H floats (any content).  ws as v2 but sized
// 2H + ceil(2H / 256) + ceil(H / 512) floats.
//
// dsum (nullable, small-H path only): column sums of dx accumulated into it
// (same dtype as dgamma) -- the bias gradient of the Linear that produced
// the residual input; returns 1 when it was written, 0 when not (fallback
// path: the caller keeps the Linear's own bias reduction).
extern "C" int dw_norm_bwd3(const void* dy, const void* x, const void* gamma, const void* mean, const void* rstd,
                            const void* dres, void* dx, void* dgamma, void* dbeta, void* ws, void* part,
                            int64_t part_floats, int64_t rows, int H, int rms, int out_fp32, int accumulate,
                            void* dsum, int* dsum_done, void* stream, void* det) {
  // accumulate: bit 0 -- dgamma / dbeta accumulate; bit 1 -- dsum is
  // OVERWRITTEN (its parameter's first gradient contribution of the step)
  const int acc2 = (accumulate & 2) ? 0 : 1;
  accumulate &= 1;
  // every workgroup resident at once, each wave striding over rows: H > 1024
  // (VPL 4) needs ~310-370 VGPRs, one workgroup per CU; smaller H two
  const int64_t nb = std::min<int64_t>((rows + 3) / 4,
                                       (H > 1024 && !DWAMD_NORM_BWD_LDSACC && !DWAMD_NORM_BWD_W2) ? 256 : 512);
  const int pw = dsum ? 3 : 2;
  if (dsum_done) *dsum_done = 0;
  static const bool off = getenv_flag("DWAMD_NORM_BWD_PART_OFF");  // A/B switch
  const bool quad = DWAMD_NORM_BWD_QUAD && H >= 2048 && H <= 4096;
  if (off || !part || !(dgamma || dbeta) || H % 8 != 0 || (H >= 2048 && !quad) || (!quad && nb * pw * H > part_floats))
    return dw_norm_bwd2(dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, ws, rows, H, rms, out_fp32, accumulate,
                        stream, det);
  hipStream_t s = (hipStream_t)stream;
  static const bool pair_on = [] {  // A/B: DWAMD_NORM_BWD_PAIR=0 keeps the one-wave-per-row kernel
    const char* e = getenv("DWAMD_NORM_BWD_PAIR");
    return !(e && e[0] == '0');
  }();
  if ((pair_on && H > 1024 && H < 2048) || quad) {
    const int NP = DWAMD_NORM_BWD_PAIR_WAVES / (quad ? 4 : 2);
    const int64_t nbp = std::min<int64_t>((rows + NP - 1) / NP, 256);  // one workgroup per CU, resident
    if (nbp * pw * H > part_floats && quad)
      return dw_norm_bwd2(dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, ws, rows, H, rms, out_fp32, accumulate,
                          stream, det);
    if (nbp * pw * H <= part_floats) {
#define NBWG(RM, DSV, G)                                                                                          \
  hipLaunchKernelGGL((norm_bwd_pair_kernel<RM, DSV, G>), dim3((unsigned)nbp), dim3(64 * DWAMD_NORM_BWD_PAIR_WAVES), 0, \
                     s, (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)gamma,                               \
                     RM ? nullptr : (const float*)mean, (const float*)rstd, (const bf16_t*)dres, (bf16_t*)dx,          \
                     (float*)part, rows, H)
#define NBW(RM, DSV)        \
  do {                      \
    if (quad)               \
      NBWG(RM, DSV, 4);     \
    else                    \
      NBWG(RM, DSV, 2);     \
  } while (0)
      if (rms) {
        if (dsum) NBW(true, true); else NBW(true, false);
      } else {
        if (dsum) NBW(false, true); else NBW(false, false);
      }
#undef NBW
#undef NBWG
      if (dsum_done) *dsum_done = dsum ? 1 : 0;
      const int H2 = pw * H;
      const int splits = (int)colsum_f32_splits(nbp);
      const int per = (int)((nbp + splits - 1) / splits);
      dim3 g((H2 + 255) / 256, (unsigned)((nbp + per - 1) / per));
      hipLaunchKernelGGL(colsum_f32_kernel, g, dim3(256), 0, s, (const float*)part, (int)nbp, H2, per, (float*)ws,
                         dgamma, rms ? nullptr : dbeta, out_fp32, accumulate, H, dsum, acc2, (float*)det);
      DW_LAUNCH_RET;
    }
  }
#define NBP(RM, DSV)                                                                                          \
  hipLaunchKernelGGL((norm_bwd_part_kernel<VPL, RM, DSV>), dim3((unsigned)nb), dim3(256), 0, s,              \
                     (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)gamma, RM ? nullptr : (const float*)mean, \
                     (const float*)rstd, (const bf16_t*)dres, (bf16_t*)dx, (float*)part, rows, H)
  DISPATCH_VPL2(H, {
    if constexpr (VPL <= 4) {
      if (rms) {
        if (dsum) NBP(true, true); else NBP(true, false);
      } else {
        if (dsum) NBP(false, true); else NBP(false, false);
      }
    }
  });
#undef NBP
  if (dsum_done) *dsum_done = dsum ? 1 : 0;
  const int H2 = pw * H;
  const int splits = (int)colsum_f32_splits(nb);
  const int per = (int)((nb + splits - 1) / splits);
  dim3 g((H2 + 255) / 256, (unsigned)((nb + per - 1) / per));
  hipLaunchKernelGGL(colsum_f32_kernel, g, dim3(256), 0, s, (const float*)part, (int)nb, H2, per, (float*)ws,
                     dgamma, rms ? nullptr : dbeta, out_fp32, accumulate, H, dsum, acc2, (float*)det);
  DW_LAUNCH_RET;
}

DW_PRELOAD(colred_kernel<0>);
