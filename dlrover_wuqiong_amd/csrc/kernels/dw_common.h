// Shared device helpers for the gfx950 kernels of dlrover_wuqiong_amd.
//
// Conventions used by every kernel TU:
//  * wave64 everywhere (CDNA4): lane = threadIdx.x & 63, reductions use
//    __shfl_xor over 64 lanes;
//  * bf16 tensors are moved as 16-byte vectors (8 x bf16) — hipcc does not
//    auto-vectorise 2-byte loads (guide G13);
//  * conversions use the native __bf16 type so hipcc emits
//    v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN preserving);
//  * every launcher is `extern "C" int dw_xxx(..., void* stream)` returning
//    the hipError_t of the launch, operating on PyTorch's current stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short bf16_t;  // storage type
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

// Element strides (batch, sequence row) of the BSHD attention tensors, so
// q/k/v can be views into one fused [B, S, 3, H, D] QKV projection output
// and the gradients can be written straight into the packed dQKV buffer.
struct AttnStrides {
  long long q_bs, q_rs, k_bs, k_rs, v_bs, v_rs, o_bs, o_rs;
  long long do_bs, do_rs, dq_bs, dq_rs, dk_bs, dk_rs, dv_bs, dv_rs;
};

#define DW_LAUNCH_RET return (int)hipGetLastError()

// Code-object preload: with deferred loading a TU's fat binary is loaded at
// the first launch of any of its kernels.  Every TU registers one kernel
// (DW_PRELOAD, at static-init time of the library); dw_preload_code_objects
// (preload.hip) queries each one's attributes, which loads every code object
// up front -- an import-mode standby does this while it waits, so the worker
// it becomes launches from warm modules (elastic_agent/warm_profile.py).
extern "C" void dw_register_preload(const void* kernel);
struct DwPreloadReg {
  explicit DwPreloadReg(const void* k) { dw_register_preload(k); }
};
#define DW_PRELOAD_CAT2(a, b) a##b
#define DW_PRELOAD_CAT(a, b) DW_PRELOAD_CAT2(a, b)
#define DW_PRELOAD(kernel) static DwPreloadReg DW_PRELOAD_CAT(dw_preload_reg_, __LINE__)((const void*)(kernel))

__device__ __forceinline__ float bf2f(bf16_t u) {
  return __uint_as_float(((unsigned int)u) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// unpack / pack 8 bf16 held in a 16-byte vector
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned int w = v[i];
    f[2 * i] = __uint_as_float(w << 16);
    f[2 * i + 1] = __uint_as_float(w & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned int lo = f2bf(f[2 * i]);
    unsigned int hi = f2bf(f[2 * i + 1]);
    v[i] = lo | (hi << 16);
  }
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `red` must hold
// NT/64 floats of LDS. Result broadcast to every thread.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// Grid size for memory-bound grid-stride kernels (guide G11): enough blocks
// to fill 256 CUs several times, capped.
static inline int dw_grid_for(int64_t work_items, int per_block, int cap = 2048) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// Deterministic grid-wide sum (replaces one float atomicAdd per block, whose
// order -- hence the last bits of the result -- varies run to run): every
// block stores its partial into ws[blockIdx.x] with an agent-scope atomic
// store, drains its stores, bumps the counter ws[GRID_SUM_MAX]; the LAST
// block sums the partials in a fixed order and adds the total to *out (one
// writer).  ws: float[GRID_SUM_MAX + 1], counter word zero on entry, left zero.
// No device-scope fence (an L2 write-back + invalidate per block on gfx950):
// the partials live at the coherent level (atomic stores / loads) and each
// block's stores have completed before its counter increment is issued.
constexpr int GRID_SUM_MAX = 2048;
template <int THREADS>
__device__ __forceinline__ void grid_sum_finish(float block_total, float* ws, float* out, float* red) {
  __shared__ int is_last;
  if (threadIdx.x == 0) {
    __hip_atomic_store(ws + blockIdx.x, block_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    is_last = __hip_atomic_fetch_add((unsigned*)(ws + GRID_SUM_MAX), 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!is_last) return;
  float a = 0.f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += THREADS)
    a += __hip_atomic_load(ws + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  a = block_sum<THREADS>(a, red);
  if (threadIdx.x == 0) {
    *out += a;
    __hip_atomic_store((unsigned*)(ws + GRID_SUM_MAX), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// tanh-approximate GELU and its derivative (GPT-2 MLP).  tanh(u) =
// 1 - 2 / (1 + 2^(2u log2 e)) with the hardware exp2 / rcp (a few VALU ops
// instead of libm tanhf's ~20: the GELU passes are VALU-bound otherwise);
// saturates correctly (exp2 -> inf gives 1, -> 0 gives -1); ~1e-6 relative.
__device__ __forceinline__ float fast_tanh(float u) {
  const float e = __builtin_amdgcn_exp2f(u * 2.8853900817779268f);  // 2 * log2(e)
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + fast_tanh(u));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * (x + k1 * x2 * x);
  const float t = fast_tanh(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x2);
}
