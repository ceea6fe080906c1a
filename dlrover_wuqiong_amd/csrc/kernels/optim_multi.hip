// Multi-tensor fused optimizers: one launch updates every parameter of an
// optimizer, whatever its storage (FSDP2 DTensor local shards, TP shards, plain
// DDP parameters), without first packing them into a flat buffer.
//
// The host builds two device tables once per step (re-uploaded only when a
// gradient pointer changes):
//   MTDesc  per tensor : param / grad / fp32 master / exp_avg / exp_avg_sq
//                        pointers, element count, dtype + alignment flags,
//                        param-group index, weight in the global grad norm;
//   MTChunk per chunk  : (tensor, chunk) pairs of MT_CHUNK elements.
// Workgroups grid-stride over the chunk table; a chunk lives in one tensor, so
// the dtype/alignment branches are uniform per workgroup (no divergence) and
// a 16-byte aligned tensor streams through 8-element vectors (28 B/elem for
// bf16 params + fp32 master/moments, 32 B/elem with an fp32 grad).
//
// Hyper-parameters are per param group (<= MT_MAX_GROUPS) and passed by value,
// so an LR scheduler changing group["lr"] costs no upload.  The gradient scale
// (1/world, global-norm clip coefficient) is a device scalar: no host sync.
//
// Parity: torch.optim.AdamW / Adam math (decoupled or L2 decay) and ATorch
// AGD (atorch/atorch/optimizers/agd.py:84-150), as in optim.hip; the apex /
// DeepSpeed multi_tensor_apply they replace in atorch/atorch/optimizers/*.
#include "dw_common.h"

#define MT_MAX_GROUPS 16
#define MT_CHUNK 16384
#define MT_THREADS 256

struct MTDesc {
  void* p;
  const void* g;
  float* master;
  float* m;
  float* v;
  int64_t n;
  int32_t flags;  // bit0: param bf16, bit1: grad bf16, bit2: all pointers 16 B aligned
  int32_t group;
  float norm_w;   // weight of this tensor's squared grad in the global norm
  int32_t pad;
};
static_assert(sizeof(MTDesc) == 64, "MTDesc layout is shared with python");

struct MTChunk {
  int32_t t;
  int32_t c;
};

struct MTHyper {
  float lr[MT_MAX_GROUPS], wd[MT_MAX_GROUPS], b1[MT_MAX_GROUPS], b2[MT_MAX_GROUPS];
  float eps[MT_MAX_GROUPS];   // Adam eps / AGD delta
  float bc1[MT_MAX_GROUPS], bc2[MT_MAX_GROUPS], bc1_prev[MT_MAX_GROUPS];
  float clip[MT_MAX_GROUPS];  // AGD update clip (0: off)
  int adamw;                  // Adam: 1 decoupled decay, 0 L2 in the gradient
};

__device__ __forceinline__ float ldf(const void* p, int64_t i, bool bf) {
  return bf ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
__device__ __forceinline__ void stf(void* p, int64_t i, float v, bool bf) {
  if (bf) ((bf16_t*)p)[i] = f2bf(v); else ((float*)p)[i] = v;
}
__device__ __forceinline__ void ld8v(const void* p, int64_t i, float* f, bool bf) {
  if (bf) {
    unpack8(*(const u32x4*)((const bf16_t*)p + i), f);
  } else {
    const f32x4 a = *(const f32x4*)((const float*)p + i), b = *(const f32x4*)((const float*)p + i + 4);
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  }
}
__device__ __forceinline__ void st8v(void* p, int64_t i, const float* f, bool bf) {
  if (bf) {
    *(u32x4*)((bf16_t*)p + i) = pack8(f);
  } else {
    *(f32x4*)((float*)p + i) = f32x4{f[0], f[1], f[2], f[3]};
    *(f32x4*)((float*)p + i + 4) = f32x4{f[4], f[5], f[6], f[7]};
  }
}

// One element of the update, in registers.  AGD=false: Adam(W).
template <bool AGD>
__device__ __forceinline__ void upd(float g, float& w, float& m, float& v, float lr, float wd, float b1, float b2,
                                    float eps, float bc1, float rbc2, float sqbc2, float bc1_prev, float clip,
                                    int adamw) {
  if (!AGD) {
    if (!adamw) g += wd * w;
    m = b1 * m + (1.f - b1) * g;
    v = b2 * v + (1.f - b2) * g * g;
    const float denom = sqrtf(v) * rbc2 + eps;
    if (adamw) w -= lr * wd * w;
    w -= (lr / bc1) * m / denom;
  } else {
    w *= 1.f - lr * wd;
    const float mprev = m;
    m = b1 * mprev + (1.f - b1) * g;
    const float s = (bc1_prev > 0.f) ? (m / bc1 - mprev / bc1_prev) : m / bc1;
    v = b2 * v + (1.f - b2) * s * s;
    float u = m / fmaxf(sqrtf(v), eps * sqbc2);
    if (clip > 0.f) u = fminf(fmaxf(u, -clip), clip);
    w -= lr * sqbc2 / bc1 * u;
  }
}

template <bool AGD>
__global__ void __launch_bounds__(MT_THREADS) mt_step_kernel(const MTDesc* __restrict__ descs,
                                                             const MTChunk* __restrict__ chunks, int64_t nchunks,
                                                             const float* __restrict__ gscale, MTHyper h) {
  const float gs = gscale ? *gscale : 1.f;
  for (int64_t ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const MTChunk ch = chunks[ci];
    const MTDesc d = descs[ch.t];
    const int gi = d.group;
    const float lr = h.lr[gi], wd = h.wd[gi], b1 = h.b1[gi], b2 = h.b2[gi], eps = h.eps[gi];
    const float bc1 = h.bc1[gi], rbc2 = rsqrtf(h.bc2[gi]), sqbc2 = sqrtf(h.bc2[gi]);
    const float bc1p = h.bc1_prev[gi], clip = h.clip[gi];
    const bool pbf = d.flags & 1, gbf = d.flags & 2, vec = d.flags & 4;
    const int64_t start = (int64_t)ch.c * MT_CHUNK;
    const int64_t end = min(start + (int64_t)MT_CHUNK, d.n);
    float* master = d.master;
    int64_t vend = start;
    if (vec) {
      vend = start + ((end - start) & ~(int64_t)7);
      for (int64_t i = start + threadIdx.x * 8; i < vend; i += MT_THREADS * 8) {
        float g[8], w[8], m[8], v[8];
        ld8v(d.g, i, g, gbf);
        if (master) ld8v(master, i, w, false); else ld8v(d.p, i, w, pbf);
        ld8v(d.m, i, m, false);
        ld8v(d.v, i, v, false);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          upd<AGD>(g[k] * gs, w[k], m[k], v[k], lr, wd, b1, b2, eps, bc1, rbc2, sqbc2, bc1p, clip, h.adamw);
        st8v(d.m, i, m, false);
        st8v(d.v, i, v, false);
        if (master) st8v(master, i, w, false);
        st8v(d.p, i, w, pbf);
      }
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += MT_THREADS) {
      float w = master ? master[i] : ldf(d.p, i, pbf);
      float m = d.m[i], v = d.v[i];
      upd<AGD>(ldf(d.g, i, gbf) * gs, w, m, v, lr, wd, b1, b2, eps, bc1, rbc2, sqbc2, bc1p, clip, h.adamw);
      d.m[i] = m;
      d.v[i] = v;
      if (master) master[i] = w;
      stf(d.p, i, w, pbf);
    }
  }
}

// sum over tensors of norm_w * ||grad||^2 -> added to *out (zeroed by the
// caller on the stream) by a deterministic fixed-order grid sum.
__global__ void __launch_bounds__(MT_THREADS) mt_sumsq_kernel(const MTDesc* __restrict__ descs,
                                                              const MTChunk* __restrict__ chunks, int64_t nchunks,
                                                              float* out, float* ws) {
  __shared__ float red[MT_THREADS / 64];
  float acc = 0.f;
  for (int64_t ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const MTChunk ch = chunks[ci];
    const MTDesc d = descs[ch.t];
    const bool gbf = d.flags & 2, vec = d.flags & 4;
    const int64_t start = (int64_t)ch.c * MT_CHUNK;
    const int64_t end = min(start + (int64_t)MT_CHUNK, d.n);
    float a = 0.f;
    int64_t vend = start;
    if (vec) {
      vend = start + ((end - start) & ~(int64_t)7);
      for (int64_t i = start + threadIdx.x * 8; i < vend; i += MT_THREADS * 8) {
        float g[8];
        ld8v(d.g, i, g, gbf);
#pragma unroll
        for (int k = 0; k < 8; ++k) a += g[k] * g[k];
      }
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += MT_THREADS) {
      const float x = ldf(d.g, i, gbf);
      a += x * x;
    }
    acc += a * d.norm_w;
  }
  acc = block_sum<MT_THREADS>(acc, red);
  __syncthreads();  // red is reused by the finish
  grid_sum_finish<MT_THREADS>(acc, ws, out, red);
}

static int mt_grid(int64_t nchunks) {
  // enough workgroups to cover 256 CUs x 8 waves several times; each walks
  // a strided subset of the chunk table
  int64_t g = nchunks < 8192 ? nchunks : 8192;
  return (int)(g < 1 ? 1 : g);
}

// max_blocks > 0 caps the grid: an update running beside other work (the
// optimizer inside the FSDP backward, optimizers/in_backward.py) then holds
// at most that many workgroups' worth of CUs at a time
extern "C" int dw_mt_adam_grid(const void* descs, const void* chunks, int64_t nchunks, const void* gscale,
                               const void* hyper, int agd, int max_blocks, void* stream) {
  if (nchunks <= 0) return 0;
  const MTHyper h = *(const MTHyper*)hyper;
  hipStream_t s = (hipStream_t)stream;
  int g = mt_grid(nchunks);
  if (max_blocks > 0 && g > max_blocks) g = max_blocks;
  if (agd)
    hipLaunchKernelGGL(mt_step_kernel<true>, dim3(g), dim3(MT_THREADS), 0, s, (const MTDesc*)descs,
                       (const MTChunk*)chunks, nchunks, (const float*)gscale, h);
  else
    hipLaunchKernelGGL(mt_step_kernel<false>, dim3(g), dim3(MT_THREADS), 0, s, (const MTDesc*)descs,
                       (const MTChunk*)chunks, nchunks, (const float*)gscale, h);
  DW_LAUNCH_RET;
}

extern "C" int dw_mt_adam(const void* descs, const void* chunks, int64_t nchunks, const void* gscale,
                          const void* hyper, int agd, void* stream) {
  return dw_mt_adam_grid(descs, chunks, nchunks, gscale, hyper, agd, 0, stream);
}

// ws: float[GRID_SUM_MAX + 1] (see grid_sum_finish)
extern "C" int dw_mt_sumsq(const void* descs, const void* chunks, int64_t nchunks, void* out, void* ws,
                           void* stream) {
  if (nchunks <= 0) return 0;
  const int grid = mt_grid(nchunks) < GRID_SUM_MAX ? mt_grid(nchunks) : GRID_SUM_MAX;
  hipLaunchKernelGGL(mt_sumsq_kernel, dim3(grid), dim3(MT_THREADS), 0, (hipStream_t)stream, (const MTDesc*)descs,
                     (const MTChunk*)chunks, nchunks, (float*)out, (float*)ws);
  DW_LAUNCH_RET;
}

extern "C" int dw_mt_hyper_size() { return (int)sizeof(MTHyper); }
extern "C" int dw_mt_chunk() { return MT_CHUNK; }

DW_PRELOAD(mt_sumsq_kernel);
