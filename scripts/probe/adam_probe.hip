// Flat AdamW streaming-layout probe (mixed precision: bf16 param + grad, fp32
// master / m / v = 28 B per element).  Times layout variants of the update on
// a GPT2-1.5B-sized flat buffer and prints one JSON line per variant:
//   0  8 consecutive elements per lane (optim.hip adam_flat_kernel layout)
//   1  4 elements per lane at two 256-element halves of a 512-element wave
//      slab: every load / store instruction covers one contiguous span
//   2  variant 1 with non-temporal loads / stores
//   3  variant 0 with non-temporal loads / stores
//   9  same bytes moved, no arithmetic (bandwidth ceiling)
// build: hipcc --offload-arch=gfx950 -O3 -o adam_probe adam_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>

typedef unsigned short bf16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ float bf2f(unsigned int u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ unsigned int pk2(float a, float b) {
  typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
  typedef float f32x2_v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned int, __builtin_convertvector((f32x2_v){a, b}, bf16x2_v));
}

struct A { float lr, b1, b2, eps, wd, bc1, bc2; int64_t n; const unsigned char* mask; };

template <int NT>
__device__ __forceinline__ f32x4 ldf(const float* p) {
  if (NT) return __builtin_nontemporal_load((const f32x4*)p);
  return *(const f32x4*)p;
}
template <int NT>
__device__ __forceinline__ void stf(float* p, f32x4 v) {
  if (NT) __builtin_nontemporal_store(v, (f32x4*)p); else *(f32x4*)p = v;
}

__device__ __forceinline__ void upd(float& w, float& m, float& v, float g, bool decay, float step, float rbc2,
                                    const A& a) {
  m = a.b1 * m + (1.f - a.b1) * g;
  v = a.b2 * v + (1.f - a.b2) * g * g;
  const float den = sqrtf(v) * rbc2 + a.eps;
  if (decay) w -= a.lr * a.wd * w;
  w -= step * m / den;
}

// variant 0 / 3: 8 consecutive elements per lane
template <int NT>
__global__ void __launch_bounds__(256) k_v0(bf16_t* p, float* ms, const bf16_t* gr, float* m, float* v, A a) {
  const float step = a.lr / a.bc1, rbc2 = rsqrtf(a.bc2);
  const int64_t nvec = a.n >> 3;
  for (int64_t vi = blockIdx.x * 256ll + threadIdx.x; vi < nvec; vi += (int64_t)gridDim.x * 256) {
    const int64_t i = vi << 3;
    u32x4 gg = NT ? __builtin_nontemporal_load((const u32x4*)(gr + i)) : *(const u32x4*)(gr + i);
    f32x4 w0 = ldf<NT>(ms + i), w1 = ldf<NT>(ms + i + 4);
    f32x4 m0 = ldf<NT>(m + i), m1 = ldf<NT>(m + i + 4);
    f32x4 v0 = ldf<NT>(v + i), v1 = ldf<NT>(v + i + 4);
    const bool d = a.mask[i >> 6] != 0;
    float g[8];
    for (int k = 0; k < 4; ++k) { g[2 * k] = bf2f(gg[k] & 0xffff); g[2 * k + 1] = bf2f(gg[k] >> 16); }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float x0 = w0[k], y0 = m0[k], z0 = v0[k], x1 = w1[k], y1 = m1[k], z1 = v1[k];
      upd(x0, y0, z0, g[k], d, step, rbc2, a);
      upd(x1, y1, z1, g[4 + k], d, step, rbc2, a);
      w0[k] = x0; m0[k] = y0; v0[k] = z0; w1[k] = x1; m1[k] = y1; v1[k] = z1;
    }
    stf<NT>(m + i, m0); stf<NT>(m + i + 4, m1);
    stf<NT>(v + i, v0); stf<NT>(v + i + 4, v1);
    stf<NT>(ms + i, w0); stf<NT>(ms + i + 4, w1);
    u32x4 o = {pk2(w0[0], w0[1]), pk2(w0[2], w0[3]), pk2(w1[0], w1[1]), pk2(w1[2], w1[3])};
    if (NT) __builtin_nontemporal_store(o, (u32x4*)(p + i)); else *(u32x4*)(p + i) = o;
  }
}

// variant 1 / 2: a wave owns a 512-element slab; lane l: 4 elements at 4l and
// at 256 + 4l
template <int NT, int UNR>
__global__ void __launch_bounds__(256) k_v1(bf16_t* p, float* ms, const bf16_t* gr, float* m, float* v, A a) {
  const float step = a.lr / a.bc1, rbc2 = rsqrtf(a.bc2);
  const int lane = threadIdx.x & 63;
  const int64_t nslab = a.n >> 9;
  const int64_t w0i = blockIdx.x * 4ll + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  for (int64_t s = w0i; s < nslab; s += nw * UNR) {
    f32x4 w[UNR][2], mm[UNR][2], vv[UNR][2];
    u32x2 gg[UNR][2];
    bool d[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t su = s + u * nw;
      if (su >= nslab) continue;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int64_t i = (su << 9) + 256 * hf + 4 * lane;
        gg[u][hf] = NT ? __builtin_nontemporal_load((const u32x2*)(gr + i)) : *(const u32x2*)(gr + i);
        w[u][hf] = ldf<NT>(ms + i);
        mm[u][hf] = ldf<NT>(m + i);
        vv[u][hf] = ldf<NT>(v + i);
      }
      d[u] = a.mask[((su << 9) + 4 * lane) >> 6] != 0;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t su = s + u * nw;
      if (su >= nslab) continue;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int64_t i = (su << 9) + 256 * hf + 4 * lane;
        const bool dd = hf ? (a.mask[i >> 6] != 0) : d[u];
        float g[4] = {bf2f(gg[u][hf][0] & 0xffff), bf2f(gg[u][hf][0] >> 16), bf2f(gg[u][hf][1] & 0xffff),
                      bf2f(gg[u][hf][1] >> 16)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float x = w[u][hf][k], y = mm[u][hf][k], z = vv[u][hf][k];
          upd(x, y, z, g[k], dd, step, rbc2, a);
          w[u][hf][k] = x; mm[u][hf][k] = y; vv[u][hf][k] = z;
        }
        stf<NT>(m + i, mm[u][hf]);
        stf<NT>(v + i, vv[u][hf]);
        stf<NT>(ms + i, w[u][hf]);
        u32x2 o = {pk2(w[u][hf][0], w[u][hf][1]), pk2(w[u][hf][2], w[u][hf][3])};
        if (NT) __builtin_nontemporal_store(o, (u32x2*)(p + i)); else *(u32x2*)(p + i) = o;
      }
    }
  }
}

// bandwidth ceiling: the same 28 B / element moved, no update arithmetic
__global__ void __launch_bounds__(256) k_copy(bf16_t* p, float* ms, const bf16_t* gr, float* m, float* v, A a) {
  const int lane = threadIdx.x & 63;
  const int64_t nslab = a.n >> 9;
  const int64_t w0i = blockIdx.x * 4ll + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  for (int64_t s = w0i; s < nslab; s += nw) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int64_t i = (s << 9) + 256 * hf + 4 * lane;
      u32x2 g = *(const u32x2*)(gr + i);
      f32x4 x = *(const f32x4*)(ms + i), y = *(const f32x4*)(m + i), z = *(const f32x4*)(v + i);
      *(f32x4*)(m + i) = x + 1.f;
      *(f32x4*)(v + i) = y + 1.f;
      *(f32x4*)(ms + i) = z + 1.f;
      *(u32x2*)(p + i) = g;
    }
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1557611200ll;  // GPT2-1.5B, 64-aligned pieces
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t nn = (n + 511) / 512 * 512;
  bf16_t *p, *g; float *ms, *m, *v; unsigned char* mask;
  CK(hipMalloc(&p, nn * 2)); CK(hipMalloc(&g, nn * 2));
  CK(hipMalloc(&ms, nn * 4)); CK(hipMalloc(&m, nn * 4)); CK(hipMalloc(&v, nn * 4));
  CK(hipMalloc(&mask, nn / 64));
  CK(hipMemset(p, 0x3f, nn * 2)); CK(hipMemset(g, 0x3c, nn * 2));
  CK(hipMemset(ms, 0, nn * 4)); CK(hipMemset(m, 0, nn * 4)); CK(hipMemset(v, 0, nn * 4));
  CK(hipMemset(mask, 1, nn / 64));
  A a = {1e-4f, 0.9f, 0.95f, 1e-8f, 0.1f, 0.1f, 0.05f, nn, mask};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int grids[] = {1024, 2048, 4096, 8192};
  const int variants[] = {0, 1, 2, 3, 4, 9};
  for (int vi = 0; vi < 6; ++vi) {
    for (int gi = 0; gi < 4; ++gi) {
      const int var = variants[vi], grid = grids[gi];
      auto launch = [&]() {
        switch (var) {
          case 0: hipLaunchKernelGGL((k_v0<0>), dim3(grid), dim3(256), 0, 0, p, ms, g, m, v, a); break;
          case 1: hipLaunchKernelGGL((k_v1<0, 1>), dim3(grid), dim3(256), 0, 0, p, ms, g, m, v, a); break;
          case 2: hipLaunchKernelGGL((k_v1<1, 1>), dim3(grid), dim3(256), 0, 0, p, ms, g, m, v, a); break;
          case 3: hipLaunchKernelGGL((k_v0<1>), dim3(grid), dim3(256), 0, 0, p, ms, g, m, v, a); break;
          case 4: hipLaunchKernelGGL((k_v1<0, 2>), dim3(grid), dim3(256), 0, 0, p, ms, g, m, v, a); break;
          default: hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, p, ms, g, m, v, a); break;
        }
      };
      launch(); launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms_t = 0;
      CK(hipEventElapsedTime(&ms_t, e0, e1));
      const double t = ms_t / reps;
      printf("{\"variant\": %d, \"grid\": %d, \"ms\": %.3f, \"TBps\": %.2f}\n", var, grid, t, 28.0 * nn / (t * 1e-3) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
