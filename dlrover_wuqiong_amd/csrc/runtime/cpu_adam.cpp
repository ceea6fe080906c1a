// Host-side AdamW for optimizer-state offload (ZeRO-Offload style).
//
// The fp32 master weights and both Adam moments live in pinned host memory;
// the GPU keeps bf16 parameters and gradients.  Per chunk, the Python driver
// (optimizers/offload.py) streams bf16 gradients D2H on one HIP stream, this
// kernel updates the chunk on all host cores, and the rounded bf16 weights go
// back H2D on a second stream -- PCIe/xGMI-to-host traffic in both directions
// overlaps the CPU math.  The update is split over std::threads; the inner
// loop is compiled for AVX2+FMA when the host supports it (every EPYC host of
// an MI355X node does) and falls back to portable scalar code otherwise.
//
// Parity: ATorch atorch/optimizers/adam_offload.py (PartitionAdam swaps
// optimizer state between CPU and GPU); DeepSpeed-style CPU Adam semantics.

#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

namespace {

inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f32_to_bf16(float f) {  // round to nearest even, NaN preserved
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct AdamArgs {
  float* p;
  const void* g;
  int g_bf16;
  float* m;
  float* v;
  uint16_t* p_out;  // optional bf16 copy of the updated weights
  float lr, b1, b2, eps, wd, bc1, bc2, gscale;
};

void adam_scalar(const AdamArgs& a, uint64_t lo, uint64_t hi) {
  const float step = a.lr / a.bc1;
  const float inv_sqrt_bc2 = 1.0f / std::sqrt(a.bc2);
  const float decay = 1.0f - a.lr * a.wd;
  for (uint64_t i = lo; i < hi; ++i) {
    float g = a.g_bf16 ? bf16_to_f32(((const uint16_t*)a.g)[i]) : ((const float*)a.g)[i];
    g *= a.gscale;
    float m = a.b1 * a.m[i] + (1.0f - a.b1) * g;
    float v = a.b2 * a.v[i] + (1.0f - a.b2) * g * g;
    a.m[i] = m;
    a.v[i] = v;
    float p = a.p[i] * decay - step * m / (std::sqrt(v) * inv_sqrt_bc2 + a.eps);
    a.p[i] = p;
    if (a.p_out) a.p_out[i] = f32_to_bf16(p);
  }
}

__attribute__((target("avx2,fma"))) void adam_avx2(const AdamArgs& a, uint64_t lo, uint64_t hi) {
  const __m256 b1 = _mm256_set1_ps(a.b1), nb1 = _mm256_set1_ps(1.0f - a.b1);
  const __m256 b2 = _mm256_set1_ps(a.b2), nb2 = _mm256_set1_ps(1.0f - a.b2);
  const __m256 gs = _mm256_set1_ps(a.gscale);
  const __m256 step = _mm256_set1_ps(a.lr / a.bc1);
  const __m256 isb = _mm256_set1_ps(1.0f / std::sqrt(a.bc2));
  const __m256 eps = _mm256_set1_ps(a.eps);
  const __m256 decay = _mm256_set1_ps(1.0f - a.lr * a.wd);
  const __m256i rnd = _mm256_set1_epi32(0x7fff), one = _mm256_set1_epi32(1);
  uint64_t i = lo;
  for (; i + 8 <= hi; i += 8) {
    __m256 g;
    if (a.g_bf16) {
      __m128i h = _mm_loadu_si128((const __m128i*)((const uint16_t*)a.g + i));
      g = _mm256_castsi256_ps(_mm256_slli_epi32(_mm256_cvtepu16_epi32(h), 16));
    } else {
      g = _mm256_loadu_ps((const float*)a.g + i);
    }
    g = _mm256_mul_ps(g, gs);
    __m256 m = _mm256_fmadd_ps(b1, _mm256_loadu_ps(a.m + i), _mm256_mul_ps(nb1, g));
    __m256 v = _mm256_fmadd_ps(b2, _mm256_loadu_ps(a.v + i), _mm256_mul_ps(nb2, _mm256_mul_ps(g, g)));
    _mm256_storeu_ps(a.m + i, m);
    _mm256_storeu_ps(a.v + i, v);
    __m256 den = _mm256_fmadd_ps(_mm256_sqrt_ps(v), isb, eps);
    __m256 p = _mm256_fnmadd_ps(step, _mm256_div_ps(m, den), _mm256_mul_ps(_mm256_loadu_ps(a.p + i), decay));
    _mm256_storeu_ps(a.p + i, p);
    if (a.p_out) {
      // round-to-nearest-even bf16 (finite weights; NaN handled by the scalar tail rules only)
      __m256i u = _mm256_castps_si256(p);
      __m256i lsb = _mm256_and_si256(_mm256_srli_epi32(u, 16), one);
      u = _mm256_srli_epi32(_mm256_add_epi32(u, _mm256_add_epi32(rnd, lsb)), 16);
      __m128i lo16 = _mm256_castsi256_si128(u), hi16 = _mm256_extracti128_si256(u, 1);
      _mm_storeu_si128((__m128i*)(a.p_out + i), _mm_packus_epi32(lo16, hi16));
    }
  }
  adam_scalar(a, i, hi);
}

}  // namespace

extern "C" {

// Returns 0 on success.  n elements starting at the given pointers.
int dw_cpu_adamw(float* p, const void* g, int g_bf16, float* m, float* v, uint16_t* p_out, uint64_t n, float lr,
                 float b1, float b2, float eps, float wd, float bc1, float bc2, float gscale, int nthreads) {
  AdamArgs a{p, g, g_bf16, m, v, p_out, lr, b1, b2, eps, wd, bc1, bc2, gscale};
  static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  auto run = [&](uint64_t lo, uint64_t hi) {
    if (avx2)
      adam_avx2(a, lo, hi);
    else
      adam_scalar(a, lo, hi);
  };
  if (nthreads <= 1 || n < (1u << 16)) {
    run(0, n);
    return 0;
  }
  // 64-element aligned slices so every thread starts on a full vector
  uint64_t per = ((n + nthreads - 1) / nthreads + 63) & ~uint64_t(63);
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t lo = t * per, hi = std::min<uint64_t>(n, lo + per);
    if (lo >= hi) break;
    ts.emplace_back(run, lo, hi);
  }
  for (auto& t : ts) t.join();
  return 0;
}

// Sum of squares of a bf16/fp32 host vector (grad-norm clipping on host).
double dw_cpu_sumsq(const void* g, int g_bf16, uint64_t n) {
  double acc = 0.0;
  if (g_bf16) {
    const uint16_t* h = (const uint16_t*)g;
    for (uint64_t i = 0; i < n; ++i) {
      double x = bf16_to_f32(h[i]);
      acc += x * x;
    }
  } else {
    const float* f = (const float*)g;
    for (uint64_t i = 0; i < n; ++i) acc += (double)f[i] * f[i];
  }
  return acc;
}

}  // extern "C"
