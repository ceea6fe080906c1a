// Split-KV decode attention over a static KV cache (gfx950, bf16 in/out).
//
// q [B, H, D] (one new token per sequence), k/v cache [B, Smax, Hkv, D] with
// arbitrary batch / row strides, lens [B] int32 ON THE DEVICE (keys 0..len-1
// are valid), out [B, H, D].  D in {64, 128}; GQA group G = H / Hkv.
//
// Decode is HBM-bound: every cached K/V byte is read exactly once per step.
//  * pass 1: grid (split, head group, b * Hkv); a 4-wave block owns a
//    `chunk`-key slice of one KV head and up to 8 of its query heads.  D/8
//    lanes cover one key row with 16-byte loads, so a wave streams 64/(D/8)
//    keys per step; the q.k partial dots reduce over those lanes with xor
//    shuffles, each lane group keeps an online softmax (m, l) and its 8-wide
//    slice of the output per head; lane groups, then waves (through LDS),
//    merge their states and the block writes (m, l, o) partials (fp32);
//  * pass 2: per (b, h) merge the splits' partials -> out.
// Lengths come from device memory and the grid depends only on Smax, so a
// decode step is capturable in a HIP graph and replayed as the cache grows.
#include "dw_common.h"

namespace {

constexpr int DEC_WAVES = 4;
constexpr int DEC_GMAX = 8;  // query heads per block

template <int D>
struct DecCfg {
  static constexpr int LPK = D / 8;        // lanes per key row
  static constexpr int KPW = 64 / LPK;     // keys a wave handles per step
};

template <int D>
__global__ void __launch_bounds__(64 * DEC_WAVES) attn_decode_split_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const int* __restrict__ lens, float* __restrict__ part_o, float* __restrict__ part_ml, int H, int HKV,
    int nsplit, int chunk, float scale_log2, long long q_bs, long long k_bs, long long k_rs, long long v_bs,
    long long v_rs) {
  using C = DecCfg<D>;
  __shared__ float sm_ml[DEC_WAVES][DEC_GMAX][2];
  __shared__ float sm_o[DEC_WAVES][DEC_GMAX][D];

  const int split = blockIdx.x, hg = blockIdx.y;
  const int b = blockIdx.z / HKV, hk = blockIdx.z % HKV;
  const int G = H / HKV;
  const int g0 = hg * DEC_GMAX;
  const int ng = min(DEC_GMAX, G - g0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = lane / C::LPK, sl = lane % C::LPK;  // key slot in the wave, 8-wide d slice
  const int len = lens[b];
  const int k_lo = split * chunk, k_hi = min(len, k_lo + chunk);

  float qv[DEC_GMAX][8];
#pragma unroll
  for (int g = 0; g < DEC_GMAX; ++g) {
    if (g < ng) {
      const u32x4 w = *(const u32x4*)(Q + (long long)b * q_bs + (long long)(hk * G + g0 + g) * D + 8 * sl);
      unpack8(w, qv[g]);
#pragma unroll
      for (int i = 0; i < 8; ++i) qv[g][i] *= scale_log2;  // scores in log2 units
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) qv[g][i] = 0.f;
    }
  }
  float m[DEC_GMAX], l[DEC_GMAX], acc[DEC_GMAX][8];
#pragma unroll
  for (int g = 0; g < DEC_GMAX; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[g][i] = 0.f;
  }

  const bf16_t* Kb = K + (long long)b * k_bs + (long long)hk * D + 8 * sl;
  const bf16_t* Vb = V + (long long)b * v_bs + (long long)hk * D + 8 * sl;
  // U keys per lane group per step, all their loads issued before any math
  // (8 x 16 B in flight per lane instead of 2)
  constexpr int U = 4;
  constexpr int STEP = DEC_WAVES * C::KPW;
  for (int key0 = k_lo + wid * C::KPW + grp; key0 < k_hi; key0 += U * STEP) {
    u32x4 kw[U], vw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int key = key0 + u * STEP;
      if (key < k_hi) {
        kw[u] = *(const u32x4*)(Kb + (long long)key * k_rs);
        vw[u] = *(const u32x4*)(Vb + (long long)key * v_rs);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (key0 + u * STEP >= k_hi) break;  // uniform within the lane group
      float kf[8], vf[8];
      unpack8(kw[u], kf);
      unpack8(vw[u], vf);
#pragma unroll
      for (int g = 0; g < DEC_GMAX; ++g) {
        if (g >= ng) break;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = __builtin_fmaf(qv[g][i], kf[i], s);
#pragma unroll
        for (int off = C::LPK / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        const float mn = fmaxf(m[g], s);
        const float alpha = __builtin_amdgcn_exp2f(m[g] - mn);  // m = -inf -> 0
        const float p = __builtin_amdgcn_exp2f(s - mn);
        l[g] = l[g] * alpha + p;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[g][i] = __builtin_fmaf(p, vf[i], acc[g][i] * alpha);
        m[g] = mn;
      }
    }
  }

  // merge the KPW key slots of this wave (lanes sl, sl + LPK, ...)
#pragma unroll
  for (int g = 0; g < DEC_GMAX; ++g) {
    if (g >= ng) break;
#pragma unroll
    for (int off = C::LPK; off < 64; off <<= 1) {
      const float mo = __shfl_xor(m[g], off, 64), lo = __shfl_xor(l[g], off, 64);
      const float mn = fmaxf(m[g], mo);
      const float a = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m[g] - mn);
      const float c = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mo - mn);
      l[g] = l[g] * a + lo * c;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float ao = __shfl_xor(acc[g][i], off, 64);
        acc[g][i] = acc[g][i] * a + ao * c;
      }
      m[g] = mn;
    }
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) sm_o[wid][g][8 * sl + i] = acc[g][i];
      if (sl == 0) {
        sm_ml[wid][g][0] = m[g];
        sm_ml[wid][g][1] = l[g];
      }
    }
  }
  __syncthreads();

  // merge the waves: thread t handles (head g, d) pairs
  const long long pbase = (((long long)b * H + hk * G + g0) * nsplit + split);
  for (int e = tid; e < ng * D; e += 64 * DEC_WAVES) {
    const int g = e / D, d = e % D;
    float mx = -INFINITY;
#pragma unroll
    for (int w = 0; w < DEC_WAVES; ++w) mx = fmaxf(mx, sm_ml[w][g][0]);
    float lt = 0.f, ot = 0.f;
#pragma unroll
    for (int w = 0; w < DEC_WAVES; ++w) {
      const float c = mx == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(sm_ml[w][g][0] - mx);
      lt += sm_ml[w][g][1] * c;
      ot += sm_o[w][g][d] * c;
    }
    const long long pi = pbase + (long long)g * nsplit;  // row (b, h, split)
    part_o[pi * D + d] = ot;
    if (d == 0) {
      part_ml[2 * pi] = mx;
      part_ml[2 * pi + 1] = lt;
    }
  }
}

// one wave per (b, h): lanes over d (D/64 values each)
template <int D>
__global__ void __launch_bounds__(64) attn_decode_merge_kernel(const float* __restrict__ part_o,
                                                               const float* __restrict__ part_ml,
                                                               bf16_t* __restrict__ O, int nsplit,
                                                               long long o_bs, int H) {
  const int bh = blockIdx.x, lane = threadIdx.x;
  const int b = bh / H, h = bh % H;
  const long long base = (long long)bh * nsplit;
  float mx = -INFINITY;
  for (int s = 0; s < nsplit; ++s) mx = fmaxf(mx, part_ml[2 * (base + s)]);
  constexpr int PER = D / 64;
  float o[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) o[i] = 0.f;
  float lt = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float ms = part_ml[2 * (base + s)];
    if (ms == -INFINITY) continue;
    const float c = __builtin_amdgcn_exp2f(ms - mx);
    lt += part_ml[2 * (base + s) + 1] * c;
#pragma unroll
    for (int i = 0; i < PER; ++i) o[i] += part_o[(base + s) * D + lane + 64 * i] * c;
  }
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  bf16_t* Ob = O + (long long)b * o_bs + (long long)h * D;
#pragma unroll
  for (int i = 0; i < PER; ++i) Ob[lane + 64 * i] = f2bf(o[i] * inv);
}

}  // namespace

// Workspace: part_o float [B*H*nsplit*D], part_ml float [B*H*nsplit*2].
// strides (elements): q_bs, k_bs, k_rs, v_bs, v_rs, o_bs.
extern "C" int dw_attn_decode(const void* q, const void* k, const void* v, const void* lens, void* out,
                              void* part_o, void* part_ml, int B, int H, int HKV, int D, int nsplit, int chunk,
                              const long long* strides, float softmax_scale, void* stream) {
  if (H % HKV != 0 || nsplit <= 0 || chunk <= 0) return (int)hipErrorInvalidValue;
  const float scale_log2 = softmax_scale * 1.4426950408889634f;
  const int G = H / HKV;
  dim3 grid((unsigned)nsplit, (unsigned)((G + DEC_GMAX - 1) / DEC_GMAX), (unsigned)(B * HKV));
  hipStream_t s = (hipStream_t)stream;
  const long long q_bs = strides[0], k_bs = strides[1], k_rs = strides[2], v_bs = strides[3], v_rs = strides[4],
                  o_bs = strides[5];
  if (D == 128) {
    hipLaunchKernelGGL(attn_decode_split_kernel<128>, grid, dim3(64 * DEC_WAVES), 0, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, (const int*)lens, (float*)part_o, (float*)part_ml, H,
                       HKV, nsplit, chunk, scale_log2, q_bs, k_bs, k_rs, v_bs, v_rs);
    hipLaunchKernelGGL(attn_decode_merge_kernel<128>, dim3(B * H), dim3(64), 0, s, (const float*)part_o,
                       (const float*)part_ml, (bf16_t*)out, nsplit, o_bs, H);
  } else if (D == 64) {
    hipLaunchKernelGGL(attn_decode_split_kernel<64>, grid, dim3(64 * DEC_WAVES), 0, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, (const int*)lens, (float*)part_o, (float*)part_ml, H,
                       HKV, nsplit, chunk, scale_log2, q_bs, k_bs, k_rs, v_bs, v_rs);
    hipLaunchKernelGGL(attn_decode_merge_kernel<64>, dim3(B * H), dim3(64), 0, s, (const float*)part_o,
                       (const float*)part_ml, (bf16_t*)out, nsplit, o_bs, H);
  } else {
    return (int)hipErrorInvalidValue;
  }
  DW_LAUNCH_RET;
}

DW_PRELOAD(attn_decode_merge_kernel<128>);
