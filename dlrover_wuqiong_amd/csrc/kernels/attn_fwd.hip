// Flash attention forward for gfx950 (bf16 in/out, fp32 accumulate).
//
// Layout: q [B, S, H, D], k/v [B, S, Hkv, D] (GQA: H % Hkv == 0), o like q,
// lse [B, H, S] fp32 (natural log), D in {64, 128}.
//
// CDNA4 design (cdna_hip_programming.md App. B "fused attention prefill"):
//  * Swapped product: S^T = K * Q^T with v_mfma_f32_16x16x32_bf16, so the
//    accumulator puts the QUERY on the lane (col = lane&15) and 4 keys in the
//    registers.  Row statistics (max / sum over keys) are then in-lane plus
//    two xor-shuffles across the 4 lane groups — no LDS round trip.
//  * O^T = V^T * P^T: the P^T accumulator registers ARE the B operand of the
//    second MFMA (k order permuted identically on both operands), V^T comes
//    from the row-major V tile via ds_read_b64_tr_b16 (hardware transpose
//    read, T10) — P never touches LDS.
//  * K tile read with ds_read_b128 from an XOR-swizzled image (T2) so the 16
//    lanes of a group (16 different key rows, same d chunk) hit 16 different
//    16-byte slots.
//  * Block = 4 waves x 32 queries = 128 queries of one (b, h); K/V tiles of
//    64 keys staged through LDS by all 256 threads (16-byte loads, register
//    staged so the global loads of tile t+1 are issued before the MFMAs of
//    tile t — T14 issue-early / write-late).
//  * exp2 with the softmax scale folded into log2(e); causal tiles above the
//    diagonal are skipped entirely.
#include "dw_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int D>
struct AttnCfg {
  static constexpr int BQ = 128;           // queries per block
  static constexpr int BK = 64;            // keys per tile
  static constexpr int NCH = D / 8;        // 16-byte chunks per row
  static constexpr int KSTEPS = D / 32;    // MFMA k-steps over head dim
  static constexpr int DT = D / 16;        // 16-wide d tiles of O^T
  static constexpr int TILE_BYTES = BK * D * 2;
  static constexpr int VEC_PER_THREAD = BK * NCH / 256;  // 16B vectors per thread per tile
};

// byte offset of 16-byte chunk `c` of row `r` in a swizzled [rows][D] tile
template <int D>
__device__ __forceinline__ int swz(int r, int c) {
  constexpr int NCH = D / 8;
  return (r * NCH + (c ^ (r & (NCH - 1)))) * 16;
}

__device__ __forceinline__ bf16x8_t as_bf16x8(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }

__device__ __forceinline__ unsigned int pack2(float a, float b) {
  return (unsigned int)f2bf(a) | ((unsigned int)f2bf(b) << 16);
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, (D <= 64 ? 2 : 1))
attn_fwd_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
                bf16_t* __restrict__ O, float* __restrict__ LSE, int S, int H, int HKV, float scale_log2,
                AttnStrides st) {
  using C = AttnCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* k_lds = smem;
  char* v_lds = smem + C::TILE_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  const int hk = h / (H / HKV);
  // causal: the longest (last) query blocks are dispatched first so the
  // short ones fill in the tail of the grid
  const int qblk = CAUSAL ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
  const int q_blk0 = qblk * C::BQ;
  const int q0 = q_blk0 + wid * 32;
  const int64_t q_rs = st.q_rs, k_rs = st.k_rs, v_rs = st.v_rs;
  const bf16_t* Qb = Q + (int64_t)b * st.q_bs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * st.k_bs + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * st.v_bs + (int64_t)hk * D;

  // ---- Q fragments (B operand): lane holds Q[q0+16qt+li][32kk + 8g .. +7]
  u32x4 qf[2][C::KSTEPS];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
#pragma unroll
    for (int kk = 0; kk < C::KSTEPS; ++kk) {
      if (q < S) qf[qt][kk] = *(const u32x4*)(Qb + (int64_t)q * q_rs + 32 * kk + 8 * g);
      else qf[qt][kk] = (u32x4){0, 0, 0, 0};
    }
  }

  f32x4 o[C::DT][2];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) o[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m_i[2] = {-INFINITY, -INFINITY}, l_i[2] = {0.f, 0.f};

  int n_tiles = (S + C::BK - 1) / C::BK;
  if (CAUSAL) {
    const int last_q = min(S - 1, q_blk0 + C::BQ - 1);
    n_tiles = min(n_tiles, last_q / C::BK + 1);
  }

  // register staging of the next K/V tile (T14)
  u32x4 kst[C::VEC_PER_THREAD], vst[C::VEC_PER_THREAD];
  auto issue_load = [&](int t) {
#pragma unroll
    for (int i = 0; i < C::VEC_PER_THREAD; ++i) {
      const int v = tid + 256 * i;
      const int r = v / C::NCH, c = v % C::NCH;
      const int key = t * C::BK + r;
      if (key < S) {
        kst[i] = *(const u32x4*)(Kb + (int64_t)key * k_rs + c * 8);
        vst[i] = *(const u32x4*)(Vb + (int64_t)key * v_rs + c * 8);
      } else {
        kst[i] = (u32x4){0, 0, 0, 0};
        vst[i] = (u32x4){0, 0, 0, 0};
      }
    }
  };
  auto write_lds = [&]() {
#pragma unroll
    for (int i = 0; i < C::VEC_PER_THREAD; ++i) {
      const int v = tid + 256 * i;
      const int r = v / C::NCH, c = v % C::NCH;
      *(u32x4*)(k_lds + swz<D>(r, c)) = kst[i];
      *(u32x4*)(v_lds + swz<D>(r, c)) = vst[i];
    }
  };

  issue_load(0);
  for (int t = 0; t < n_tiles; ++t) {
    __syncthreads();  // previous tile fully consumed
    write_lds();
    __syncthreads();
    if (t + 1 < n_tiles) issue_load(t + 1);  // in flight during this tile's math
    const int k0 = t * C::BK;

    // ---- S^T = K Q^T : acc[i][qt], key tile i (16 keys), query tile qt
    f32x4 s[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[i][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < C::KSTEPS; ++kk) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u32x4 kf = *(const u32x4*)(k_lds + swz<D>(16 * i + li, 4 * kk + g));
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          s[i][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(kf), as_bf16x8(qf[qt][kk]), s[i][qt], 0, 0, 0);
      }
    }

    // ---- online softmax (query on the lane)
    const bool need_mask = (k0 + C::BK > S) || (CAUSAL && (k0 + C::BK - 1 > q0));
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = q0 + 16 * qt + li;
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = s[i][qt][r] * scale_log2;
          if (need_mask) {
            const int key = k0 + 16 * i + 4 * g + r;
            if (key >= S || (CAUSAL && key > q)) x = -INFINITY;
          }
          s[i][qt][r] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_i[qt], mx);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = exp2f(m_i[qt] - m_use);
      float rs = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[i][qt][r] - m_use);
          s[i][qt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      l_i[qt] = l_i[qt] * alpha + rs;
      m_i[qt] = m_new;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dt][qt][r] *= alpha;
    }

    // ---- O^T += V^T P^T   (2 k-steps of 32 keys)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 pf[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const f32x4 a = s[2 * ks][qt], c2 = s[2 * ks + 1][qt];
        pf[qt] = (u32x4){pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(c2[0], c2[1]), pack2(c2[2], c2[3])};
      }
      const int qrow = li >> 2, p = li & 3;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        const int col = 16 * dt + 4 * p;  // element column
        const int r0 = 32 * ks + 4 * g + qrow, r1 = r0 + 16;
        const int off0 = swz<D>(r0, col >> 3) + (col & 7) * 2;
        const int off1 = swz<D>(r1, col >> 3) + (col & 7) * 2;
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(v_lds + off0));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(v_lds + off1));
        u32x4 vf;
        vf[0] = (unsigned short)v0[0] | ((unsigned int)(unsigned short)v0[1] << 16);
        vf[1] = (unsigned short)v0[2] | ((unsigned int)(unsigned short)v0[3] << 16);
        vf[2] = (unsigned short)v1[0] | ((unsigned int)(unsigned short)v1[1] << 16);
        vf[3] = (unsigned short)v1[2] | ((unsigned int)(unsigned short)v1[3] << 16);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(vf), as_bf16x8(pf[qt]), o[dt][qt], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: O = O^T / l ; lse
  bf16_t* Ob = O + (int64_t)b * st.o_bs + (int64_t)h * D;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + 16 * qt + li;
    if (q >= S) continue;
    const float inv = l_i[qt] > 0.f ? 1.f / l_i[qt] : 0.f;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const f32x4 a = o[dt][qt];
      uint2 w;
      w.x = pack2(a[0] * inv, a[1] * inv);
      w.y = pack2(a[2] * inv, a[3] * inv);
      *(uint2*)(Ob + (int64_t)q * st.o_rs + 16 * dt + 4 * g) = w;
    }
    if (g == 0 && LSE) {
      const float lse = (l_i[qt] > 0.f) ? (m_i[qt] + log2f(l_i[qt])) * 0.6931471805599453f : -INFINITY;
      LSE[((int64_t)b * H + h) * S + q] = lse;
    }
  }
}

template <int D>
static void launch_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S, int H, int HKV,
                       int causal, float scale_log2, const AttnStrides& st, hipStream_t s) {
  dim3 grid((S + AttnCfg<D>::BQ - 1) / AttnCfg<D>::BQ, H, B), block(256);
  const int lds = 2 * AttnCfg<D>::TILE_BYTES;
  if (causal)
    hipLaunchKernelGGL((attn_fwd_kernel<D, true>), grid, block, lds, s, (const bf16_t*)q, (const bf16_t*)k,
                       (const bf16_t*)v, (bf16_t*)o, (float*)lse, S, H, HKV, scale_log2, st);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<D, false>), grid, block, lds, s, (const bf16_t*)q, (const bf16_t*)k,
                       (const bf16_t*)v, (bf16_t*)o, (float*)lse, S, H, HKV, scale_log2, st);
}

// strides: int64[8] = q_bs, q_rs, k_bs, k_rs, v_bs, v_rs, o_bs, o_rs (elements)
extern "C" int dw_attn_fwd_strided(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S,
                                   int H, int HKV, int D, const long long* strides, int causal, float softmax_scale,
                                   int flags, void* stream) {
  if (H % HKV != 0) return (int)hipErrorInvalidValue;
  AttnStrides st = {};
  st.q_bs = strides[0]; st.q_rs = strides[1]; st.k_bs = strides[2]; st.k_rs = strides[3];
  st.v_bs = strides[4]; st.v_rs = strides[5]; st.o_bs = strides[6]; st.o_rs = strides[7];
  const float scale_log2 = softmax_scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  if (D == 128) launch_fwd<128>(q, k, v, o, lse, B, S, H, HKV, causal, scale_log2, st, s);
  else if (D == 64) launch_fwd<64>(q, k, v, o, lse, B, S, H, HKV, causal, scale_log2, st, s);
  else return (int)hipErrorInvalidValue;
  DW_LAUNCH_RET;
}

extern "C" int dw_attn_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S,
                           int H, int HKV, int D, int causal, float softmax_scale, int flags, void* stream) {
  const long long st[8] = {(long long)S * H * D, (long long)H * D, (long long)S * HKV * D, (long long)HKV * D,
                           (long long)S * HKV * D, (long long)HKV * D, (long long)S * H * D, (long long)H * D};
  return dw_attn_fwd_strided(q, k, v, o, lse, B, S, H, HKV, D, st, causal, softmax_scale, flags, stream);
}
