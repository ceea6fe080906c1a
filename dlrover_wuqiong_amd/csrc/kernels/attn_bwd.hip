// Flash attention backward for gfx950 (bf16 in/out, fp32 accumulate).
//
// Recompute P from Q, K and the forward's LSE; five MFMA products per tile
// (S = Q K^T, dP = dO V^T, dV^T += dO^T P, dK^T += Q^T dS, dQ += dS K).
//
// Structure (cdna_hip_programming.md App. B "Attention backward"):
//  * one block = 4 waves = 128 keys of one (batch, kv-head); each wave owns
//    32 keys and keeps dK^T, dV^T for them in registers while the block
//    sweeps every query head of the GQA group x 32-query slices, so dK/dV
//    need no cross-block sum (written once, bf16).
//  * KEY on the lane: S and dP accumulators (query in registers, key on the
//    lane) are directly the B operands of dV^T and dK^T (query order permuted
//    identically on both operands); dO^T and Q^T come from LDS with the
//    ds_read_b64_tr_b16 transpose read.  K/V fragments of the wave's keys
//    stay in registers for the whole sweep.
//  * only dS crosses LDS (once), for dQ = dS K; dQ partial tiles are summed
//    across key blocks with fp32 atomics into a workspace (atomic bytes per
//    FLOP sized per Guideline 12), converted to bf16 by a final pass.
//  * softmax scale folded into dS; causal slices fully below the diagonal
//    are skipped.
#include "dw_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int D>
__device__ __forceinline__ int swzb(int r, int c) {  // byte offset of chunk c of row r
  constexpr int NCH = D / 8;
  return (r * NCH + (c ^ (r & (NCH - 1)))) * 16;
}
// dS tile: [32 q][128 keys] bf16, rows of 256 B (16 chunks)
__device__ __forceinline__ int swz_ds(int r, int c) { return (r * 16 + (c ^ (r & 15))) * 16; }

__device__ __forceinline__ bf16x8_t as_bf(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }
__device__ __forceinline__ unsigned int pk2(float a, float b) {
  return (unsigned int)f2bf(a) | ((unsigned int)f2bf(b) << 16);
}
__device__ __forceinline__ u32x4 tr_pair(const char* base, int off0, int off1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(base + off0));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(base + off1));
  u32x4 v;
  v[0] = (unsigned short)a[0] | ((unsigned int)(unsigned short)a[1] << 16);
  v[1] = (unsigned short)a[2] | ((unsigned int)(unsigned short)a[3] << 16);
  v[2] = (unsigned short)b[0] | ((unsigned int)(unsigned short)b[1] << 16);
  v[3] = (unsigned short)b[2] | ((unsigned int)(unsigned short)b[3] << 16);
  return v;
}

// delta[b,h,q] = sum_d dO*O.  D/8 lanes per (b, s, h) row (16-byte loads),
// 64/(D/8) rows per wave; rows are (b, s, h) in BSHD order.
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_pre_kernel(const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                           float* __restrict__ delta, int B, int S, int H,
                                                           AttnStrides st) {
  constexpr int LPR = D / 8;            // lanes per row
  constexpr int RPW = 64 / LPR;         // rows per wave
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const int c = lane % LPR;
  const bool ok = row < (int64_t)B * S * H;
  float acc = 0.f;
  int h = 0, s = 0, b = 0;
  if (ok) {
    h = (int)(row % H);
    const int64_t bs = row / H;
    s = (int)(bs % S);
    b = (int)(bs / S);
    float a[8], d[8];
    unpack8(*(const u32x4*)(O + (int64_t)b * st.o_bs + (int64_t)s * st.o_rs + h * D + c * 8), a);
    unpack8(*(const u32x4*)(dO + (int64_t)b * st.do_bs + (int64_t)s * st.do_rs + h * D + c * 8), d);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += a[k] * d[k];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (ok && c == 0) delta[((int64_t)b * H + h) * S + s] = acc;
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, (D <= 64 ? 2 : 1))  // D=64: keep 2 waves/SIMD (<= 256 VGPR+AGPR)
attn_bwd_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
                const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                float* __restrict__ dQacc, bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int S, int H, int HKV,
                float scale, float scale_log2, AttnStrides st) {
  constexpr int KS = D / 32;   // k-steps over d
  constexpr int DT = D / 16;   // d tiles
  constexpr int NCH = D / 8;
  constexpr int BKB = 128;     // keys per block
  constexpr int QI = 32;       // queries per iteration
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* k_lds = smem;                              // [128][D]
  char* ds_lds = k_lds + BKB * D * 2;              // [32][128]
  char* qbuf = ds_lds + QI * BKB * 2;              // 2 x {Q [32][D], dO [32][D], lse_log2[32], delta[32]}
  constexpr int QBUF = 2 * QI * D * 2 + 2 * QI * 4;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int b = blockIdx.z, hk = blockIdx.y;
  // causal: the key blocks with the most queries (the first ones) go first
  const int kb0 = blockIdx.x * BKB;  // causal: the first key blocks (most queries) dispatch first
  const int kw0 = kb0 + 32 * wid;  // this wave's first key
  const int group = H / HKV;
  const int64_t q_acc_rs = (int64_t)H * D;  // fp32 dQ workspace is contiguous BSHD
  const bf16_t* Kb = K + (int64_t)b * st.k_bs + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * st.v_bs + (int64_t)hk * D;

  // K block -> LDS (for the dQ transpose reads); K,V fragments -> registers
  for (int v = tid; v < BKB * NCH; v += 256) {
    const int r = v / NCH, c = v % NCH;
    const int key = kb0 + r;
    u32x4 x = (u32x4){0, 0, 0, 0};
    if (key < S) x = *(const u32x4*)(Kb + (int64_t)key * st.k_rs + c * 8);
    *(u32x4*)(k_lds + swzb<D>(r, c)) = x;
  }
  u32x4 kf[2][KS], vf[2][KS];  // B operand frags: [key = li][d = 32kk + 8g..]
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = kw0 + 16 * kt + li;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      if (key < S) {
        kf[kt][kk] = *(const u32x4*)(Kb + (int64_t)key * st.k_rs + 32 * kk + 8 * g);
        vf[kt][kk] = *(const u32x4*)(Vb + (int64_t)key * st.v_rs + 32 * kk + 8 * g);
      } else {
        kf[kt][kk] = (u32x4){0, 0, 0, 0};
        vf[kt][kk] = (u32x4){0, 0, 0, 0};
      }
    }
  }
  f32x4 dk[DT][2], dv[DT][2];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      dk[dt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      dv[dt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }

  const int q_start = CAUSAL ? (kb0 / QI) * QI : 0;
  const int nq = (S - q_start + QI - 1) / QI;  // query slices per head
  const int n_it = group * nq;
  // Software pipeline over (head, query slice): the Q / dO rows, LSE and
  // delta of slice i+1 are loaded into registers while slice i computes and
  // written to the other LDS buffer after its dQ pass (T14 issue-early /
  // write-late): HBM latency stays off the critical path even at one wave
  // per SIMD.  Two barriers per slice.
  constexpr int LV = QI * NCH / 256;  // 16-byte vectors per thread per tensor
  u32x4 q_st[LV], do_st[LV];
  float lse_st = INFINITY, del_st = 0.f;
  auto issue_slice = [&](int it) {
    const int h = hk * group + it / nq;
    const int qb = q_start + (it % nq) * QI;
    const bf16_t* Qb = Q + (int64_t)b * st.q_bs + (int64_t)h * D;
    const bf16_t* dOb = dO + (int64_t)b * st.do_bs + (int64_t)h * D;
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int v = tid + 256 * i;
      const int r = v / NCH, c = v % NCH;
      const int q = qb + r;
      if (q < S) {
        q_st[i] = *(const u32x4*)(Qb + (int64_t)q * st.q_rs + c * 8);
        do_st[i] = *(const u32x4*)(dOb + (int64_t)q * st.do_rs + c * 8);
      } else {
        q_st[i] = (u32x4){0, 0, 0, 0};
        do_st[i] = (u32x4){0, 0, 0, 0};
      }
    }
    if (tid < QI) {
      const int q = qb + tid;
      const int64_t off = ((int64_t)b * H + h) * S + q;
      lse_st = q < S ? LSE[off] * 1.4426950408889634f : INFINITY;
      del_st = q < S ? DELTA[off] : 0.f;
    }
  };
  auto write_slice = [&](int buf) {
    char* ql = qbuf + buf * QBUF;
    char* dl = ql + QI * D * 2;
    float* stl = (float*)(dl + QI * D * 2);
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      const int v = tid + 256 * i;
      const int r = v / NCH, c = v % NCH;
      *(u32x4*)(ql + swzb<D>(r, c)) = q_st[i];
      *(u32x4*)(dl + swzb<D>(r, c)) = do_st[i];
    }
    if (tid < QI) {
      stl[tid] = lse_st;
      stl[QI + tid] = del_st;
    }
  };
  if (n_it > 0) {
    issue_slice(0);
    write_slice(0);
  }
  __syncthreads();  // K block + first slice visible
  for (int it = 0; it < n_it; ++it) {
    const int h = hk * group + it / nq;
    const int qb = q_start + (it % nq) * QI;
    float* dQb = dQacc + (int64_t)b * S * q_acc_rs + (int64_t)h * D;
    const char* q_lds = qbuf + (it & 1) * QBUF;
    const char* do_lds = q_lds + QI * D * 2;
    const float* stat_lds = (const float*)(do_lds + QI * D * 2);
    if (it + 1 < n_it) issue_slice(it + 1);
    {
      // S = Q K^T and dP = dO V^T : [qt][kt], lane holds [q = 4g + r][key = li]
      f32x4 s[2][2], dp[2][2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[qt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
          dp[qt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const u32x4 qa = *(const u32x4*)(q_lds + swzb<D>(16 * qt + li, 4 * kk + g));
          const u32x4 da = *(const u32x4*)(do_lds + swzb<D>(16 * qt + li, 4 * kk + g));
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(qa), as_bf(kf[kt][kk]), s[qt][kt], 0, 0, 0);
            dp[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(da), as_bf(vf[kt][kk]), dp[qt][kt], 0, 0, 0);
          }
        }
      }
      // P and dS (scaled) in place
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 16 * qt + 4 * g + r;
          const int q = qb + ql;
          const float lse2 = stat_lds[ql], dl = stat_lds[QI + ql];
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            const int key = kw0 + 16 * kt + li;
            float p = exp2f(s[qt][kt][r] * scale_log2 - lse2);
            if (key >= S || q >= S || (CAUSAL && key > q)) p = 0.f;
            s[qt][kt][r] = p;
            dp[qt][kt][r] = p * (dp[qt][kt][r] - dl) * scale;
          }
        }
      // dV^T += dO^T P ; dK^T += Q^T dS  (k = 32 queries, permuted order)
      {
        u32x4 pb[2], sb[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const f32x4 a = s[0][kt], c = s[1][kt];
          pb[kt] = (u32x4){pk2(a[0], a[1]), pk2(a[2], a[3]), pk2(c[0], c[1]), pk2(c[2], c[3])};
          const f32x4 e = dp[0][kt], f = dp[1][kt];
          sb[kt] = (u32x4){pk2(e[0], e[1]), pk2(e[2], e[3]), pk2(f[0], f[1]), pk2(f[2], f[3])};
        }
        const int qrow = li >> 2, p4 = li & 3;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int col = 16 * dt + 4 * p4;
          const int r0 = 4 * g + qrow, r1 = r0 + 16;
          const int o0 = swzb<D>(r0, col >> 3) + (col & 7) * 2;
          const int o1 = swzb<D>(r1, col >> 3) + (col & 7) * 2;
          const u32x4 doT = tr_pair(do_lds, o0, o1);
          const u32x4 qT = tr_pair(q_lds, o0, o1);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            dv[dt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(doT), as_bf(pb[kt]), dv[dt][kt], 0, 0, 0);
            dk[dt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(qT), as_bf(sb[kt]), dk[dt][kt], 0, 0, 0);
          }
        }
      }
      // dS -> LDS as [q][key_in_block] bf16
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ql = 16 * qt + 4 * g + r;
            const int kl = 32 * wid + 16 * kt + li;
            *(bf16_t*)(ds_lds + swz_ds(ql, kl >> 3) + (kl & 7) * 2) = f2bf(dp[qt][kt][r]);
          }
      __syncthreads();
      // dQ[q][d] = sum_key dS[q][key] K[key][d]; wave -> q tile (wid&1), d tiles (wid>>1)*DT/2..
      {
        const int qt = wid & 1;
        constexpr int DTW = DT / 2;
        const int dt0 = (wid >> 1) * DTW;
        f32x4 acc[DTW];
#pragma unroll
        for (int i = 0; i < DTW; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < BKB / 32; ++ks) {
          // A = dS[q = li][key = 32ks + perm]: keys 32ks + 4g + j (j<4), 32ks+16+4g+j-4
          // build from two 8-byte pieces of the row
          const int qr = 16 * qt + li;
          const int ka = 32 * ks + 4 * g, kb = ka + 16;
          const uint2 pa = *(const uint2*)(ds_lds + swz_ds(qr, ka >> 3) + (ka & 7) * 2);
          const uint2 pbv = *(const uint2*)(ds_lds + swz_ds(qr, kb >> 3) + (kb & 7) * 2);
          const u32x4 af = (u32x4){pa.x, pa.y, pbv.x, pbv.y};
          const int qrow = li >> 2, p4 = li & 3;
#pragma unroll
          for (int i = 0; i < DTW; ++i) {
            const int col = 16 * (dt0 + i) + 4 * p4;
            const int r0 = 32 * ks + 4 * g + qrow, r1 = r0 + 16;
            const u32x4 kT = tr_pair(k_lds, swzb<D>(r0, col >> 3) + (col & 7) * 2,
                                     swzb<D>(r1, col >> 3) + (col & 7) * 2);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(af), as_bf(kT), acc[i], 0, 0, 0);
          }
        }
        // C: [q = 4g + r][d = li]
#pragma unroll
        for (int i = 0; i < DTW; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = qb + 16 * qt + 4 * g + r;
            if (q < S) atomicAdd(dQb + (int64_t)q * q_acc_rs + 16 * (dt0 + i) + li, acc[i][r]);
          }
      }
    }
    // next slice -> the other buffer (last read in iteration it-1, which every
    // wave finished before the dS barrier above); dS / this buffer free after
    if (it + 1 < n_it) write_slice((it + 1) & 1);
    __syncthreads();
  }
  // write dK, dV: lane holds [d = 16dt + 4g + r][key = kw0 + 16kt + li]
  bf16_t* dKb = dK + (int64_t)b * st.dk_bs + (int64_t)hk * D;
  bf16_t* dVb = dV + (int64_t)b * st.dv_bs + (int64_t)hk * D;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = kw0 + 16 * kt + li;
    if (key >= S) continue;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      uint2 wk, wv;
      wk.x = pk2(dk[dt][kt][0], dk[dt][kt][1]);
      wk.y = pk2(dk[dt][kt][2], dk[dt][kt][3]);
      wv.x = pk2(dv[dt][kt][0], dv[dt][kt][1]);
      wv.y = pk2(dv[dt][kt][2], dv[dt][kt][3]);
      *(uint2*)(dKb + (int64_t)key * st.dk_rs + 16 * dt + 4 * g) = wk;
      *(uint2*)(dVb + (int64_t)key * st.dv_rs + 16 * dt + 4 * g) = wv;
    }
  }
}

// dQ workspace (contiguous fp32 BSHD) -> bf16 dq with its own batch/row strides
__global__ void dq_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t rows, int S, int HD,
                                  long long bs, long long rs) {
  const int per_row = HD / 8;
  const int64_t nv = rows * per_row;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / per_row;  // (b, s)
    const int c = (int)(i % per_row);
    const int64_t b = row / S, sq = row % S;
    const f32x4 a = *(const f32x4*)(x + i * 8), bb = *(const f32x4*)(x + i * 8 + 4);
    const float f[8] = {a[0], a[1], a[2], a[3], bb[0], bb[1], bb[2], bb[3]};
    *(u32x4*)(y + b * bs + sq * rs + c * 8) = pack8(f);
  }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  const int64_t nv = n >> 3;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 a = *(const f32x4*)(x + i * 8), b = *(const f32x4*)(x + i * 8 + 4);
    const float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    *(u32x4*)(y + i * 8) = pack8(f);
  }
}

// workspace: dq_acc fp32 [B,S,H,D] + delta fp32 [B,H,S]
extern "C" int64_t dw_attn_bwd_workspace(int B, int S, int H, int D) {
  return (int64_t)B * S * H * D * 4 + (int64_t)B * H * S * 4 + 256;
}

template <int D>
static size_t bwd_lds_bytes() {
  return 128 * D * 2 + 32 * 128 * 2 + 2 * (2 * 32 * D * 2 + 2 * 32 * 4);
}

template <int D>
static void launch_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const void* lse,
                       float* dq_acc, float* delta, void* dk, void* dv, int B, int S, int H, int HKV, int causal,
                       float softmax_scale, const AttnStrides& st, hipStream_t s) {
  const int64_t rows = (int64_t)B * S * H;
  constexpr int RPB = 4 * (64 / (D / 8));  // rows per 256-thread block
  hipLaunchKernelGGL(attn_bwd_pre_kernel<D>, dim3((unsigned)((rows + RPB - 1) / RPB)), dim3(256), 0, s,
                     (const bf16_t*)o, (const bf16_t*)dout, delta, B, S, H, st);
  const float scale_log2 = softmax_scale * 1.4426950408889634f;
  dim3 grid((S + 127) / 128, HKV, B);
  const size_t lds = bwd_lds_bytes<D>();
  if (causal)
    hipLaunchKernelGGL((attn_bwd_kernel<D, true>), grid, dim3(256), lds, s, (const bf16_t*)q, (const bf16_t*)k,
                       (const bf16_t*)v, (const bf16_t*)dout, (const float*)lse, delta, dq_acc, (bf16_t*)dk,
                       (bf16_t*)dv, S, H, HKV, softmax_scale, scale_log2, st);
  else
    hipLaunchKernelGGL((attn_bwd_kernel<D, false>), grid, dim3(256), lds, s, (const bf16_t*)q, (const bf16_t*)k,
                       (const bf16_t*)v, (const bf16_t*)dout, (const float*)lse, delta, dq_acc, (bf16_t*)dk,
                       (bf16_t*)dv, S, H, HKV, softmax_scale, scale_log2, st);
}

// strides: int64[16] = q, k, v, o, do, dq, dk, dv  x (batch, row) in elements
extern "C" int dw_attn_bwd_strided(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                   const void* lse, void* dq, void* dk, void* dv, void* workspace, int B, int S,
                                   int H, int HKV, int D, const long long* strides, int causal, float softmax_scale,
                                   int flags, void* stream) {
  if (H % HKV != 0 || (D != 64 && D != 128)) return (int)hipErrorInvalidValue;
  AttnStrides st;
  long long* f = &st.q_bs;
  for (int i = 0; i < 16; ++i) f[i] = strides[i];
  hipStream_t s = (hipStream_t)stream;
  float* dq_acc = (float*)workspace;
  float* delta = dq_acc + (int64_t)B * S * H * D;
  hipError_t e = hipMemsetAsync(dq_acc, 0, (size_t)B * S * H * D * 4, s);
  if (e != hipSuccess) return (int)e;
  if (D == 128) launch_bwd<128>(q, k, v, o, dout, lse, dq_acc, delta, dk, dv, B, S, H, HKV, causal, softmax_scale,
                                st, s);
  else launch_bwd<64>(q, k, v, o, dout, lse, dq_acc, delta, dk, dv, B, S, H, HKV, causal, softmax_scale, st, s);
  const int64_t rows = (int64_t)B * S;
  const int64_t nv = rows * H * D / 8;
  hipLaunchKernelGGL(dq_to_bf16_kernel, dim3(dw_grid_for(nv, 256, 4096)), dim3(256), 0, s, dq_acc, (bf16_t*)dq,
                     rows, S, H * D, st.dq_bs, st.dq_rs);
  DW_LAUNCH_RET;
}

extern "C" int dw_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                           const void* lse, void* dq, void* dk, void* dv, void* workspace, void* unused,
                           int B, int S, int H, int HKV, int D, int causal, float softmax_scale, int flags,
                           void* stream) {
  const long long qs = (long long)S * H * D, qr = (long long)H * D, ks = (long long)S * HKV * D,
                  kr = (long long)HKV * D;
  const long long st[16] = {qs, qr, ks, kr, ks, kr, qs, qr, qs, qr, qs, qr, ks, kr, ks, kr};
  return dw_attn_bwd_strided(q, k, v, o, dout, lse, dq, dk, dv, workspace, B, S, H, HKV, D, st, causal,
                             softmax_scale, flags, stream);
}
