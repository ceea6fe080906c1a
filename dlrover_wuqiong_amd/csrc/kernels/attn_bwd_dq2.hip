// Query-major dQ kernel for D = 128, one wave per SIMD.
//
// Same algorithm as attn_bwd_dq_kernel (attn_bwd.hip): per key tile,
// S^T = K Q^T and dP^T = V dO^T with the key on the MFMA row, dS^T =
// exp2(S') * (dP - delta) in registers, dQ^T += K^T dS^T with the packed dS^T
// accumulator as the B operand -- no atomics, dQ written once in bf16.
//
// What changes is the shape of the work per wave, for the CDNA4 register
// file: a workgroup is 4 waves (one per SIMD, the whole 512-entry register
// file each) and every wave owns 64 queries as two 32-query groups.  Each K /
// V fragment read from LDS then feeds two MFMAs (one per group), halving the
// LDS reads per MFMA of the 8-wave / 32-query form, and the two groups are
// independent MFMA chains the scheduler interleaves with the other group's
// exp / multiply / pack (MI355X_MICROARCH 'one wave per SIMD: single-issue
// instructions hidden per MFMA gap': up to 5 per 32x32x16 gap; this body has
// ~2.5).  In the 8-wave form the S / dP chains waited on LDS reads issued one
// MFMA ahead (the 256-VGPR cap left no room to prefetch) and the two waves of
// a SIMD, barrier-aligned, ran their softmax phases together.
//
// Workgroup = 256 queries of one (batch, head), as before (same grid size);
// K / V tiles of 64 keys double-buffered in the T10(a) LDS image (64 KB).
#include "attn_bwd_common.h"

#include <cstdlib>
#include <type_traits>

#ifndef DWAMD_DQ2_FENCE
#define DWAMD_DQ2_FENCE 1
#endif
#ifndef DWAMD_DQ2_RI
// row constants as loop-invariant MFMA C operands (attn_bwd_dq_kernel's RI):
// off -- at D = 128 its 64 extra registers crash the ROCm 7.2 register
// allocator; at D = 64 the allocator trades the saved fma / sub for as many
// AGPR copies (148 per tile).  1 on; 2 -delta only
#define DWAMD_DQ2_RI 0
#endif

#ifndef DWAMD_DQ2_AACC
// dQ accumulators in the accumulator (AGPR) file through inline-asm MFMAs:
// frees 128 arch VGPRs at D = 128 for the S / dP side.  hipcc pads nothing
// inside asm: the packed dS operand is fresh from v_cvt_pk (VALU -> MFMA
// operand: s_nop 1 in the string), and the accumulators are read only after
// an s_nop pad that covers the last MFMA's 8-pass latency.
#define DWAMD_DQ2_AACC 0
#endif

namespace {
__device__ __forceinline__ void mfma_acc_agpr(f32x16& acc, const u32x4& a, const u32x4& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int DD>
struct Dq2Cfg {
  static constexpr int D = DD;
  // one wave per SIMD (D = 64 at two per SIMD spills 112 registers)
  static constexpr int MINW = 1;
  static constexpr int WAVES = 4;
  static constexpr int G = 2;  // 32-query groups per wave
  static constexpr int BQ = 32 * G * WAVES;
  static constexpr int BK = 64;
  static constexpr int NCH = D / 8;
  static constexpr int KK = D / 16;
  static constexpr int DT = D / 32;
  static constexpr int TILE = BK * D * 2;
};
}  // namespace

template <int DD, bool CAUSAL>
__global__ void __launch_bounds__(64 * Dq2Cfg<DD>::WAVES, Dq2Cfg<DD>::MINW)
attn_bwd_dq2_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
                    const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                    bf16_t* __restrict__ dQ, int S, int H, int HKV, float scale, float scale_log2, AttnStrides st,
                    AttnVarlen vl) {
  using C = Dq2Cfg<DD>;
  constexpr int D = C::D, G = C::G;
  constexpr bool RI = DWAMD_DQ2_RI == 1;
  constexpr bool RID = DWAMD_DQ2_RI == 2;  // -delta only as dP's initial accumulator
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + C::BQ - 1) / C::BQ;
  const BlockXYZ bc = xcd_block(nqb, H);
  const int b = bc.z, h = bc.y;
  const int hk = h / (H / HKV);
  const int qblk = CAUSAL ? nqb - 1 - bc.x : bc.x;  // causal: heaviest blocks first
  const int q_blk0 = qblk * C::BQ;
  const SeqRange sr = seq_range(vl, b, h, H, S);
  if (q_blk0 >= sr.sq) return;
  const int SQ = sr.sq, SK = sr.sk, co = SK - SQ;
  const int q0 = q_blk0 + wid * 32 * G;  // the wave's first query
  const bf16_t* Qb = Q + (int64_t)b * st.q_bs + (int64_t)sr.q_off * st.q_rs + (int64_t)h * D;
  const bf16_t* dOb = dO + (int64_t)b * st.do_bs + (int64_t)sr.q_off * st.do_rs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * st.k_bs + (int64_t)sr.k_off * st.k_rs + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * st.v_bs + (int64_t)sr.k_off * st.v_rs + (int64_t)hk * D;

  // Q (prescaled into the exp2 domain when RI) and dO fragments: B operands,
  // lane holds query q0 + 32 g + r, d = 16 kk + 8 hh .. +7
  u32x4 qf[G][C::KK], dof[G][C::KK];
  float lse2[G], dl[G];
  f32x16 s_init[G], dp_init[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int q = q0 + 32 * g + r;
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk) {
      if (q < SQ) {
        qf[g][kk] = *(const u32x4*)(Qb + (int64_t)q * st.q_rs + 16 * kk + 8 * hh);
        if (RI) qf[g][kk] = scaled8(qf[g][kk], scale_log2);
        dof[g][kk] = *(const u32x4*)(dOb + (int64_t)q * st.do_rs + 16 * kk + 8 * hh);
      } else {
        qf[g][kk] = (u32x4){0, 0, 0, 0};
        dof[g][kk] = (u32x4){0, 0, 0, 0};
      }
    }
    const int64_t so = sr.lse_base + q;
    const float lse_v = q < SQ ? LSE[so] : -INFINITY;
    lse2[g] = lse_v > -INFINITY ? lse_v * 1.4426950408889634f : INFINITY;  // no visible key: p = 0
    dl[g] = q < SQ ? DELTA[so] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s_init[g][i] = -lse2[g];
      dp_init[g][i] = -dl[g];
    }
  }
  f32x16 acc[G][C::DT];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[g][dt][i] = 0.f;

  int n_tiles = (SK + C::BK - 1) / C::BK;
  if (CAUSAL) {
    const int last = min(SK - 1, min(SQ - 1, q_blk0 + C::BQ - 1) + co);
    n_tiles = last < 0 ? 0 : min(n_tiles, last / C::BK + 1);
  }

  // K / V tiles arrive by LDS-DMA (global_load_lds_dwordx4: no staging
  // registers, no ds_write): one instruction fills 1 KB of the image
  // lane-linearly, so each lane fetches the global 16 bytes that img_off
  // places at its LDS position (the swizzle moves to the source address).
  // A tile is 16 pieces per tensor, 4 per wave; ragged-end keys are clamped
  // to the last key (finite data; the mask zeroes their probabilities).
  auto issue_tile = [&](int t, int buf) {
    char* kl = smem + buf * 2 * C::TILE;
#pragma unroll
    for (int j = 0; j < C::TILE / 1024 / C::WAVES; ++j) {
      const int piece = wid + C::WAVES * j;
      const int o = 1024 * piece + 16 * lane;
      const int rem = o % (D * 16), sub = rem % 512;
      const int row = 8 * (o / (D * 16)) + sub / 64;
      const int ch = 4 * (rem / 512) + (((sub % 64) / 16) ^ ((row >> 2) & 3));
      const int key = min(t * C::BK + row, SK - 1);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(Kb + (int64_t)key * st.k_rs + ch * 8),
                                       (__attribute__((address_space(3))) void*)(kl + 1024 * piece), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(Vb + (int64_t)key * st.v_rs + ch * 8),
                                       (__attribute__((address_space(3))) void*)(kl + C::TILE + 1024 * piece), 16, 0, 0);
    }
  };
  if (n_tiles > 0) issue_tile(0, 0);
  __syncthreads();  // (waits for the DMA: vmcnt(0) before the barrier)
  const int rwl[2] = {row_lane<D>(lane, 0), row_lane<D>(lane, 1)};
  const int trl[2] = {tr_lane<D>(lane, 0), tr_lane<D>(lane, 1)};

  for (int t = 0; t < n_tiles; ++t) {
    const int k0 = t * C::BK;
    // the next tile into the other buffer (read by tile t - 1, which every
    // wave finished before the last barrier); it lands during this tile
    if (t + 1 < n_tiles) issue_tile(t + 1, (t + 1) & 1);
    const char* kl = smem + (t & 1) * 2 * C::TILE;
    const char* vlds = kl + C::TILE;
    if (!CAUSAL || k0 <= q0 + 32 * G - 1 + co) {  // wave-uniform: some query of the wave sees a key
      const bool need_mask = (k0 + C::BK > SK) || (CAUSAL && (k0 + C::BK - 1 > q0 + co));
      // instantiated with and without the mask: an interior tile is one basic
      // block over both subtiles and both groups
      auto tile = [&](auto mask_c) {
        constexpr bool MASK = decltype(mask_c)::value;
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
#if DWAMD_DQ2_FENCE
          __builtin_amdgcn_sched_barrier(0);  // no hoisting across subtiles (register pressure)
#endif
          f32x16 s[G], dp[G];
          if (!RI) {
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
              for (int i = 0; i < 16; ++i) {
                s[g][i] = 0.f;
                if (!RID) dp[g][i] = 0.f;
              }
          }
#pragma unroll
          for (int kk = 0; kk < C::KK; ++kk) {
            const u32x4 kf = *(const u32x4*)(kl + rwl[kk & 1] + row_const<D>(32 * sb, kk));
            const u32x4 vf = *(const u32x4*)(vlds + rwl[kk & 1] + row_const<D>(32 * sb, kk));
#pragma unroll
            for (int g = 0; g < G; ++g) {
              s[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(kf), as_bf(qf[g][kk]),
                                                             (RI && kk == 0) ? s_init[g] : s[g], 0, 0, 0);
              dp[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(vf), as_bf(dof[g][kk]),
                                                              ((RI || RID) && kk == 0) ? dp_init[g] : dp[g], 0, 0, 0);
            }
          }
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (MASK) {
              const int q = q0 + 32 * g + r;
              const int lim = CAUSAL ? min(SK, q + co + 1) : SK;  // keys < lim are visible to this lane's query
              const int rel = lim - k0 - 32 * sb - 4 * hh;
#pragma unroll
              for (int i = 0; i < 16; ++i) s[g][i] = ((i & 3) + 8 * (i >> 2)) < rel ? s[g][i] : -INFINITY;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              if (RI) {
                s[g][i] = __builtin_amdgcn_exp2f(s[g][i]) * dp[g][i];  // dS^T (scale in the epilogue)
              } else {
                const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[g][i], scale_log2, -lse2[g]));
                s[g][i] = p * (RID ? dp[g][i] : dp[g][i] - dl[g]);
              }
            }
          }
          // dQ^T += K^T dS^T: 2 k-steps of 16 keys, K^T by transposed reads
          // shared by both groups
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            u32x4 pf[G];
#pragma unroll
            for (int g = 0; g < G; ++g)
              pf[g] = (u32x4){pk2(s[g][8 * s2 + 0], s[g][8 * s2 + 1]), pk2(s[g][8 * s2 + 2], s[g][8 * s2 + 3]),
                              pk2(s[g][8 * s2 + 4], s[g][8 * s2 + 5]), pk2(s[g][8 * s2 + 6], s[g][8 * s2 + 7])};
#pragma unroll
            for (int dt = 0; dt < C::DT; ++dt) {
              const u32x4 kt = tr_frag<D>(kl, 32 * sb + 16 * s2, 32 * dt, trl);
#pragma unroll
              for (int g = 0; g < G; ++g)
                if constexpr (DWAMD_DQ2_AACC)
                  mfma_acc_agpr(acc[g][dt], kt, pf[g]);
                else
                  acc[g][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(kt), as_bf(pf[g]), acc[g][dt], 0, 0, 0);
            }
          }
        }
      };
      if (need_mask)
        tile(std::true_type{});
      else
        tile(std::false_type{});
    }
    __syncthreads();  // tile t + 1 landed (vmcnt(0)), buffer t & 1 free
  }
  if constexpr (DWAMD_DQ2_AACC) asm volatile("s_nop 15\n\ts_nop 3" ::: "memory");  // last MFMA's result lands
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int q = q0 + 32 * g + r;
    if (q < SQ) {
      bf16_t* dQq = dQ + (int64_t)b * st.dq_bs + (int64_t)h * D + (int64_t)(sr.q_off + q) * st.dq_rs;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint2 w;
          w.x = pk2(acc[g][dt][4 * j + 0] * scale, acc[g][dt][4 * j + 1] * scale);
          w.y = pk2(acc[g][dt][4 * j + 2] * scale, acc[g][dt][4 * j + 3] * scale);
          *(uint2*)(dQq + 32 * dt + 8 * j + 4 * hh) = w;
        }
    }
  }
}

template <int DD>
static void launch_dq2_d(const void* q, const void* k, const void* v, const void* dout, const void* lse,
                         const float* delta, void* dq, int B, int Sq, int H, int HKV, int causal, float softmax_scale,
                         float scale_log2, const AttnStrides& st, const AttnVarlen& vl, hipStream_t s) {
  using C = Dq2Cfg<DD>;
  dim3 grid((unsigned)((Sq + C::BQ - 1) / C::BQ * H * B));  // 1-D: xcd_block()
  if (causal)
    hipLaunchKernelGGL((attn_bwd_dq2_kernel<DD, true>), grid, dim3(64 * C::WAVES), 4 * C::TILE, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, (const float*)lse, delta, (bf16_t*)dq,
                       Sq, H, HKV, softmax_scale, scale_log2, st, vl);
  else
    hipLaunchKernelGGL((attn_bwd_dq2_kernel<DD, false>), grid, dim3(64 * C::WAVES), 4 * C::TILE, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, (const float*)lse, delta, (bf16_t*)dq,
                       Sq, H, HKV, softmax_scale, scale_log2, st, vl);
}

bool launch_dq2(const void* q, const void* k, const void* v, const void* dout, const void* lse, const float* delta,
                void* dq, int B, int Sq, int H, int HKV, int D, int causal, float softmax_scale, float scale_log2,
                const AttnStrides& st, const AttnVarlen& vl, hipStream_t s) {
  // DWAMD_ATTN_DQ2: unset / 0 = never (the 8-wave kernel); 1 = D 128; 2 = D
  // 64 and 128.  Opt-in: measured SLOWER than the 8-wave kernel -- GQA S=8192
  // backward 659 vs 715 TF/s, S=4096 569 vs 632, GPT2 shape (D=64) 315 vs 347
  // (profiles/r4/attn_dq2_ab.md): with one wave per SIMD the exp / multiply /
  // pack VALU (7.9 VALU per MFMA after the compiler's AGPR copies) is no
  // longer hidden behind a partner wave's MFMAs.
  static const int mode = [] {
    const char* e = std::getenv("DWAMD_ATTN_DQ2");
    return e ? std::atoi(e) : 0;
  }();
  if (mode == 0) return false;
  if (D == 128) {
    launch_dq2_d<128>(q, k, v, dout, lse, delta, dq, B, Sq, H, HKV, causal, softmax_scale, scale_log2, st, vl, s);
    return true;
  }
  if (D == 64 && mode == 2) {
    launch_dq2_d<64>(q, k, v, dout, lse, delta, dq, B, Sq, H, HKV, causal, softmax_scale, scale_log2, st, vl, s);
    return true;
  }
  return false;
}

DW_PRELOAD((attn_bwd_dq2_kernel<128, true>));
DW_PRELOAD((attn_bwd_dq2_kernel<128, false>));
DW_PRELOAD((attn_bwd_dq2_kernel<64, true>));
DW_PRELOAD((attn_bwd_dq2_kernel<64, false>));
