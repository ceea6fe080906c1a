// Flash attention backward for gfx950 (bf16 in/out, fp32 accumulate).
//
// Recompute P from Q, K and the forward's LSE (per query row); with
// delta = rowsum(dO * O) and dS = P * (dP - delta):
//   dV = P^T dO,  dK = scale * dS^T Q,  dQ = scale * dS K.
//
// Split into two atomic-free kernels built on v_mfma_f32_32x32x16_bf16
// (cdna_hip_programming.md App. B "Attention backward"; why split: the fused
// form sums dQ across key blocks with float atomics, which at S = 4096 cost
// ~40 % of its time against the 1.3 TB/s chip-wide atomic rate):
//  * attn_bwd_dkdv_kernel -- key-major: each wave owns 32 keys ON THE MFMA
//    LANE; S = Q K^T and dP = dO V^T (K, V fragments of the wave's keys stay
//    in registers) put queries in the accumulator registers, so P and dS,
//    packed pairwise to bf16, ARE the B operands of dV^T += dO^T P and
//    dK^T += Q^T dS ("accumulator as the next MFMA's operand", guide §3);
//    dO^T / Q^T come from ds_read_b64_tr_b16 of the same LDS images the row
//    reads use (T10 (a)).  Q / dO / LSE / delta tiles of 64 queries are
//    register-staged one tile ahead into double-buffered LDS (T14), one
//    barrier per tile.  One query head per workgroup (grid.y = H): GQA
//    groups write fp32 partials that a tiny pass sums per kv head, so every
//    (b, head, key block) is an independent workgroup (fills 256 CUs even at
//    batch 1).
//  * attn_bwd_dq_kernel -- query-major twin of the forward kernel: dQ summed
//    in registers and written once in bf16.
// Softmax scale folded into the exponent FMA and applied to dK / dQ in the
// epilogues; causal tiles wholly above a wave's diagonal are skipped.
#include "attn_common.h"

#include <cstdlib>
#include <type_traits>

#ifndef DWAMD_DQ_RI
#define DWAMD_DQ_RI 1  // A/B: -DDWAMD_DQ_RI=0 builds the previous dQ form
#endif
#ifndef DWAMD_DKDV_W1
// A/B: dK/dV at D = 128 with one wave per SIMD, V fragments in registers and
// each S / dP chain's Q / dO fragments read ahead of its MFMAs (the 2-wave form
// waits on an LDS read before every MFMA)
#define DWAMD_DKDV_W1 0
#endif
#ifndef DWAMD_DKDV64_W3
// dK/dV at D = 64 capped at 168 VGPRs -- three workgroups (12 waves) per CU
// instead of two (the 2-workgroup form waits 47 % of its wave cycles, PMC):
// GPT2 shape backward 323 -> 334 TF/s packed, 354 -> 371 unpacked
// (profiles/r4/attn_dkdv64_w3_ab.jsonl).  -DDWAMD_DKDV64_W3=0: the 2-wave form
#define DWAMD_DKDV64_W3 1
#endif
#ifndef DWAMD_DKDV_DMA
// The D = 64 dK/dV kernel's Q / dO tiles by LDS-DMA (global_load_lds_dwordx4:
// each wave one 1-KiB 8-row group per tensor and chunk, the T10 swizzle folded
// into the per-lane source addresses) instead of register staging + ds_write:
// 168 VGPRs + 2 spills -> 155, GPT2-shape kernel 105.7 -> 101.0 us alone,
// backward 171-174 -> 169.5-170 us (profiles/r6/attn_dkdv64_dma_ab.jsonl); 0:
// register staging
#define DWAMD_DKDV_DMA 1
#endif
#ifndef DWAMD_DQ_DMA
#define DWAMD_DQ_DMA 1  // the D = 64 dQ kernel's K / V tiles by LDS-DMA (0: register staging)
#endif
#ifndef DWAMD_DKDV_VDMA
// the dK/dV kernel's block V image by LDS-DMA: GPT2 shape 101.4 -> 99.2 us,
// D = 128 neutral (profiles/r6/attn_dkdv_vdma_ab.jsonl)
#define DWAMD_DKDV_VDMA 1
#endif
#ifndef DWAMD_DMA128
// LDS-DMA staging in the D = 128 dK/dV and dQ kernels too: S=4096 GQA causal
// dK/dV 1320 -> 1226 us, dQ 1031 -> 996 us (profiles/r6/attn_dma128_ab.jsonl)
#define DWAMD_DMA128 1
#endif
#ifndef DWAMD_DKDV64_BQT
#define DWAMD_DKDV64_BQT 64  // A/B: queries per staged tile of the D = 64 dK/dV kernel (32 / 64 / 128)
#endif
#ifndef DWAMD_DQ_SPLIT
#define DWAMD_DQ_SPLIT 1  // A/B: 0 keeps the D=64 mask a runtime branch inside one tile body
#endif
#ifndef DWAMD_DQ_MINW
#define DWAMD_DQ_MINW 1  // A/B: minimum waves per SIMD the dQ kernel is compiled for (3: <= 168 VGPRs)
#endif
#ifndef DWAMD_DQ64_O3
// The D = 64 dQ kernel at three waves per SIMD -- one tile body with a
// runtime mask branch (no split), row constants subtracted after the MFMAs
// instead of held as 32 registers of accumulator init: 166 VGPRs, no spills
// (238 otherwise, two waves per SIMD).  GPT2 shape backward 366 -> 381 TF/s
// unpacked, 340 -> 350 packed (profiles/r5/attn_dq64_o3_ab.jsonl); 0: the
// split two-wave form
#define DWAMD_DQ64_O3 1
#endif

#ifndef DWAMD_DQ_AUG
// A/B: the dQ kernel's row constants as one extra MFMA k-step per chain:
// Q (prescaled by scale * log2 e) and dO get a 17th..18th "column" holding
// -lse2 resp. -delta split into bf16 hi + lo, K and V a matching column of
// ones, so S^T arrives as S * scale * log2 e - lse2 and dP^T as dP - delta:
// P = exp2(S'), dS = P * dP' -- one exp and one multiply per element and no
// per-subtile accumulator initialisation, for two more MFMAs per 32 keys
// (9.7 VALU per MFMA, MFMA busy 14 %).  Measured: 30 % fewer VALU in the
// tile body, no gain (GPT2 bwd 389 -> 382 TF/s, D=128 S=8k 737 -> 730;
// profiles/r5/attn_dq_aug_ab.jsonl): dQ runs beside dK/dV and waits on
// memory, so it stays off
#define DWAMD_DQ_AUG 0
#endif

#include "attn_bwd_common.h"

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


// ---------------------------------------------------------------------------
// Key-major dK / dV kernel.
template <int D>
struct DkvCfg {
  // 4 waves x 32 keys, 32-query tiles: a wave's dK^T + dV^T accumulators
  // are 128 registers at D = 128; with K fragments, S / dP and a 16-register
  // staging slot it still fits 256, so two workgroups (2 waves per SIMD,
  // ~65 KiB LDS each) share a CU
  static constexpr int WAVES = 4;
  static constexpr int BKB = 32 * WAVES;   // keys per workgroup
  static constexpr int BQT = D == 64 ? DWAMD_DKDV64_BQT : 32;  // queries per tile
  static constexpr int NCH = D / 8;
  static constexpr int KK = D / 16;
  static constexpr int DT = D / 32;
  static constexpr int TILE = BQT * D * 2;            // one [64][D] bf16 image
  static constexpr int BUF = 2 * TILE + 2 * BQT * 4;  // Q, dO, lse2[64], delta[64]
  static constexpr int VPT = BQT * NCH / (64 * WAVES);
  static constexpr int VIMG = BKB * D * 2;            // the block's V rows (LDS-resident)
};

template <int D, bool CAUSAL, bool PARTIAL, bool EXT>
__global__ void __launch_bounds__(64 * DkvCfg<D>::WAVES,
                                  (DWAMD_DKDV_W1 && D == 128 && !EXT) ? 1 : ((DWAMD_DKDV64_W3 && D == 64 && !EXT) ? 3 : 2))
attn_bwd_dkdv_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
                     const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                     bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, float* __restrict__ dKp,
                     float* __restrict__ dVp, int S, int H, int HKV, float scale, float scale_log2,
                     AttnStrides st, AttnVarlen vl, AttnExt ex) {
  using C = DkvCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar wave index
  const int r = lane & 31, hh = lane >> 5;
  const BlockXYZ bc = xcd_block((S + C::BKB - 1) / C::BKB, H);
  const int b = bc.z, h = bc.y;
  const int hk = h / (H / HKV);
  const int kb0 = bc.x * C::BKB;  // causal: low key blocks (most queries) dispatch first
  const SeqRange sr = seq_range(vl, b, h, H, S);  // S: the grid's (maximum) key length
  if (kb0 >= sr.sk) return;
  const int SQ = sr.sq, SK = sr.sk, co = SK - SQ;  // co: bottom-right causal offset
  const int kw0 = kb0 + 32 * wid;
  const int key = kw0 + r;
  const bf16_t* Qb = Q + (int64_t)b * st.q_bs + (int64_t)sr.q_off * st.q_rs + (int64_t)h * D;
  const bf16_t* dOb = dO + (int64_t)b * st.do_bs + (int64_t)sr.q_off * st.do_rs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * st.k_bs + (int64_t)sr.k_off * st.k_rs + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * st.v_bs + (int64_t)sr.k_off * st.v_rs + (int64_t)hk * D;
  const float* lse_b = LSE + sr.lse_base;
  const float* del_b = DELTA + sr.lse_base;

  // K fragments of this wave's keys stay in registers (B operand of S):
  // K[key][16 kk + 8 hh .. +7]; the block's V rows live in LDS (B operand of
  // dP, row-read per k-step) -- registers for 2 waves per SIMD.
  char* v_img = smem + 2 * C::BUF;
  // (VDMA: the V image by LDS-DMA too, drained by the prologue's vmcnt(0);
  // keys past the sequence read the last key -- only their own, unwritten,
  // dK / dV rows see it)
  constexpr bool VDMA = DWAMD_DKDV_VDMA && DWAMD_DKDV_DMA && (D == 64 || DWAMD_DMA128) && !EXT &&
                        !(DWAMD_DKDV_W1 && D == 128) && (C::VIMG / 1024) % C::WAVES == 0;
  if constexpr (VDMA) {
    constexpr int NGV = C::VIMG / 1024 / C::WAVES;
#pragma unroll
    for (int j = 0; j < NGV; ++j) {
      const int ci = NGV * wid + j;
      int row, ch;
      dma_rc<D>(ci, lane, row, ch);
      const int kv = min(kb0 + row, SK - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Vb + (int64_t)kv * st.v_rs + ch * 8),
                                       LDS_PTR(v_img + 1024 * ci), 16, 0, 0);
    }
  }
  for (int v = tid; v < (VDMA ? 0 : C::BKB * C::NCH); v += 64 * C::WAVES) {
    int row, c;
    stage_rc<D>(v, row, c);
    const int kv = kb0 + row;
    *(u32x4*)(v_img + img_off<D>(row, c)) =
        kv < SK ? *(const u32x4*)(Vb + (int64_t)kv * st.v_rs + c * 8) : (u32x4){0, 0, 0, 0};
  }
  // D=64: this wave's V fragments (16 VGPRs) live in registers too
  // D=64 V fragments in registers measured 10 % slower (bwd 334 -> 300 TF/s)
  constexpr bool W1 = DWAMD_DKDV_W1 && D == 128 && !EXT;
  constexpr bool VREG = W1;
  u32x4 vr[VREG ? C::KK : 1];
  // K (only used for S here) prescaled by softmax_scale * log2(e)
  u32x4 kf[C::KK];
#pragma unroll
  for (int kk = 0; kk < C::KK; ++kk)
    kf[kk] = key < SK ? scaled8(*(const u32x4*)(Kb + (int64_t)key * st.k_rs + 16 * kk + 8 * hh), scale_log2)
                      : (u32x4){0, 0, 0, 0};
  f32x16 dk[C::DT], dv[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      dk[dt][i] = 0.f;
      dv[dt][i] = 0.f;
    }

  // first query that sees key kb0: key <= q + co
  const int pre = EXT && ex.prefix ? min(SK, ex.prefix[b]) : 0;
  int q_lo = CAUSAL ? (max(0, kb0 - co) / C::BQT) * C::BQT : 0;
  int q_end = SQ;  // EXT: queries past the last window that reaches these keys see none of them
  if (EXT) {
    if (kb0 < pre) {
      q_lo = 0;  // prefix keys in the block: every query sees them
    } else {
      // query q sees key k iff -win_l <= k - (q + co) <= win_r
      if (ex.win_r >= 0) q_lo = (max(0, kb0 - co - ex.win_r) / C::BQT) * C::BQT;
      if (ex.win_l >= 0) q_end = max(0, min(SQ, kb0 + C::BKB - 1 - co + ex.win_l + 1));
    }
  }
  const int n_it = max(0, (q_end - q_lo + C::BQT - 1) / C::BQT);
  const long long bh = vl.cu_q ? (long long)h : (long long)b * H + h;  // dropout hash row
  const float al2 = EXT ? ext_alibi2(ex, b, h) : 0.f;
  constexpr bool DMA = DWAMD_DKDV_DMA && (D == 64 || DWAMD_DMA128) && !EXT && !W1 &&
                       (C::TILE / 1024) % C::WAVES == 0;
  constexpr int NG = C::TILE / 1024 / C::WAVES;  // 1 KiB DMA chunks per wave per tensor
  static_assert(!VDMA || DMA, "the V image's DMA is drained by the tile DMA's prologue wait");
  u32x4 q_st[DMA ? 1 : C::VPT], do_st[DMA ? 1 : C::VPT];
  float lse_st = -INFINITY, del_st = 0.f;  // the tile's LSE / delta (raw)
  // LDS-DMA of the tile's Q and dO images (attn_common.h dma_rc); rows past
  // the sequence read the last row (their LSE is -inf: p = 0, no contribution)
  auto dma = [&](int it, int buf) {
    const int q0 = q_lo + it * C::BQT;
    char* ql = smem + buf * C::BUF;
    char* dl = ql + C::TILE;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int ci = NG * wid + j;
      int row, ch;
      dma_rc<D>(ci, lane, row, ch);
      const int q = min(q0 + row, SQ - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Qb + (int64_t)q * st.q_rs + ch * 8), LDS_PTR(ql + 1024 * ci),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(dOb + (int64_t)q * st.do_rs + ch * 8), LDS_PTR(dl + 1024 * ci),
                                       16, 0, 0);
    }
  };
  auto issue = [&](int it) {
    const int q0 = q_lo + it * C::BQT;
#pragma unroll
    for (int i = 0; i < (DMA ? 0 : C::VPT); ++i) {
      const int v = tid + 64 * C::WAVES * i;
      int row, c;
      stage_rc<D>(v, row, c);
      const int q = q0 + row;
      if (q < SQ) {
        q_st[i] = *(const u32x4*)(Qb + (int64_t)q * st.q_rs + c * 8);
        do_st[i] = *(const u32x4*)(dOb + (int64_t)q * st.do_rs + c * 8);
      } else {
        q_st[i] = (u32x4){0, 0, 0, 0};
        do_st[i] = (u32x4){0, 0, 0, 0};
      }
    }
    if (tid < C::BQT) {
      // raw values: negated / scaled at write(), after the tile's compute --
      // arithmetic here waited on the load at once, with the tile barrier
      // right behind it
      const int q = q0 + tid;
      lse_st = q < SQ ? lse_b[q] : -INFINITY;
      del_st = q < SQ ? del_b[q] : 0.f;
    }
  };
  auto write = [&](int buf) {
    char* ql = smem + buf * C::BUF;
    char* dl = ql + C::TILE;
    float* stl = (float*)(dl + C::TILE);
#pragma unroll
    for (int i = 0; i < (DMA ? 0 : C::VPT); ++i) {
      const int v = tid + 64 * C::WAVES * i;
      int row, c;
      stage_rc<D>(v, row, c);
      *(u32x4*)(ql + img_off<D>(row, c)) = q_st[i];
      *(u32x4*)(dl + img_off<D>(row, c)) = do_st[i];
    }
    if (tid < C::BQT) {
      // row constants NEGATED: they are the initial accumulators of S' and dP';
      // a row that saw no key (lse = -inf) contributes nothing: p = 2^-inf
      stl[tid] = lse_st > -INFINITY ? -lse_st * 1.4426950408889634f : -INFINITY;
      stl[C::BQT + tid] = -del_st;
    }
  };
  if (n_it > 0) {
    if constexpr (DMA) dma(0, 0);
    issue(0);
    write(0);
    if (!DMA && n_it > 1) issue(1);
  }
  if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's DMA landed
  __syncthreads();
  if (DMA && n_it > 1) {
    dma(1, 1);
    issue(1);
  }
  // per-lane LDS read offsets; the rest of each address is an immediate
  const int rwl[2] = {row_lane<D>(lane, 0), row_lane<D>(lane, 1)};
  const int trl[2] = {tr_lane<D>(lane, 0), tr_lane<D>(lane, 1)};
  if constexpr (VREG) {
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk) vr[kk] = *(const u32x4*)(v_img + rwl[kk & 1] + row_const<D>(32 * wid, kk));
  }

  for (int it = 0; it < n_it; ++it) {
    const int q0 = q_lo + it * C::BQT;
    const char* ql = smem + (it & 1) * C::BUF;
    const char* dl = ql + C::TILE;
    const float* stl = (const float*)(dl + C::TILE);
    // all queries of this tile precede this wave's keys: nothing to add
    if (!CAUSAL || q0 + C::BQT - 1 + co >= kw0 || (EXT && kw0 < pre)) {
      const bool need_mask = EXT || (q0 + C::BQT > SQ) || (kw0 + 32 > SK) || (CAUSAL && kw0 + 31 > q0 + co);
#pragma unroll
      for (int qs = 0; qs < C::BQT / 32; ++qs) {
        // S = Q K^T, dP = dO V^T for 32 queries: key on the lane, query in the registers
        // row constants as the initial accumulators: S' = S*c - lse2, dP' = dP - delta
        f32x16 s, dp;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qi = 32 * qs + 8 * g + 4 * hh;
          const f32x4 l4 = *(const f32x4*)(stl + qi);
          const f32x4 d4 = *(const f32x4*)(stl + C::BQT + qi);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            s[4 * g + j] = l4[j];
            dp[4 * g + j] = d4[j];
          }
        }
        if constexpr (W1) {
          // every Q / dO fragment of the chain in flight before its MFMAs
          u32x4 qa[C::KK], da[C::KK];
#pragma unroll
          for (int kk = 0; kk < C::KK; ++kk) {
            qa[kk] = *(const u32x4*)(ql + rwl[kk & 1] + row_const<D>(32 * qs, kk));
            da[kk] = *(const u32x4*)(dl + rwl[kk & 1] + row_const<D>(32 * qs, kk));
          }
#pragma unroll
          for (int kk = 0; kk < C::KK; ++kk) {
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(qa[kk]), as_bf(kf[kk]), s, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(da[kk]), as_bf(vr[VREG ? kk : 0]), dp, 0, 0, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x100, 2 * C::KK, 0);  // the DS reads first
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * C::KK, 0);  // then the MFMAs
        } else {
#pragma unroll
          for (int kk = 0; kk < C::KK; ++kk) {
            const u32x4 qa = *(const u32x4*)(ql + rwl[kk & 1] + row_const<D>(32 * qs, kk));
            const u32x4 da = *(const u32x4*)(dl + rwl[kk & 1] + row_const<D>(32 * qs, kk));
            const u32x4 vb = VREG ? vr[VREG ? kk : 0]
                                  : *(const u32x4*)(v_img + rwl[kk & 1] + row_const<D>(32 * wid, kk));
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(qa), as_bf(kf[kk]), s, 0, 0, 0);
            dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(da), as_bf(vb), dp, 0, 0, 0);
          }
        }
        if (!EXT) {
          // P, then (diagonal / ragged tiles only) the mask, then dS: the
          // empty volatile asm keeps the mask a scalar branch (need_mask is
          // wave-uniform) instead of per-element selects or branches
          if (need_mask) {
            __asm__ volatile("");
            // register i holds query q0 + 4 hh + c, c = 32 qs + 8 (i >> 2) + (i & 3)
            const int base = q0 + 4 * hh;
            const int qlim = key < SK ? SQ - base : -1;  // c < qlim: a real query (and a real key)
            const int kmin = key - co - base;            // c >= kmin: causal, the key is visible
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int c = 32 * qs + 8 * (i >> 2) + (i & 3);
              const bool keep = (c < qlim) && (!CAUSAL || c >= kmin);
              s[i] = keep ? s[i] : -INFINITY;  // p = 2^-inf = 0
            }
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            s[i] = __builtin_amdgcn_exp2f(s[i]);
            dp[i] = s[i] * dp[i];  // dS (scale applied in the epilogue)
          }
        }
        // rows of register group g: queries 32 qs + 8 g + 4 hh + 0..3
#pragma unroll
        for (int g = 0; g < 4 && EXT; ++g) {
          const int qi = 32 * qs + 8 * g + 4 * hh;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * g + j;
            {
              const int q = q0 + qi + j;
              const bool vis = (q < SQ) && ext_visible(ex, CAUSAL, q, key, co, SK, pre);
              float add = (vis && ex.bias)
                  ? ex.bias[(int64_t)b * ex.bias_bs + (int64_t)h * ex.bias_hs + (int64_t)q * ex.bias_qs + key] *
                        1.4426950408889634f
                  : 0.f;
              add -= al2 * fabsf((float)(key - q - co));
              const float p = vis ? __builtin_amdgcn_exp2f(s[i] + add) : 0.f;
              if (ex.dropout) {
                // dV takes the dropped probabilities; dS = P (Z dP / (1-p) - delta)
                const float del = -stl[C::BQT + qi + j];
                const bool kp = attn_keep(ex, bh, (long long)sr.q_off + q, (long long)sr.k_off + key);
                s[i] = kp ? p * ex.inv_keep : 0.f;
                dp[i] = p * (kp ? (dp[i] + del) * ex.inv_keep - del : -del);
              } else {
                s[i] = p;
                dp[i] = p * dp[i];
              }
            }
          }
        }
        // dV^T += dO^T P ; dK^T += Q^T dS : 2 k-steps of 16 queries
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const u32x4 pf = {pk2(s[8 * s2 + 0], s[8 * s2 + 1]), pk2(s[8 * s2 + 2], s[8 * s2 + 3]),
                            pk2(s[8 * s2 + 4], s[8 * s2 + 5]), pk2(s[8 * s2 + 6], s[8 * s2 + 7])};
          const u32x4 sf = {pk2(dp[8 * s2 + 0], dp[8 * s2 + 1]), pk2(dp[8 * s2 + 2], dp[8 * s2 + 3]),
                            pk2(dp[8 * s2 + 4], dp[8 * s2 + 5]), pk2(dp[8 * s2 + 6], dp[8 * s2 + 7])};
#pragma unroll
          for (int dt = 0; dt < C::DT; ++dt) {
            const u32x4 doT = tr_frag<D>(dl, 32 * qs + 16 * s2, 32 * dt, trl);
            dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(doT), as_bf(pf), dv[dt], 0, 0, 0);
          }
#pragma unroll
          for (int dt = 0; dt < C::DT; ++dt) {
            const u32x4 qT = tr_frag<D>(ql, 32 * qs + 16 * s2, 32 * dt, trl);
            dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(qT), as_bf(sf), dk[dt], 0, 0, 0);
          }
        }
      }
    }
    if (it + 1 < n_it) {
      write((it + 1) & 1);  // buffer last read in iteration it-1
      if (!DMA && it + 2 < n_it) issue(it + 2);
    }
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile it+1's DMA landed
    __syncthreads();
    if (DMA && it + 2 < n_it) {  // buffer it & 1 is free: every wave is past this tile
      dma(it + 2, it & 1);
      issue(it + 2);
    }
  }
  if (key >= SK) return;
  // accumulator rows = d: register i of tile dt is d = 32 dt + 8 (i>>2) + 4 hh + (i&3)
  if (PARTIAL) {
    // partials [rows, H, D]: rows = B*S (dense) or total_k (packed)
    const int64_t prow = vl.cu_q ? (int64_t)sr.k_off + key : (int64_t)b * S + key;
    float* kp = dKp + (prow * H + h) * D;
    float* vp = dVp + (prow * H + h) * D;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * hh;
        *(f32x4*)(kp + d) = (f32x4){dk[dt][4 * g] * scale, dk[dt][4 * g + 1] * scale, dk[dt][4 * g + 2] * scale,
                                    dk[dt][4 * g + 3] * scale};
        *(f32x4*)(vp + d) = (f32x4){dv[dt][4 * g], dv[dt][4 * g + 1], dv[dt][4 * g + 2], dv[dt][4 * g + 3]};
      }
  } else {
    bf16_t* dKk = dK + (int64_t)b * st.dk_bs + (int64_t)hk * D + (int64_t)(sr.k_off + key) * st.dk_rs;
    bf16_t* dVk = dV + (int64_t)b * st.dv_bs + (int64_t)hk * D + (int64_t)(sr.k_off + key) * st.dv_rs;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * hh;
        uint2 wk, wv;
        wk.x = pk2(dk[dt][4 * g] * scale, dk[dt][4 * g + 1] * scale);
        wk.y = pk2(dk[dt][4 * g + 2] * scale, dk[dt][4 * g + 3] * scale);
        wv.x = pk2(dv[dt][4 * g], dv[dt][4 * g + 1]);
        wv.y = pk2(dv[dt][4 * g + 2], dv[dt][4 * g + 3]);
        *(uint2*)(dKk + d) = wk;
        *(uint2*)(dVk + d) = wv;
      }
  }
}

// GQA: dK[b, s, hk, :] = sum over the group's query heads of the fp32 partials
// (8 elements per thread; partial layout [B, S, H, D]).
template <int D>
__global__ void gqa_reduce_kernel(const float* __restrict__ pk, const float* __restrict__ pv, bf16_t* __restrict__ dK,
                                  bf16_t* __restrict__ dV, int64_t BS, int S, int H, int HKV, AttnStrides st) {
  const int group = H / HKV;
  const int64_t nv = BS * HKV * (D / 8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % (D / 8));
    const int64_t t = i / (D / 8);
    const int hk = (int)(t % HKV);
    const int64_t bs = t / HKV;
    const int64_t b = bs / S, sq = bs % S;
    float fk[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int g = 0; g < group; ++g) {
      const int64_t off = (bs * H + hk * group + g) * D + c * 8;
      const f32x4 a0 = *(const f32x4*)(pk + off), a1 = *(const f32x4*)(pk + off + 4);
      const f32x4 b0 = *(const f32x4*)(pv + off), b1 = *(const f32x4*)(pv + off + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fk[j] += a0[j];
        fk[4 + j] += a1[j];
        fv[j] += b0[j];
        fv[4 + j] += b1[j];
      }
    }
    *(u32x4*)(dK + b * st.dk_bs + sq * st.dk_rs + hk * D + c * 8) = pack8(fk);
    *(u32x4*)(dV + b * st.dv_bs + sq * st.dv_rs + hk * D + c * 8) = pack8(fv);
  }
}

// ---------------------------------------------------------------------------
// Query-major dQ kernel (split backward: no atomics).
//
// dQ = scale * sum_keys dS K with dS = P * (dP - delta), P = exp2(S*c - lse2).
// Same structure as the forward kernel: per wave 32 queries on the MFMA lane
// (swapped products S^T = K Q^T and dP^T = V dO^T with v_mfma_f32_32x32x16),
// K/V tiles of 64 keys double-buffered in the T10(a) LDS image, and
// dQ^T += K^T dS^T with the packed dS^T accumulator as the B operand and K^T
// from ds_read_b64_tr_b16.  Every dQ element is summed in registers by one
// wave and written once, in bf16, straight into the (possibly packed) dQ
// view: no fp32 workspace, no memset, no conversion pass -- the fused
// kernel's atomics (1.3 TB/s chip-wide, ~40 % of its time at S = 4096) are
// gone at the price of recomputing S and dP here.
template <int D>
struct DqCfg {
  // D=64: 4 waves (128 queries): twice the blocks of the 8-wave form, two per
  // CU -- the causal tail of a short sequence (GPT2: 4 query blocks of 256
  // per head) left the 8-wave form at 200 us vs 123 for the dK/dV kernel
  static constexpr int WAVES = D == 64 ? 4 : 8;
  static constexpr int BQ = 32 * WAVES;
  static constexpr int BK = 64;
  static constexpr int NCH = D / 8;
  static constexpr int KK = D / 16;
  static constexpr int DT = D / 32;
  static constexpr int TILE = BK * D * 2;
  static constexpr int VPT = BK * NCH / (64 * WAVES);
};

template <int D, bool CAUSAL, bool EXT>
__global__ void __launch_bounds__(64 * DqCfg<D>::WAVES, (D == 64 && !EXT) ? (DWAMD_DQ64_O3 ? 3 : DWAMD_DQ_MINW) : 1)
attn_bwd_dq_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
                   const bf16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                   bf16_t* __restrict__ dQ, int S, int H, int HKV, float scale, float scale_log2, AttnStrides st,
                   AttnVarlen vl, AttnExt ex) {
  using C = DqCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar wave index
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + C::BQ - 1) / C::BQ;
  const BlockXYZ bc = xcd_block(nqb, H);
  const int b = bc.z, h = bc.y;
  const int hk = h / (H / HKV);
  const int qblk = CAUSAL ? nqb - 1 - bc.x : bc.x;
  const int q_blk0 = qblk * C::BQ;
  const SeqRange sr = seq_range(vl, b, h, H, S);  // S: the grid's (maximum) query length
  if (q_blk0 >= sr.sq) return;
  const int SQ = sr.sq, SK = sr.sk, co = SK - SQ;
  const int q0 = q_blk0 + wid * 32;
  const int q = q0 + r;
  const bf16_t* Qb = Q + (int64_t)b * st.q_bs + (int64_t)sr.q_off * st.q_rs + (int64_t)h * D;
  const bf16_t* dOb = dO + (int64_t)b * st.do_bs + (int64_t)sr.q_off * st.do_rs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * st.k_bs + (int64_t)sr.k_off * st.k_rs + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * st.v_bs + (int64_t)sr.k_off * st.v_rs + (int64_t)hk * D;

  // Row constants as the accumulators' INITIAL VALUES (RI, dense masks):
  // Q is prescaled by softmax_scale * log2(e) so S^T leaves the MFMA in the
  // exp2 domain, and the first MFMA of each chain takes a loop-invariant C
  // operand holding -lse2 (resp. -delta) -- a lane's 16 registers all belong
  // to its query -- so P = exp2(S'), dS = P * dP' cost one exp and one mul
  // per element instead of fma + exp + sub + mul.
  constexpr bool AUG = DWAMD_DQ_AUG && !EXT;
  constexpr bool RI = DWAMD_DQ_RI && !EXT && !(D == 64 && DWAMD_DQ64_O3) && !AUG;
  // Q and dO fragments (B operands): lane holds row q, d = 16 kk + 8 hh .. +7
  u32x4 qf[C::KK], dof[C::KK];
#pragma unroll
  for (int kk = 0; kk < C::KK; ++kk) {
    if (q < SQ) {
      qf[kk] = *(const u32x4*)(Qb + (int64_t)q * st.q_rs + 16 * kk + 8 * hh);
      if (RI || AUG) qf[kk] = scaled8(qf[kk], scale_log2);
      dof[kk] = *(const u32x4*)(dOb + (int64_t)q * st.do_rs + 16 * kk + 8 * hh);
    } else {
      qf[kk] = (u32x4){0, 0, 0, 0};
      dof[kk] = (u32x4){0, 0, 0, 0};
    }
  }
  const int64_t so = sr.lse_base + q;
  const float lse_v = q < SQ ? LSE[so] : -INFINITY;
  const float lse2 = lse_v > -INFINITY ? lse_v * 1.4426950408889634f : INFINITY;  // no visible key: p = 0
  const float dl = q < SQ ? DELTA[so] : 0.f;

  f32x16 acc[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[dt][i] = 0.f;
  constexpr bool DPI = D == 64 && !EXT && !RI;  // dP^T initialised with -delta
  f32x16 s_init, dp_init;  // RI: the loop-invariant C operands
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    s_init[i] = -lse2;
    dp_init[i] = -dl;
  }
  // AUG: the augmented k-step's operands.  B side (this lane's query row,
  // k-index 8 hh .. +7): -lse2 and -delta as bf16 hi + lo in k-indices 0, 1;
  // A side (key rows): ones there.  No visible key (lse2 = inf): -inf + 0.
  u32x4 qaug = {0, 0, 0, 0}, doaug = {0, 0, 0, 0}, ones = {0, 0, 0, 0};
  if (AUG && hh == 0) {
    const float nl = -lse2, nd = -dl;
    const float nl_hi = bf2f(f2bf(nl)), nd_hi = bf2f(f2bf(nd));
    qaug[0] = pk2(nl_hi, nl > -INFINITY ? nl - nl_hi : 0.f);
    doaug[0] = pk2(nd_hi, nd - nd_hi);
    ones[0] = pk2(1.f, 1.f);
  }
  const f32x16 zero16 = {};

  int n_tiles = (SK + C::BK - 1) / C::BK;
  int t_begin = 0;
  const int pre = EXT && ex.prefix ? min(SK, ex.prefix[b]) : 0;
  if (CAUSAL || EXT) {
    const int q_last = min(SQ - 1, q_blk0 + C::BQ - 1);
    int last = SK - 1;
    if (CAUSAL) last = min(last, q_last + co);
    if (EXT && ex.win_r >= 0) last = min(last, q_last + co + ex.win_r);
    if (EXT && pre > 0) last = max(last, pre - 1);
    n_tiles = last < 0 ? 0 : min(n_tiles, last / C::BK + 1);
    if (EXT && ex.win_l >= 0 && pre == 0) t_begin = min(n_tiles, max(0, q_blk0 + co - ex.win_l) / C::BK);
  }
  const int n_run = n_tiles - t_begin;
  const long long bh = vl.cu_q ? (long long)h : (long long)b * H + h;
  const float al2 = EXT ? ext_alibi2(ex, b, h) : 0.f;
  const float* brow = nullptr;
  if (EXT && ex.bias && q < SQ)
    brow = ex.bias + (int64_t)b * ex.bias_bs + (int64_t)h * ex.bias_hs + (int64_t)q * ex.bias_qs;

  // (D = 64: K / V tiles by LDS-DMA, as the dK/dV kernel's Q / dO; keys past
  // the sequence read the last key -- masked, p = 0)
  constexpr bool DMA = DWAMD_DQ_DMA && (D == 64 || DWAMD_DMA128) && !EXT && (C::TILE / 1024) % C::WAVES == 0;
  constexpr int NG = C::TILE / 1024 / C::WAVES;  // 1 KiB DMA chunks per wave per tensor
  u32x4 kst[DMA ? 1 : C::VPT], vst[DMA ? 1 : C::VPT];
  auto dma = [&](int t, int buf) {
    char* kl = smem + buf * 2 * C::TILE;
    char* vl = kl + C::TILE;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int ci = NG * wid + j;
      int row, ch;
      dma_rc<D>(ci, lane, row, ch);
      const int key = min(t * C::BK + row, SK - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Kb + (int64_t)key * st.k_rs + ch * 8), LDS_PTR(kl + 1024 * ci),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(Vb + (int64_t)key * st.v_rs + ch * 8), LDS_PTR(vl + 1024 * ci),
                                       16, 0, 0);
    }
  };
  auto issue_load = [&](int t) {
#pragma unroll
    for (int i = 0; i < (DMA ? 0 : C::VPT); ++i) {
      const int v = tid + 64 * C::WAVES * i;
      int row, c;
      stage_rc<D>(v, row, c);
      const int key = t * C::BK + row;
      if (key < SK) {
        kst[i] = *(const u32x4*)(Kb + (int64_t)key * st.k_rs + c * 8);
        vst[i] = *(const u32x4*)(Vb + (int64_t)key * st.v_rs + c * 8);
      } else {
        kst[i] = (u32x4){0, 0, 0, 0};
        vst[i] = (u32x4){0, 0, 0, 0};
      }
    }
  };
  auto write_lds = [&](int buf) {
    char* kl = smem + buf * 2 * C::TILE;
    char* vl = kl + C::TILE;
#pragma unroll
    for (int i = 0; i < (DMA ? 0 : C::VPT); ++i) {
      const int v = tid + 64 * C::WAVES * i;
      int row, c;
      stage_rc<D>(v, row, c);
      *(u32x4*)(kl + img_off<D>(row, c)) = kst[i];
      *(u32x4*)(vl + img_off<D>(row, c)) = vst[i];
    }
  };
  if constexpr (DMA) {
    if (n_run > 0) dma(t_begin, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    issue_load(t_begin);
    write_lds(0);
    if (n_run > 1) issue_load(t_begin + 1);
  }
  __syncthreads();
  if (DMA && n_run > 1) dma(t_begin + 1, 1);
  const int rwl[2] = {row_lane<D>(lane, 0), row_lane<D>(lane, 1)};
  const int trl[2] = {tr_lane<D>(lane, 0), tr_lane<D>(lane, 1)};

  for (int tt = 0; tt < n_run; ++tt) {
    const int t = t_begin + tt;
    const int k0 = t * C::BK;
    const char* kl = smem + (tt & 1) * 2 * C::TILE;
    const char* vl = kl + C::TILE;
    bool active = !CAUSAL || k0 <= q0 + 31 + co;
    if (EXT) {
      if (k0 < pre) active = true;
      if (ex.win_r >= 0) active = active && (k0 <= q0 + 31 + co + ex.win_r);
      if (ex.win_l >= 0 && k0 >= pre) active = active && (k0 + C::BK - 1 >= q0 + co - ex.win_l);
    }
    if (active) {
      const bool need_mask = (k0 + C::BK > SK) || (CAUSAL && (k0 + C::BK - 1 > q0 + co));
      const int lim = CAUSAL ? min(SK, q + co + 1) : SK;  // keys < lim are visible to this lane's query
      // The tile body is instantiated twice -- with and without the mask --
      // so an interior tile (most of them) is ONE basic block over both
      // subtiles and the scheduler can overlap subtile 1's S / dP MFMAs with
      // subtile 0's softmax (a runtime mask branch split them).
      // (D=64 only: at D=128 the overlap needs ~200 more VGPRs than the 256 of
      // two waves per SIMD and spills; there the mask stays a runtime branch.)
      constexpr bool SPLIT = DWAMD_DQ_SPLIT && D == 64 && !DWAMD_DQ64_O3;
      auto tile = [&](auto mask_c) {
        constexpr bool MASK = decltype(mask_c)::value;
      // one 32-key subtile at a time keeps S^T / dP^T at 32 registers
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        // dP^T starts at -delta (row constant as the initial accumulator) at
        // D=64; at D=128 that form cost this kernel 40+ spilled VGPRs
        f32x16 s, dp;
        if (AUG) {
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(ones), as_bf(qaug), zero16, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(ones), as_bf(doaug), zero16, 0, 0, 0);
        } else if (!RI) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            s[i] = 0.f;
            dp[i] = DPI ? -dl : 0.f;
          }
        }
#pragma unroll
        for (int kk = 0; kk < C::KK; ++kk) {
          const u32x4 kf = *(const u32x4*)(kl + rwl[kk & 1] + row_const<D>(32 * sb, kk));
          const u32x4 vf = *(const u32x4*)(vl + rwl[kk & 1] + row_const<D>(32 * sb, kk));
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(kf), as_bf(qf[kk]), (RI && kk == 0) ? s_init : s, 0,
                                                      0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(vf), as_bf(dof[kk]), (RI && kk == 0) ? dp_init : dp,
                                                       0, 0, 0);
        }
        if (!EXT) {
          if (MASK || (!SPLIT && need_mask)) {  // diagonal / ragged tiles only
            if (!SPLIT) __asm__ volatile("");  // keep the runtime test a scalar branch
            const int rel = lim - k0 - 32 * sb - 4 * hh;  // register i's key offset must be < rel
#pragma unroll
            for (int i = 0; i < 16; ++i) s[i] = ((i & 3) + 8 * (i >> 2)) < rel ? s[i] : -INFINITY;  // p = 0
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            if (RI || AUG) {
              s[i] = __builtin_amdgcn_exp2f(s[i]) * dp[i];  // dS^T (scale applied in the epilogue)
            } else {
              const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[i], scale_log2, -lse2));
              s[i] = p * (DPI ? dp[i] : dp[i] - dl);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 16 && EXT; ++i) {
          {
            const int key = k0 + 32 * sb + (i & 3) + 8 * (i >> 2) + 4 * hh;
            const bool vis = (q < SQ) && ext_visible(ex, CAUSAL, q, key, co, SK, pre);
            float add = (vis && brow) ? brow[key] * 1.4426950408889634f : 0.f;
            add -= al2 * fabsf((float)(key - q - co));
            const float p = vis ? __builtin_amdgcn_exp2f(__builtin_fmaf(s[i], scale_log2, add - lse2)) : 0.f;
            float dpe = dp[i];
            if (ex.dropout)
              dpe = attn_keep(ex, bh, (long long)sr.q_off + q, (long long)sr.k_off + key) ? dpe * ex.inv_keep : 0.f;
            s[i] = p * (dpe - dl);
          }
        }
        // dQ^T += K^T dS^T : 2 k-steps of 16 keys, K^T from transposed reads
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const u32x4 pf = {pk2(s[8 * s2 + 0], s[8 * s2 + 1]), pk2(s[8 * s2 + 2], s[8 * s2 + 3]),
                            pk2(s[8 * s2 + 4], s[8 * s2 + 5]), pk2(s[8 * s2 + 6], s[8 * s2 + 7])};
#pragma unroll
          for (int dt = 0; dt < C::DT; ++dt) {
            const u32x4 kt = tr_frag<D>(kl, 32 * sb + 16 * s2, 32 * dt, trl);
            acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(kt), as_bf(pf), acc[dt], 0, 0, 0);
          }
        }
      }
      };
      if (SPLIT && (need_mask || EXT))
        tile(std::true_type{});
      else
        tile(std::false_type{});
    }
    if (!DMA && tt + 1 < n_run) {
      write_lds((tt + 1) & 1);
      if (tt + 2 < n_run) issue_load(t + 2);
    }
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile tt+1 landed
    __syncthreads();
    if (DMA && tt + 2 < n_run) dma(t + 2, tt & 1);  // buffer tt & 1 is free
  }
  if (q < SQ) {
    bf16_t* dQq = dQ + (int64_t)b * st.dq_bs + (int64_t)h * D + (int64_t)(sr.q_off + q) * st.dq_rs;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 w;
        w.x = pk2(acc[dt][4 * g + 0] * scale, acc[dt][4 * g + 1] * scale);
        w.y = pk2(acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale);
        *(uint2*)(dQq + 32 * dt + 8 * g + 4 * hh) = w;
      }
  }
}

// workspace: delta fp32 [B, H, S] (+ GQA fp32 partials 2 x [B, S, H, D])
extern "C" int64_t dw_attn_bwd_workspace(int B, int S, int H, int D) {
  return (int64_t)B * H * S * 4 + 2 * (int64_t)B * S * H * D * 4 + 512;
}

// dQ runs on a second stream concurrently with dK/dV (both only read q, k,
// v, dO, lse and delta): each kernel alone leaves the CUs half occupied
// (8 waves / CU) and has a causal tail; together they fill each other's
// gaps.  Fork / join through events, so it is also capturable in a graph.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

static SideStream* side_stream() {
  static thread_local SideStream per_dev[16];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 16) return nullptr;
  SideStream& ss = per_dev[d];
  if (!ss.s) {
    if (hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ss.join, hipEventDisableTiming) != hipSuccess)
      return nullptr;
  }
  return &ss;
}

static bool bwd_concurrent() {
  static const bool on = [] {
    const char* v = getenv("DWAMD_ATTN_BWD_CONCURRENT");
    return !(v && v[0] == '0');
  }();
  return on;
}

template <int D>
static void launch_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const void* lse,
                       char* ws, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int H, int HKV, int causal,
                       float softmax_scale, const AttnStrides& st, const AttnVarlen& vl, hipStream_t s,
                       const AttnExt* ext = nullptr) {
  const AttnExt none = {};
  const AttnExt& ex = ext ? *ext : none;
  // workspace layout (dw_attn_bwd_workspace with S = max(Sq, Sk)): delta, then
  // the GQA partials; packed batches use [H, total_q] / [total_k, H, D] inside
  const int Smax = Sq > Sk ? Sq : Sk;
  float* delta = (float*)ws;
  // delta rows: (b, s, h) of the dense tensor, or (row, h) of the packed one
  const int pre_b = vl.cu_q ? 1 : B, pre_s = vl.cu_q ? vl.total_q : Sq;
  const int64_t rows = (int64_t)pre_b * pre_s * H;
  constexpr int RPB = 4 * (64 / (D / 8));  // rows per 256-thread block
  hipLaunchKernelGGL(attn_bwd_pre_kernel<D>, dim3((unsigned)((rows + RPB - 1) / RPB)), dim3(256), 0, s,
                     (const bf16_t*)o, (const bf16_t*)dout, delta, pre_b, pre_s, H, st);
  const float scale_log2 = softmax_scale * 1.4426950408889634f;
  SideStream* side = bwd_concurrent() ? side_stream() : nullptr;
  hipStream_t sq = s;
  if (side && hipEventRecord(side->fork, s) == hipSuccess && hipStreamWaitEvent(side->s, side->fork, 0) == hipSuccess)
    sq = side->s;
  // key-major dK / dV
  using KC = DkvCfg<D>;
  const bool partial = H != HKV;
  float* pk = (float*)(ws + (((int64_t)B * H * Smax * 4 + 255) / 256) * 256);
  float* pv = pk + (int64_t)B * Smax * H * D;
  dim3 gk((unsigned)((Sk + KC::BKB - 1) / KC::BKB * H * B));  // 1-D: xcd_block()
  const int lk = 2 * KC::BUF + KC::VIMG;
#define DKDV(CA, PA, EX)                                                                                      \
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, CA, PA, EX>), gk, dim3(64 * KC::WAVES), lk, s, (const bf16_t*)q, \
                     (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, (const float*)lse, delta,        \
                     (bf16_t*)dk, (bf16_t*)dv, pk, pv, Sk, H, HKV, softmax_scale, scale_log2, st, vl, ex)
  if (ext) {
    if (causal) {
      if (partial) DKDV(true, true, true); else DKDV(true, false, true);
    } else {
      if (partial) DKDV(false, true, true); else DKDV(false, false, true);
    }
  } else if (causal) {
    if (partial) DKDV(true, true, false); else DKDV(true, false, false);
  } else {
    if (partial) DKDV(false, true, false); else DKDV(false, false, false);
  }
#undef DKDV
  if (partial) {
    // partial rows: B*Sk (dense) or total_k (packed, one "batch")
    const int64_t prow = vl.cu_q ? (int64_t)vl.total_k : (int64_t)B * Sk;
    const int pS = vl.cu_q ? vl.total_k : Sk;
    const int64_t nv = prow * HKV * (D / 8);
    hipLaunchKernelGGL(gqa_reduce_kernel<D>, dim3(dw_grid_for(nv, 256, 4096)), dim3(256), 0, s, pk, pv,
                       (bf16_t*)dk, (bf16_t*)dv, prow, pS, H, HKV, st);
  }
  // query-major dQ (on the side stream when concurrent)
  using DC = DqCfg<D>;
  dim3 gq((unsigned)((Sq + DC::BQ - 1) / DC::BQ * H * B));  // 1-D: xcd_block()
  const int lq = 4 * DC::TILE;
#define DQ(CA, EX)                                                                                            \
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, CA, EX>), gq, dim3(64 * DC::WAVES), lq, sq, (const bf16_t*)q,      \
                     (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, (const float*)lse, delta,        \
                     (bf16_t*)dq, Sq, H, HKV, softmax_scale, scale_log2, st, vl, ex)
  bool dq_done = false;
  if (!ext)  // dense masks: the 4-wave, 64-queries-per-wave form (attn_bwd_dq2.hip)
    dq_done = launch_dq2(q, k, v, dout, lse, delta, dq, B, Sq, H, HKV, D, causal, softmax_scale, scale_log2, st, vl,
                         sq);
  if (dq_done) {
  } else if (ext) {
    if (causal) DQ(true, true); else DQ(false, true);
  } else if (causal) {
    DQ(true, false);
  } else {
    DQ(false, false);
  }
#undef DQ
  if (sq != s) {  // join: the caller's stream continues after both
    hipEventRecord(side->join, sq);
    hipStreamWaitEvent(s, side->join, 0);
  }
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
  char* ws = (char*)workspace;
  const AttnVarlen vl = {nullptr, nullptr, 0, 0};
  if (D == 128)
    launch_bwd<128>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, S, S, H, HKV, causal, softmax_scale, st, vl, s);
  else
    launch_bwd<64>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, S, S, H, HKV, causal, softmax_scale, st, vl, s);
  DW_LAUNCH_RET;
}

// Packed variable-length batch (see dw_attn_fwd_varlen).  row_strides
// int64[8] = q, k, v, o, do, dq, dk, dv row strides (elements).  Workspace:
// dw_attn_bwd_workspace(B, max(max_seqlen_q, max_seqlen_k), H, D).
extern "C" int dw_attn_bwd_varlen(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                  const void* lse, void* dq, void* dk, void* dv, void* workspace, const void* cu_q,
                                  const void* cu_k, int B, int max_seqlen_q, int max_seqlen_k, int total_q,
                                  int total_k, int H, int HKV, int D, const long long* row_strides, int causal,
                                  float softmax_scale, void* stream) {
  if (H % HKV != 0 || (D != 64 && D != 128) || !cu_q || !cu_k) return (int)hipErrorInvalidValue;
  AttnStrides st = {};
  st.q_rs = row_strides[0]; st.k_rs = row_strides[1]; st.v_rs = row_strides[2]; st.o_rs = row_strides[3];
  st.do_rs = row_strides[4]; st.dq_rs = row_strides[5]; st.dk_rs = row_strides[6]; st.dv_rs = row_strides[7];
  const AttnVarlen vl = {(const int*)cu_q, (const int*)cu_k, total_q, total_k};
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  if (D == 128)
    launch_bwd<128>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, max_seqlen_q, max_seqlen_k, H, HKV, causal,
                    softmax_scale, st, vl, s);
  else
    launch_bwd<64>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, max_seqlen_q, max_seqlen_k, H, HKV, causal,
                   softmax_scale, st, vl, s);
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

// Extended masks (attn_common.h AttnExtArgs); dense layout as dw_attn_bwd_strided.
extern "C" int dw_attn_bwd_ext(const void* q, const void* k, const void* v, const void* o, const void* dout,
                               const void* lse, void* dq, void* dk, void* dv, void* workspace, int B, int S, int H,
                               int HKV, int D, const long long* strides, int causal, float softmax_scale,
                               const AttnExtArgs* args, void* stream) {
  if (H % HKV != 0 || (D != 64 && D != 128)) return (int)hipErrorInvalidValue;
  AttnStrides st;
  long long* f = &st.q_bs;
  for (int i = 0; i < 16; ++i) f[i] = strides[i];
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const AttnVarlen vl = {nullptr, nullptr, 0, 0};
  const AttnExt ex = make_ext(args, S, S);
  const AttnExt* ep = ext_active(args) ? &ex : nullptr;
  if (D == 128)
    launch_bwd<128>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, S, S, H, HKV, causal, softmax_scale, st, vl, s, ep);
  else
    launch_bwd<64>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, S, S, H, HKV, causal, softmax_scale, st, vl, s, ep);
  DW_LAUNCH_RET;
}

extern "C" int dw_attn_bwd_varlen_ext(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                      const void* lse, void* dq, void* dk, void* dv, void* workspace, const void* cu_q,
                                      const void* cu_k, int B, int max_seqlen_q, int max_seqlen_k, int total_q,
                                      int total_k, int H, int HKV, int D, const long long* row_strides, int causal,
                                      float softmax_scale, const AttnExtArgs* args, void* stream) {
  if (H % HKV != 0 || (D != 64 && D != 128) || !cu_q || !cu_k ||
      (args && (args->bias || args->prefix || (args->alibi && args->alibi_bs))))
    return (int)hipErrorInvalidValue;
  AttnStrides st = {};
  st.q_rs = row_strides[0]; st.k_rs = row_strides[1]; st.v_rs = row_strides[2]; st.o_rs = row_strides[3];
  st.do_rs = row_strides[4]; st.dq_rs = row_strides[5]; st.dk_rs = row_strides[6]; st.dv_rs = row_strides[7];
  const AttnVarlen vl = {(const int*)cu_q, (const int*)cu_k, total_q, total_k};
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const AttnExt ex = make_ext(args, total_q, total_k);
  const AttnExt* ep = ext_active(args) ? &ex : nullptr;
  if (D == 128)
    launch_bwd<128>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, max_seqlen_q, max_seqlen_k, H, HKV, causal,
                    softmax_scale, st, vl, s, ep);
  else
    launch_bwd<64>(q, k, v, o, dout, lse, ws, dq, dk, dv, B, max_seqlen_q, max_seqlen_k, H, HKV, causal,
                   softmax_scale, st, vl, s, ep);
  DW_LAUNCH_RET;
}

DW_PRELOAD(attn_bwd_pre_kernel<128>);
