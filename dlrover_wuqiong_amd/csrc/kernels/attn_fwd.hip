// Flash attention forward for gfx950 (bf16 in/out, fp32 accumulate).
//
// Layout: q [B, S, H, D], k/v [B, S, Hkv, D] (GQA: H % Hkv == 0), o like q,
// lse [B, H, S] fp32 (natural log), D in {64, 128}; arbitrary batch / row
// strides (q/k/v may be views into one packed QKV projection).
//
// CDNA4 design (cdna_hip_programming.md App. B "fused attention prefill"):
//  * W waves x 32 query rows per workgroup (D=128: 8 -> 256 queries; D=64: 4
//    -> 128); K/V tiles of 64
//    keys double-buffered in LDS (one barrier per tile); every tile is read
//    from HBM once per 256 queries.
//  * v_mfma_f32_32x32x16_bf16 with the swapped product S^T = K * Q^T: the
//    accumulator puts the QUERY on the lane (col = lane & 31) and 16 keys in
//    the registers, so the row max / sum are in-lane over 32 values plus ONE
//    exchange with lane ^ 32 for the max (the sum stays a per-half partial
//    until the epilogue).
//  * O^T += V^T * P^T: the S^T accumulator registers, packed pairwise to
//    bf16, ARE the B operand of the second MFMA ("an accumulator tile as the
//    next MFMA's operand", guide §3): P never touches LDS.  The V^T operand
//    comes from the row-major V tile via ds_read_b64_tr_b16 (T10), two reads
//    per 16-key k-step.
//  * One LDS image per tile in the "8-row x 32-column subtile" layout of
//    guide T10 (a): conflict-free for the K row reads (ds_read_b128, A
//    operand of S^T) and the V transposed reads.
//  * K/V tiles fetched one tile ahead: D = 64 by LDS-DMA straight into the
//    image, D = 128 register-staged (T14 issue-early / write-late); exp2 with the softmax scale folded into log2(e); causal:
//    tiles above a wave's diagonal are skipped by that wave, the longest
//    query blocks are dispatched first.
#include "attn_common.h"

#ifndef DWAMD_FWD_DIAG_SKIP
// causal diagonal tiles: a wave skips the QK^T / PV MFMAs of the 32-key
// subtiles that lie wholly after its 32 queries (A/B; 0 = compute and mask).
// Measured SLOWER despite fewer MFMAs -- the per-subtile scalar branches
// break the interleaved MFMA chains: GPT2 shape fwd 65.5 -> 73.1 us, D=128
// S=4k 649 -> 702 us (profiles/r4/attn_fwd_diag_skip_ab.jsonl)
#define DWAMD_FWD_DIAG_SKIP 0
#endif

#ifndef DWAMD_FWD64_BK
#define DWAMD_FWD64_BK 128  // keys per K/V tile at D = 64 (launch_fwd)
#endif
#ifndef DWAMD_FWD_DMA
// D = 64 K / V tiles by LDS-DMA (0: register staging).  GPT2 shape (B8 S1024
// H25 causal) kernel 70.3 -> 65.0 us, S=4096 120.9 -> 111.8 us; with DMA the
// 64-key form drops to 150 VGPRs (3 waves / SIMD) and wins at S <= 2048
// (63.5 us), the 128-key form at longer S (profiles/r6/attn_fwd64_dma_ab.jsonl)
#define DWAMD_FWD_DMA 1
#endif
#ifndef DWAMD_FWD128_BK
#define DWAMD_FWD128_BK 64  // A/B: keys per K/V tile at D = 128 (128: same speed, profiles/r6/attn_fwd128_bk128_ab.jsonl)
#endif
#ifndef DWAMD_FWD_DMA128
// the D = 128 K / V tiles by LDS-DMA too (214 -> 194 VGPRs): GQA S=4096 forward
// 652 -> 594 us, S=8192 1006 -> 1077 TF/s (profiles/r6/attn_fwd128_dma_ab.jsonl)
#define DWAMD_FWD_DMA128 1
#endif
#ifndef DWAMD_FWD64_BK64_MAX_S
#define DWAMD_FWD64_BK64_MAX_S 2048
#endif

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

template <int D, int W = 8, int BKT = 64>
struct Fwd2Cfg {
  // W waves share each K/V tile.  D=128: 8 waves (236 VGPRs, one block per
  // CU); D=64: 4 waves (see launch_fwd).
  static constexpr int WAVES = W;
  static constexpr int BQ = 32 * WAVES;  // queries per block
  static constexpr int BK = BKT;         // keys per tile
  static constexpr int NSB = BK / 32;    // 32-key subtiles (S^T accumulators)
  static constexpr int NCH = D / 8;      // 16-byte chunks per row
  static constexpr int KK = D / 16;      // MFMA k-steps over the head dim
  static constexpr int DT = D / 32;      // 32-wide d tiles of O^T
  static constexpr int TILE = BK * D * 2;
  static constexpr int VPT = BK * NCH / (64 * WAVES);  // staged 16-B vectors per thread per tensor
};

__device__ __forceinline__ bf16x8_t as_bf16x8(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }

__device__ __forceinline__ unsigned int pack2(float a, float b) {
  // one v_cvt_pk_bf16_f32 (RNE) for the pair
  typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
  typedef float f32x2_v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned int, __builtin_convertvector((f32x2_v){a, b}, bf16x2_v));
}

template <int D, bool CAUSAL, bool EXT, int W = 8, int MINW = 1, int BKT = 64>
__global__ void __launch_bounds__(64 * W, MINW)
attn_fwd_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
                bf16_t* __restrict__ O, float* __restrict__ LSE, int S, int H, int HKV, float scale_log2,
                AttnStrides st, AttnVarlen vl, AttnExt ex) {
  using C = Fwd2Cfg<D, W, BKT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  // wave index as a scalar: keeps q0 / causal skips / mask decisions in SGPRs
  // (a VGPR wid turns every per-element mask into an exec-mask branch)
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + C::BQ - 1) / C::BQ;
  const BlockXYZ bc = xcd_block(nqb, H);
  const int b = bc.z, h = bc.y;
  const int hk = h / (H / HKV);
  const int qblk = CAUSAL ? nqb - 1 - bc.x : bc.x;  // causal: heaviest query blocks first
  const int q_blk0 = qblk * C::BQ;
  // this (batch | packed sequence)'s query / key extents; S is the grid's
  // (maximum) length
  const SeqRange sr = seq_range(vl, b, h, H, S);
  if (q_blk0 >= sr.sq) return;  // whole block past a short sequence
  const int SQ = sr.sq, SK = sr.sk, co = SK - SQ;  // co: bottom-right causal offset
  const int q0 = q_blk0 + wid * 32;
  const bf16_t* Qb = Q + (int64_t)b * st.q_bs + (int64_t)sr.q_off * st.q_rs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * st.k_bs + (int64_t)sr.k_off * st.k_rs + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * st.v_bs + (int64_t)sr.k_off * st.v_rs + (int64_t)hk * D;

  // ---- Q fragments (B operand of S^T): lane holds Q[q0 + r][16 kk + 8 hh .. +7]
  // Q is prescaled by softmax_scale * log2(e) once (guide: operand prescale),
  // so the scores come out of the MFMA already in the exp2 domain
  u32x4 qf[C::KK];
  {
    const int q = q0 + r;
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk) {
      const u32x4 raw =
          (q < SQ) ? *(const u32x4*)(Qb + (int64_t)q * st.q_rs + 16 * kk + 8 * hh) : (u32x4){0, 0, 0, 0};
      float f[8];
      unpack8(raw, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= scale_log2;
      qf[kk] = (u32x4){pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7])};
    }
  }

  f32x16 o[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  // m_i: the row's reference offset (exp2 domain), only raised when a tile's
  // max exceeds it by more than RESCALE_T (deferred rescale, guide T13): p
  // may reach 2^RESCALE_T, harmless in fp32 / bf16, and O / l are rescaled
  // on a handful of tiles instead of nearly every one.  l_i: this
  // lane-half's partial row sum.
  constexpr float RESCALE_T = 8.f;
  float m_i = 0.f, l_i = 0.f;
  // -m_i in all 16 registers: the loop-invariant C operand of each S chain's
  // first MFMA (a lane's registers all belong to its query), rewritten only
  // when m_i moves -- instead of 16 v_mov per subtile per tile
  f32x16 minit;
#pragma unroll
  for (int i = 0; i < 16; ++i) minit[i] = 0.f;
  bool seeded = false;  // the row's offset was set from its first visible scores

  int n_tiles = (SK + C::BK - 1) / C::BK;
  int t_begin = 0;  // EXT sliding window: tiles left of every query's window are skipped
  const int pre = EXT && ex.prefix ? min(SK, ex.prefix[b]) : 0;
  if (CAUSAL || EXT) {
    const int q_last = min(SQ - 1, q_blk0 + C::BQ - 1);
    int last = SK - 1;  // last key the block's queries see
    if (CAUSAL) last = min(last, q_last + co);
    if (EXT && ex.win_r >= 0) last = min(last, q_last + co + ex.win_r);
    if (EXT && pre > 0) last = max(last, pre - 1);
    n_tiles = last < 0 ? 0 : min(n_tiles, last / C::BK + 1);
    if (EXT && ex.win_l >= 0 && pre == 0) t_begin = min(n_tiles, max(0, q_blk0 + co - ex.win_l) / C::BK);
  }
  const int n_run = n_tiles - t_begin;
  const long long bh = vl.cu_q ? (long long)h : (long long)b * H + h;  // dropout hash row
  const float al2 = EXT ? ext_alibi2(ex, b, h) : 0.f;
  const float* brow = nullptr;  // this lane's query row of the additive bias
  if (EXT && ex.bias && q0 + r < SQ)
    brow = ex.bias + (int64_t)b * ex.bias_bs + (int64_t)h * ex.bias_hs + (int64_t)(q0 + r) * ex.bias_qs;

  // D = 64: K / V tiles go global -> LDS by DMA (global_load_lds_dwordx4: one
  // wave instruction fills one 8-row x 64-column group of the T10 image, the
  // swizzle lives in the per-lane source address); no staging registers, no
  // ds_write.  Keys past the sequence read the last key: masked, p = 0.
  constexpr bool DMA = DWAMD_FWD_DMA && (D == 64 || DWAMD_FWD_DMA128) && !EXT && (C::TILE / 1024) % C::WAVES == 0;
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

  // per-lane LDS read offsets (attn_common.h row_lane / tr_lane); the rest
  // of every read address is a compile-time immediate
  const int kro[2] = {row_lane<D>(lane, 0), row_lane<D>(lane, 1)};
  const int vtr[2] = {tr_lane<D>(lane, 0), tr_lane<D>(lane, 1)};

  for (int tt = 0; tt < n_run; ++tt) {
    const int t = t_begin + tt;
    const int k0 = t * C::BK;
    const char* kl = smem + (tt & 1) * 2 * C::TILE;
    const char* vl = kl + C::TILE;
    // a wave whose 32 queries all lie before this tile has nothing to do here
    bool active = !CAUSAL || (k0 <= q0 + 31 + co);
    if (EXT) {
      if (k0 < pre) active = true;
      if (ex.win_r >= 0) active = active && (k0 <= q0 + 31 + co + ex.win_r);
      if (ex.win_l >= 0 && k0 >= pre) active = active && (k0 + C::BK - 1 >= q0 + co - ex.win_l);
    }
    if (active) {
      // ---- S'^T = K Q'^T - m : two 32-key subtiles; the accumulator starts at
      // -m_i (row constant as the initial accumulator), so p = exp2(S') needs
      // no subtraction
      f32x16 s[C::NSB];
      // subtiles [sb_hi, NSB) hold only keys after this wave's last query
      // (causal, non-EXT): every score there is masked to -inf below
      int sb_hi = C::NSB;
      if (DWAMD_FWD_DIAG_SKIP && CAUSAL && !EXT && k0 + C::BK - 1 > q0 + 31 + co)
        sb_hi = min(C::NSB, max(1, (q0 + 31 + co - k0) / 32 + 1));
      if (EXT) {  // (the EXT instances keep the explicit init: minit would spill them)
#pragma unroll
        for (int sb = 0; sb < C::NSB; ++sb)
#pragma unroll
          for (int i = 0; i < 16; ++i) s[sb][i] = -m_i;
      }
      // the two subtiles' chains interleaved: no MFMA waits on its predecessor
      if constexpr (D == 64 && C::NSB == 2) {
        // all 8 K fragments (32 VGPRs) in flight at once: one LDS latency per
        // tile instead of one per MFMA
        u32x4 kf[C::KK][2];
#pragma unroll
        for (int kk = 0; kk < C::KK; ++kk)
#pragma unroll
          for (int sb = 0; sb < C::NSB; ++sb)
            kf[kk][sb] = *(const u32x4*)(kl + kro[kk & 1] + row_const<D>(32 * sb, kk));
#pragma unroll
        for (int kk = 0; kk < C::KK; ++kk)
#pragma unroll
          for (int sb = 0; sb < C::NSB; ++sb)
            s[sb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kf[kk][sb]), as_bf16x8(qf[kk]),
                                                            (kk == 0 && !EXT) ? minit : s[sb], 0, 0, 0);
        // the machine scheduler would sink each read next to its MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * C::KK, 0);  // DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * C::KK, 0);  // then the MFMAs
      } else {
#pragma unroll
        for (int kk = 0; kk < C::KK; ++kk)
#pragma unroll
          for (int sb = 0; sb < C::NSB; ++sb) {
            if (DWAMD_FWD_DIAG_SKIP && sb >= sb_hi) continue;  // wholly masked below
            const u32x4 kf = *(const u32x4*)(kl + kro[kk & 1] + row_const<D>(32 * sb, kk));
            s[sb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kf), as_bf16x8(qf[kk]),
                                                            (kk == 0 && !EXT) ? minit : s[sb], 0, 0, 0);
          }
      }

      // ---- online softmax: lane = query q0 + r, its 32 keys in registers
      const int q = q0 + r;
      const bool need_mask = (k0 + C::BK > SK) || (CAUSAL && (k0 + C::BK - 1 > q0 + co));
      if (EXT) {
        // window / prefix visibility and the additive bias (exp2 domain)
#pragma unroll
        for (int sb = 0; sb < C::NSB; ++sb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = k0 + 32 * sb + (i & 3) + 8 * (i >> 2) + 4 * hh;
            const bool vis = ext_visible(ex, CAUSAL, q, key, co, SK, pre);
            float add = (brow && vis) ? brow[key] * 1.4426950408889634f : 0.f;
            add -= al2 * fabsf((float)(key - q - co));
            s[sb][i] = vis ? s[sb][i] + add : -INFINITY;
          }
      } else if (need_mask) {
        // diagonal / ragged-end tiles only (need_mask is wave-uniform): the
        // empty volatile asm keeps this a scalar branch -- if-converted, the
        // 64 compares + selects would run on every tile
        __asm__ volatile("");
        // keys < lim are visible to this lane's query; the register's key
        // offset within the tile is a compile-time constant
        const int rel = (CAUSAL ? min(SK, q + co + 1) : SK) - k0 - 4 * hh;
#pragma unroll
        for (int sb = 0; sb < C::NSB; ++sb)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            s[sb][i] = (32 * sb + (i & 3) + 8 * (i >> 2)) < rel ? s[sb][i] : -INFINITY;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int sb = 0; sb < C::NSB; ++sb)
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[sb][i]);
      mx = half_max(mx);  // the row's max above its offset
      // move the offset of the rows that outgrew it, and seed it from the
      // first visible scores of a row (they may sit far below 0); O and l follow
      const bool fresh = !seeded && mx > -INFINITY;
      const bool shift = (mx > RESCALE_T) || fresh;
      seeded = seeded || (mx > -INFINITY);
      if (__any(shift)) {
        const float d = shift ? mx : 0.f;
        // a fresh row has l = O = 0; its seed may lie far below 0 (ALiBi over
        // a long distance) where exp2(-d) overflows and 0 * inf would be NaN
        const float alpha = fresh ? 1.f : __builtin_amdgcn_exp2f(-d);
        m_i += d;
        if (!EXT) {
#pragma unroll
          for (int i = 0; i < 16; ++i) minit[i] = -m_i;
        }
        l_i *= alpha;
#pragma unroll
        for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
#pragma unroll
        for (int sb = 0; sb < C::NSB; ++sb)
#pragma unroll
          for (int i = 0; i < 16; ++i) s[sb][i] -= d;
      }
      float rs = 0.f;
#pragma unroll
      for (int sb = 0; sb < C::NSB; ++sb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(s[sb][i]);
          s[sb][i] = p;
          rs += p;
        }
      l_i += rs;
      if (EXT && ex.dropout) {
        // O accumulates the dropped probabilities; l (hence LSE) the full ones
#pragma unroll
        for (int sb = 0; sb < C::NSB; ++sb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = k0 + 32 * sb + (i & 3) + 8 * (i >> 2) + 4 * hh;
            const bool keep = attn_keep(ex, bh, (long long)sr.q_off + q, (long long)sr.k_off + key);
            s[sb][i] = keep ? s[sb][i] * ex.inv_keep : 0.f;
          }
      }

      // ---- O^T += V^T P^T : 4 k-steps of 16 keys
#pragma unroll
      for (int sb = 0; sb < C::NSB; ++sb) {
        if (DWAMD_FWD_DIAG_SKIP && sb >= sb_hi) continue;  // P == 0 there
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const f32x16& a = s[sb];
          const u32x4 pf = {pack2(a[8 * s2 + 0], a[8 * s2 + 1]), pack2(a[8 * s2 + 2], a[8 * s2 + 3]),
                            pack2(a[8 * s2 + 4], a[8 * s2 + 5]), pack2(a[8 * s2 + 6], a[8 * s2 + 7])};
          const int k0 = 32 * sb + 16 * s2;  // this k-step's 16 key rows
#pragma unroll
          for (int dt = 0; dt < C::DT; ++dt) {
            const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4*)LDS_PTR(vl + vtr[0] + tr_const<D>(k0, dt, 0)));
            const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4*)LDS_PTR(vl + vtr[1] + tr_const<D>(k0, dt, 1)));
            const u32x4 vf = join_tr(v0, v1);
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(vf), as_bf16x8(pf), o[dt], 0, 0, 0);
          }
        }
      }
    }
    if (!DMA && tt + 1 < n_run) {
      write_lds((tt + 1) & 1);
      if (tt + 2 < n_run) issue_load(t + 2);
    }
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile tt+1 landed
    __syncthreads();
    if (DMA && tt + 2 < n_run) dma(t + 2, tt & 1);  // buffer tt & 1 is free
  }

  // ---- epilogue: O = O^T / l ; lse
  const float l_tot = half_sum(l_i);
  const int q = q0 + r;
  if (q < SQ) {
    bf16_t* Oq = O + (int64_t)b * st.o_bs + (int64_t)h * D + (int64_t)(sr.q_off + q) * st.o_rs;
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 w;
        w.x = pack2(o[dt][4 * g + 0] * inv, o[dt][4 * g + 1] * inv);
        w.y = pack2(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
        *(uint2*)(Oq + 32 * dt + 8 * g + 4 * hh) = w;
      }
    if (hh == 0 && LSE) {
      const float lse = (l_tot > 0.f) ? (m_i + log2f(l_tot)) * 0.6931471805599453f : -INFINITY;
      LSE[sr.lse_base + q] = lse;
    }
  }
}

template <int D, bool CAUSAL, bool EXT, int W, int MINW, int BKT = 64>
static void launch_fwd_v(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S, int H,
                         int HKV, float scale_log2, const AttnStrides& st, const AttnVarlen& vl, const AttnExt& ex,
                         hipStream_t s) {
  using C = Fwd2Cfg<D, W, BKT>;
  dim3 grid((unsigned)((S + C::BQ - 1) / C::BQ * H * B)), block(64 * W);  // 1-D: xcd_block()
  hipLaunchKernelGGL((attn_fwd_kernel<D, CAUSAL, EXT, W, MINW, BKT>), grid, block, 4 * C::TILE, s, (const bf16_t*)q,
                     (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, (float*)lse, S, H, HKV, scale_log2, st, vl, ex);
}

// one-wave-per-SIMD D = 128 forward (attn_fwd2.hip); false: not taken
bool launch_fwd2(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S, int H, int HKV,
                 int causal, float scale_log2, const AttnStrides& st, const AttnVarlen& vl, hipStream_t s);

template <int D>
static void launch_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S, int H, int HKV,
                       int causal, float scale_log2, const AttnStrides& st, const AttnVarlen& vl, hipStream_t s,
                       const AttnExt* ext = nullptr, int variant = 0) {
  if (D == 128 && !ext && variant == 0 && launch_fwd2(q, k, v, o, lse, B, S, H, HKV, causal, scale_log2, st, vl, s))
    return;
  // D=64: 4 waves (128 queries per block, two blocks per CU):
  // twice the blocks of the 8-wave form for a finer causal balance; measured
  // against 8 waves capped at 128 VGPRs (spills) / uncapped and 4 waves
  // capped: 289-311 vs 239-288 TF/s (profiles/r2/attn_fwd64_variants.jsonl)
  constexpr int W = D == 64 ? 4 : 8;
  if (ext) {
    return causal ? launch_fwd_v<D, true, true, W, 1>(q, k, v, o, lse, B, S, H, HKV, scale_log2, st, vl, *ext, s)
                  : launch_fwd_v<D, false, true, W, 1>(q, k, v, o, lse, B, S, H, HKV, scale_log2, st, vl, *ext, s);
  }
  const AttnExt none = {};
  // D=64: 128-key tiles -- twice the MFMAs per barrier and per staging pass,
  // 252 VGPRs: +4-8 % over 64-key tiles (GPT2 shape 354 -> 369 TF/s, S=4096
  // 578 -> 626; profiles/r3/attn_fwd64_bk128_ab.jsonl).  D=128 keeps 64 (128
  // spills).  flags=1 selects the 64-key form for A/B runs; with DMA staging
  // the 64-key form is the faster one up to S = DWAMD_FWD64_BK64_MAX_S.
  constexpr int BKT = D == 64 ? DWAMD_FWD64_BK : DWAMD_FWD128_BK;
  if (D == 64 && (variant == 1 || (DWAMD_FWD_DMA && S <= DWAMD_FWD64_BK64_MAX_S)))
    return causal ? launch_fwd_v<D, true, false, W, 1, 64>(q, k, v, o, lse, B, S, H, HKV, scale_log2, st, vl, none, s)
                  : launch_fwd_v<D, false, false, W, 1, 64>(q, k, v, o, lse, B, S, H, HKV, scale_log2, st, vl, none, s);
  return causal ? launch_fwd_v<D, true, false, W, 1, BKT>(q, k, v, o, lse, B, S, H, HKV, scale_log2, st, vl, none, s)
                : launch_fwd_v<D, false, false, W, 1, BKT>(q, k, v, o, lse, B, S, H, HKV, scale_log2, st, vl, none, s);
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
  const AttnVarlen vl = {nullptr, nullptr, 0, 0};
  // flags: kernel variant for tuning A/B runs (0 = the default choice)
  if (D == 128) launch_fwd<128>(q, k, v, o, lse, B, S, H, HKV, causal, scale_log2, st, vl, s, nullptr, flags);
  else if (D == 64) launch_fwd<64>(q, k, v, o, lse, B, S, H, HKV, causal, scale_log2, st, vl, s, nullptr, flags);
  else return (int)hipErrorInvalidValue;
  DW_LAUNCH_RET;
}

// Packed variable-length batch: q [total_q, H, D], k/v [total_k, HKV, D] (row
// strides given: rows_strides int64[4] = q, k, v, o), cu_seqlens int32 [B+1]
// on the device, lse [H, total_q].  max_seqlen_q sizes the grid; blocks past
// a sequence's end exit at once.
extern "C" int dw_attn_fwd_varlen(const void* q, const void* k, const void* v, void* o, void* lse,
                                  const void* cu_q, const void* cu_k, int B, int max_seqlen_q, int total_q, int H,
                                  int HKV, int D, const long long* row_strides, int causal, float softmax_scale,
                                  void* stream) {
  if (H % HKV != 0 || !cu_q || !cu_k) return (int)hipErrorInvalidValue;
  AttnStrides st = {};
  st.q_rs = row_strides[0]; st.k_rs = row_strides[1]; st.v_rs = row_strides[2]; st.o_rs = row_strides[3];
  const AttnVarlen vl = {(const int*)cu_q, (const int*)cu_k, total_q, 0};
  const float scale_log2 = softmax_scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  if (D == 128) launch_fwd<128>(q, k, v, o, lse, B, max_seqlen_q, H, HKV, causal, scale_log2, st, vl, s);
  else if (D == 64) launch_fwd<64>(q, k, v, o, lse, B, max_seqlen_q, H, HKV, causal, scale_log2, st, vl, s);
  else return (int)hipErrorInvalidValue;
  DW_LAUNCH_RET;
}

extern "C" int dw_attn_fwd(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S,
                           int H, int HKV, int D, int causal, float softmax_scale, int flags, void* stream) {
  const long long st[8] = {(long long)S * H * D, (long long)H * D, (long long)S * HKV * D, (long long)HKV * D,
                           (long long)S * HKV * D, (long long)HKV * D, (long long)S * H * D, (long long)H * D};
  return dw_attn_fwd_strided(q, k, v, o, lse, B, S, H, HKV, D, st, causal, softmax_scale, flags, stream);
}

// Extended masks (window / GLM prefix / additive bias / dropout; attn_common.h
// AttnExtArgs).  Dense: strides as dw_attn_fwd_strided, Sq = Sk = S.
extern "C" int dw_attn_fwd_ext(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S, int H,
                               int HKV, int D, const long long* strides, int causal, float softmax_scale,
                               const AttnExtArgs* args, void* stream) {
  if (H % HKV != 0) return (int)hipErrorInvalidValue;
  AttnStrides st = {};
  st.q_bs = strides[0]; st.q_rs = strides[1]; st.k_bs = strides[2]; st.k_rs = strides[3];
  st.v_bs = strides[4]; st.v_rs = strides[5]; st.o_bs = strides[6]; st.o_rs = strides[7];
  const float scale_log2 = softmax_scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  const AttnVarlen vl = {nullptr, nullptr, 0, 0};
  const AttnExt ex = make_ext(args, S, S);
  const AttnExt* ep = ext_active(args) ? &ex : nullptr;
  if (D == 128) launch_fwd<128>(q, k, v, o, lse, B, S, H, HKV, causal, scale_log2, st, vl, s, ep);
  else if (D == 64) launch_fwd<64>(q, k, v, o, lse, B, S, H, HKV, causal, scale_log2, st, vl, s, ep);
  else return (int)hipErrorInvalidValue;
  DW_LAUNCH_RET;
}

// Packed batches with window / dropout (no bias / prefix: their indexing is dense).
extern "C" int dw_attn_fwd_varlen_ext(const void* q, const void* k, const void* v, void* o, void* lse,
                                      const void* cu_q, const void* cu_k, int B, int max_seqlen_q, int total_q,
                                      int total_k, int H, int HKV, int D, const long long* row_strides, int causal,
                                      float softmax_scale, const AttnExtArgs* args, void* stream) {
  if (H % HKV != 0 || !cu_q || !cu_k || (args && (args->bias || args->prefix || (args->alibi && args->alibi_bs))))
    return (int)hipErrorInvalidValue;
  AttnStrides st = {};
  st.q_rs = row_strides[0]; st.k_rs = row_strides[1]; st.v_rs = row_strides[2]; st.o_rs = row_strides[3];
  const AttnVarlen vl = {(const int*)cu_q, (const int*)cu_k, total_q, total_k};
  const float scale_log2 = softmax_scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  const AttnExt ex = make_ext(args, total_q, total_k);
  const AttnExt* ep = ext_active(args) ? &ex : nullptr;
  if (D == 128) launch_fwd<128>(q, k, v, o, lse, B, max_seqlen_q, H, HKV, causal, scale_log2, st, vl, s, ep);
  else if (D == 64) launch_fwd<64>(q, k, v, o, lse, B, max_seqlen_q, H, HKV, causal, scale_log2, st, vl, s, ep);
  else return (int)hipErrorInvalidValue;
  DW_LAUNCH_RET;
}

// The dropout keep-mask the kernels use, materialised (tests / references):
// out uint8 [B, H, S, S] (dense index space, tq = tk = S), 1 = kept.
__global__ void attn_dropout_mask_kernel(unsigned char* out, int B, int H, int S, AttnExt ex) {
  const long long n = (long long)B * H * S * S;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long key = i % S, q = (i / S) % S, bh = i / ((long long)S * S);
    out[i] = attn_keep(ex, bh, q, key) ? 1 : 0;
  }
}

extern "C" int dw_attn_dropout_mask(void* out, int B, int H, int S, float p, unsigned long long seed,
                                    unsigned long long offset, void* stream) {
  AttnExtArgs a = {};
  a.win_l = a.win_r = -1;
  a.p_drop = p;
  a.seed = seed;
  a.offset = offset;
  const AttnExt ex = make_ext(&a, S, S);
  hipLaunchKernelGGL(attn_dropout_mask_kernel, dim3(1024), dim3(256), 0, (hipStream_t)stream, (unsigned char*)out, B,
                     H, S, ex);
  DW_LAUNCH_RET;
}

DW_PRELOAD(attn_dropout_mask_kernel);
