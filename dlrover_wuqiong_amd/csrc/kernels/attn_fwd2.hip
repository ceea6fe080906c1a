// Flash attention forward for D = 128, one wave per SIMD (dense masks).
//
// attn_fwd.hip's algorithm (S^T = K Q'^T with the query on the MFMA lane,
// online softmax in registers with the deferred rescale, O^T += V^T P^T with
// the packed probabilities as the B operand) re-shaped for the CDNA4
// register file the way cdna_hip_programming.md describes its fastest
// compiler-scheduled attention body: a workgroup is 4 waves, one per SIMD,
// each owning 64 queries as two 32-query groups, so
//  * every K row fragment (S) and V transposed fragment (PV) read from LDS
//    feeds two MFMAs -- half the LDS reads per MFMA of the 8-wave form;
//  * the two groups are independent MFMA chains the scheduler interleaves
//    with the other group's max / exp / sum / pack (no partner wave on the
//    SIMD to steal issue slots: MI355X_MICROARCH 'one wave per SIMD');
//  * K / V tiles arrive by LDS-DMA (global_load_lds_dwordx4, swizzle on the
//    source address), so no staging registers and no ds_write pass.
// Workgroup = 256 queries of one (batch, head) as before (same grid).
#include "attn_common.h"

#include <cstdlib>
#include <type_traits>

typedef __attribute__((ext_vector_type(4))) short s16x4_f2;
typedef __attribute__((address_space(3))) s16x4_f2 lds_s16x4_f2;

namespace {
struct Fwd2x {
  static constexpr int D = 128;
  static constexpr int WAVES = 4;
  static constexpr int G = 2;
  static constexpr int BQ = 32 * G * WAVES;
  static constexpr int BK = 64;
  static constexpr int NSB = BK / 32;
  static constexpr int KK = D / 16;
  static constexpr int DT = D / 32;
  static constexpr int TILE = BK * D * 2;
};

__device__ __forceinline__ bf16x8_t bf8(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }

__device__ __forceinline__ unsigned int pk2f(float a, float b) {
  typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
  typedef float f32x2_v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned int, __builtin_convertvector((f32x2_v){a, b}, bf16x2_v));
}
}  // namespace

template <bool CAUSAL>
__global__ void __launch_bounds__(64 * Fwd2x::WAVES, 1)
attn_fwd2_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
                 bf16_t* __restrict__ O, float* __restrict__ LSE, int S, int H, int HKV, float scale_log2,
                 AttnStrides st, AttnVarlen vl) {
  using C = Fwd2x;
  constexpr int D = C::D, G = C::G;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = (S + C::BQ - 1) / C::BQ;
  const BlockXYZ bc = xcd_block(nqb, H);
  const int b = bc.z, h = bc.y;
  const int hk = h / (H / HKV);
  const int qblk = CAUSAL ? nqb - 1 - bc.x : bc.x;  // causal: heaviest query blocks first
  const int q_blk0 = qblk * C::BQ;
  const SeqRange sr = seq_range(vl, b, h, H, S);
  if (q_blk0 >= sr.sq) return;
  const int SQ = sr.sq, SK = sr.sk, co = SK - SQ;
  const int q0 = q_blk0 + wid * 32 * G;
  const bf16_t* Qb = Q + (int64_t)b * st.q_bs + (int64_t)sr.q_off * st.q_rs + (int64_t)h * D;
  const bf16_t* Kb = K + (int64_t)b * st.k_bs + (int64_t)sr.k_off * st.k_rs + (int64_t)hk * D;
  const bf16_t* Vb = V + (int64_t)b * st.v_bs + (int64_t)sr.k_off * st.v_rs + (int64_t)hk * D;

  // Q fragments prescaled by softmax_scale * log2(e): scores leave the MFMA
  // in the exp2 domain
  u32x4 qf[G][C::KK];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int q = q0 + 32 * g + r;
#pragma unroll
    for (int kk = 0; kk < C::KK; ++kk) {
      const u32x4 raw =
          (q < SQ) ? *(const u32x4*)(Qb + (int64_t)q * st.q_rs + 16 * kk + 8 * hh) : (u32x4){0, 0, 0, 0};
      float f[8];
      unpack8(raw, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= scale_log2;
      qf[g][kk] = (u32x4){pk2f(f[0], f[1]), pk2f(f[2], f[3]), pk2f(f[4], f[5]), pk2f(f[6], f[7])};
    }
  }
  f32x16 o[G][C::DT];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[g][dt][i] = 0.f;
  // deferred rescale (attn_fwd.hip): the row offset m only moves when a
  // tile's max exceeds it by more than RESCALE_T
  constexpr float RESCALE_T = 8.f;
  float m_i[G], l_i[G];
  bool seeded[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m_i[g] = 0.f;
    l_i[g] = 0.f;
    seeded[g] = false;
  }

  int n_tiles = (SK + C::BK - 1) / C::BK;
  if (CAUSAL) {
    const int last = min(SK - 1, min(SQ - 1, q_blk0 + C::BQ - 1) + co);
    n_tiles = last < 0 ? 0 : min(n_tiles, last / C::BK + 1);
  }
  // K / V tile t into LDS buffer `buf` by LDS-DMA (see attn_bwd_dq2.hip)
  auto issue_tile = [&](int t, int buf) {
    char* kl = smem + buf * 2 * C::TILE;
#pragma unroll
    for (int j = 0; j < C::TILE / 1024 / C::WAVES; ++j) {
      const int piece = wid + C::WAVES * j;
      const int o_ = 1024 * piece + 16 * lane;
      const int rem = o_ % (D * 16), sub = rem % 512;
      const int row = 8 * (o_ / (D * 16)) + sub / 64;
      const int ch = 4 * (rem / 512) + (((sub % 64) / 16) ^ ((row >> 2) & 3));
      const int key = min(t * C::BK + row, SK - 1);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(Kb + (int64_t)key * st.k_rs + ch * 8),
          (__attribute__((address_space(3))) void*)(kl + 1024 * piece), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(Vb + (int64_t)key * st.v_rs + ch * 8),
          (__attribute__((address_space(3))) void*)(kl + C::TILE + 1024 * piece), 16, 0, 0);
    }
  };
  if (n_tiles > 0) issue_tile(0, 0);
  __syncthreads();
  const int kro[2] = {row_lane<D>(lane, 0), row_lane<D>(lane, 1)};
  const int vtr[2] = {tr_lane<D>(lane, 0), tr_lane<D>(lane, 1)};

  for (int t = 0; t < n_tiles; ++t) {
    const int k0 = t * C::BK;
    if (t + 1 < n_tiles) issue_tile(t + 1, (t + 1) & 1);
    const char* kl = smem + (t & 1) * 2 * C::TILE;
    const char* vl2 = kl + C::TILE;
    if (!CAUSAL || k0 <= q0 + 32 * G - 1 + co) {
      const bool need_mask = (k0 + C::BK > SK) || (CAUSAL && (k0 + C::BK - 1 > q0 + co));
      // one 32-key subtile at a time (S of both groups = 32 registers): the
      // online softmax steps per 32 keys, which keeps O (128) + S + the
      // fragments inside the 256 arch VGPRs
      auto tile = [&](auto mask_c) {
        constexpr bool MASK = decltype(mask_c)::value;
#pragma unroll
        for (int sb = 0; sb < C::NSB; ++sb) {
          f32x16 s[G];
#pragma unroll
          for (int g = 0; g < G; ++g)
#pragma unroll
            for (int i = 0; i < 16; ++i) s[g][i] = 0.f;
#pragma unroll
          for (int kk = 0; kk < C::KK; ++kk) {
            const u32x4 kf = *(const u32x4*)(kl + kro[kk & 1] + row_const<D>(32 * sb, kk));
#pragma unroll
            for (int g = 0; g < G; ++g)
              s[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf8(kf), bf8(qf[g][kk]), s[g], 0, 0, 0);
          }
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (MASK) {
              const int q = q0 + 32 * g + r;
              const int rel = (CAUSAL ? min(SK, q + co + 1) : SK) - k0 - 32 * sb - 4 * hh;
#pragma unroll
              for (int i = 0; i < 16; ++i) s[g][i] = ((i & 3) + 8 * (i >> 2)) < rel ? s[g][i] : -INFINITY;
            }
            float mx = -INFINITY;
#pragma unroll
            for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[g][i]);
            mx = half_max(mx) - m_i[g];  // the row's max above its offset
            const bool fresh = !seeded[g] && mx > -INFINITY;
            const bool shift = (mx > RESCALE_T) || fresh;
            seeded[g] = seeded[g] || (mx > -INFINITY);
            if (__any(shift)) {
              const float d = shift ? mx : 0.f;
              const float alpha = fresh ? 1.f : __builtin_amdgcn_exp2f(-d);
              m_i[g] += d;
              l_i[g] *= alpha;
#pragma unroll
              for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[g][dt][i] *= alpha;
            }
            float rs = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float p = __builtin_amdgcn_exp2f(s[g][i] - m_i[g]);
              s[g][i] = p;
              rs += p;
            }
            l_i[g] += rs;
          }
          // O^T += V^T P^T over this subtile's 32 keys; each V^T fragment feeds both groups
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            u32x4 pf[G];
#pragma unroll
            for (int g = 0; g < G; ++g)
              pf[g] = (u32x4){pk2f(s[g][8 * s2 + 0], s[g][8 * s2 + 1]), pk2f(s[g][8 * s2 + 2], s[g][8 * s2 + 3]),
                              pk2f(s[g][8 * s2 + 4], s[g][8 * s2 + 5]), pk2f(s[g][8 * s2 + 6], s[g][8 * s2 + 7])};
            const int kr = 32 * sb + 16 * s2;
#pragma unroll
            for (int dt = 0; dt < C::DT; ++dt) {
              const s16x4_f2 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (lds_s16x4_f2*)((__attribute__((address_space(3))) void*)(vl2 + vtr[0] + tr_const<D>(kr, dt, 0))));
              const s16x4_f2 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                  (lds_s16x4_f2*)((__attribute__((address_space(3))) void*)(vl2 + vtr[1] + tr_const<D>(kr, dt, 1))));
              const u32x4 vf = join_tr(v0, v1);
#pragma unroll
              for (int g = 0; g < G; ++g)
                o[g][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf8(vf), bf8(pf[g]), o[g][dt], 0, 0, 0);
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

#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float l_tot = half_sum(l_i[g]);
    const int q = q0 + 32 * g + r;
    if (q < SQ) {
      bf16_t* Oq = O + (int64_t)b * st.o_bs + (int64_t)h * D + (int64_t)(sr.q_off + q) * st.o_rs;
      const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint2 w;
          w.x = pk2f(o[g][dt][4 * j + 0] * inv, o[g][dt][4 * j + 1] * inv);
          w.y = pk2f(o[g][dt][4 * j + 2] * inv, o[g][dt][4 * j + 3] * inv);
          *(uint2*)(Oq + 32 * dt + 8 * j + 4 * hh) = w;
        }
      if (hh == 0 && LSE)
        LSE[sr.lse_base + q] = (l_tot > 0.f) ? (m_i[g] + log2f(l_tot)) * 0.6931471805599453f : -INFINITY;
    }
  }
}

bool launch_fwd2(const void* q, const void* k, const void* v, void* o, void* lse, int B, int S, int H, int HKV,
                 int causal, float scale_log2, const AttnStrides& st, const AttnVarlen& vl, hipStream_t s) {
  // opt-in (DWAMD_ATTN_FWD2=1): measured SLOWER than the 8-wave kernel, GQA
  // S=8192 forward 636 vs 979 TF/s (profiles/r4/attn_dq2_ab.md): the branchy
  // per-group rescale makes the allocator shuttle O between AGPRs and VGPRs
  static const bool off = [] {
    const char* e = std::getenv("DWAMD_ATTN_FWD2");
    return !(e && e[0] == '1');
  }();
  if (off) return false;
  using C = Fwd2x;
  dim3 grid((unsigned)((S + C::BQ - 1) / C::BQ * H * B));
  if (causal)
    hipLaunchKernelGGL(attn_fwd2_kernel<true>, grid, dim3(64 * C::WAVES), 4 * C::TILE, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, (float*)lse, S, H, HKV, scale_log2, st, vl);
  else
    hipLaunchKernelGGL(attn_fwd2_kernel<false>, grid, dim3(64 * C::WAVES), 4 * C::TILE, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, (float*)lse, S, H, HKV, scale_log2, st, vl);
  return true;
}

DW_PRELOAD(attn_fwd2_kernel<true>);
DW_PRELOAD(attn_fwd2_kernel<false>);
