// Helpers shared by the 32x32x16-MFMA attention kernels (attn_fwd.hip,
// attn_bwd.hip's query-major dQ kernel).
#pragma once
#include "dw_common.h"

typedef __attribute__((ext_vector_type(16))) float f32x16;

// Byte offset of 16-byte chunk `ch` of row `row` in a [rows][D] bf16 tile
// stored as 8-row x 32-column subtiles (cdna_hip_programming.md T10 layout
// (a)): conflict-free for ds_read_b128 row reads (32x32x16 A operand) and for
// ds_read_b64_tr_b16 transposed reads of 4-row blocks.
template <int D>
__device__ __forceinline__ int img_off(int row, int ch) {
  return (D * 16) * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// img_off split into a per-lane part (computed once per kernel) and a
// compile-time part (folded into the ds_read offset field), for the two
// MFMA operand reads of the attention kernels -- with img_off written out
// per read, the compiler kept ~30 per-lane offset registers and spent one
// v_add per LDS read (~1.5 VALU per MFMA, the VALU issue slots are the
// kernels' bound: MI355X_MICROARCH 'vector-instruction ISSUE cost').
//  * row reads (32x32x16 A operand): lane row r = lane & 31 of the 32-row
//    subtile at row0 (a multiple of 16), chunk 2*kk + hh:
//      img_off(row0 + r, 2kk + hh) = row_lane(lane, kk & 1) + row_const(row0, kk)
//  * transposed reads (ds_read_b64_tr_b16 pair of tr_frag): key rows
//    k0 + 4hh + tq (+8 for the second read, p8), k0 a multiple of 16, d tile dt:
//      img_off(k0 + 4hh + tq + 8p8, 4dt + 2(g4&1) + (tp>>1)) + 8(tp&1)
//        = tr_lane(lane, p8) + tr_const(k0, dt, p8)
template <int D>
__device__ __forceinline__ int row_lane(int lane, int kodd) {
  const int r = lane & 31, hh = lane >> 5;
  return (D * 16) * (r >> 3) + 64 * (r & 7) + 16 * ((2 * kodd + hh) ^ ((r >> 2) & 3));
}

template <int D>
__host__ __device__ constexpr int row_const(int row0, int kk) {
  return (D * 16) * (row0 >> 3) + 512 * (kk >> 1);
}

template <int D>
__device__ __forceinline__ int tr_lane(int lane, int p8) {
  const int hh = lane >> 5, g4 = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  return 64 * (4 * hh + tq) + 16 * ((2 * (g4 & 1) + (tp >> 1)) ^ ((hh + 2 * p8) & 3)) + 8 * (tp & 1);
}

template <int D>
__host__ __device__ constexpr int tr_const(int k0, int dt, int p8) {
  return (D * 16) * ((k0 >> 3) + p8) + 512 * dt;
}

// (row, 16-byte chunk) that staged vector v (0 .. rows * D/8 - 1) carries in
// a tile written through img_off: 8 consecutive lanes take 2 rows x 4 chunks
// of one 8x32 subtile = 128 contiguous LDS bytes, so a ds_write_b128 lane
// group (8 lanes) hits every bank once.  Row-major lanes (a row's chunks on
// 8 consecutive lanes) put the row's two subtiles 512 B apart: 2-way
// conflicts on every staging store, all the bank conflicts of these kernels.
template <int D>
__device__ __forceinline__ void stage_rc(int v, int& row, int& c) {
  constexpr int CG = D / 32;  // 4-chunk groups per row
  const int rest = v >> 3;
  row = (rest / CG) * 2 + ((v >> 2) & 1);
  c = (rest % CG) * 4 + (v & 3);
}

// LDS-DMA (global_load_lds_dwordx4) into an img_off tile: one wave
// instruction writes 1 KiB, lane L to LDS byte 1024 ci + 16 L (the
// instruction's LDS base is wave-uniform), so a chunk ci covers 8 rows x 64
// columns and the swizzle moves into the per-lane SOURCE address: lane L
// fetches (row, ch) with img_off<D>(row, ch) == 1024 ci + 16 L
template <int D>
__device__ __forceinline__ void dma_rc(int ci, int lane, int& row, int& ch) {
  constexpr int HALVES = D / 64;  // 1 KiB chunks per 8-row group
  row = 8 * (ci / HALVES) + ((lane & 31) >> 2);
  ch = 4 * (2 * (ci % HALVES) + (lane >> 5)) + ((lane & 3) ^ ((row >> 2) & 3));
}

// Block coordinates of a 1-D launch over nx * ny * nz workgroups (x fastest).
// Hardware hands consecutive workgroup ids to the 8 XCDs round-robin, and each
// XCD has a private L2; the remap gives every XCD a contiguous chunk of the
// logical grid, so the x-blocks of one (head, batch) -- which all stream the
// same K/V (forward, dQ) or Q/dO (dK/dV) -- meet in one L2 instead of eight
// (cdna_hip_programming.md T1).  Bijective; a grid not divisible by 8 keeps
// its tail unmapped.
struct BlockXYZ {
  int x, y, z;
};

__device__ __forceinline__ BlockXYZ xcd_block(int nx, int ny) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int cpx = nwg >> 3;
  const int l = bid < (cpx << 3) ? (bid & 7) * cpx + (bid >> 3) : bid;
  BlockXYZ r;
  r.x = l % nx;
  const int yz = l / nx;
  r.y = yz % ny;
  r.z = yz / ny;
  return r;
}

// Variable-length (packed) batches, flash-attn "varlen" convention: q rows of
// sequence b are [cu_q[b], cu_q[b+1]) of a [total_q, H, D] tensor, k/v rows
// [cu_k[b], cu_k[b+1]); LSE / delta are [H, total_q].  cu_q == nullptr: dense
// [B, S, H, D] with LSE [B, H, S].  Causal masks align bottom-right
// (key <= q + len_k - len_q), as flash-attn does for len_q != len_k.
struct AttnVarlen {
  const int* cu_q;
  const int* cu_k;
  int total_q, total_k;
};

struct SeqRange {
  int q_off, k_off, sq, sk;
  long long lse_base;  // LSE / delta index of (b, h, query 0)
};

__device__ __forceinline__ SeqRange seq_range(const AttnVarlen& vl, int b, int h, int H, int S) {
  SeqRange r;
  if (vl.cu_q) {
    r.q_off = vl.cu_q[b];
    r.k_off = vl.cu_k[b];
    r.sq = vl.cu_q[b + 1] - r.q_off;
    r.sk = vl.cu_k[b + 1] - r.k_off;
    r.lse_base = (long long)h * vl.total_q + r.q_off;
  } else {
    r.q_off = r.k_off = 0;
    r.sq = r.sk = S;
    r.lse_base = ((long long)b * H + h) * S;
  }
  return r;
}

// two ds_read_b64_tr_b16 results -> one MFMA operand (pure register
// renaming: the 4 shorts of each read are already the packed bf16 pairs)
template <typename V>
__device__ __forceinline__ u32x4 join_tr(const V& a, const V& b) {
  static_assert(sizeof(V) == 8, "8-byte transposed read");
  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  const u32x2_t x = __builtin_bit_cast(u32x2_t, a), y = __builtin_bit_cast(u32x2_t, b);
  return (u32x4){x[0], x[1], y[0], y[1]};
}

// max over lanes i and i ^ 32 (a row split across the two wave halves):
// v_permlane32_swap exchanges the halves in one VALU op, where __shfl_xor
// goes through ds_bpermute (address math + an LDS round trip)
__device__ __forceinline__ float half_max(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}

__device__ __forceinline__ float half_sum(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

__device__ __forceinline__ unsigned int pack_s16(short a, short b) {
  return (unsigned int)(unsigned short)a | ((unsigned int)(unsigned short)b << 16);
}

// ---------------------------------------------------------------------------
// Extended masking for the attention kernels (instantiated only when EXT is a
// template parameter of true; the plain causal / full kernels never see it):
//   * sliding window: key visible iff -win_l <= key - (q + co) <= win_r
//     (flash-attn window_size; < 0 = unbounded on that side);
//   * GLM prefix ("break point"): keys < prefix[b] are visible to every query
//     of batch b on top of the causal mask (ATorch fa2_with_glm_mask);
//   * additive bias / mask [B|1, H|1, Sq|1, Sk] fp32 (strides 0 broadcast),
//     added to the scaled scores (-inf = masked); no gradient;
//   * ALiBi: -slope[b, h] * |key - (q + co)| added to the scaled scores
//     (flash-attn alibi_slopes [H] or [B, H], fp32);
//   * dropout on the probabilities used for O (LSE over the undropped ones,
//     FA2 semantics) with a counter-based hash of (seed, head, query, key):
//     stateless, so the backward regenerates the identical mask.
// Host ABI (ctypes, ops/attention.py): AttnExtArgs.
struct AttnExtArgs {
  long long bias_bs, bias_hs, bias_qs;
  const float* bias;
  const int* prefix;
  unsigned long long seed, offset;
  int win_l, win_r;
  float p_drop;
  int pad_;
  const float* alibi;
  long long alibi_bs;  // 0: slopes [H] shared by the batch
};

struct AttnExt {
  const float* bias;
  long long bias_bs, bias_hs, bias_qs;
  const int* prefix;
  const float* alibi;
  long long alibi_bs;
  unsigned long long seed, offset;
  long long tq, tk;  // rows of the query / key index space of the hash
  unsigned int drop_thresh;  // keep iff hash >= thresh
  float inv_keep;            // 1 / (1 - p)
  int win_l, win_r;
  bool dropout;
};

static inline AttnExt make_ext(const AttnExtArgs* a, long long tq, long long tk) {
  AttnExt e = {};
  e.win_l = e.win_r = -1;
  e.inv_keep = 1.f;
  if (!a) return e;
  e.bias = a->bias;
  e.bias_bs = a->bias_bs;
  e.bias_hs = a->bias_hs;
  e.bias_qs = a->bias_qs;
  e.prefix = a->prefix;
  e.alibi = a->alibi;
  e.alibi_bs = a->alibi_bs;
  e.seed = a->seed;
  e.offset = a->offset;
  e.tq = tq;
  e.tk = tk;
  e.win_l = a->win_l;
  e.win_r = a->win_r;
  e.dropout = a->p_drop > 0.f;
  if (e.dropout) {
    const double t = (double)a->p_drop * 4294967296.0;
    e.drop_thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (unsigned int)t;
    e.inv_keep = 1.f / (1.f - a->p_drop);
  }
  return e;
}

static inline bool ext_active(const AttnExtArgs* a) {
  return a && (a->bias || a->prefix || a->alibi || a->win_l >= 0 || a->win_r >= 0 || a->p_drop > 0.f);
}

// splitmix64 finalizer over (seed, element index): the keep decision of one
// attention probability.  Identical in the forward, both backward kernels and
// dw_attn_dropout_mask (the test / reference mask).
__device__ __forceinline__ unsigned int attn_hash(unsigned long long seed, unsigned long long idx) {
  unsigned long long z = seed + (idx + 1ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (unsigned int)((z ^ (z >> 31)) >> 32);
}

// element index of (head row bh, global query qg, global key kg)
__device__ __forceinline__ bool attn_keep(const AttnExt& e, long long bh, long long qg, long long kg) {
  const unsigned long long idx = ((unsigned long long)bh * e.tq + qg) * e.tk + kg + e.offset;
  return attn_hash(e.seed, idx) >= e.drop_thresh;
}

// key visibility beyond the plain causal / length checks
__device__ __forceinline__ bool ext_visible(const AttnExt& e, bool causal, int q, int key, int co, int SK, int pre) {
  if (key >= SK) return false;
  if (key < pre) return true;  // GLM prefix: bidirectional
  const int d = key - (q + co);
  bool v = !causal || d <= 0;
  if (e.win_r >= 0) v = v && d <= e.win_r;
  if (e.win_l >= 0) v = v && d >= -e.win_l;
  return v;
}

// ALiBi slope of (b, h) pre-multiplied by log2(e) (0 without ALiBi)
__device__ __forceinline__ float ext_alibi2(const AttnExt& e, int b, int h) {
  return e.alibi ? e.alibi[(long long)b * e.alibi_bs + h] * 1.4426950408889634f : 0.f;
}
