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

__device__ __forceinline__ unsigned int pack_s16(short a, short b) {
  return (unsigned int)(unsigned short)a | ((unsigned int)(unsigned short)b << 16);
}
