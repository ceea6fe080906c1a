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

__device__ __forceinline__ unsigned int pack_s16(short a, short b) {
  return (unsigned int)(unsigned short)a | ((unsigned int)(unsigned short)b << 16);
}
