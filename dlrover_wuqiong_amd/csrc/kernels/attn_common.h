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

__device__ __forceinline__ unsigned int pack_s16(short a, short b) {
  return (unsigned int)(unsigned short)a | ((unsigned int)(unsigned short)b << 16);
}
