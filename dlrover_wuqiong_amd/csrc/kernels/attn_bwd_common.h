// Operand helpers shared by the attention backward kernels (attn_bwd.hip,
// attn_bwd_dq2.hip).
#pragma once
#include "attn_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ bf16x8_t as_bf(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }
// 8 bf16 scaled by c (operand prescale: scores then leave the MFMA in the exp2 domain)
__device__ __forceinline__ u32x4 scaled8(const u32x4& v, float c);

__device__ __forceinline__ unsigned int pk2(float a, float b) {
  // one v_cvt_pk_bf16_f32 (RNE) for the pair
  typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
  typedef float f32x2_v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned int, __builtin_convertvector((f32x2_v){a, b}, bf16x2_v));
}

// A operand of a 32x32x16 MFMA that sums over 16 rows of a row-major LDS
// image (rows r0 .. r0+15, columns d0 .. d0+31): element j of lane half h is
__device__ __forceinline__ u32x4 scaled8(const u32x4& v, float c) {
  float f[8];
  unpack8(v, f);
  return (u32x4){pk2(f[0] * c, f[1] * c), pk2(f[2] * c, f[3] * c), pk2(f[4] * c, f[5] * c), pk2(f[6] * c, f[7] * c)};
}

// row r0 + 8(j>>2) + 4h + (j&3), matching the k order of a packed 32x32
// accumulator used as the B operand.  Two ds_read_b64_tr_b16 per fragment.
// (r0 a multiple of 16, d0 of 32; tr[p] = tr_lane<D>(lane, p), attn_common.h)
template <int D>
__device__ __forceinline__ u32x4 tr_frag(const char* img, int r0, int d0, const int (&tr)[2]) {
  const s16x4 v0 =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(img + tr[0] + tr_const<D>(r0, d0 / 32, 0)));
  const s16x4 v1 =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(img + tr[1] + tr_const<D>(r0, d0 / 32, 1)));
  return join_tr(v0, v1);
}

// One-wave-per-SIMD dQ kernel (attn_bwd_dq2.hip): returns false
// when it does not apply (then the caller launches attn_bwd_dq_kernel).
bool launch_dq2(const void* q, const void* k, const void* v, const void* dout, const void* lse, const float* delta,
                void* dq, int B, int Sq, int H, int HKV, int D, int causal, float softmax_scale, float scale_log2,
                const AttnStrides& st, const AttnVarlen& vl, hipStream_t s);
