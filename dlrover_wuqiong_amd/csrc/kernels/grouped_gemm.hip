// Grouped GEMM for mixture-of-experts layers (bf16 in/out, fp32 accumulate).
//
// The token rows routed to expert e are the contiguous rows
// [offs[e], offs[e+1]) of one activation buffer (MoELayer sorts them), and the
// group offsets stay ON THE DEVICE: one launch per GEMM covers every expert,
// no per-expert host synchronisation, no padding to a capacity.
//
// Three forms cover an expert linear layer's forward and backward
// (W [E, N, K] is the nn.Linear weight of each expert):
//   NT  (forward)  Y[r, n]    = sum_k X[r, k]  * W[e, n, k]      rows r of group e
//   NN  (dgrad)    dX[r, k]   = sum_n dY[r, n] * W[e, n, k]
//   TN  (wgrad)    dW[e, n, k] = sum_{r in e} dY[r, n] * X[r, k]
//
// CDNA4 structure (cdna_hip_programming.md §5, 128²-tile row: "grouped GEMM
// at 2-3 blocks/CU: glds ~ register stage"): 128x128 output tile per 4-wave
// workgroup (2x2 waves of 64x64 = 2x2 v_mfma_f32_32x32x16_bf16 tiles), BK = 64,
// register-staged double-buffered LDS images in the T10 (a) "8-row x 32-col
// subtile" layout shared with the attention kernels: operands whose reduction
// index is contiguous in memory are read as rows (ds_read_b128), operands
// whose reduction index is the memory row (dW's both operands, dX's weight)
// with ds_read_b64_tr_b16; when the two operand kinds are mixed, the row
// reads follow the transposed reads' k order (the MFMA only needs A and B to
// agree on it).  The epilogue stages the bf16 tile through LDS so the global
// stores are 16-byte row chunks.  NT / NN workgroups find their (expert, row
// block) by scanning the device offsets; the grid is sized for the worst case
// (ceil(T/128) + E row blocks) and surplus workgroups exit at once.
//
// Parity: ATorch grouped-GEMM MoE experts (atorch/atorch/modules/moe/
// grouped_gemm_moe.py:46-112, which calls the CUDA grouped_gemm package).
#include "attn_common.h"

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
constexpr int IMG = BM * BK * 2;  // bytes of one operand image (both shapes)

enum { MODE_NT = 0, MODE_NN = 1, MODE_TN = 2 };

struct GGArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  const int* offs;  // [E+1] group row offsets (device)
  int E;
  int M;            // TN: output rows per expert (N of the layer)
  int Nout;         // output columns
  int R;            // reduction length (NT: K, NN: N); TN: per group
  long long lda, ldb, ldc;
  long long b_es, c_es;  // per-expert strides of B (NT/NN weights) / C (TN dW), elements
  int tiles_n, tiles_m;  // grid decomposition
};

__device__ __forceinline__ bf16x8_t as_bf(const u32x4& v) { return __builtin_bit_cast(bf16x8_t, v); }

// ROW image: [128 rows][64 cols], img_off<64>.  K-major image: [64 rows][128 cols], img_off<128>.
__device__ __forceinline__ u32x4 frag_row(const char* img, int row, int kk, int hh) {
  return *(const u32x4*)(img + img_off<64>(row, 2 * kk + hh));
}
// same 8 values in the transposed reads' k order: k = 16kk + 8(j>>2) + 4hh + (j&3)
__device__ __forceinline__ u32x4 frag_row_perm(const char* img, int row, int kk, int hh) {
  const uint2 lo = *(const uint2*)(img + img_off<64>(row, 2 * kk) + 8 * hh);
  const uint2 hi = *(const uint2*)(img + img_off<64>(row, 2 * kk + 1) + 8 * hh);
  return (u32x4){lo.x, lo.y, hi.x, hi.y};
}
// transposed read of a K-major image: lane -> column c0 + (lane & 31), 8
// reduction rows 16kk + 8(j>>2) + 4hh + (j&3)
__device__ __forceinline__ u32x4 frag_tr(const char* img, int kk, int c0, int lane) {
  const int g4 = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3, h = lane >> 5;
  const int row = 16 * kk + 4 * h + tq;
  const int ch = (c0 + 16 * (g4 & 1)) / 8 + (tp >> 1);
  const s16x4 v0 =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(img + img_off<128>(row, ch) + 8 * (tp & 1)));
  const s16x4 v1 =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)LDS_PTR(img + img_off<128>(row + 8, ch) + 8 * (tp & 1)));
  return (u32x4){pack_s16(v0[0], v0[1]), pack_s16(v0[2], v0[3]), pack_s16(v1[0], v1[1]), pack_s16(v1[2], v1[3])};
}

// Staged global loads of one operand tile (4 x 16 B per thread).
//  ROW:  rows [0, nrows) x reduction cols [r0, r0 + 64) of src (ld), valid rows < rows_ok, cols < rlim
//  KMAJ: reduction rows [r0, r0 + 64) x cols [0, 128) of src (ld), valid rows < rlim, cols < cols_ok
struct Stage {
  u32x4 v[4];
};

__device__ __forceinline__ void load_row(Stage& s, const bf16_t* src, long long ld, int rows_ok, int r0, int rlim,
                                         int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + NTHR * i;
    const int row = q >> 3, c = q & 7;
    const int col = r0 + 8 * c;
    s.v[i] = (row < rows_ok && col < rlim) ? *(const u32x4*)(src + (long long)row * ld + col) : (u32x4){0, 0, 0, 0};
  }
}
__device__ __forceinline__ void store_row(const Stage& s, char* img, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + NTHR * i;
    *(u32x4*)(img + img_off<64>(q >> 3, q & 7)) = s.v[i];
  }
}
__device__ __forceinline__ void load_kmaj(Stage& s, const bf16_t* src, long long ld, int r0, int rlim, int cols_ok,
                                          int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + NTHR * i;
    const int row = q >> 4, c = q & 15;
    const int r = r0 + row;
    s.v[i] = (r < rlim && 8 * c < cols_ok) ? *(const u32x4*)(src + (long long)r * ld + 8 * c) : (u32x4){0, 0, 0, 0};
  }
}
__device__ __forceinline__ void store_kmaj(const Stage& s, char* img, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + NTHR * i;
    *(u32x4*)(img + img_off<128>(q >> 4, q & 15)) = s.v[i];
  }
}

}  // namespace

template <int MODE>
__global__ void __launch_bounds__(NTHR, 2) grouped_gemm_kernel(GGArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;  // 2x2 waves of 64x64

  // ---- which tile: (expert, output row block, output column block)
  int e = 0, row0 = 0, m_ok = 0, R = a.R;
  const BlockXYZ bc = xcd_block(a.tiles_n, a.tiles_m);
  const int tn = bc.x;
  if (MODE == MODE_TN) {
    e = bc.z;
    row0 = a.offs[e];
    R = a.offs[e + 1] - row0;  // reduction over the group's rows
    m_ok = min(BM, a.M - bc.y * BM);
  } else {
    int mt = bc.y;
    e = -1;
    for (int g = 0; g < a.E; ++g) {
      const int lo = a.offs[g], cnt = a.offs[g + 1] - lo;
      const int nt = (cnt + BM - 1) / BM;
      if (mt < nt) {
        e = g;
        row0 = lo + mt * BM;
        m_ok = min(BM, cnt - mt * BM);
        break;
      }
      mt -= nt;
    }
    if (e < 0) return;  // surplus row block (the grid is sized for the worst case)
  }
  const int n0 = tn * BN;
  const int n_ok = min(BN, a.Nout - n0);

  // ---- operand bases
  const bf16_t *Abase, *Bbase;
  if (MODE == MODE_NT) {
    Abase = a.A + (long long)row0 * a.lda;                 // X rows, k contiguous
    Bbase = a.B + (long long)e * a.b_es + (long long)n0 * a.ldb;  // W[e] rows n, k contiguous
  } else if (MODE == MODE_NN) {
    Abase = a.A + (long long)row0 * a.lda;                 // dY rows, n contiguous
    Bbase = a.B + (long long)e * a.b_es + n0;              // W[e][n][k0 + ..]: reduction rows n
  } else {
    Abase = a.A + (long long)row0 * a.lda + (long long)bc.y * BM;  // dY[r][m0 + ..]
    Bbase = a.B + (long long)row0 * a.ldb + n0;                    // X[r][n0 + ..]
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int n_it = (R + BK - 1) / BK;
  Stage sa, sb;
  auto issue = [&](int it) {
    const int r0 = it * BK;
    if (MODE == MODE_TN) {
      load_kmaj(sa, Abase, a.lda, r0, R, m_ok, tid);
      load_kmaj(sb, Bbase, a.ldb, r0, R, n_ok, tid);
    } else if (MODE == MODE_NN) {
      load_row(sa, Abase, a.lda, m_ok, r0, R, tid);
      load_kmaj(sb, Bbase, a.ldb, r0, R, n_ok, tid);
    } else {
      load_row(sa, Abase, a.lda, m_ok, r0, R, tid);
      load_row(sb, Bbase, a.ldb, n_ok, r0, R, tid);
    }
  };
  auto write = [&](int buf) {
    char* ai = smem + buf * 2 * IMG;
    char* bi = ai + IMG;
    if (MODE == MODE_TN) store_kmaj(sa, ai, tid); else store_row(sa, ai, tid);
    if (MODE == MODE_NT) store_row(sb, bi, tid); else store_kmaj(sb, bi, tid);
  };

  if (n_it > 0) {
    issue(0);
    write(0);
    if (n_it > 1) issue(1);
  }
  __syncthreads();
  for (int it = 0; it < n_it; ++it) {
    const char* ai = smem + (it & 1) * 2 * IMG;
    const char* bi = ai + IMG;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      u32x4 fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int mrow = wm * 64 + t * 32;  // output rows of this MFMA tile
        const int ncol = wn * 64 + t * 32;  // output cols
        if (MODE == MODE_NT) {
          fa[t] = frag_row(ai, mrow + (lane & 31), kk, hh);
          fb[t] = frag_row(bi, ncol + (lane & 31), kk, hh);
        } else if (MODE == MODE_NN) {
          fa[t] = frag_row_perm(ai, mrow + (lane & 31), kk, hh);
          fb[t] = frag_tr(bi, kk, ncol, lane);
        } else {
          fa[t] = frag_tr(ai, kk, mrow, lane);
          fb[t] = frag_tr(bi, kk, ncol, lane);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(fa[i]), as_bf(fb[j]), acc[i][j], 0, 0, 0);
    }
    if (it + 1 < n_it) {
      write((it + 1) & 1);
      if (it + 2 < n_it) issue(it + 2);
    }
    __syncthreads();
  }

  // ---- epilogue: bf16 tile through LDS ([128][128 + 8] padded rows), 16-byte stores
  constexpr int LDC = BN + 8;
  bf16_t* tile = (bf16_t*)smem;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = wn * 64 + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wm * 64 + i * 32 + 8 * (r >> 2) + 4 * hh + (r & 3);
        tile[m * LDC + n] = f2bf(acc[i][j][r]);
      }
    }
  __syncthreads();
  bf16_t* Cb = (MODE == MODE_TN) ? a.C + (long long)e * a.c_es + (long long)bc.y * BM * a.ldc + n0
                                 : a.C + (long long)row0 * a.ldc + n0;
#pragma unroll
  for (int i = 0; i < (BM * BN / 8) / NTHR; ++i) {
    const int q = tid + NTHR * i;
    const int m = q >> 4, c = q & 15;
    if (m < m_ok && 8 * c < n_ok) *(u32x4*)(Cb + (long long)m * a.ldc + 8 * c) = *(const u32x4*)(tile + m * LDC + 8 * c);
  }
}

static_assert(BM * (BN + 8) * 2 <= 4 * IMG, "epilogue tile must fit the operand LDS");

// mode: 0 NT (y = x W^T), 1 NN (dx = dy W), 2 TN (dW = dy^T x per group).
//  NT: A = x [T, K] (lda), B = W [E, N, K], C = y [T, N];   Nout = N, R = K
//  NN: A = dy [T, N] (lda), B = W [E, N, K], C = dx [T, K]; Nout = K, R = N
//  TN: A = dy [T, N] (lda), B = x [T, K] (ldb), C = dW [E, N, K]; M = N, Nout = K
// T (total rows) sizes the NT / NN grid.  All inner dimensions % 8 == 0,
// row strides % 8 == 0 (16-byte vectors).
extern "C" int dw_grouped_gemm(int mode, const void* A, const void* B, void* C, const void* offs, int E, int T,
                               int M, int Nout, int R, long long lda, long long ldb, long long ldc, long long b_es,
                               long long c_es, void* stream) {
  if (E <= 0 || Nout % 8 || lda % 8 || ldb % 8 || ldc % 8 || (mode != MODE_TN && R % 8) ||
      (mode == MODE_TN && M % 8))
    return (int)hipErrorInvalidValue;
  GGArgs g;
  g.A = (const bf16_t*)A;
  g.B = (const bf16_t*)B;
  g.C = (bf16_t*)C;
  g.offs = (const int*)offs;
  g.E = E;
  g.M = M;
  g.Nout = Nout;
  g.R = R;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.b_es = b_es;
  g.c_es = c_es;
  g.tiles_n = (Nout + BN - 1) / BN;
  hipStream_t s = (hipStream_t)stream;
  const int lds = 4 * IMG;
  if (mode == MODE_TN) {
    g.tiles_m = (M + BM - 1) / BM;
    dim3 grid((unsigned)(g.tiles_n * g.tiles_m * E));
    hipLaunchKernelGGL(grouped_gemm_kernel<MODE_TN>, grid, dim3(NTHR), lds, s, g);
  } else {
    g.tiles_m = (T + BM - 1) / BM + E;  // worst case: every group adds one partial block
    if (T <= 0) return 0;
    dim3 grid((unsigned)(g.tiles_n * g.tiles_m));
    if (mode == MODE_NT)
      hipLaunchKernelGGL(grouped_gemm_kernel<MODE_NT>, grid, dim3(NTHR), lds, s, g);
    else
      hipLaunchKernelGGL(grouped_gemm_kernel<MODE_NN>, grid, dim3(NTHR), lds, s, g);
  }
  DW_LAUNCH_RET;
}

DW_PRELOAD(grouped_gemm_kernel<MODE_TN>);
