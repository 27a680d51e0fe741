// int8 MFMA tile GEMM shared by the GRM kernels:
//   C(128x128, int32) = sum_s A[i][s] * B[j][s]
// where A and B are 128-row tiles of the kernel form's packed panel (rows of pk_row bytes, 64-SNP
// block kb at + 16 kb), unpacked to int8 on the way into LDS.
// 256 threads = 4 waves in a 2x2 grid, each wave a 64x64 block of 2x2
// v_mfma_i32_32x32x32_i8 tiles (lane l holds 16 k of row l&31).
// Genotypes are {0,1,2}: every partial sum is an exact integer.
#pragma once
#include "tblup_internal.h"

namespace tblup {

// ---- 2-bit packed genotypes ----
// A packed row holds 4 genotypes per byte, animal 4j+i at bits 2i of byte j.  One 32-bit
// word (16 animals) unpacks to the 16 int8 MFMA operand bytes with two ops per dword:
// dword q = (x >> 2q) & 0x03030303, i.e. byte m of dword q is animal 4m+q.  This fixed
// permutation of the 16 animals is the same for every row, so A.B^T contractions are
// unchanged.
__device__ __forceinline__ v4i unpack16(uint32_t x) {
  return v4i{(int)(x & 0x03030303u), (int)((x >> 2) & 0x03030303u), (int)((x >> 4) & 0x03030303u),
             (int)((x >> 6) & 0x03030303u)};
}


// [128 rows][64 B]; 16-B chunk c of row r stored at c ^ ((r >> 2) & 3):
// conflict-free ds_read_b128 for the 32x32x32 i8 fragment pattern.
__device__ __forceinline__ int lds_off_i8(int row, int chunk) { return row * 64 + 16 * (chunk ^ ((row >> 2) & 3)); }

// lds: >= 32 KiB (two buffers x A/B x 8 KiB).  a_base/b_base point at the first packed row of the
// two 128-row tiles; rows are pk_row bytes apart.  Dword c of a row's block kb (16 SNPs) becomes the
// row's 16-B int8 chunk c (unpack16: the same SNP order in every row).
__device__ __forceinline__ void i8_tile_gemm(const uint8_t* __restrict__ a_base, const uint8_t* __restrict__ b_base,
                                             bool same, int64_t nblk, int64_t pk_row, int8_t* lds,
                                             v16i (&acc)[2][2]) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0;
  if (nblk <= 0) return;
  constexpr int TB = TILE * KBLK;  // 8 KiB
  v4i ra[2], rb[2];
  auto gload = [&](int64_t kb) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = t + 256 * e, row = q >> 2, c = q & 3;
      const int64_t o = (int64_t)row * pk_row + 16 * kb + 4 * c;
      ra[e] = unpack16(*reinterpret_cast<const uint32_t*>(a_base + o));
      if (!same) rb[e] = unpack16(*reinterpret_cast<const uint32_t*>(b_base + o));
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = t + 256 * e, row = q >> 2, c = q & 3;
      *reinterpret_cast<v4i*>(lds + (2 * buf) * TB + lds_off_i8(row, c)) = ra[e];
      if (!same) *reinterpret_cast<v4i*>(lds + (2 * buf + 1) * TB + lds_off_i8(row, c)) = rb[e];
    }
  };
  gload(0);
  swrite(0);
  __syncthreads();
  for (int64_t kb = 0; kb < nblk; ++kb) {
    const int cur = (int)(kb & 1);
    if (kb + 1 < nblk) gload(kb + 1);
    const int8_t* As = lds + (2 * cur) * TB;
    const int8_t* Bs = same ? As : lds + (2 * cur + 1) * TB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = (l >> 5) + 2 * kk;
      v4i a[2], bb[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) a[m] = *reinterpret_cast<const v4i*>(As + lds_off_i8(64 * wr + 32 * m + (l & 31), chunk));
#pragma unroll
      for (int n = 0; n < 2; ++n) bb[n] = *reinterpret_cast<const v4i*>(Bs + lds_off_i8(64 * wc + 32 * n + (l & 31), chunk));
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[m], bb[n], acc[m][n], 0, 0, 0);
    }
    if (kb + 1 < nblk) swrite(cur ^ 1);
    __syncthreads();
  }
}

// Row / column (within the 128x128 tile) of accumulator element r of block (m, n) for lane l.
__device__ __forceinline__ int i8_row(int wr, int m, int r, int l) { return 64 * wr + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }
__device__ __forceinline__ int i8_col(int wc, int n, int l) { return 64 * wc + 32 * n + (l & 31); }

// System value from the exact integer count c = (A A^T)_ij:
//   dual   (c - (u_i + u_j)/N + q/N^2) / d       (sm = 0)
//   primal (c - s_a s_b / n_T) / d                (sa = cN = 0, sm = 1/n_T)
__device__ __forceinline__ double grm_value(int32_t c, double ui, double uj, double sa, double cN, double invd,
                                            double sm) {
  return ((double)c - (ui + uj) * sa - ui * uj * sm + cN) * invd;
}

}  // namespace tblup
