// GRM block kernel: K_{R,T} = (A_R A_T^T - (u_R + u_T)/N + q/N^2) / d (+ lambda I on TT)
// for every individual of the batch, on int8 MFMA (v_mfma_i32_32x32x32_i8).
//
// Restates tblup/utils.py:7-18 (make_grm) for the rows the solve needs and the
// kernel-form system of both reference branches (evaluator.py:275-284 and the
// Ridge fit of evaluator.py:311-314): genotypes are {0,1,2}, so A A^T is an
// exact integer product (int32 accumulation never overflows for k < 2^28),
// and the centring is an exact-integer rank-1 correction applied in fp64.
//
// Tiling: one 256-thread workgroup per 128x128 output tile (4 waves, 64x64 each
// = 2x2 MFMA 32x32 blocks); K steps of 64 SNPs read from the animal-major
// panel (one 128x64 operand tile = 8 KB contiguous).  Only the tiles the
// Cholesky and the prediction read are computed: the TT lower triangle
// (diagonal tiles in full) and the VT block.  Workgroups of one individual are
// kept on one XCD (xcd_remap) so the individual's panel is re-read from L2.
#include "tblup_internal.h"

namespace tblup {

namespace {

__device__ __forceinline__ int lds_off_i8(int row, int chunk) {
  // [128 rows][64 B]; 16-B chunk c of row r stored at chunk c ^ ((r >> 2) & 3):
  // conflict-free ds_read_b128 for the 32x32x32 i8 fragment pattern.
  return row * 64 + 16 * (chunk ^ ((row >> 2) & 3));
}

}  // namespace

__global__ __launch_bounds__(256) void k_grm(const int8_t* __restrict__ panel, int64_t panel_stride,
                                             const int64_t* __restrict__ off, const double* __restrict__ u,
                                             const double* __restrict__ scal, int64_t nT, int64_t nTp, int64_t nV,
                                             int64_t nRp, int NT, int64_t tiles_per, double* __restrict__ K) {
  __shared__ __attribute__((aligned(16))) int8_t lds[2][2][TILE * KBLK];  // [buf][A/B]
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int64_t logical = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t b = logical / tiles_per;
  int64_t tt = logical % tiles_per;
  int ti, tj;
  const int64_t ntri = (int64_t)NT * (NT + 1) / 2;
  if (tt < ntri) {
    int r = (int)((sqrt(8.0 * (double)tt + 1.0) - 1.0) * 0.5);
    while ((int64_t)(r + 1) * (r + 2) / 2 <= tt) ++r;
    while ((int64_t)r * (r + 1) / 2 > tt) --r;
    ti = r;
    tj = (int)(tt - (int64_t)r * (r + 1) / 2);
  } else {
    tt -= ntri;
    ti = NT + (int)(tt / NT);
    tj = (int)(tt % NT);
  }
  const bool same = (ti == tj);
  const int64_t k = off[b + 1] - off[b];
  const int64_t nblk = (k + KBLK - 1) / KBLK;
  const int8_t* pb = panel + b * panel_stride;

  v16i acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0;

  v4i ra[2], rb[2];
  auto gload = [&](int64_t kb) {
    const int8_t* A = pb + (kb * nRp + (int64_t)ti * TILE) * KBLK;
    const int8_t* Bp = pb + (kb * nRp + (int64_t)tj * TILE) * KBLK;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = t + 256 * e;
      ra[e] = *reinterpret_cast<const v4i*>(A + 16 * q);
      if (!same) rb[e] = *reinterpret_cast<const v4i*>(Bp + 16 * q);
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = t + 256 * e, row = q >> 2, c = q & 3;
      *reinterpret_cast<v4i*>(&lds[buf][0][lds_off_i8(row, c)]) = ra[e];
      if (!same) *reinterpret_cast<v4i*>(&lds[buf][1][lds_off_i8(row, c)]) = rb[e];
    }
  };

  if (nblk > 0) {
    gload(0);
    swrite(0);
    __syncthreads();
    for (int64_t kb = 0; kb < nblk; ++kb) {
      const int cur = (int)(kb & 1);
      if (kb + 1 < nblk) gload(kb + 1);
      const int8_t* As = lds[cur][0];
      const int8_t* Bs = same ? lds[cur][0] : lds[cur][1];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = (l >> 5) + 2 * kk;
        v4i a[2], bb[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int row = 64 * wr + 32 * m + (l & 31);
          a[m] = *reinterpret_cast<const v4i*>(As + lds_off_i8(row, chunk));
        }
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int row = 64 * wc + 32 * n + (l & 31);
          bb[n] = *reinterpret_cast<const v4i*>(Bs + lds_off_i8(row, chunk));
        }
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[m], bb[n], acc[m][n], 0, 0, 0);
      }
      if (kb + 1 < nblk) swrite(cur ^ 1);
      __syncthreads();
    }
  }

  // epilogue: exact-integer centring in fp64, padding rows/cols -> identity
  const double* sc = scal + b * 8;
  const double invN = sc[0], cN = sc[1], invd = sc[2], lam = sc[4];
  const double* ub = u + b * nRp;
  double* Kb = K + b * nRp * nTp;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int64_t gj = (int64_t)tj * TILE + 64 * wc + 32 * n + (l & 31);
      const double uj = ub[gj];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gi = (int64_t)ti * TILE + 64 * wr + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
        double val;
        const bool real_i = (gi < nT) || (gi >= nTp && gi < nTp + nV);
        if (gj >= nT || !real_i) {
          val = (gi == gj) ? 1.0 : 0.0;
        } else {
          val = ((double)acc[m][n][r] - (ub[gi] + uj) * invN + cN) * invd;
          if (gi == gj) val += lam;
        }
        Kb[gi * nTp + gj] = val;
      }
    }
  }
}

hipError_t launch_grm(const int8_t* panel, int64_t panel_stride, const int64_t* off, const double* u,
                      const double* scal, const EvalDims& d, int64_t B, double* K, hipStream_t s) {
  const int64_t tiles_per = (int64_t)d.NT * (d.NT + 1) / 2 + (int64_t)(d.NR - d.NT) * d.NT;
  const int64_t nwg = tiles_per * B;
  hipLaunchKernelGGL(k_grm, dim3((unsigned)nwg), dim3(256), 0, s, panel, panel_stride, off, u, scal, d.nT, d.nTp, d.nV,
                     d.nRp, d.NT, tiles_per, K);
  return hipGetLastError();
}

}  // namespace tblup
