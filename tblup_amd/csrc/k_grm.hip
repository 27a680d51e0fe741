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
// panel (one 128x64 operand tile = 128 packed 16-B row blocks, unpacked into LDS).  Only the tiles the
// Cholesky and the prediction read are computed: the TT lower triangle
// (diagonal tiles in full) and the VT block.  Workgroups of one individual are
// kept on one XCD (xcd_remap) so the individual's panel is re-read from L2.
#include "i8_tile.h"

namespace tblup {

__global__ __launch_bounds__(256) void k_grm(const uint8_t* __restrict__ panel, int64_t panel_stride, int64_t pk_row,
                                             const int64_t* __restrict__ off, const double* __restrict__ u,
                                             const double* __restrict__ scal, int64_t nT, int64_t nTp, int64_t nV,
                                             int64_t nRp, int NT, int64_t tiles_per, double* __restrict__ K) {
  __shared__ __attribute__((aligned(16))) int8_t lds[4 * TILE * KBLK];
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
  const int64_t k = off[b + 1] - off[b];
  const uint8_t* pb = panel + b * panel_stride;
  v16i acc[2][2];
  i8_tile_gemm(pb + (int64_t)ti * TILE * pk_row, pb + (int64_t)tj * TILE * pk_row, ti == tj, (k + KBLK - 1) / KBLK,
               pk_row, lds, acc);

  // epilogue: exact-integer centring in fp64, padding rows/cols -> identity
  const double* sc = scal + b * SCAL;
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

hipError_t launch_grm(const uint8_t* panel, int64_t panel_stride, int64_t pk_row, const int64_t* off, const double* u,
                      const double* scal, const EvalDims& d, int64_t B, double* K, hipStream_t s) {
  const int64_t tiles_per = (int64_t)d.NT * (d.NT + 1) / 2 + (int64_t)(d.NR - d.NT) * d.NT;
  const int64_t nwg = tiles_per * B;
  hipLaunchKernelGGL(k_grm, dim3((unsigned)nwg), dim3(256), 0, s, panel, panel_stride, pk_row, off, u, scal, d.nT, d.nTp, d.nV,
                     d.nRp, d.NT, tiles_per, K);
  return hipGetLastError();
}

}  // namespace tblup
