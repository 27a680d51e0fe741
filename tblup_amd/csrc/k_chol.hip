// Batched left-looking tile Cholesky of (K_TT + lambda I), fp64, 128x128 tiles.
//
// Replaces the reference's per-individual dense solves
//   gblup:    G_inv = np.linalg.inv(G_TT + lambda I)          (tblup/evaluator.py:280-284)
//   snp_blup: Ridge(alpha).fit -> scipy.linalg.solve(assume_a="pos") (evaluator.py:311-312,
//             scikit-learn 1.7.2 _ridge.py _solve_cholesky[_kernel])
// by one Cholesky factorisation per individual, batched over the population:
// for each tile column J
//   k_chol_diag    (one WG per individual): T = A_JJ - sum_L L_JL L_JL^T on fp64 MFMA,
//                  in-register right-looking factorisation of T that also produces
//                  inv(L_JJ) (row operations applied to I) and the forward-substitution
//                  block z_J = L_JJ^{-1}(y_J - mu - sum_L L_JL z_L)
//   k_chol_offdiag (one WG per individual x tile row I > J):
//                  T = A_IJ - sum_L L_IL L_JL^T, then L_IJ = T inv(L_JJ)^T, both on MFMA.
// fp64 MFMA: v_mfma_f64_16x16x4_f64, A[i=l&15][k=l>>4], B[k=l>>4][j=l&15],
// C/D row=(l>>4)+4r, col=l&15 (verified on gfx950 by tools/mfma_probe.hip).
#include "tblup_internal.h"

namespace tblup {

namespace {

constexpr int BKD = 16;               // fp64 K step (128 B per row)
constexpr int STAGE = TILE * BKD;     // doubles per operand stage
constexpr int TS = 144;               // row stride (doubles) of the diag kernel's LDS tile

__device__ __forceinline__ int st_off(int row, int k) {
  // [128 rows][16 doubles]; 16-B chunk c=k>>1 of row r stored at c ^ ((r>>1)&7):
  // conflict-free ds_read_b64 for the f64 16x16x4 fragment pattern.
  return row * BKD + 2 * ((k >> 1) ^ ((row >> 1) & 7)) + (k & 1);
}

__device__ __forceinline__ int t_off(int row, int col) {
  // [128][128] doubles, 16-B chunk swizzle by (row & 15): conflict-free A-fragment reads.
  return row * TILE + 2 * ((col >> 1) ^ (row & 15)) + (col & 1);
}

__device__ __forceinline__ v4d mfma64(double a, double b, v4d c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// acc[m][n] += sum_{k < kmax} A[64wr+16m+i][k] * Bm[64wc+16n+j][k]  (row-major, ld)
// 256 threads, double-buffered LDS staging with register prefetch.
// OnStage(buf_ptr, k0) is called by every thread once per staged A panel.
template <bool SAME, typename OnStage>
__device__ __forceinline__ void gemm_nt_f64(const double* __restrict__ A, const double* __restrict__ Bm, int64_t ld,
                                            int kmax, v4d (&acc)[4][4], double* lds, OnStage on_stage) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  double* As0 = lds;
  double* As1 = lds + (SAME ? 1 : 2) * STAGE;
  double* Bs0 = SAME ? As0 : lds + STAGE;
  double* Bs1 = SAME ? As1 : lds + 3 * STAGE;
  v2d ra[4], rb[4];
  const int nst = kmax / BKD;
  if (nst == 0) return;
  auto gload = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 256 * e, r = q >> 3, c = q & 7;
      ra[e] = *reinterpret_cast<const v2d*>(A + (int64_t)r * ld + k0 + 2 * c);
      if (!SAME) rb[e] = *reinterpret_cast<const v2d*>(Bm + (int64_t)r * ld + k0 + 2 * c);
    }
  };
  auto swrite = [&](double* as, double* bs) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 256 * e, r = q >> 3, c = q & 7;
      const int o = r * BKD + 2 * (c ^ ((r >> 1) & 7));
      *reinterpret_cast<v2d*>(as + o) = ra[e];
      if (!SAME) *reinterpret_cast<v2d*>(bs + o) = rb[e];
    }
  };
  gload(0);
  swrite(As0, Bs0);
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const bool odd = (s & 1) != 0;
    const double* As = odd ? As1 : As0;
    const double* Bs = odd ? Bs1 : Bs0;
    if (s + 1 < nst) gload((s + 1) * BKD);
    on_stage(As, s * BKD);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * kk + (l >> 4);
      double a[4], bv[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = As[st_off(64 * wr + 16 * m + (l & 15), k)];
#pragma unroll
      for (int n = 0; n < 4; ++n) bv[n] = Bs[st_off(64 * wc + 16 * n + (l & 15), k)];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma64(a[m], bv[n], acc[m][n]);
    }
    if (s + 1 < nst) swrite(odd ? As0 : As1, odd ? Bs0 : Bs1);
    __syncthreads();
  }
}

struct NoStage {
  __device__ void operator()(const double*, int) const {}
};

struct ElimState {
  double (&v)[8][8];
  double (&rv)[8];
  double (*colbuf)[TILE];
  double (*erow)[TILE];
  double* rbuf;
  double* pivs;
  double* Kb;
  int64_t nTp, j0;
  int t, tr, tc;
};

// Steps j = 16*JB .. 16*JB+15 of the in-register elimination of the diagonal
// tile.  Thread (tr, tc) owns elements (tr + 16a, tc + 16bb); JB is a
// template parameter so every register index is static.  Element (i,c), i >= c:
//   c > j : Schur update  T_ic -= T_ij T_cj / piv_j
//   c == j: becomes E_ij = -T_ij/piv_j (i > j) or 1 (i == j)   [E = L'^{-1}]
//   c < j : E_ic -= (T_ij/piv_j) E_jc
// L column j (= T_ij / sqrt(piv_j)) is written to K as it is published; the
// right-hand side r is eliminated alongside (forward substitution).
template <int JB>
__device__ __forceinline__ void elim_block(ElimState& S) {
  double(&v)[8][8] = S.v;
  double(&rv)[8] = S.rv;
  const int tr = S.tr, tc = S.tc;
  for (int jj = 0; jj < 16; ++jj) {
    const int j = 16 * JB + jj;
    const int buf = j & 1;
    if (tc == jj) {
#pragma unroll
      for (int a = JB; a < 8; ++a) {
        const int i = tr + 16 * a;
        if (i >= j) S.colbuf[buf][i] = v[a][JB];
      }
    }
    if (tr == jj) {
#pragma unroll
      for (int bb = 0; bb <= JB; ++bb) {
        const int c = tc + 16 * bb;
        if (c < j) S.erow[buf][c] = v[JB][bb];
      }
      if (tc == 15) S.rbuf[buf] = rv[JB];
    }
    __syncthreads();
    const double piv = S.colbuf[buf][j];
    const double ip = 1.0 / piv;
    const double rj = S.rbuf[buf];
    if (S.t == 0) S.pivs[j] = piv;
    if (tc == jj) {
      const double rs = 1.0 / sqrt(piv);
#pragma unroll
      for (int a = JB; a < 8; ++a) {
        const int i = tr + 16 * a;
        if (i >= j) S.Kb[(S.j0 + i) * S.nTp + S.j0 + j] = v[a][JB] * rs;
      }
    }
#pragma unroll
    for (int a = JB; a < 8; ++a) {
      const int i = tr + 16 * a;
      const double li = (i >= j) ? S.colbuf[buf][i] * ip : 0.0;
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        const int c = tc + 16 * bb;
        if (bb > JB) {
          if (i >= c) v[a][bb] -= li * S.colbuf[buf][c];
        } else if (bb == JB) {
          if (c > j) {
            if (i >= c) v[a][bb] -= li * S.colbuf[buf][c];
          } else if (c == j) {
            if (i >= j) v[a][bb] = (i == j) ? 1.0 : -li;
          } else {
            if (i > j) v[a][bb] -= li * S.erow[buf][c];
          }
        } else {
          if (i > j) v[a][bb] -= li * S.erow[buf][c];
        }
      }
      if (tc == 15 && i > j) rv[a] -= li * rj;
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// diagonal tile: SYRK update, factorisation, inverse and forward substitution
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_chol_diag(double* __restrict__ K, int64_t nTp, int64_t nT, int64_t mstride,
                                                   int J, double* __restrict__ Dinv, double* __restrict__ z,
                                                   const double* __restrict__ yT, const double* __restrict__ scal) {
  __shared__ __attribute__((aligned(16))) double lds[TILE * TS];  // 144 KiB: staging, then the T tile
  __shared__ double colbuf[2][TILE], erow[2][TILE], rbuf[2], pivs[TILE], rsh[TILE], wsh[TILE];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int64_t b = blockIdx.x;
  double* Kb = K + b * mstride;
  const int64_t j0 = (int64_t)J * TILE;
  const double* zb = z + b * nTp;
  const double mu = scal[b * 8 + 3];

  v4d acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = v4d{0.0, 0.0, 0.0, 0.0};

  // forward-substitution partial sums w_i = sum_{k<j0} L[j0+i][k] z[k], fused into the staging loop
  double wpart = 0.0;
  auto on_stage = [&](const double* As, int k0) {
    if (t < TILE) {
#pragma unroll
      for (int kk = 0; kk < BKD; ++kk) wpart += As[st_off(t, kk)] * zb[k0 + kk];
    }
  };
  if (J > 0) gemm_nt_f64<true>(Kb + j0 * nTp, Kb + j0 * nTp, nTp, (int)j0, acc, lds, on_stage);
  __syncthreads();

  // T = A_JJ - acc  -> LDS (stride TS); r = y_J - mu - w
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 64 * wr + 16 * m + (l >> 4) + 4 * r, col = 64 * wc + 16 * n + (l & 15);
        lds[row * TS + col] = Kb[(j0 + row) * nTp + j0 + col] - acc[m][n][r];
      }
  if (t < TILE) {
    const int64_t gi = j0 + t;
    wsh[t] = wpart;
    rsh[t] = (gi < nT) ? (yT[gi] - mu - wpart) : 0.0;
  }
  __syncthreads();

  // ownership: thread (tr, tc) holds elements (tr + 16a, tc + 16bb)
  const int tr = t >> 4, tc = t & 15;
  double v[8][8];
  double rv[8];
#pragma unroll
  for (int a = 0; a < 8; ++a) {
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) v[a][bb] = lds[(tr + 16 * a) * TS + tc + 16 * bb];
    rv[a] = rsh[tr + 16 * a];
  }

  // Right-looking elimination with unscaled pivots (see elim_block).
  ElimState st{v, rv, colbuf, erow, rbuf, pivs, Kb, nTp, j0, t, tr, tc};
  elim_block<0>(st);
  elim_block<1>(st);
  elim_block<2>(st);
  elim_block<3>(st);
  elim_block<4>(st);
  elim_block<5>(st);
  elim_block<6>(st);
  elim_block<7>(st);
  __syncthreads();

  // X = L^{-1} = D^{-1/2} E ; z_J = D^{-1/2} r
  double* Db = Dinv + (b * (nTp / TILE) + J) * (int64_t)(TILE * TILE);
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int i = tr + 16 * a;
    const double rs = 1.0 / sqrt(pivs[i]);
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) {
      const int c = tc + 16 * bb;
      Db[i * TILE + c] = (i >= c) ? v[a][bb] * rs : 0.0;
    }
    if (tc == 15) z[b * nTp + j0 + i] = rv[a] * rs;
  }
}

hipError_t launch_chol_diag(double* K, const EvalDims& d, int64_t B, int J, double* Dinv, double* z,
                            const double* yT, const double* scal, hipStream_t s) {
  hipLaunchKernelGGL(k_chol_diag, dim3((unsigned)B), dim3(256), 0, s, K, d.nTp, d.nT, d.nRp * d.nTp, J, Dinv, z, yT,
                     scal);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// off-diagonal tiles of column J: L_IJ = (A_IJ - sum_L L_IL L_JL^T) inv(L_JJ)^T
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_chol_offdiag(double* __restrict__ K, int64_t nTp, int64_t mstride, int J,
                                                      int NT, const double* __restrict__ Dinv) {
  __shared__ __attribute__((aligned(16))) double lds[TILE * TILE + STAGE];  // T tile + X stage (144 KiB)
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int nI = NT - J - 1;
  const int64_t logical = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t b = logical / nI;
  const int I = J + 1 + (int)(logical % nI);
  double* Kb = K + b * mstride;
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)J * TILE;

  v4d acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = v4d{0.0, 0.0, 0.0, 0.0};
  if (J > 0) gemm_nt_f64<false>(Kb + i0 * nTp, Kb + j0 * nTp, nTp, (int)j0, acc, lds, NoStage{});
  __syncthreads();

  double* Tl = lds;
  double* Xs = lds + TILE * TILE;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 64 * wr + 16 * m + (l >> 4) + 4 * r, col = 64 * wc + 16 * n + (l & 15);
        Tl[t_off(row, col)] = Kb[(i0 + row) * nTp + j0 + col] - acc[m][n][r];
        acc[m][n][r] = 0.0;
      }

  // out[i][j] = sum_c T[i][c] X[j][c], X = inv(L_JJ) lower triangular (X[j][c] = 0 for c > j)
  const double* X = Dinv + (b * NT + J) * (int64_t)(TILE * TILE);
  v2d rx[4];
  auto gload = [&](int s) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 256 * e, r = q >> 3, c = q & 7;
      rx[e] = *reinterpret_cast<const v2d*>(X + r * TILE + s * BKD + 2 * c);
    }
  };
  gload(0);
  for (int s = 0; s < TILE / BKD; ++s) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 256 * e, r = q >> 3, c = q & 7;
      *reinterpret_cast<v2d*>(Xs + r * BKD + 2 * (c ^ ((r >> 1) & 7))) = rx[e];
    }
    __syncthreads();
    if (s + 1 < TILE / BKD) gload(s + 1);
    if (wc == 1 || s < (TILE / BKD) / 2) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = 4 * kk + (l >> 4);
        double a[4], bv[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = Tl[t_off(64 * wr + 16 * m + (l & 15), s * BKD + k)];
#pragma unroll
        for (int n = 0; n < 4; ++n) bv[n] = Xs[st_off(64 * wc + 16 * n + (l & 15), k)];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[m][n] = mfma64(a[m], bv[n], acc[m][n]);
      }
    }
  }

#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 64 * wr + 16 * m + (l >> 4) + 4 * r, col = 64 * wc + 16 * n + (l & 15);
        Kb[(i0 + row) * nTp + j0 + col] = acc[m][n][r];
      }
}

hipError_t launch_chol_offdiag(double* K, const EvalDims& d, int64_t B, int J, const double* Dinv, hipStream_t s) {
  const int nI = d.NT - J - 1;
  if (nI <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_chol_offdiag, dim3((unsigned)(B * nI)), dim3(256), 0, s, K, d.nTp, d.nRp * d.nTp, J, d.NT,
                     Dinv);
  return hipGetLastError();
}

}  // namespace tblup
