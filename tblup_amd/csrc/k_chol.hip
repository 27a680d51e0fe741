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
#include "i8_tile.h"

namespace tblup {

namespace {

constexpr int BKD = 16;               // fp64 K step (128 B per row)
constexpr int STAGE = TILE * BKD;     // doubles per operand stage

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
template <bool SAME, typename OnStage, bool NEG_A = false>
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
      *reinterpret_cast<v2d*>(as + o) = NEG_A ? -ra[e] : ra[e];
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

// ---- SYRK restricted to the 36 lower 16x16 blocks of a 128x128 tile ----
// Block e (row-major over q >= s) goes to wave e % 4: 9 blocks per wave, so the
// lower triangle costs 36 block-MFMA streams instead of the 64 of a full GEMM.
__host__ __device__ constexpr int tri_q(int e) {
  int q = 0;
  while ((q + 1) * (q + 2) / 2 <= e) ++q;
  return q;
}
__host__ __device__ constexpr int tri_s(int e) { return e - tri_q(e) * (tri_q(e) + 1) / 2; }

template <int W>
__device__ __forceinline__ void syrk_stage(const double* As, v4d (&acc)[9], int l) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 4 * kk + (l >> 4);
    double a8[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) a8[q] = As[st_off(16 * q + (l & 15), k)];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int e = W + 4 * i;
      acc[i] = mfma64(a8[tri_q(e)], a8[tri_s(e)], acc[i]);
    }
  }
}

// acc[i] (block e = w + 4i) += sum_{k < kmax} A[16q + r][k] A[16s + c][k]; staging as gemm_nt_f64<true>.
template <typename OnStage>
__device__ __forceinline__ void syrk_lower_f64(const double* __restrict__ A, int64_t ld, int kmax, v4d (&acc)[9],
                                               double* lds, OnStage on_stage) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  double* As0 = lds;
  double* As1 = lds + STAGE;
  v2d ra[4];
  const int nst = kmax / BKD;
  if (nst == 0) return;
  auto gload = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 256 * e, r = q >> 3, c = q & 7;
      ra[e] = *reinterpret_cast<const v2d*>(A + (int64_t)r * ld + k0 + 2 * c);
    }
  };
  auto swrite = [&](double* as) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 256 * e, r = q >> 3, c = q & 7;
      *reinterpret_cast<v2d*>(as + r * BKD + 2 * (c ^ ((r >> 1) & 7))) = ra[e];
    }
  };
  gload(0);
  swrite(As0);
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    const bool odd = (s & 1) != 0;
    const double* As = odd ? As1 : As0;
    if (s + 1 < nst) gload((s + 1) * BKD);
    on_stage(As, s * BKD);
    if (w == 0) syrk_stage<0>(As, acc, l);
    else if (w == 1) syrk_stage<1>(As, acc, l);
    else if (w == 2) syrk_stage<2>(As, acc, l);
    else syrk_stage<3>(As, acc, l);
    if (s + 1 < nst) swrite(odd ? As0 : As1);
    __syncthreads();
  }
}

// ---- packed lower-triangular 16x16 block storage of a 128x128 tile in LDS ----
constexpr int NB = 16;                       // base block edge
constexpr int NBLK = TILE / NB;              // 8 block rows
constexpr int NPACK = NBLK * (NBLK + 1) / 2; // 36 lower blocks
constexpr int BLKD = NB * NB;                // doubles per block

__device__ __forceinline__ int pk(int q, int s) { return (q * (q + 1) / 2 + s) * BLKD; }
// element (r, c) of a 16x16 block; 16-B chunk swizzle makes the fragment reads conflict-free
__device__ __forceinline__ int bo(int r, int c) { return r * NB + 2 * ((c >> 1) ^ ((r >> 1) & 7)) + (c & 1); }

// acc (16x16, f64 MFMA C layout) += A(16x16) * B(16x16)^T, both blocks in LDS
__device__ __forceinline__ v4d mma_abt(const double* A, const double* Bt, v4d acc, int l) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 4 * kk + (l >> 4);
    acc = mfma64(A[bo(l & 15, k)], Bt[bo(l & 15, k)], acc);
  }
  return acc;
}

// Factor the 16x16 SPD block D in place with ONE wave (no barriers): D <- L (lower),
// X <- L^{-1} (lower, zeros above).  Lane l holds row i = l&15, columns 4g..4g+3
// (g = l>>4).  Right-looking elimination with unscaled pivots; a column, once
// eliminated, turns into the matching column of E = L'^{-1} (row operations on I):
//   c > j : T_ic -= T_ij T_cj / piv_j
//   c == j: E_ij = -T_ij / piv_j (i > j), 1 (i == j)
//   c < j : E_ic -= (T_ij / piv_j) E_jc
// L = L' D^{1/2}  ->  L_ij = T_ij / sqrt(piv_j);  X = D^{-1/2} E.
__device__ __forceinline__ void factor16(double* D, double* X, int l) {
  const int i = l & 15, g = l >> 4;
  double v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = D[bo(i, 4 * g + q)];
  double piv_own = 1.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int jg = j >> 2, jq = j & 3;
    const double ci = __shfl(v[jq], i + 16 * jg);
    const double piv = __shfl(v[jq], j + 16 * jg);
    double cc[4], ej[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cc[q] = __shfl(v[jq], 4 * g + q + 16 * jg);
      ej[q] = __shfl(v[q], j + 16 * g);
    }
    if (g == jg && i >= j) D[bo(i, j)] = ci / sqrt(piv);
    if (i == j) piv_own = piv;
    const double li = ci / piv;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * g + q;
      if (c > j) {
        if (i >= c) v[q] -= li * cc[q];
      } else if (c == j) {
        if (i >= j) v[q] = (i == j) ? 1.0 : -li;
      } else {
        if (i > j) v[q] -= li * ej[q];
      }
    }
  }
  const double rs = 1.0 / sqrt(piv_own);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * g + q;
    X[bo(i, c)] = (i >= c) ? v[q] * rs : 0.0;
  }
}

}  // namespace

// Per-launch arguments shared by the two Cholesky kernels.
struct CholArgs {
  double* L;                // [B][nTp][nTp] factor (TT lower tiles)
  double* Dinv;             // [B][NT][128][128]
  double* z;                // [B][nTp]
  const double* yT;         // [nTp]
  const int8_t* panel;      // [B] x pstride
  int64_t pstride;
  const int64_t* off;       // [B+1]
  const double* u;          // [B][nRp]
  const double* scal;       // [B][8]
  int64_t nT, nTp, nRp;
  int NT, J;
  int skip;                 // diagnostic ablation mask (TBLUP_DBG_SKIP); 0 in production
};

// ---------------------------------------------------------------------------
// diagonal tile: fused GRM tile, SYRK update, blocked factorisation, blocked
// inverse, forward solve
// ---------------------------------------------------------------------------
//   0. K_JJ from the panel on int8 MFMA (exact counts + fp64 centring) -> packed lower blocks
//   A. acc = sum_{L<J} L_JL L_JL^T (fp64 MFMA), w = sum_{L<J} L_JL z_L (fused)
//   B. T = K_JJ - acc (in place, packed lower 16x16 blocks); r = y_J - mu - w
//   C. for panel p: one wave factors T_pp (-> L_pp, X_pp = L_pp^{-1});
//      all waves: L_qp = T_qp X_pp^T (q > p); T_qs -= L_qp L_sp^T (q >= s > p)   [MFMA]
//   D. blocked inverse X = L^{-1}: X_{j+d,j} = -X_{j+d,j+d} sum_{l=j}^{j+d-1} L_{j+d,l} X_{l,j}
//   E. write L (lower blocks), X to Dinv (zeros above the diagonal), z_J = X r
__global__ __launch_bounds__(256) void k_chol_diag(CholArgs a) {
  __shared__ __attribute__((aligned(16))) double lds[2 * NPACK * BLKD];  // 144 KiB: T blocks | X blocks (+staging)
  __shared__ double rsh[TILE];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int64_t b = blockIdx.x, nTp = a.nTp;
  const int J = a.J;
  double* Lb = a.L + b * nTp * nTp;
  const int64_t j0 = (int64_t)J * TILE;
  const double* zb = a.z + b * nTp;
  const double* sc = a.scal + b * 8;
  const double invN = sc[0], cN = sc[1], invd = sc[2], mu = sc[3], lam = sc[4];
  const double* ub = a.u + b * a.nRp;
  double* Tp = lds;
  double* Xp = lds + NPACK * BLKD;   // also the staging area of steps 0 and A

  // 0. fused GRM tile K_JJ (lower 16x16 blocks only)
  if (!(a.skip & 1)) {
    const int64_t k = a.off[b + 1] - a.off[b];
    const int8_t* pj = a.panel + b * a.pstride + j0 * KBLK;
    v16i ci[2][2];
    i8_tile_gemm_ring<true, 8>(pj, pj, (k + KBLK - 1) / KBLK, a.nRp * KBLK, reinterpret_cast<int8_t*>(Xp), ci);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = i8_col(wc, n, l);
        const int64_t gj = j0 + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = i8_row(wr, m, r, l);
          if ((row >> 4) >= (col >> 4)) {
            const int64_t gi = j0 + row;
            double v;
            if (gi < a.nT && gj < a.nT) {
              v = grm_value(ci[m][n][r], ub[gi], ub[gj], invN, cN, invd);
              if (gi == gj) v += lam;
            } else {
              v = (gi == gj) ? 1.0 : 0.0;
            }
            Tp[pk(row >> 4, col >> 4) + bo(row & 15, col & 15)] = v;
          }
        }
      }
  }

  v4d acc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] = v4d{0.0, 0.0, 0.0, 0.0};
  double wpart = 0.0;
  auto on_stage = [&](const double* As, int k0) {
    if (t < TILE) {
#pragma unroll
      for (int kk = 0; kk < BKD; ++kk) wpart += As[st_off(t, kk)] * zb[k0 + kk];
    }
  };
  __syncthreads();
  if (J > 0 && !(a.skip & 2)) syrk_lower_f64(Lb + j0 * nTp, nTp, (int)j0, acc, Xp, on_stage);

  // B. T = K_JJ - acc on the lower blocks (wave w holds blocks e = w + 4i)
  if (J > 0) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int e = w + 4 * i, q = tri_q(e), sb = tri_s(e);
#pragma unroll
      for (int r = 0; r < 4; ++r) Tp[pk(q, sb) + bo((l >> 4) + 4 * r, l & 15)] -= acc[i][r];
    }
  }
  if (t < TILE) {
    const int64_t gi = j0 + t;
    rsh[t] = (gi < a.nT) ? (a.yT[gi] - mu - wpart) : 0.0;
  }
  __syncthreads();

  // C. blocked right-looking factorisation over 16-column panels
  for (int p = 0; p < ((a.skip & 4) ? 0 : NBLK); ++p) {
    if (w == 0 && !(a.skip & 256)) factor16(Tp + pk(p, p), Xp + pk(p, p), l);
    __syncthreads();
    for (int q = p + 1 + w; q < ((a.skip & 512) ? 0 : NBLK); q += 4) {
      v4d x = {0.0, 0.0, 0.0, 0.0};
      x = mma_abt(Tp + pk(q, p), Xp + pk(p, p), x, l);
#pragma unroll
      for (int r = 0; r < 4; ++r) Tp[pk(q, p) + bo((l >> 4) + 4 * r, l & 15)] = x[r];
    }
    __syncthreads();
    const int nb = NBLK - 1 - p;
    for (int e = w; e < ((a.skip & 512) ? 0 : nb * (nb + 1) / 2); e += 4) {
      int qq = 0;
      while ((qq + 1) * (qq + 2) / 2 <= e) ++qq;
      const int q = p + 1 + qq, sb = p + 1 + (e - qq * (qq + 1) / 2);
      v4d x = {0.0, 0.0, 0.0, 0.0};
      x = mma_abt(Tp + pk(q, p), Tp + pk(sb, p), x, l);
      double* dst = Tp + pk(q, sb);
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[bo((l >> 4) + 4 * r, l & 15)] -= x[r];
    }
    __syncthreads();
  }

  // D. blocked inverse, one block diagonal per round
  for (int dd = 1; dd < ((a.skip & 8) ? 0 : NBLK); ++dd) {
    for (int jb = w; jb + dd < NBLK; jb += 4) {
      const int q = jb + dd;
      v4d sacc = {0.0, 0.0, 0.0, 0.0};
      for (int lb = jb; lb < q; ++lb) {
        const double* A = Tp + pk(q, lb);
        const double* Xb = Xp + pk(lb, jb);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = 4 * kk + (l >> 4);
          sacc = mfma64(A[bo(l & 15, k)], Xb[bo(k, l & 15)], sacc);
        }
      }
      // X_{q,jb} = -X_{q,q} S ; S in C layout feeds the B operand directly (k = 4kk + (l>>4))
      v4d xo = {0.0, 0.0, 0.0, 0.0};
      const double* Xqq = Xp + pk(q, q);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) xo = mfma64(Xqq[bo(l & 15, 4 * kk + (l >> 4))], sacc[kk], xo);
#pragma unroll
      for (int r = 0; r < 4; ++r) Xp[pk(q, jb) + bo((l >> 4) + 4 * r, l & 15)] = -xo[r];
    }
    __syncthreads();
  }

  // E. outputs
  double* Db = a.Dinv + (b * a.NT + J) * (int64_t)(TILE * TILE);
  if (a.skip & 16) return;
  for (int e = t; e < TILE * TILE; e += 256) {
    const int rr = e >> 7, cc = e & 127, q = rr >> 4, sb = cc >> 4;
    double xv = 0.0;
    if (q >= sb) {
      xv = Xp[pk(q, sb) + bo(rr & 15, cc & 15)];
      if (rr >= cc) Lb[(j0 + rr) * nTp + j0 + cc] = Tp[pk(q, sb) + bo(rr & 15, cc & 15)];
    }
    Db[e] = xv;
  }
  if (t < TILE) {
    const int q = t >> 4;
    double acc_z = 0.0;
    for (int sb = 0; sb <= q; ++sb) {
      const double* Xb = Xp + pk(q, sb);
#pragma unroll
      for (int c = 0; c < NB; ++c) acc_z += Xb[bo(t & 15, c)] * rsh[16 * sb + c];
    }
    a.z[b * nTp + j0 + t] = acc_z;
  }
}

// ---------------------------------------------------------------------------
// off-diagonal tiles of column J: L_IJ = (K_IJ - sum_L L_IL L_JL^T) inv(L_JJ)^T
//   0. K_IJ from the panel (int8 MFMA) -> fp64 image in LDS -> accumulators
//   1. acc -= sum_L L_IL L_JL^T (fp64 MFMA, A operand negated at staging)
//   2. L_IJ = T X^T with X = inv(L_JJ) lower triangular (fp64 MFMA)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_chol_offdiag(CholArgs a) {
  __shared__ __attribute__((aligned(16))) double lds[TILE * TILE + STAGE];  // T image + X stage (144 KiB)
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wr = w >> 1, wc = w & 1;
  const int J = a.J, NT = a.NT;
  const int nI = NT - J - 1;
  const int64_t logical = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t b = logical / nI;
  const int I = J + 1 + (int)(logical % nI);
  const int64_t nTp = a.nTp;
  double* Lb = a.L + b * nTp * nTp;
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)J * TILE;
  double* Tl = lds;
  double* Xs = lds + TILE * TILE;

  // 0. fused GRM tile
  if (!(a.skip & 32)) {
    const int64_t k = a.off[b + 1] - a.off[b];
    const int8_t* pb = a.panel + b * a.pstride;
    v16i ci[2][2];
    i8_tile_gemm_ring<false, 8>(pb + i0 * KBLK, pb + j0 * KBLK, (k + KBLK - 1) / KBLK, a.nRp * KBLK,
                                reinterpret_cast<int8_t*>(lds), ci);
    const double* sc = a.scal + b * 8;
    const double invN = sc[0], cN = sc[1], invd = sc[2];
    const double* ub = a.u + b * a.nRp;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = i8_col(wc, n, l);
        const int64_t gj = j0 + col;
        const double uj = ub[gj];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = i8_row(wr, m, r, l);
          const int64_t gi = i0 + row;
          Tl[t_off(row, col)] = (gi < a.nT && gj < a.nT) ? grm_value(ci[m][n][r], ub[gi], uj, invN, cN, invd) : 0.0;
        }
      }
  }
  __syncthreads();
  v4d acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[m][n][r] = Tl[t_off(64 * wr + 16 * m + (l >> 4) + 4 * r, 64 * wc + 16 * n + (l & 15))];
  __syncthreads();
  if (J > 0 && !(a.skip & 64)) gemm_nt_f64<false, NoStage, true>(Lb + i0 * nTp, Lb + j0 * nTp, nTp, (int)j0, acc, lds, NoStage{});
  __syncthreads();

#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 64 * wr + 16 * m + (l >> 4) + 4 * r, col = 64 * wc + 16 * n + (l & 15);
        Tl[t_off(row, col)] = acc[m][n][r];
        acc[m][n][r] = 0.0;
      }

  // out[i][j] = sum_c T[i][c] X[j][c], X = inv(L_JJ) lower triangular (X[j][c] = 0 for c > j)
  const double* X = a.Dinv + (b * NT + J) * (int64_t)(TILE * TILE);
  v2d rx[4];
  auto gload = [&](int s) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 256 * e, r = q >> 3, c = q & 7;
      rx[e] = *reinterpret_cast<const v2d*>(X + r * TILE + s * BKD + 2 * c);
    }
  };
  gload(0);
  for (int s = 0; s < ((a.skip & 128) ? 0 : TILE / BKD); ++s) {
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
        double av[4], bv[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) av[m] = Tl[t_off(64 * wr + 16 * m + (l & 15), s * BKD + k)];
#pragma unroll
        for (int n = 0; n < 4; ++n) bv[n] = Xs[st_off(64 * wc + 16 * n + (l & 15), k)];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[m][n] = mfma64(av[m], bv[n], acc[m][n]);
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
        Lb[(i0 + row) * nTp + j0 + col] = acc[m][n][r];
      }
}

hipError_t launch_chol(const CholLaunch& c, int J, hipStream_t s, bool diag) {
  CholArgs a{c.L, c.Dinv, c.z, c.yT, c.panel, c.pstride, c.off, c.u, c.scal, c.d.nT, c.d.nTp, c.d.nRp, c.d.NT, J,
             c.skip};
  if (diag) {
    hipLaunchKernelGGL(k_chol_diag, dim3((unsigned)c.B), dim3(256), 0, s, a);
  } else {
    const int nI = c.d.NT - J - 1;
    if (nI <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_chol_offdiag, dim3((unsigned)(c.B * nI)), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace tblup
