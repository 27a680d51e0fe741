// Per-individual scalars of one system, for one 256-thread workgroup: k_indiv_stats (k_prep.hip) and
// the SNP-form launch that forms K_JJ + lambda I of the tiles J < 2 after k_sys_tiles_st
// (k_stats_diag_counts, k_chol.hip) run this same code, so the scalars are the same bits either way.
//
// Reference behaviour restated (ianwhale/tblup): allele frequency p = column mean / 2 over ALL rows for
// gblup (utils.py:14 via evaluator.py:275) and over TRAIN rows for snp_blup (evaluator.py:304);
// d = 2 sum p(1-p) (utils.py:18, evaluator.py:305); lambda = (1-h2)/h2 (evaluator.py:277).
#pragma once
#include "tblup_internal.h"

namespace tblup {

constexpr int STATS_THREADS = 256;

// LDS of stats_wg
struct StatsShared {
  int64_t r1[STATS_THREADS / 64], r2[STATS_THREADS / 64];   // per-wave partial sums
  double sc[SCAL];
};

// Individual (system) b: branch, 1/N, q/N^2, 1/d, mu flag, lambda ... into sh.sc (every thread reads
// them after the call) and, scal != null, into scal[b].  An index outside [-P, P) sets *err (vector
// store; every writer stores 1) and SC_BAD.
__device__ __forceinline__ void stats_wg(const int64_t* __restrict__ idx, const int64_t* __restrict__ off,
                                         const FoldTab& ft, const int32_t* __restrict__ csA, int64_t n, int64_t nT,
                                         int64_t nTp, int64_t P, int form, int64_t ns, int pad_first, int nt,
                                         int branch, double h2, int64_t b, double* __restrict__ scal,
                                         int32_t* __restrict__ err, StatsShared& sh) {
  const int t = threadIdx.x;
  const int64_t o0 = off[b], k = off[b + 1] - o0;
  const int32_t* __restrict__ csT = ft.csT[fold_of(ft, b)];   // the system's split
  int mode = branch;
  if (mode == 0) mode = (k > n) ? 1 : 2;  // evaluator.py:257
  const int32_t* cs = (mode == 1) ? csA : csT;
  const bool primal = form == FORM_PRIMAL;   // snp branch only (host guarantees)
  int64_t m1 = 0, q = 0;
  int bad = 0;
  for (int64_t s = t; s < k; s += STATS_THREADS) {
    const int64_t p = idx[o0 + s];
    bad |= (p < -P || p >= P);
    const int64_t m = cs[snp_col(p, P)];
    m1 += m;
    q += m * m;
  }
  // exact integer sums: wave shuffles, then the four waves' partials through LDS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m1 += __shfl_xor(m1, o);
    q += __shfl_xor(q, o);
  }
  if ((t & 63) == 0) {
    sh.r1[t >> 6] = m1;
    sh.r2[t >> 6] = q;
  }
  const int any_bad = __syncthreads_or(bad);
  if (any_bad && t == 0) *err = 1;
  if (t == 0) {
    int64_t s1 = 0, s2 = 0;
    for (int w = 0; w < STATS_THREADS / 64; ++w) {
      s1 += sh.r1[w];
      s2 += sh.r2[w];
    }
    const double N = (mode == 1) ? (double)n : (double)nT;
    const double M1 = (double)s1, Q = (double)s2;
    const double d = M1 / N - Q / (2.0 * N * N);  // 2 sum p(1-p)
    double* sc = sh.sc;
    // primal (SNP-space) form: C_ab = (X^T X)_ab - s_a s_b / n_T over train rows
    sc[SC_SA] = primal ? 0.0 : 1.0 / N;
    sc[SC_CN] = primal ? 0.0 : Q / (N * N);
    sc[SC_INVD] = 1.0 / d;
    sc[SC_MUF] = (mode == 2) ? 1.0 : 0.0;
    sc[SC_LAM] = (1.0 - h2) / h2;
    sc[SC_D] = d;
    sc[SC_MODE] = (double)mode;
    sc[SC_K] = (double)k;
    sc[SC_SM] = primal ? 1.0 / (double)nT : 0.0;
    sc[SC_NROW] = primal ? (double)k : (double)nT;
    sc[SC_CBLK] = primal ? (double)(nTp / KBLK) : (double)((k + KBLK - 1) / KBLK);
    sc[SC_BAD] = any_bad ? 1.0 : 0.0;
    sc[SC_PAD] = (primal && pad_first) ? (double)(ns - k) : 0.0;
    for (int e = SC_PAD + 1; e < SCAL; ++e) sc[e] = 0.0;
  }
  __syncthreads();
  if (scal && t < SCAL && t <= SC_PAD) scal[b * SCAL + t] = sh.sc[t];
}

// Primal form, after stats_wg: u[b][a] = s_a and rhs[b][t][a] = xty[t][p_a] / d over the system rows
// a0 <= a < a1 (zero on padding rows)
__device__ __forceinline__ void stats_rows(const int64_t* __restrict__ idx, const int64_t* __restrict__ off,
                                           const FoldTab& ft, int64_t P, int64_t ns, int pad_first, int nt,
                                           int64_t b, double* __restrict__ u, double* __restrict__ rhs,
                                           const StatsShared& sh, int64_t a0, int64_t a1) {
  const int t = threadIdx.x;
  const int64_t o0 = off[b], k = off[b + 1] - o0;
  const int32_t* __restrict__ csT = ft.csT[fold_of(ft, b)];
  const double* __restrict__ xty = ft.xty[fold_of(ft, b)];
  // u_a = s_a (train allele count), rhs_ta = X_c^T (y_T,t - mu_t) / d = xty[t][p_a] / d
  // (the sklearn primal right-hand side in 1/d units); zero on padding rows (system row a holds
  // selected SNP a - pad)
  const double invd = sh.sc[SC_INVD];
  const int64_t pad = pad_first ? ns - k : 0;
  for (int64_t a = a0 + t; a < a1; a += STATS_THREADS) {
    const bool real = sys_real(a, pad, k);
    const int64_t p = real ? snp_col(idx[o0 + a - pad], P) : 0;
    u[b * ns + a] = real ? (double)csT[p] : 0.0;
    for (int tr = 0; tr < nt; ++tr) rhs[(b * nt + tr) * ns + a] = real ? xty[tr * P + p] * invd : 0.0;
  }
}

}  // namespace tblup
