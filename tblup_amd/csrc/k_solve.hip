// Back substitution, prediction and fitness, one 1024-thread workgroup per individual.
//
//   alpha = L^{-T} z                       (z = L^{-1} rhs from k_chol_diag)
//   dual:   EBV_V = K_VT alpha + mu, K_VT applied in factored form from the packed panel
//                                          gblup: evaluator.py:284 (G[:,T] Ginv y_T, mu = 0)
//                                          snp:   evaluator.py:314 (clf.predict, intercept mean(y_T))
//   primal: EBV_V = (X_V - 2p) beta + mean(y_T), beta = alpha (sklearn primal Ridge coef_)
//   fitness = |pearsonr(EBV_V, y_V)|       evaluator.py:286 / :314, scipy 1.15.3 pearsonr
//            (multi-trait, BASELINE config 5: the mean over traits of |r|; build-defined):
//            exact-equality constant input -> NaN; mean-centre; max-abs scaled
//            norms; clip to [-1, 1]; round when n == 2.
#include "tblup_internal.h"

namespace tblup {

namespace {

constexpr int NTH = 1024;

template <int NTH_ = NTH>
__device__ __forceinline__ double block_sum(double v, double* red) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NTH_ / 64; ++i) s += red[i];
  return s;
}

template <int NTH_ = NTH>
__device__ __forceinline__ double block_max(double v, double* red) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < NTH_ / 64; ++i) s = fmax(s, red[i]);
  return s;
}

// N sums (max: N maxima) in one pass: each component reduced exactly as block_sum / block_max
// reduce it alone (red: N x 16 slots)
template <int NTH_, int N, bool MAX>
__device__ __forceinline__ void block_reduce(double (&v)[N], double* red) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] = MAX ? fmax(v[k], __shfl_xor(v[k], o)) : v[k] + __shfl_xor(v[k], o);
  __syncthreads();
  if (l == 0)
#pragma unroll
    for (int k = 0; k < N; ++k) red[k * 16 + w] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    double s = MAX ? red[k * 16] : 0.0;
#pragma unroll
    for (int i = MAX ? 1 : 0; i < NTH_ / 64; ++i) s = MAX ? fmax(s, red[k * 16 + i]) : s + red[k * 16 + i];
    v[k] = s;
  }
}

}  // namespace

// (NTH_ may be below the block size: the threads past it hold no elements; red needs a slot per wave)
template <int NTH_ = NTH>
__device__ __forceinline__ double pearson_abs(const double* e, const double* yV, int64_t nV, double* red) {
  const int t = threadIdx.x < NTH_ ? (int)threadIdx.x : (int)nV;
  const double yb = yV[0], eb = e[0];
  // red: 4 x 16 slots; four reductions (sums and non-constant counts, maxima, squares, products)
  double m4[4] = {0.0, 0.0, 0.0, 0.0};   // sx, sy, ncx, ncy
  for (int64_t v = t; v < nV; v += NTH_) {
    m4[0] += e[v];
    m4[1] += yV[v];
    m4[2] += (e[v] != eb) ? 1.0 : 0.0;
    m4[3] += (yV[v] != yb) ? 1.0 : 0.0;
  }
  block_reduce<NTH_, 4, false>(m4, red);
  const double mx = m4[0] / (double)nV, my = m4[1] / (double)nV;
  const double nonconst_x = m4[2], nonconst_y = m4[3];
  double a2[2] = {0.0, 0.0};
  for (int64_t v = t; v < nV; v += NTH_) {
    a2[0] = fmax(a2[0], fabs(e[v] - mx));
    a2[1] = fmax(a2[1], fabs(yV[v] - my));
  }
  block_reduce<NTH_, 2, true>(a2, red);
  const double xmax = a2[0], ymax = a2[1];
  double q2[2] = {0.0, 0.0};
  for (int64_t v = t; v < nV; v += NTH_) {
    const double a = (e[v] - mx) / xmax, c = (yV[v] - my) / ymax;
    q2[0] = __builtin_fma(a, a, q2[0]);
    q2[1] = __builtin_fma(c, c, q2[1]);
  }
  block_reduce<NTH_, 2, false>(q2, red);
  const double nx = xmax * sqrt(q2[0]);
  const double ny = ymax * sqrt(q2[1]);
  double r1[1] = {0.0};
  for (int64_t v = t; v < nV; v += NTH_) r1[0] = __builtin_fma((e[v] - mx) / nx, (yV[v] - my) / ny, r1[0]);
  block_reduce<NTH_, 1, false>(r1, red);
  double r = r1[0];
  if (r == r) r = fmin(fmax(r, -1.0), 1.0);  // np.clip keeps NaN (fmin/fmax would drop it)
  if (nonconst_x == 0.0 || nonconst_y == 0.0) r = __builtin_nan("");
  if (nV == 2) r = rint(r);
  return fabs(r);
}


// Sum over the 8 lanes 8m .. 8m + 7 (every lane gets it), by DPP instead of ds_bpermute: xor 1 and xor 2
// by quad_perm, then each lane adds the other quad's sum through row_half_mirror (lane i <-> 7 - i of
// each 8): the same two quad sums the xor-4 butterfly adds, so the same bits; DPP moves 32 bits, so a
// double crosses in two halves.
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double sum8(double v) {
  v += dpp64<0xB1>(v);    // quad_perm [1, 0, 3, 2]: xor 1
  v += dpp64<0x4E>(v);    // quad_perm [2, 3, 0, 1]: xor 2
  v += dpp64<0x141>(v);   // row_half_mirror
  return v;
}

// ---- arithmetic shared by k_solve and k_solve_chain (the SNP-form results of the two are
// bit-identical, so the launcher may pick either per batch) ----
constexpr int PCTH = 512;   // Pearson / centring-term reductions as over 512 threads

// The tile stream's mapping: the 8 threads of a row take its 16-B chunks interleaved -- thread seg
// chunks seg, seg + 8, .., seg + 56 -- so each load instruction of a wave covers 8 whole 128-B lines
// (8 rows) instead of 64 lines 16 B apart (thread seg once held 16 consecutive doubles: every load then
// touched a line per lane -- PMC at config 2: the texture address unit stalled by the L1 for 87M
// cycles per k_solve launch, profiles/r05_pmc_units.json), and the beta_J reads of one instruction hit 8
// consecutive 16-B LDS chunks (bank-conflict free).
// v of the X_J products (vsh) keeps 2 doubles of padding after every 16: the 16-element segment s
// that the row's thread s reads starts at 18 s, so a wave's 8 segments fall on 8 distinct bank groups
// (unpadded, 128 B apart, they fell on 2: 4-way conflicts; 52.9M SQ_LDS_BANK_CONFLICT cycles per
// k_solve launch with the old tile mapping).
constexpr int TPAD = TILE + TILE / 8;
__device__ __forceinline__ int vpi(int i) { return i + 2 * (i >> 4); }

// p = (L_JI^T beta_J)[row] over the row's chunks of thread seg (x[e]: doubles 2 (seg + 8 e), +1 of the
// row), xor-reduced over the row's 8 threads: every thread of the row holds p
template <int NTR>
__device__ __forceinline__ void tile_row_partial(const v2d (&x)[8], const double* beta, int64_t stride, int seg,
                                                 double (&p)[NTR]) {
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) p[tr] = 0.0;
#pragma unroll
  for (int e = 0; e < 8; ++e)   // explicit fmas: no contraction choice left to the compiler
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr)
      p[tr] = __builtin_fma(x[e][1], beta[tr * stride + 2 * seg + 16 * e + 1],
                            __builtin_fma(x[e][0], beta[tr * stride + 2 * seg + 16 * e], p[tr]));
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) {
    p[tr] = sum8(p[tr]);
  }
}

// beta[row] = (X^T v)[row] = sum_i X[i][row] v[i]: Dinv holds the lower blocks of X transposed, so
// thread (row, seg) reads row row%16 of block (seg, row/16) -- 16 contiguous i -- which exists iff
// seg >= row/16; xor-reduced over the row's 8 threads
__device__ __forceinline__ bool xrow_load(const double* Dj, int row, int seg, v2d (&xr)[8]) {
  const bool ok = seg >= (row >> 4);
  const double* xb = Dj + (ok ? pk(seg, row >> 4) + (row & 15) * NB : 0);
#pragma unroll
  for (int m = 0; m < 8; ++m) xr[m] = *reinterpret_cast<const v2d*>(xb + 2 * m);
  return ok;
}
template <int NTR>
__device__ __forceinline__ void xrow_apply(const v2d (&xr)[8], bool ok, int row, int seg, const double (*vsh)[TPAD],
                                           double (&s2)[NTR]) {
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) s2[tr] = 0.0;
  if (ok) {
    const int sw = (row >> 1) & 7;   // bo(): 16-B chunk m of the row holds columns 2(m ^ sw), +1
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const v2d xv = xr[m];
      const int i0 = 18 * seg + 2 * (m ^ sw);   // vpi(16 seg + 2 (m ^ sw))
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) s2[tr] = __builtin_fma(xv[1], vsh[tr][i0 + 1], __builtin_fma(xv[0], vsh[tr][i0], s2[tr]));
    }
  }
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) {
    s2[tr] = sum8(s2[tr]);
  }
}

// block J's share of the SNP-form prediction for animals 4 qd .. 4 qd + 3, every trait: sum over
// the block's rows r = rg, rg + 8, .. < nr of x_va beta_r (the 2-bit packed split rows: one byte
// holds the four animals, animal 4q + i at bits 2i; V animals from byte nTp / 4 -- a quarter of the
// int8 rows' bytes; beta[tr * bstride + r]), then xor-reduced over the 8 row groups
template <int NTR>
__device__ __forceinline__ void pred_share(const uint8_t* gp, int64_t gp_row, const int32_t* rowp, const double* beta,
                                           int64_t bstride, int nr, int64_t qoff, int rg, double (&acc)[NTR][4]) {
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[tr][j] = 0.0;
#pragma unroll 4
  for (int r = rg; r < nr; r += 8) {
    const uint32_t xb = gp[(int64_t)rowp[r] * gp_row + qoff];
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr) {
      const double bv = beta[tr * bstride + r];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[tr][j] = __builtin_fma((double)((xb >> (2 * j)) & 3u), bv, acc[tr][j]);
    }
  }
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[tr][j] = sum8(acc[tr][j]);
    }
}

template <int NTR>
__global__ __launch_bounds__(NTH) void k_solve(CholLaunch c, double* __restrict__ fit, double* __restrict__ ebv) {
  extern __shared__ double dyn[];  // alpha[nt][ns], e[nt][nV], then (primal) int32 rowp[ns]
  __shared__ double part[NTH / 64][2 * TILE];   // reused as [64][64]
  __shared__ double vsh[MAXT][TPAD];
  __shared__ double wblk[4 * KBLK];   // kernel form: w_s of one 256-SNP stage
  __shared__ double red[4 * 16];
  const int64_t nTp = c.d.nTp, nT = c.d.nT, nV = c.d.nV, ns = c.sd.ns, prow = c.sd.prow;
  const int NT = c.sd.NT;
  constexpr int nt = NTR;
  double* alpha = dyn;
  double* eall = dyn + nt * ns;
  int32_t* rowp = reinterpret_cast<int32_t*>(eall + nt * nV);   // [ns] primal: split row per SNP
  const int t = threadIdx.x;
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);   // the XCD that factorised it
  const double* Lb = c.L + b * l_stride(NT);
  const double* Db = c.Dinv + b * (int64_t)NT * NPACK * BLKD;
  const double* sc = c.scal + b * SCAL;
  const double invN = sc[SC_SA], cN = sc[SC_CN], invd = sc[SC_INVD], muf = sc[SC_MUF];
  const int fo = fold_of(c.ft, b);   // the system's split

  // alpha = L^{-T} z for every trait in one pass over L, block rows from the bottom, using
  // the stored diagonal inverses.  (L_JI^T alpha_J)[c] = sum_r Lt_(J,I)[c][r] alpha_J[r]:
  // row c of the transposed tile, 8 threads per row (16 contiguous r each), lane shuffles.
  const int rc = t >> 3, seg = t & 7;
  // z into alpha's slots up front (alpha_I replaces z_I once computed): no global load on
  // the block-row chain except the tiles and X_I
  if (c.skip & 8192) return;
  for (int64_t i = t; i < nt * ns; i += NTH) alpha[i] = c.z[b * nt * ns + i];
  __syncthreads();
  for (int I = NT - 1; I >= 0; --I) {
    // s = sum_{J > I} (L_JI^T alpha_J), one tile's row partial at a time, J descending (the
    // chained solve's order: its pull units get alpha_J from the bottom up)
    double s[NTR] = {};
    // two tiles per step: 256 B per thread (256 KiB per workgroup) in flight
    for (int J = (c.skip & 1024) ? I : NT - 1; J > I; J -= 2) {
      const bool two = J - 1 > I;
      const double* row0 = Lb + ((int64_t)J * NT + I) * TILE * TILE + rc * TILE + 2 * seg;
      const double* row1 = two ? row0 - (int64_t)NT * TILE * TILE : row0;
      v2d x0[8], x1[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x0[e] = *reinterpret_cast<const v2d*>(row0 + 16 * e);
#pragma unroll
      for (int e = 0; e < 8; ++e) x1[e] = *reinterpret_cast<const v2d*>(row1 + 16 * e);
      double p[NTR];
      tile_row_partial<NTR>(x0, alpha + J * TILE, ns, seg, p);
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) s[tr] += p[tr];
      if (two) {
        tile_row_partial<NTR>(x1, alpha + (J - 1) * TILE, ns, seg, p);
#pragma unroll
        for (int tr = 0; tr < NTR; ++tr) s[tr] += p[tr];
      }
    }
    // alpha_I = X_I^T v, X_I's row loaded before the barrier so that its latency overlaps it
    v2d xr[8];
    const bool xrow = xrow_load(Db + (int64_t)I * NPACK * BLKD, rc, seg, xr);
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr)
      if (seg == 0) vsh[tr][vpi(rc)] = alpha[tr * ns + (int64_t)I * TILE + rc] - s[tr];
    __syncthreads();
    double s2[NTR];
    xrow_apply<NTR>(xr, xrow, rc, seg, vsh, s2);
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr)
      if (seg == 0) alpha[tr * ns + I * TILE + rc] = s2[tr];
    __syncthreads();
  }

  if (c.skip & 4096) return;
  const double* ub = c.u + b * prow;
  const uint8_t* pb = c.panel + b * c.pstride;   // kernel form: packed animal rows (dual_pk_row bytes)
  if (c.sd.form == FORM_PRIMAL) {
    // system row r holds selected SNP r - pad (leading padding rows: the zero split row P)
    const int64_t kk = (int64_t)sc[SC_K], o0 = c.off[b], pad = (int64_t)sc[SC_PAD];
    for (int64_t r = t; r < pad + kk; r += NTH) {
      rowp[r] = (r < pad) ? (int32_t)c.d.P : (int32_t)snp_col(c.idx[o0 + r - pad], c.d.P);
    }
    __syncthreads();
  }
  double* pw = &part[0][0];             // kernel form: [16 waves][256]
  double fsum = 0.0;
  if (c.sd.form == FORM_PRIMAL) {
    // EBV_v = sum_J e_J[v] - (sum_J mb_J) / n_T + mu with block J's shares e_J[v] = sum_{a in J}
    // x_va beta_a and mb_J = sum_{a in J} s_a beta_a, J ascending (the chained solve's order),
    // every trait in one pass over the rows
    const int64_t kk = (int64_t)sc[SC_K] + (int64_t)sc[SC_PAD];   // rows up to the last real one
    const int rg8 = t & 7;
    const int64_t nq = (nV + 3) / 4;
    double mbt[NTR];
    for (int J = 0; J < NT; ++J) {
      const int nr = (int)max((int64_t)0, min((int64_t)TILE, kk - (int64_t)J * TILE));
      for (int64_t qd = t >> 3; qd < ((c.skip & 2048) ? 0 : nq); qd += NTH / 8) {
        double acc[NTR][4];
        pred_share<NTR>(c.ft.gpk[fo], c.gpk_row, rowp + J * TILE, alpha + J * TILE, ns, nr, nTp / 4 + qd, rg8, acc);
#pragma unroll
        for (int tr = 0; tr < NTR; ++tr)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t v = 4 * qd + j;
            if (rg8 == 0 && v < nV) eall[tr * nV + v] = (J == 0) ? acc[tr][j] : eall[tr * nV + v] + acc[tr][j];
          }
      }
      double m[NTR];
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr)
        m[tr] = (t < nr && t < PCTH) ? ub[(int64_t)J * TILE + t] * alpha[tr * ns + (int64_t)J * TILE + t] : 0.0;
      block_reduce<PCTH, NTR, false>(m, red);
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) mbt[tr] = (J == 0) ? m[tr] : mbt[tr] + m[tr];
    }
    __syncthreads();
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr) {
      const double MB = mbt[tr] * sc[SC_SM], mu = muf * c.ft.ymu[fo][tr];
      for (int64_t v = t; v < nV; v += NTH) eall[tr * nV + v] = eall[tr * nV + v] - MB + mu;
    }
    __syncthreads();
  }
  for (int tr = 0; tr < nt; ++tr) {
    const double* al = alpha + tr * ns;
    double* e = eall + tr * nV;
    const double* yV = c.ft.yV[fo] + tr * nV;
    const double mu = muf * c.ft.ymu[fo][tr];
    if (c.sd.form == FORM_PRIMAL) {
      // (the EBVs above)
    } else {
      // EBV_V = K_VT alpha + mu without materialising K_VT (exact-integer factored form):
      //   sum_t K_vt alpha_t = [sum_s a_vs w_s - u_v S/N - (u_T . alpha)/N + cN S] / d,
      //   w_s = sum_t a_ts alpha_t,  S = sum_t alpha_t
      double s_a = 0.0, s_ua = 0.0;
      for (int64_t r = t; r < nT; r += NTH) {
        s_a += al[r];
        s_ua += ub[r] * al[r];
      }
      const double S = block_sum(s_a, red);
      const double UA = block_sum(s_ua, red);
      for (int64_t v = t; v < nV; v += NTH) e[v] = 0.0;
      // 256-SNP stages (64 B of each packed row): thread (rh, hq) = (t >> 5, t & 31) sums half-dword
      // hq of its rows (SNPs 8 hq .. 8 hq + 7 of the stage, 2 bits each); a wave's two row groups by
      // a shuffle, then the 16 waves' partials in LDS
      const int64_t nst = ((int64_t)sc[SC_CBLK] + 3) / 4;
      const int64_t pkr = c.pstride / prow;   // packed row bytes (dual_pk_row)
      const int hq = t & 31, rh = t >> 5;
      for (int64_t st = 0; st < nst; ++st) {
        const uint8_t* sp = pb + st * 64;
        double p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = 0.0;
        for (int64_t r = rh; r < nT; r += NTH / 32) {
          const uint32_t x = *reinterpret_cast<const uint16_t*>(sp + r * pkr + 2 * hq);
          const double ar = al[r];
#pragma unroll
          for (int j = 0; j < 8; ++j) p[j] += (double)((x >> (2 * j)) & 3) * ar;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] += __shfl_xor(p[j], 32);
        __syncthreads();
        if ((t & 63) < 32) {
#pragma unroll
          for (int j = 0; j < 8; ++j) pw[(t >> 6) * 4 * KBLK + 8 * hq + j] = p[j];
        }
        __syncthreads();
        if (t < 4 * KBLK) {
          double acc = 0.0;
          for (int q = 0; q < NTH / 64; ++q) acc += pw[q * 4 * KBLK + t];
          wblk[t] = acc;
        }
        __syncthreads();
        for (int64_t v = t; v < nV; v += NTH) {
          const uint4* row = reinterpret_cast<const uint4*>(sp + (nTp + v) * pkr);
          double acc = 0.0;
#pragma unroll 1
          for (int h = 0; h < 4; ++h) {   // (not unrolled: wblk's 256 loads are not hoisted out of the v loop)
            const uint4 q = row[h];
            const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int d = 0; d < 4; ++d)
#pragma unroll
              for (int j = 0; j < 16; ++j) acc += (double)((qw[d] >> (2 * j)) & 3) * wblk[16 * (4 * h + d) + j];
          }
          e[v] += acc;
        }
      }
      __syncthreads();
      for (int64_t v = t; v < nV; v += NTH) e[v] = (e[v] - ub[nTp + v] * S * invN - UA * invN + cN * S) * invd + mu;
      __syncthreads();
    }
    // Pearson correlation (scipy.stats.pearsonr restated); multi-trait fitness is the mean |r|
    fsum += pearson_abs<PCTH>(e, yV, nV, red);
    if (ebv != nullptr) {
      for (int64_t v = t; v < nV; v += NTH) ebv[(b * nt + tr) * nV + v] = e[v];
    }
  }
  if (t == 0) fit[b] = sc[SC_BAD] != 0.0 ? __builtin_nan("") : (nt == 1) ? fsum : fsum / (double)nt;
}


// ===========================================================================
// Chained back substitution (SNP form): an individual's solve spread over the chip, one 512-thread
// unit U(b, J) per block row J:
//   while it waits: X_J (72 KiB) into LDS by LDS-DMA and tile (J, J-1) into registers;
//   v = z_J - sum_{K > J} c_{K->J} (K ascending; c_{K->J} from unit K), beta_J = X_J^T v;
//   c_{J->J-1} = L_{J,J-1}^T beta_J from the registers, published at once -- the chain's only
//   hand-off per block row -- then the tiles (J, I), I = J-2 .. 0, streamed (each c_{J->I} published
//   as it is done: unit I takes its terms in K order, and the nearest rows are needed first);
//   then block J's share of the prediction, sum_{a in J} x_va beta_a, and of the centring term;
//   U(b, 0) finally adds the shares (J ascending) and forms the fitness.
// The one-workgroup-per-individual k_solve streams an individual's 4.7 MB (config 2) through one
// CU at ~30 GB/s and waits out the block-row chain on top; here the tile stream of every block row
// runs on its own CU beside the chain.  (Round 3's form -- a unit per tile, each holding its tile in
// registers until beta_J arrived, and two hand-offs per block row (F -> T -> F) -- spent most of its
// time with the chip's unit slots full of waiting tile units: 0.162 ms at pop 128.)
// Pull units (round 5, the default; TBLUP_SOLVE_PULL=0 keeps the push units above): U(b, J) takes
// the tiles of its block COLUMN instead -- it publishes only beta_J (ch.beta, flag_beta), and pulls
// c_{K->J} = L_KJ^T beta_K itself for K = NT-1 .. J+1 as the beta_K arrive (tile (K-1, J) loading while
// it waits for beta_{K-1}), then v, beta_J = X_J^T v, beta_J published.  The chain still costs one
// hand-off and one tile product per block row, but the work of a unit is 7 - J tiles instead of J:
// the first-dispatched levels (large J) end at once and free their slots, where the push units of
// level NT-1 streamed NT-1 tiles while the low levels, which the chain ends on, waited for a slot
// (pop 128: 1024 units on 512 slots, levels 3 .. 0 dispatched 66-102 us in,
// profiles/r04_solve_trace_pop128.txt).  Every c_{K->J} sum runs K descending, in k_solve too.
// Grid order: level J = NT-1 .. 0, individuals within a level.  A unit waits only on units with
// smaller block ids (U(b, J) on U(b, K > J)), and each XCD dispatches its share in block-id order, so
// the waits drain.  Argument: let u be the smallest block id not yet dispatched.  u's XCD is full,
// and every block resident there has an id < u, so the smallest waiting unit w anywhere has w < u:
// every unit it waits on (ids < w) is dispatched, and, being smaller than w, is not waiting -- it
// runs to completion.  Workgroups of other kernels (other streams, other processes) holding CU
// slots only delay dispatch; they end on their own.  The one assumption is the per-XCD in-order
// dispatch of one kernel's blocks, an observed hardware behaviour, not a documented guarantee --
// hence the bound on every wait: CHAIN_SPIN_MAX polls, after which the unit stores the call's seq
// into its expiry-ring slot ch.err (every later wait of the same call gives up at once); the host
// entries read that slot and re-solve the chunk's factor through k_solve (bit-identical), device
// entries see the context's sticky status word ch.expired (tblup_solve_error /
// tblup_status_async) -- a recovery or an error, never a silent NaN fitness.  Every
// sum has a fixed order, the same as k_solve's, so the results do not depend on B, the timing or
// the grid, and equal k_solve's bit for bit.  With 8 | B an individual's units share one XCD
// (block id = level * B + b), so its hand-offs stay in one L2.
// ===========================================================================
constexpr int CTH = 512;
enum { WGT_SROW = 7 };
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// profiling only (TBLUP_WG_TRACE): {start, end, kind << 56 | I << 40 | b, J | (first wait done - start) << 16}
struct ChainTrace {
  uint64_t* rec = nullptr;
  uint64_t t0 = 0, tw = 0;
  __device__ explicit ChainTrace(uint64_t* base) {
    if (base) {
      rec = base + (int64_t)blockIdx.x * WGT_REC;
      t0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ void waited() {
    if (rec && tw == 0) tw = __builtin_amdgcn_s_memrealtime();
  }
  __device__ void done(int kind, int J, int I, int64_t b) {
    if (!rec) return;
    __syncthreads();
    if (threadIdx.x == 0) {
      rec[0] = t0;
      rec[1] = __builtin_amdgcn_s_memrealtime();
      rec[2] = ((uint64_t)kind << 56) | ((uint64_t)I << 40) | (uint64_t)b;
      rec[3] = (uint64_t)J | ((tw ? tw - t0 : 0) << 16);
    }
  }
};

__device__ __forceinline__ int32_t* flag_part(const SolveChain& ch, int64_t b, int NT, int I, int J) {
  return ch.flags + b * chain_flags(NT) + NT + I * NT + J;
}
__device__ __forceinline__ int32_t* flag_e(const SolveChain& ch, int64_t b, int NT, int J) {
  return ch.flags + b * chain_flags(NT) + NT + NT * NT + J;
}
// pull units: beta_K published (the first NT flags of an individual)
__device__ __forceinline__ int32_t* flag_beta(const SolveChain& ch, int64_t b, int NT, int K) {
  return ch.flags + b * chain_flags(NT) + K;
}

// Exchange through coherent (sc1) accesses: the producer stores its data and, once every wave's
// stores have completed (s_waitcnt vmcnt(0) + barrier), the flag; the consumer polls the flag
// and reads the data with sc1 loads.  No acquire/release fences: on gfx950 those are an L2
// invalidate (buffer_inv sc1) per poll and an L2 write-back (buffer_wbl2 sc1) per publish, which
// measured 25 us per hand-off and slowed every other workgroup of the XCD.  This relies on the
// gfx950 (CDNA3/4) coherence of sc1 accesses, so the library is built for gfx950 only (Makefile);
// mode (TBLUP_CHAIN_SYNC): 0 = this, 1 = acquire/release atomics on the flag (reference;
// tests/test_gpu_shapes.py checks the two bit for bit).
template <typename T>
__device__ __forceinline__ T cload(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void cstore(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The whole workgroup waits until *f == seq (one lane polls).  False: gave up.
__device__ bool chain_wait(const int32_t* f, const SolveChain& ch, int* sh) {
  const int32_t seq = ch.seq;
  if (threadIdx.x == 0) {
    int ok = 1;
    for (int it = 0;; ++it) {
      const int32_t v = ch.mode == 1 ? __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) : cload(f);
      if (v == seq) break;
      if (it >= ch.spin_max || cload(ch.err) == seq) {   // this call's waits already expired elsewhere
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) {
      cstore(ch.err, seq);          // the call's sequence number: later calls start unaffected
      cstore(ch.expired, (int32_t)1);   // sticky until the host reads it
    }
    *sh = ok;
  }
  __syncthreads();
  const int ok = *sh;
  __syncthreads();
  return ok != 0;
}

// every wave's stores completed, then the flag
__device__ __forceinline__ void chain_publish(int32_t* f, int32_t seq, int mode) {
  if (mode == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (mode == 1)
      __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else
      cstore(f, seq);
  }
}

// rows rc and rc + 64 of tile (J, I) (transposed storage: row r = column 128 I + r of L, block J),
// the row's 16-B chunks seg + 8 e (tile_row_partial's mapping)
__device__ __forceinline__ void chain_tile_load(const CholLaunch& c, int64_t b, int J, int I, int rc, int seg,
                                                v2d (&x)[2][8]) {
  const int NT = c.sd.NT;
  const double* tile = c.L + b * l_stride(NT) + ((int64_t)J * NT + I) * TILE * TILE + 2 * seg;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) x[h][e] = *reinterpret_cast<const v2d*>(tile + (rc + 64 * h) * TILE + 16 * e);
}

// push units: c_{J->I} = L_JI^T beta_J (beta_J in bsh) -> cpart, then its flag
template <int NTR>
__device__ __forceinline__ void chain_tile_publish(const SolveChain& ch, int64_t b, int NT, int J, int I,
                                                   const v2d (&x)[2][8], const double (*bsh)[TILE], int rc,
                                                   int seg) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double p[NTR];
    tile_row_partial<NTR>(x[h], &bsh[0][0], TILE, seg, p);
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr)
      if (seg == 0) cstore(ch.cpart + (((b * NT + I) * NT + J) * NTR + tr) * TILE + rc + 64 * h, p[tr]);
  }
  chain_publish(flag_part(ch, b, NT, I, J), ch.seq, ch.mode);
}

// The unit of block row J.  xl: 72 KiB of LDS -- X_J, then (U(b, 0)) the EBVs.
template <int NTR, bool PULL>
__device__ void chain_unit(const CholLaunch& c, const SolveChain& ch, int64_t b, int J, double* fit, double* ebv,
                           double* xl, int* sh, ChainTrace& tr_) {
  __shared__ double vsh[NTR][TPAD];   // z_J, then v (padded: vpi)
  __shared__ double bsh[NTR][TILE];   // beta_J
  __shared__ int32_t rowp[TILE];
  __shared__ double red[4 * 16];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int NT = c.sd.NT;
  const int64_t ns = c.sd.ns, nV = c.d.nV, nTp = c.d.nTp;
  const double* sc = c.scal + b * SCAL;
  const int64_t kk = (int64_t)sc[SC_K], o0 = c.off[b], pad = (int64_t)sc[SC_PAD];
  // rows of block J up to the last real one (system row r holds selected SNP r - pad; the leading
  // padding rows read the zero split row P)
  const int nr = (int)max((int64_t)0, min((int64_t)TILE, pad + kk - (int64_t)J * TILE));
  const int rc = t >> 3, seg = t & 7;   // rows rc and rc + 64, 8 threads per row
  // X_J (packed lower blocks, each transposed: Dinv's layout) into LDS, 9 x 16 B per thread
  {
    const double* Dj = c.Dinv + (b * NT + J) * (int64_t)NPACK * BLKD;
#pragma unroll
    for (int e = 0; e < NPACK * BLKD / 2 / CTH; ++e) {
      const int chunk = (e * (CTH / 64) + w) * 64;
      __builtin_amdgcn_global_load_lds(Dj + 2 * (chunk + l), (lds_ptr_t)(xl + 2 * chunk), 16, 0, 0);
    }
  }
  v2d x[2][8];
  constexpr bool pull = PULL;
  if constexpr (pull) {
    if (J + 1 < NT) chain_tile_load(c, b, NT - 1, J, rc, seg, x);   // the first tile pulled: (NT-1, J)
  } else if (J > 0) {
    chain_tile_load(c, b, J, J - 1, rc, seg, x);
  }
  for (int i = t; i < NTR * TILE; i += CTH) vsh[i / TILE][vpi(i % TILE)] = c.z[(b * NTR + i / TILE) * ns + (int64_t)J * TILE + i % TILE];
  for (int r = t; r < nr; r += CTH) {
    const int64_t g = (int64_t)J * TILE + r;
    rowp[r] = (g < pad) ? (int32_t)c.d.P : (int32_t)snp_col(c.idx[o0 + g - pad], c.d.P);
  }
  if constexpr (pull) {
    // c_{K->J} = L_KJ^T beta_K for K = NT-1 .. J+1 as the beta_K arrive, summed in that order (k_solve's):
    // tile (K-1, J)'s rows are loaded into the registers each half of tile K frees, so the next
    // tile is in flight while this unit waits for beta_{K-1}
    double acc[2][NTR];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) acc[h][tr] = 0.0;
    for (int K = NT - 1; K > J; --K) {
      if (!chain_wait(flag_beta(ch, b, NT, K), ch, sh)) {
        if (J == 0 && t == 0) fit[b] = __builtin_nan("");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the X_J LDS-DMA lands before the workgroup ends
        return;
      }
      if (t < NTR * TILE) bsh[t / TILE][t % TILE] = cload(ch.beta + (b * NTR + t / TILE) * ns + (int64_t)K * TILE + t % TILE);
      __syncthreads();
      const double* nxt = c.L + b * l_stride(NT) + ((int64_t)(K - 1) * NT + J) * TILE * TILE + 2 * seg;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double p[NTR];
        tile_row_partial<NTR>(x[h], &bsh[0][0], TILE, seg, p);
#pragma unroll
        for (int tr = 0; tr < NTR; ++tr) acc[h][tr] += p[tr];
        if (K - 1 > J) {
#pragma unroll
          for (int e = 0; e < 8; ++e) x[h][e] = *reinterpret_cast<const v2d*>(nxt + (rc + 64 * h) * TILE + 16 * e);
        }
      }
      __syncthreads();   // bsh is overwritten by the next beta
    }
    tr_.waited();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // X_J in LDS, z_J, the row table
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h)   // v = z_J - sum_{K > J} c_{K->J}
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr)
        if (seg == 0) vsh[tr][vpi(rc + 64 * h)] = vsh[tr][vpi(rc + 64 * h)] - acc[h][tr];
  } else {
    for (int K = J + 1; K < NT; ++K)
      if (!chain_wait(flag_part(ch, b, NT, J, K), ch, sh)) {
        if (J == 0 && t == 0) fit[b] = __builtin_nan("");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the X_J LDS-DMA lands before the workgroup ends
        return;
      }
    tr_.waited();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // X_J in LDS, z_J, the row table
    __syncthreads();
    for (int i = t; i < NTR * TILE; i += CTH) {   // v = z_J - sum_{K > J} c_{K->J}, K descending
      const int tr = i / TILE, cc = i % TILE;
      double acc = 0.0;
      for (int K = NT - 1; K > J; --K) acc += cload(ch.cpart + (((b * NT + J) * NT + K) * NTR + tr) * TILE + cc);
      vsh[tr][vpi(cc)] = vsh[tr][vpi(cc)] - acc;
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {   // beta_J = X_J^T v
    v2d xr[8];
    const bool ok = xrow_load(xl, rc + 64 * h, seg, xr);
    double s2[NTR];
    xrow_apply<NTR>(xr, ok, rc + 64 * h, seg, vsh, s2);
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr)
      if (seg == 0) bsh[tr][rc + 64 * h] = s2[tr];
  }
  __syncthreads();
  if (J > 0) {
    if (ch.delay > 0 && b == 0 && J == NT - 1) {   // debug knob (expiry test): a late producer
      for (int i = 0; i < ch.delay; ++i) __builtin_amdgcn_s_sleep(127);
    }
  }
  if constexpr (pull) {
    if (J > 0) {   // beta_J for the units of the block columns I < J
      if (t < NTR * TILE) cstore(ch.beta + (b * NTR + t / TILE) * ns + (int64_t)J * TILE + t % TILE, bsh[t / TILE][t % TILE]);
      chain_publish(flag_beta(ch, b, NT, J), ch.seq, ch.mode);
    }
  } else if (J > 0) {
    chain_tile_publish<NTR>(ch, b, NT, J, J - 1, x, bsh, rc, seg);
    for (int I = J - 2; I >= 0; --I) {
      chain_tile_load(c, b, J, I, rc, seg, x);
      chain_tile_publish<NTR>(ch, b, NT, J, I, x, bsh, rc, seg);
    }
  }

  // block J's share of the prediction and of the centring term, every trait in one pass: units
  // J > 0 to epart, U(b, 0) into LDS (X_0 is done with)
  double* eall = xl;
  const int rg = t & 7;
  const int64_t nq = (nV + 3) / 4;
  for (int64_t qd = t >> 3; qd < nq; qd += CTH / 8) {
    double acc[NTR][4];
    pred_share<NTR>(c.ft.gpk[fold_of(c.ft, b)], c.gpk_row, rowp, &bsh[0][0], TILE, nr, nTp / 4 + qd, rg, acc);
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t v = 4 * qd + j;
        if (rg == 0 && v < nV) {
          if (J > 0)
            cstore(ch.epart + ((b * NT + J) * NTR + tr) * nV + v, acc[tr][j]);
          else
            eall[tr * nV + v] = acc[tr][j];
        }
      }
  }
  double mb[NTR];
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) mb[tr] = t < nr ? c.u[b * c.sd.prow + (int64_t)J * TILE + t] * bsh[tr][t] : 0.0;
  block_reduce<PCTH, NTR, false>(mb, red);
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr)
    if (J > 0 && t == 0) cstore(ch.mbpart + (b * NT + J) * NTR + tr, mb[tr]);
  if (J > 0) {
    chain_publish(flag_e(ch, b, NT, J), ch.seq, ch.mode);
    tr_.done(WGT_SROW, J, 0, b);
    return;
  }
  // U(b, 0): EBV_v = sum_J e_J[v] - (sum_J mb_J) / n_T + mu, J ascending; then the fitness
  for (int K = 1; K < NT; ++K)
    if (!chain_wait(flag_e(ch, b, NT, K), ch, sh)) {
      if (t == 0) fit[b] = __builtin_nan("");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
  const double muf = sc[SC_MUF];
  double fsum = 0.0;
  for (int tr = 0; tr < NTR; ++tr) {
    double mbt = mb[tr];
    for (int K = 1; K < NT; ++K) mbt += cload(ch.mbpart + (b * NT + K) * NTR + tr);
    const double MB = mbt * sc[SC_SM], mu = muf * c.ft.ymu[fold_of(c.ft, b)][tr];
    double* e = eall + tr * nV;
    for (int64_t v = t; v < nV; v += CTH) {
      double acc = e[v];
      for (int K = 1; K < NT; ++K) acc += cload(ch.epart + ((b * NT + K) * NTR + tr) * nV + v);
      e[v] = acc - MB + mu;
    }
    __syncthreads();
    fsum += pearson_abs<PCTH>(e, c.ft.yV[fold_of(c.ft, b)] + tr * nV, nV, red);
    if (ebv != nullptr)
      for (int64_t v = t; v < nV; v += CTH) ebv[(b * NTR + tr) * nV + v] = e[v];
  }
  if (t == 0) fit[b] = sc[SC_BAD] != 0.0 ? __builtin_nan("") : (NTR == 1) ? fsum : fsum / (double)NTR;
  tr_.done(WGT_SROW, J, 1, b);
}

template <int NTR, bool PULL>
__global__ __launch_bounds__(CTH, NTR < 4 ? 4 : 2) void k_solve_chain(CholLaunch c, SolveChain ch, double* __restrict__ fit,
                                                     double* __restrict__ ebv) {
  __shared__ __attribute__((aligned(16))) double xl[NPACK * BLKD];   // X_J, then (U(b, 0)) the EBVs
  __shared__ int sh;
  const int NT = c.sd.NT;
  const int64_t g = blockIdx.x;
  const int J = NT - 1 - (int)(g / c.B);
  ChainTrace tr(c.wgt);
  chain_unit<NTR, PULL>(c, ch, g % c.B, J, fit, ebv, xl, &sh, tr);
}

// whether the chained solve can run this batch: the EBVs of U(b, 0) fit its 72 KiB of LDS
bool chain_fits(const CholLaunch& c) { return (int64_t)c.d.nt * c.d.nV <= (int64_t)NPACK * BLKD; }

hipError_t launch_solve(const CholLaunch& c, const SolveChain* ch, double* fitness, double* ebv, hipStream_t s) {
  const size_t shm = (size_t)c.d.nt * (size_t)(c.sd.ns + c.d.nV) * sizeof(double) + (size_t)((c.sd.ns + 1) / 2) * sizeof(double);
  auto launch = [&](const void* fn, auto kernel) -> hipError_t {
    if (shm > 64 * 1024) {
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kernel, dim3((unsigned)c.B), dim3(NTH), shm, s, c, fitness, ebv);
    return hipGetLastError();
  };
  if (ch != nullptr && c.sd.form == FORM_PRIMAL && chain_fits(c)) {
    const dim3 grid((unsigned)(c.B * c.sd.NT));
    auto launch_chain = [&](auto kernel) -> hipError_t {
      hipLaunchKernelGGL(kernel, grid, dim3(CTH), 0, s, c, *ch, fitness, ebv);
      return hipGetLastError();
    };
    const int sel = c.d.nt * 2 + (ch->pull ? 1 : 0);
    switch (sel) {
      case 2: return launch_chain(k_solve_chain<1, false>);
      case 3: return launch_chain(k_solve_chain<1, true>);
      case 4: return launch_chain(k_solve_chain<2, false>);
      case 5: return launch_chain(k_solve_chain<2, true>);
      case 6: return launch_chain(k_solve_chain<3, false>);
      case 7: return launch_chain(k_solve_chain<3, true>);
      case 8: return launch_chain(k_solve_chain<4, false>);
      case 9: return launch_chain(k_solve_chain<4, true>);
      default: return hipErrorInvalidValue;
    }
  }
  switch (c.d.nt) {
    case 1: return launch((const void*)k_solve<1>, k_solve<1>);
    case 2: return launch((const void*)k_solve<2>, k_solve<2>);
    case 3: return launch((const void*)k_solve<3>, k_solve<3>);
    case 4: return launch((const void*)k_solve<4>, k_solve<4>);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tblup
