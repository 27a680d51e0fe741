// Back substitution, prediction and fitness, one 1024-thread workgroup per individual.
//
//   alpha = L^{-T} z                       (z = L^{-1}(y_T - mu) from k_chol_diag)
//   EBV_V = K_VT alpha + mu                gblup: evaluator.py:284 (G[:,T] Ginv y_T, mu = 0)
//                                          snp:   evaluator.py:314 (clf.predict, intercept mean(y_T))
//   fitness = |pearsonr(EBV_V, y_V)|       evaluator.py:286 / :314, scipy 1.15.3 pearsonr:
//            exact-equality constant input -> NaN; mean-centre; max-abs scaled
//            norms; clip to [-1, 1]; round when n == 2.
#include "tblup_internal.h"

namespace tblup {

namespace {

constexpr int NTH = 1024;

__device__ double block_sum(double v, double* red) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NTH / 64; ++i) s += red[i];
  return s;
}

__device__ double block_max(double v, double* red) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < NTH / 64; ++i) s = fmax(s, red[i]);
  return s;
}

}  // namespace

__global__ __launch_bounds__(NTH) void k_solve(const double* __restrict__ K, int64_t nTp, int64_t nT, int64_t nV,
                                               int NT, int64_t mstride, const double* __restrict__ Dinv,
                                               const double* __restrict__ z, const double* __restrict__ yV,
                                               const double* __restrict__ scal, double* __restrict__ fit,
                                               double* __restrict__ ebv) {
  extern __shared__ double dyn[];  // alpha[nTp] then e[nV]
  __shared__ double part[NTH / 64][TILE];
  __shared__ double vsh[TILE];
  __shared__ double red[NTH / 64];
  double* alpha = dyn;
  double* e = dyn + nTp;
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int64_t b = blockIdx.x;
  const double* Kb = K + b * mstride;
  const double* Db = Dinv + b * (int64_t)NT * TILE * TILE;
  const double mu = scal[b * 8 + 3];
  const int cp = t & 63;   // column pair: columns 2cp, 2cp+1 of the tile
  const int g = t >> 6;    // row group: rows g, g+16, ...

  for (int I = NT - 1; I >= 0; --I) {
    // s = sum_{J>I} L_JI^T alpha_J
    v2d s = {0.0, 0.0};
    for (int J = I + 1; J < NT; ++J) {
      const double* base = Kb + (int64_t)J * TILE * nTp + (int64_t)I * TILE + 2 * cp;
      const double* al = alpha + J * TILE;
#pragma unroll 8
      for (int r = g; r < TILE; r += 16) {
        const v2d x = *reinterpret_cast<const v2d*>(base + (int64_t)r * nTp);
        s += x * al[r];
      }
    }
    part[g][2 * cp] = s[0];
    part[g][2 * cp + 1] = s[1];
    __syncthreads();
    if (t < TILE) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc += part[q][t];
      vsh[t] = z[b * nTp + (int64_t)I * TILE + t] - acc;
    }
    __syncthreads();
    // alpha_I = X_I^T v  (X lower triangular, zeros stored above the diagonal)
    const double* X = Db + (int64_t)I * TILE * TILE + 2 * cp;
    v2d s2 = {0.0, 0.0};
#pragma unroll 8
    for (int r = g; r < TILE; r += 16) {
      const v2d x = *reinterpret_cast<const v2d*>(X + r * TILE);
      s2 += x * vsh[r];
    }
    part[g][2 * cp] = s2[0];
    part[g][2 * cp + 1] = s2[1];
    __syncthreads();
    if (t < TILE) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc += part[q][t];
      alpha[I * TILE + t] = acc;
    }
    __syncthreads();
  }

  // EBV_V = K_VT alpha + mu : one wave per validation row
  for (int64_t v = w; v < nV; v += NTH / 64) {
    const double* row = Kb + (nTp + v) * nTp;
    double s = 0.0;
    for (int64_t c = 2 * l; c < nT; c += 128) {
      if (c + 1 < nT) {
        const v2d x = *reinterpret_cast<const v2d*>(row + c);
        s += x[0] * alpha[c] + x[1] * alpha[c + 1];
      } else {
        s += row[c] * alpha[c];
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (l == 0) e[v] = s + mu;
  }
  __syncthreads();

  // Pearson correlation (scipy.stats.pearsonr restated), fitness = |r|
  const double yb = yV[0], eb = e[0];
  double sx = 0.0, sy = 0.0, ncx = 0.0, ncy = 0.0;
  for (int64_t v = t; v < nV; v += NTH) {
    sx += e[v];
    sy += yV[v];
    ncx += (e[v] != eb) ? 1.0 : 0.0;
    ncy += (yV[v] != yb) ? 1.0 : 0.0;
  }
  const double mx = block_sum(sx, red) / (double)nV;
  const double my = block_sum(sy, red) / (double)nV;
  const double nonconst_x = block_sum(ncx, red);
  const double nonconst_y = block_sum(ncy, red);
  double ax = 0.0, ay = 0.0;
  for (int64_t v = t; v < nV; v += NTH) {
    ax = fmax(ax, fabs(e[v] - mx));
    ay = fmax(ay, fabs(yV[v] - my));
  }
  const double xmax = block_max(ax, red);
  const double ymax = block_max(ay, red);
  double qx = 0.0, qy = 0.0;
  for (int64_t v = t; v < nV; v += NTH) {
    const double a = (e[v] - mx) / xmax, c = (yV[v] - my) / ymax;
    qx += a * a;
    qy += c * c;
  }
  const double nx = xmax * sqrt(block_sum(qx, red));
  const double ny = ymax * sqrt(block_sum(qy, red));
  double rr = 0.0;
  for (int64_t v = t; v < nV; v += NTH) rr += ((e[v] - mx) / nx) * ((yV[v] - my) / ny);
  double r = block_sum(rr, red);
  if (t == 0) {
    if (r == r) r = fmin(fmax(r, -1.0), 1.0);  // np.clip keeps NaN (fmin/fmax would drop it)
    if (nonconst_x == 0.0 || nonconst_y == 0.0) r = __builtin_nan("");
    if (nV == 2) r = rint(r);
    fit[b] = fabs(r);
  }
  if (ebv != nullptr) {
    for (int64_t v = t; v < nV; v += NTH) ebv[b * nV + v] = e[v];
  }
}

hipError_t launch_solve(const double* K, const EvalDims& d, int64_t B, const double* Dinv, const double* z,
                        const double* yV, const double* scal, double* fitness, double* ebv, hipStream_t s) {
  const size_t shm = (size_t)(d.nTp + d.nV) * sizeof(double);
  hipLaunchKernelGGL(k_solve, dim3((unsigned)B), dim3(NTH), shm, s, K, d.nTp, d.nT, d.nV, d.NT, d.nRp * d.nTp, Dinv,
                     z, yV, scal, fitness, ebv);
  return hipGetLastError();
}

}  // namespace tblup
