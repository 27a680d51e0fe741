// Preparation kernels: genotype transpose, split build, per-individual scalars
// and the gathered, animal-major genotype panel with exact centring sums.
//
// Reference behaviour restated here (ianwhale/tblup):
//   * data[:, indices] fancy-index gather, duplicates gathered twice
//     (tblup/evaluator.py:275, :298)
//   * allele frequency p = column mean / 2 over ALL rows for gblup
//     (utils.py:14 via evaluator.py:275) and over TRAIN rows for snp_blup
//     (evaluator.py:304); d = 2 sum p(1-p) (utils.py:18, evaluator.py:305)
//   * lambda = (1-h2)/h2 (evaluator.py:277; evaluator.py:306 is lambda*d in
//     ridge units)
// All centring terms are carried as exact integers: with m_s the allele count
// of SNP s over the reference rows (N of them), 2p_s = m_s/N, so
//   sum_s (a_is - 2p_s)(a_js - 2p_s) = (A A^T)_ij - (u_i + u_j)/N + q/N^2
// with u_i = sum_s m_s a_is and q = sum_s m_s^2.
#include "tblup_internal.h"
#include "k_stats.h"

namespace tblup {

// ---------------------------------------------------------------------------
// animal-major [n][P] -> SNP-major [P][n]; 64x64 byte tiles through LDS.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_transpose_geno(const int8_t* __restrict__ src, int8_t* __restrict__ dst,
                                                        int64_t n, int64_t P) {
  __shared__ int8_t tile[64][65];
  const int64_t p0 = (int64_t)blockIdx.x * 64, a0 = (int64_t)blockIdx.y * 64;
  const int t = threadIdx.x;
  // load: thread t covers 16 bytes of animal row (t >> 2), SNP cols (t & 3) * 16 ..
  {
    const int ar = t >> 2, pc = (t & 3) * 16;
    const int64_t a = a0 + ar;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t p = p0 + pc + e;
      tile[ar][pc + e] = (a < n && p < P) ? src[a * P + p] : (int8_t)0;
    }
  }
  __syncthreads();
  {
    const int pr = t >> 2, ac = (t & 3) * 16;
    const int64_t p = p0 + pr;
    if (p < P) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t a = a0 + ac + e;
        if (a < n) dst[p * n + a] = tile[ac + e][pr];
      }
    }
  }
}

hipError_t launch_transpose_geno(const int8_t* src, int8_t* dst, int64_t n, int64_t P, hipStream_t s) {
  dim3 grid((unsigned)((P + 63) / 64), (unsigned)((n + 63) / 64));
  hipLaunchKernelGGL(k_transpose_geno, grid, dim3(256), 0, s, src, dst, n, P);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// per-SNP allele count over all n animals (one wave per SNP row)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_colsum_all(const int8_t* __restrict__ g, int32_t* __restrict__ cs, int64_t n,
                                                    int64_t P) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + w;
  if (p >= P) return;
  const int8_t* row = g + p * n;
  int s = 0;
  for (int64_t a = l; a < n; a += 64) s += row[a];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (l == 0) cs[p] = s;
}

hipError_t launch_colsum_all(const int8_t* geno_sm, int32_t* colsum, int64_t n, int64_t P, hipStream_t s) {
  hipLaunchKernelGGL(k_colsum_all, dim3((unsigned)((P + 3) / 4)), dim3(256), 0, s, geno_sm, colsum, n, P);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// split build: permuted 2-bit packed SNP-major rows [T | pad | V | pad] and train counts
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_build_split(const int8_t* __restrict__ g, int64_t n, int64_t P,
                                                     const int32_t* __restrict__ rowmap, int64_t nRp, int64_t nT,
                                                     const double* __restrict__ yT, const double* __restrict__ ymu,
                                                     int nt, uint8_t* __restrict__ opk,
                                                     int32_t* __restrict__ csT, double* __restrict__ xty) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + w;
  if (p > P) return;
  uint8_t* prow = opk + p * (nRp / 4);
  if (p == P) {   // the zero row
    for (int64_t q = l; q < nRp / 4; q += 64) prow[q] = 0;
    return;
  }
  const int8_t* row = g + p * n;
  for (int64_t q = l; q < nRp / 4; q += 64) {   // 2-bit packed copy: animal 4q+i at bits 2i
    uint32_t pk = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t src = rowmap[4 * q + i];
      pk |= (uint32_t)(src >= 0 ? (uint8_t)row[src] : 0u) << (2 * i);
    }
    prow[q] = (uint8_t)pk;
  }
  const int64_t nTp = (nT + TILE - 1) / TILE * TILE;
  int s = 0;
  double dot[MAXT] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t r = l; r < nT; r += 64) {
    const int32_t src = rowmap[r];
    const int8_t v = src >= 0 ? row[src] : (int8_t)0;
    {
      s += v;
#pragma unroll
      for (int t = 0; t < MAXT; ++t)
        if (t < nt) dot[t] += (double)v * (yT[t * nTp + r] - ymu[t]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
#pragma unroll
    for (int t = 0; t < MAXT; ++t) dot[t] += __shfl_xor(dot[t], o);
  }
  if (l == 0) {
    csT[p] = s;
#pragma unroll
    for (int t = 0; t < MAXT; ++t)
      if (t < nt) xty[t * P + p] = dot[t];
  }
}

hipError_t launch_build_split(const int8_t* geno_sm, int64_t n, int64_t P, const int32_t* rowmap, int64_t nRp,
                              int64_t nT, const double* yT, const double* ymu, int nt,
                              uint8_t* geno_packed, int32_t* colsum_T, double* xty, hipStream_t s) {
  hipLaunchKernelGGL(k_build_split, dim3((unsigned)((P + 1 + 3) / 4)), dim3(256), 0, s, geno_sm, n, P, rowmap, nRp,
                     nT, yT, ymu, nt, geno_packed, colsum_T, xty);
  return hipGetLastError();
}

// fold-fused offsets: system s = f * B + b takes individual b's index list from the f-th copy
__global__ void k_fold_offsets(const int64_t* __restrict__ off, int64_t B, int64_t F, int64_t sum_k,
                               int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < F * B) out[i] = (i / B) * sum_k + off[i % B];
  if (i == 0) out[F * B] = F * sum_k;
}

hipError_t launch_fold_offsets(const int64_t* off, int64_t B, int64_t F, int64_t sum_k, int64_t* out, hipStream_t s) {
  const int64_t n = F * B;
  hipLaunchKernelGGL(k_fold_offsets, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, off, B, F, sum_k, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// per-individual scalars: branch, 1/N, q/N^2, 1/d, mu, lambda
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(STATS_THREADS) void k_indiv_stats(const int64_t* __restrict__ idx, const int64_t* __restrict__ off,
                                                               FoldTab ft, const int32_t* __restrict__ csA, int64_t n, int64_t nT, int64_t nTp, int64_t P, int form,
                                                               int64_t ns, int pad_first, int nt, int branch, double h2,
                                                               double* __restrict__ scal, double* __restrict__ u,
                                                               double* __restrict__ rhs, int32_t* __restrict__ err) {
  __shared__ StatsShared sh;
  stats_wg(idx, off, ft, csA, n, nT, nTp, P, form, ns, pad_first, nt, branch, h2, blockIdx.x, scal, err, sh);
  if (form == FORM_PRIMAL) stats_rows(idx, off, ft, P, ns, pad_first, nt, blockIdx.x, u, rhs, sh, 0, ns);
}

hipError_t launch_indiv_stats(const int64_t* idx, const int64_t* off, int64_t B, const FoldTab& ft,
                              const int32_t* colsum_all, const EvalDims& d, const SysDims& sd,
                              int branch, double h2, double* scal, double* u, double* rhs, int32_t* err,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_indiv_stats, dim3((unsigned)B), dim3(STATS_THREADS), 0, s, idx, off, ft, colsum_all, d.n,
                     d.nT, d.nTp, d.P, sd.form, sd.ns, sd.pad_first, d.nt, branch, h2, scal, u, rhs, err);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// gather: panel[b][r][pk_row] (animal rows, 2-bit packed over the selected SNPs: 16 B per 64-SNP
// block, byte j holding SNPs 4j..4j+3 at bits 2i; SNPs past k are zero) + u_r = sum m_s a_rs
//   grid (nRp/128, B), 128 threads; thread t owns animal row r0 + t.
//   Each 256-SNP stage: 256 gathered packed SNP rows x 128 animals (32 B each) staged in LDS
//   (16-B row-segment loads), transposed by 2-bit reads, and stored as one 64-B piece per row.
// ---------------------------------------------------------------------------
constexpr int GST = 4 * KBLK;   // SNPs per gather stage (one 64-B packed row piece)
__global__ __launch_bounds__(128) void k_gather(FoldTab ft, const int64_t* __restrict__ idx,
                                                const int64_t* __restrict__ off,
                                                int64_t panel_stride, const int32_t* __restrict__ csA,
                                                const double* __restrict__ scal, int64_t P, int64_t nRp,
                                                int64_t pk_row, uint8_t* __restrict__ panel,
                                                double* __restrict__ u) {
  static_assert(GATHER_ROWS == 128, "two SNP rows and four 16-B row pieces per thread and stage");
  __shared__ __attribute__((aligned(16))) uint32_t tile[GST][GATHER_ROWS / 16];   // 2-bit packed
  __shared__ int64_t srow[GST];
  __shared__ int32_t sm[GST];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * GATHER_ROWS;
  const int64_t o0 = off[b], k = off[b + 1] - o0;
  const int mode = (int)scal[b * SCAL + SC_MODE];
  // the system's split (fold-fused batches), 2-bit packed SNP rows of nRp / 4 bytes
  const uint8_t* __restrict__ gp = ft.gpk[fold_of(ft, b)];
  const int32_t* cs = (mode == 1) ? csA : ft.csT[fold_of(ft, b)];
  const int64_t nst = (k + GST - 1) / GST;
  uint8_t* pb = panel + b * panel_stride + (r0 + t) * pk_row;
  int64_t uacc = 0;
  for (int64_t st = 0; st < nst; ++st) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = t + 128 * e;
      const int64_t s = st * GST + j;
      if (s < k) {
        const int64_t p = snp_col(idx[o0 + s], P);
        srow[j] = p;
        sm[j] = cs[p];
      } else {
        srow[j] = -1;
        sm[j] = 0;
      }
    }
    __syncthreads();
    // 256 SNP rows x 128 animals at 2 bits = 256 x 32 B: four 16-B chunks per thread
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = t + 128 * e, j = q >> 1, c = q & 1;
      const int64_t p = srow[j];
      v4i v = {0, 0, 0, 0};
      if (p >= 0) v = *reinterpret_cast<const v4i*>(gp + p * (nRp / 4) + r0 / 4 + 16 * c);
      *reinterpret_cast<v4i*>(&tile[j][4 * c]) = v;
    }
    __syncthreads();
    v4i out[4];
    int64_t us = 0;
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      uint32_t word = 0;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int j = d * 16 + e;
        const uint32_t g = (tile[j][t >> 4] >> (2 * (t & 15))) & 3u;   // animal r0 + t
        us += (int64_t)(sm[j] * (int32_t)g);   // <= 4n per term
        word |= g << (2 * e);
      }
      out[d >> 2][d & 3] = (int)word;
    }
    uacc += us;
    v4i* dst = reinterpret_cast<v4i*>(pb + st * 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = out[q];
    __syncthreads();
  }
  u[b * nRp + r0 + t] = (double)uacc;
}

hipError_t launch_gather(const FoldTab& ft, const int64_t* idx, const int64_t* off, int64_t panel_stride, int64_t B,
                         const int32_t* colsum_all, const double* scal, const EvalDims& d, int64_t pk_row,
                         uint8_t* panel, double* u, hipStream_t s) {
  dim3 grid((unsigned)(d.nRp / GATHER_ROWS), (unsigned)B);
  hipLaunchKernelGGL(k_gather, grid, dim3(GATHER_ROWS), 0, s, ft, idx, off, panel_stride, colsum_all,
                     scal, d.P, d.nRp, pk_row, panel, u);
  return hipGetLastError();
}

}  // namespace tblup
