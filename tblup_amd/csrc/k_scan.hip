// Per-SNP marginal regression sums over a set of animals: the data pass of the seeder's
// GWAS metric (tblup/seeder.py:144-160, 202-210: sklearn f_regression over X[train]).
//
// For every SNP s and the given animal rows R (any order, repeats allowed):
//   sx[s]  = sum_r x_rs,   sxx[s] = sum_r x_rs^2   (exact integers; x in {0,1,2})
//   sxy[s] = sum_r x_rs * yc_r                      (fp64, yc = the caller's centred phenotypes)
// which is everything r_regression needs (sklearn's X_norms from the exact moments, the
// y @ X product); F and p-values follow on the host exactly as sklearn forms them.
// One wave per SNP row of the SNP-major genotypes; the row ids and yc are staged in LDS
// once per workgroup and shared by its 8 waves.  HBM-bound: n bytes per SNP.
#include "tblup_internal.h"

namespace tblup {
namespace {

constexpr int SCAN_WAVES = 8;
constexpr int SCAN_STAGE = 4096;   // rows staged per LDS pass

__global__ __launch_bounds__(64 * SCAN_WAVES) void k_snp_scan(const int8_t* __restrict__ g, int64_t n, int64_t P,
                                                              const int32_t* __restrict__ rows, int64_t nr,
                                                              const double* __restrict__ yc, int64_t* __restrict__ sx,
                                                              int64_t* __restrict__ sxx, double* __restrict__ sxy) {
  __shared__ int32_t srow[SCAN_STAGE];
  __shared__ double sy[SCAN_STAGE];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * SCAN_WAVES + w;
  const int8_t* row = g + (p < P ? p : 0) * n;
  int64_t a1 = 0, a2 = 0;
  double ay = 0.0;
  for (int64_t r0 = 0; r0 < nr; r0 += SCAN_STAGE) {
    const int m = (int)(nr - r0 < SCAN_STAGE ? nr - r0 : SCAN_STAGE);
    __syncthreads();
    for (int t = threadIdx.x; t < m; t += 64 * SCAN_WAVES) {
      srow[t] = rows[r0 + t];
      sy[t] = yc[r0 + t];
    }
    __syncthreads();
    if (p < P) {
      for (int t = l; t < m; t += 64) {
        const int x = row[srow[t]];
        a1 += x;
        a2 += x * x;
        ay += (double)x * sy[t];
      }
    }
  }
  // fixed-order wave reduction: deterministic sums
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a1 += __shfl_xor(a1, o);
    a2 += __shfl_xor(a2, o);
    ay += __shfl_xor(ay, o);
  }
  if (p < P && l == 0) {
    sx[p] = a1;
    sxx[p] = a2;
    sxy[p] = ay;
  }
}

}  // namespace

hipError_t launch_snp_scan(const int8_t* geno_sm, int64_t n, int64_t P, const int32_t* rows, int64_t nr,
                           const double* yc, int64_t* sx, int64_t* sxx, double* sxy, hipStream_t s) {
  hipLaunchKernelGGL(k_snp_scan, dim3((unsigned)((P + SCAN_WAVES - 1) / SCAN_WAVES)), dim3(64 * SCAN_WAVES), 0, s,
                     geno_sm, n, P, rows, nr, yc, sx, sxx, sxy);
  return hipGetLastError();
}

}  // namespace tblup
