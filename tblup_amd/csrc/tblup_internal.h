// Internal declarations shared by the HIP translation units of libtblup_gpu.so.
//
// Data layout in HBM (per context = one GPU):
//   geno_sm   int8  [P][n]        SNP-major genotypes, built once (transpose of the .npy)
//   colsum_all int32 [P]          per-SNP allele count over all n animals (gblup p)
//   per split s (train T, valid V; nTp/nVp = sizes rounded up to 128):
//     geno      int8 [P][nRp]     SNP-major rows permuted to [T | 0-pad | V | 0-pad], nRp = nTp+nVp
//     colsum_T  int32 [P]         allele counts over T (snp p)
//     yT        f64 [nTp]         phenotypes of T (0 in padding), yV f64 [nV]
//   per evaluation chunk of B individuals (workspace):
//     panel  int8 [b][kblk][nRp][64]  gathered genotypes, animal-major 64-SNP blocks (stride = max kblk)
//     u      f64  [B][nRp]            u_i = sum_s m_s a_is (exact integers)
//     scal   f64  [B][8]              1/N, q/N^2, 1/d, mu, lambda, d, branch, k
//     K      f64  [B][nRp][nTp]       GRM block K_{R,T}; TT lower triangle overwritten by L
//     Dinv   f64  [B][NT][128][128]   inverse of each diagonal Cholesky tile
//     z      f64  [B][nTp]            L^{-1}(y_T - mu)
//     fit    f64  [B]
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace tblup {

constexpr int TILE = 128;      // output tile edge of the GRM and Cholesky kernels
constexpr int TBLUP_NSLOT = 5; // diagonal-tile slots per individual: 4 SYRK partials + the assembled tile
constexpr int KBLK = 64;       // SNPs per panel block (int8 MFMA K step)
constexpr int GATHER_ROWS = 128;

typedef double v2d __attribute__((ext_vector_type(2)));
typedef double v4d __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

struct EvalDims {
  int64_t n;        // animals in the panel
  int64_t P;        // SNPs in the panel
  int64_t nT, nV;   // split sizes
  int64_t nTp, nVp; // padded to TILE
  int64_t nRp;      // nTp + nVp
  int NT;           // nTp / TILE
  int NR;           // nRp / TILE
};

// ---- launchers (k_prep.hip) ----
hipError_t launch_transpose_geno(const int8_t* src, int8_t* dst, int64_t n, int64_t P, hipStream_t s);
hipError_t launch_colsum_all(const int8_t* geno_sm, int32_t* colsum, int64_t n, int64_t P, hipStream_t s);
hipError_t launch_build_split(const int8_t* geno_sm, int64_t n, int64_t P, const int32_t* rowmap,
                              int64_t nRp, int64_t nT, int8_t* geno_split, int32_t* colsum_T,
                              hipStream_t s);
hipError_t launch_indiv_stats(const int64_t* idx, const int64_t* off, int64_t B, const int32_t* colsum_T,
                              const int32_t* colsum_all, const EvalDims& d, int branch, double meanyT,
                              double h2, double* scal, hipStream_t s);
hipError_t launch_gather(const int8_t* geno_split, const int64_t* idx, const int64_t* off,
                         int64_t panel_stride, int64_t B, const int32_t* colsum_T,
                         const int32_t* colsum_all, const double* scal, const EvalDims& d,
                         int8_t* panel, double* u, hipStream_t s);

// ---- launchers (k_grm.hip) ----
hipError_t launch_grm(const int8_t* panel, int64_t panel_stride, const int64_t* off, const double* u,
                      const double* scal, const EvalDims& d, int64_t B, double* K, hipStream_t s);

// ---- launchers (k_chol.hip, k_solve.hip) ----
struct CholLaunch {
  EvalDims d;
  int64_t B;
  double* L;             // Lt tiles [B][NT][NT][128*128] (tile (I,J) holds L_IJ^T)
  double* Dinv;          // [B][NT][128][128]
  double* z;             // [B][nTp]
  double* w;             // [B][nTp] forward-substitution partial sums
  double* S;             // [B][TBLUP_NSLOT][36*256] SYRK partials + assembled diagonal tile
  double* Kd;            // [B][NT][36*256] GRM diagonal tiles
  const double* yT;      // split phenotypes [nTp]
  const double* yV;      // [nV]
  const int8_t* panel;   // gathered genotypes
  int64_t pstride;       // panel bytes per individual
  const int64_t* off;    // [B+1] device offsets
  const double* u;       // [B][nRp]
  const double* scal;    // [B][8]
  int skip;              // diagnostic ablation mask (env TBLUP_DBG_SKIP), 0 in production
};
// one tile column J of the fused GRM + Cholesky: diag=true -> k_chol_diag, else k_chol_offdiag
hipError_t launch_chol(const CholLaunch& c, int J, hipStream_t s, bool diag);
// all diagonal GRM tiles K_JJ of the batch (one launch, before the column loop)
hipError_t launch_diag_grm(const CholLaunch& c, hipStream_t s);
hipError_t launch_solve(const CholLaunch& c, double* fitness, double* ebv, hipStream_t s);

// XCD-aware bijective remap of a 1-D block id (blocks b and b+8 share an XCD
// under the observed round-robin placement; speed only, never correctness).
__device__ __forceinline__ int64_t xcd_remap(int64_t orig, int64_t nwg) {
  if (nwg <= 8) return orig;
  int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  int64_t base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

}  // namespace tblup
