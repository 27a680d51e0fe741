// Internal declarations shared by the HIP translation units of libtblup_gpu.so.
//
// Data layout in HBM (per context = one GPU):
//   geno_sm   int8  [P][n]        SNP-major genotypes, built once (transpose of the .npy)
//   colsum_all int32 [P]          per-SNP allele count over all n animals (gblup p)
//   per split s (train T, valid V; nTp/nVp = sizes rounded up to 128):
//     gpk       uint8 [P+1][nRp/4] SNP-major rows permuted to [T | 0-pad | V | 0-pad], nRp = nTp+nVp,
//                                 2-bit packed (animal 4j+i at bits 2i of byte j); row P is all zero
//                                 (padding rows of the primal form)
//     colsum_T  int32 [P]         allele counts over T (snp p)
//     xty       f64  [nt][P]      sum_t x_tp (y_t - mean y_T): the primal right-hand side, per SNP and trait
//     yT        f64 [nTp]         phenotypes of T (0 in padding), yV f64 [nV]
//   per evaluation chunk of B individuals (workspace):
//   Two equivalent forms of the per-individual system (chosen per chunk, see SysDims):
//     kernel (dual) form   rows = train animals (ns = nTp), contraction over the k SNPs
//     SNP (primal) form    rows = the k selected SNPs (ns = round_up(k)), contraction over
//                          the train animals -- sklearn Ridge's own choice when k <= n_T
//     panel  uint8 [b][nRp][dual_pk_row]  kernel form only: each system's animal rows 2-bit packed
//                                      over its k SNPs (the primal form reads gpk rows in place)
//     u      f64  [B][prow]            centring sums (dual: u_i = sum_s m_s a_is; primal: s_a)
//     scal   f64  [B][16]              see SC_* below
//     L      f64  [B][NT][NT][128^2]   Lt tiles (tile (I,J) holds L_IJ^T)
//     Dinv   f64  [B][NT][36][16x16]   X = L_JJ^{-1} of each diagonal tile, packed lower blocks
//     z      f64  [B][ns]              L^{-1} rhs
//     fit    f64  [B]
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace tblup {

constexpr int TILE = 128;      // output tile edge of the GRM and Cholesky kernels
constexpr int TBLUP_NSLOT = 2; // diagonal-tile preparation buffers per individual (slot J&1)
constexpr int KBLK = 64;       // SNPs per panel block (int8 MFMA K step)
constexpr int MAXT = 4;        // traits per context (multi-trait: one Cholesky, MAXT right-hand sides)
constexpr int GATHER_ROWS = 128;

// per-individual scalars scal[b][SCAL]
constexpr int SCAL = 16;
enum {
  SC_SA = 0,    // additive centring coefficient (dual 1/N, primal 0)
  SC_CN = 1,    // constant centring term (dual q/N^2, primal 0)
  SC_INVD = 2,  // 1/d
  SC_MUF = 3,   // intercept flag: 1 = snp branch (intercept mean(y_T) of each trait), 0 = gblup
  SC_LAM = 4,   // lambda = (1-h2)/h2
  SC_D = 5,     // d = 2 sum p(1-p)
  SC_MODE = 6,  // branch: 1 gblup, 2 snp
  SC_K = 7,     // selected SNPs
  SC_SM = 8,    // multiplicative centring coefficient (dual 0, primal 1/n_T)
  SC_NROW = 9,  // real system rows (dual n_T, primal k); the rest is identity padding
  SC_CBLK = 10, // contraction blocks of 64 for the system matrix
  SC_BAD = 11,  // 1 when an index lies outside [-P, P) (numpy would raise IndexError): fitness NaN
  SC_PAD = 12,  // leading padding rows (SNP form: ns - k, see SysDims::pad_first; kernel form 0)
};
// System row r is real (not identity padding) when pad <= r < pad + nrow.  SNP form: real row r
// holds selected SNP r - pad.  The padding leads so that its exact-zero rows and columns fall at
// the START of block column 0, where the Cholesky's contractions over L = 0 skip them
// (gemm1_a32 / syrk_lower8_32 start at row pad); trailing padding would sit in the output rows of
// the last tile row instead, split unevenly over the waves.
__host__ __device__ __forceinline__ bool sys_real(int64_t r, int64_t pad, int64_t nrow) {
  return (uint64_t)(r - pad) < (uint64_t)nrow;
}
enum { FORM_DUAL = 0, FORM_PRIMAL = 1 };

// Panel column of a selected-SNP index with numpy's fancy-index rule (the reference's
// data[:, indices], evaluator.py:275/298): -P <= p < 0 addresses column p + P.  Indices
// outside [-P, P) are rejected on the host (tblup_eval_batch) or flagged by k_indiv_stats
// (device entry); the clamp below only keeps such a flagged individual's loads in bounds.
__host__ __device__ __forceinline__ int64_t snp_col(int64_t p, int64_t P) {
  p = p < 0 ? p + P : p;
  return p < 0 ? 0 : (p >= P ? P - 1 : p);
}
constexpr int FLAG_WRITE_LJJ = 1 << 16;   // CholLaunch::skip: also store L_JJ (debug readback only)

// System dimensions of one chunk.
struct SysDims {
  int form;          // FORM_DUAL / FORM_PRIMAL
  int64_t ns;        // padded system size (multiple of TILE)
  int NT;            // ns / TILE
  int64_t prow;      // panel rows per contraction block
  int64_t cblk;      // contraction blocks per individual in the panel (max over the chunk)
  int pad_first = 0; // SNP form: padding rows lead (SC_PAD = ns - k; TBLUP_PAD_FIRST, default on)
};
// Kernel form: the gathered panel holds each system's prow (= n_Rp) animal rows 2-bit packed over its
// selected SNPs -- byte j of a row holds SNPs 4j..4j+3 at bits 2i, the SNP-form split rows' code --
// in whole 64-B (256-SNP) stages: bytes per row
inline int64_t dual_pk_row(const SysDims& sd) { return (sd.cblk + 3) / 4 * 64; }

typedef double v2d __attribute__((ext_vector_type(2)));
typedef double v4d __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

struct EvalDims {
  int64_t n;        // animals in the panel
  int64_t P;        // SNPs in the panel
  int64_t nT, nV;   // split sizes
  int64_t nTp, nVp; // padded to TILE
  int64_t nRp;      // nTp + nVp
  int NT;           // nTp / TILE
  int NR;           // nRp / TILE
  int nt;           // traits
};

// LDS-DMA of 16 B per lane (lane i -> lds + 16 i) as inline asm, for the stage rings.  The compiler
// sees __builtin_amdgcn_global_load_lds as an LDS write in flight and waits vmcnt(0) before the
// next LDS read of ANY address (ROCm 7.2, checked in the emitted code): in a ring that issues
// stage s + 1 and then reads stage s, that wait drained the prefetch, so every stage's load
// latency was exposed.  Hidden from the compiler, the DMA is ordered by the ring's own counted
// s_waitcnt + barrier, which every reader of a stage sits behind (the compiler's own counted waits
// on its loads stay correct: an extra outstanding DMA only makes them wait for more).  m0 is saved
// and restored around the DMA (its LDS address is sampled at issue), so the asm leaves m0 as the
// compiler last set it: builtin LDS-DMAs beside these rings keep whatever m0 setup the compiler
// hoisted or merged for them, by construction.  (m0 is a reserved register, so it cannot be
// declared clobbered: clang warns that the clobber is not honoured.)
__device__ __forceinline__ void glds16_asm(const void* g, const void* lds) {
  const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(la)
      : "memory");
}

// ---- packed lower-triangular 16x16 block storage of a 128x128 tile (LDS and Dinv) ----
constexpr int NB = 16;                       // base block edge
constexpr int NBLK = TILE / NB;              // 8 block rows
constexpr int NPACK = NBLK * (NBLK + 1) / 2; // 36 lower blocks
constexpr int BLKD = NB * NB;                // doubles per block

__host__ __device__ __forceinline__ int pk(int q, int s) { return (q * (q + 1) / 2 + s) * BLKD; }
// element (r, c) of a 16x16 block; 16-B chunk swizzle makes the fragment reads conflict-free
__host__ __device__ __forceinline__ int bo(int r, int c) { return r * NB + 2 * ((c >> 1) ^ ((r >> 1) & 7)) + (c & 1); }

// Per-split device data of the systems of one launch sequence.  One split: nf = 1.  Fold-fused
// evaluation (tblup_eval_folds*: IntraGCV's k folds as one batch of F x B systems, system
// s = f * bpf + b against split f; every split of equal dimensions): one entry per fold.
constexpr int MAXF = 16;
struct FoldTab {
  int64_t bpf;                 // systems per fold (the chunk's B when nf = 1)
  int nf;
  int share;                   // every fold's train + valid rows are one multiset (k_sys_tiles_folds)
  const uint8_t* gpk[MAXF];    // 2-bit packed split rows [P+1][nRp/4]
  const int32_t* csT[MAXF];    // train allele counts [P]
  const double* xty[MAXF];     // [nt][P]
  const double* yV[MAXF];      // [nt][nV]
  const double* yT[MAXF];      // [nt][nTp] (kernel form: the right-hand sides y_T - mu on the fly)
  const double* ymu[MAXF];     // [nt]
  // kernel form with shared counts (IntraGCV, share): every system's int8 count A_r . A_c is read
  // from its individual's A_R A_R^T over fold 0's split rows (k_gshare), system row r of fold f at
  // row gmap[f][r] (-1: padding) -- one int8 GEMM per individual instead of one per fold
  int32_t* gsh;                // [bpf][gsh_ld][gsh_ld] (null: counts per system, int8 MFMA in the units)
  const int32_t* gmap;         // [nf][gmap_ld]
  int64_t gsh_ld, gmap_ld;     // nRp, nTp
};
__host__ __device__ __forceinline__ int fold_of(const FoldTab& ft, int64_t s) { return (int)(s / ft.bpf); }

// ---- launchers (k_prep.hip) ----
hipError_t launch_transpose_geno(const int8_t* src, int8_t* dst, int64_t n, int64_t P, hipStream_t s);
hipError_t launch_colsum_all(const int8_t* geno_sm, int32_t* colsum, int64_t n, int64_t P, hipStream_t s);
hipError_t launch_build_split(const int8_t* geno_sm, int64_t n, int64_t P, const int32_t* rowmap,
                              int64_t nRp, int64_t nT, const double* yT, const double* ymu, int nt,
                              uint8_t* geno_packed, int32_t* colsum_T, double* xty,
                              hipStream_t s);
// fused offsets of F copies of a B-individual index list (sum_k indices each): out[F * B + 1]
hipError_t launch_fold_offsets(const int64_t* off, int64_t B, int64_t F, int64_t sum_k, int64_t* out, hipStream_t s);
// primal form (sd.form): also u[b][a] = s_a and rhs[b][t][a] = xty[t][p_a] / d over the ns rows
// (colsum_T / xty of system b: ft's fold of b)
hipError_t launch_indiv_stats(const int64_t* idx, const int64_t* off, int64_t B, const FoldTab& ft,
                              const int32_t* colsum_all, const EvalDims& d, const SysDims& sd,
                              int branch, double h2, double* scal, double* u, double* rhs, int32_t* err,
                              hipStream_t s);
// kernel form: each system's 2-bit packed animal rows (dual_pk_row bytes each) from its split's rows
// (ft: fold of system b)
hipError_t launch_gather(const FoldTab& ft, const int64_t* idx, const int64_t* off, int64_t panel_stride, int64_t B,
                         const int32_t* colsum_all, const double* scal, const EvalDims& d, int64_t pk_row,
                         uint8_t* panel, double* u, hipStream_t s);

// ---- launchers (k_grm.hip) ----
hipError_t launch_grm(const uint8_t* panel, int64_t panel_stride, int64_t pk_row, const int64_t* off, const double* u,
                      const double* scal, const EvalDims& d, int64_t B, double* K, hipStream_t s);

// ---- launchers (k_chol.hip, k_solve.hip) ----
// SNP form with k_sys_tiles_st (which reads no scalar): k_indiv_stats' inputs and outputs, when the
// scalars are formed in the launch after the system tiles (k_stats_diag_counts, fused with the
// K_JJ + lambda I epilogue of the tiles J < 2) instead of in a launch of their own before them
struct StatsFuse {
  const int32_t* csA;    // allele counts over all n animals (gblup p)
  int64_t n, nT;
  int branch;
  double h2;
  int32_t* err;          // the context's index-error status word
  double* scal;          // [B][SCAL]
  double* u;             // [B][ns]
  double* rhs;           // [B][nt][ns]
};
// 4 KiB between individuals' Lt tiles, so the same tile of different individuals does not start on the
// same HBM channel offset: off-diagonal -5 us at pop 128, solve -1% (A/B, profiles/r06_lpad_ab.txt;
// 64 KiB was slower, 260 KiB even)
#ifndef TBLUP_AB_LPAD   // A/B builds (tools/ab_build_defs.sh): doubles of padding between individuals' L
#define TBLUP_AB_LPAD 512
#endif
constexpr int64_t L_PAD = TBLUP_AB_LPAD;
// doubles from one individual's Lt tiles to the next's
__host__ __device__ inline int64_t l_stride(int NT) { return (int64_t)NT * NT * TILE * TILE + L_PAD; }
struct CholLaunch {
  EvalDims d;
  SysDims sd;
  int64_t B;
  double* L;             // Lt tiles [B][NT][NT][128*128] (tile (I,J) holds L_IJ^T)
  double* Dinv;          // [B][NT][NPACK*BLKD] X = L_JJ^{-1}, packed lower 16x16 blocks
  double* z;             // [B][nt][ns]
  double* w;             // [B][nt][ns] forward-substitution partial sums
  const double* rhs;     // [B][nt][ns] primal right-hand sides (dual: y_T - mu on the fly)
  double* S;             // [B][2][36*256] diagonal-tile preparation, slot J&1
  double* Kd;            // [B][NT][36*256] GRM diagonal tiles K_JJ + lambda I (kernel form / no system tiles)
  const double* yT;      // split phenotypes [nt][nTp] (kernel form: one split)
  const uint8_t* panel;  // kernel form: the gathered 2-bit packed animal rows (dual_pk_row bytes each)
  int64_t pstride;       // panel bytes per individual
  const int64_t* off;    // [B+1] device offsets
  const int64_t* idx;    // device SNP indices of the chunk
  int64_t gs_row;        // bytes per int8 split row (nRp): split SNP-major matrix, row P zero
  int64_t gpk_row;       // bytes per 2-bit packed split row (nRp / 4)
  FoldTab ft;            // split rows, counts, right-hand sides and phenotypes of each system's split
  const double* u;       // [B][prow]
  const double* scal;    // [B][SCAL]
  int skip;              // diagnostic ablation mask (env TBLUP_DBG_SKIP), 0 in production
  uint64_t* wgt;         // per-workgroup timestamp records of this launch (env TBLUP_WG_TRACE), else null
  int16_t* kc;           // exact off-diagonal system-tile counts from k_sys_tiles (either form), else null
  double* part;          // [2][B][NT][128*128] partial sums of the next column's tiles (ahead schedule)
  double* q;             // last-term mode: [B][36*256] diagonal tile J's last SYRK term, from launch J-1
  int padskip;           // contractions over block column 0 skip the leading padding rows (SC_PAD)
  int16_t* kd;           // with k_sys_tiles: the diagonal tiles' exact counts instead of Kd,
                         // [B][NT][36 packed lower blocks][64 lanes][4] (KD_TILE int16 per tile); the
                         // consumers form K_JJ + lambda I from them (kd_block, k_chol.hip)
  int sys_st = -1;       // k_sys_tiles_st: -1 auto, 0 never, 1 whenever it applies (TBLUP_SYS_ST)
  const StatsFuse* stats = nullptr;   // launch_sys_tiles: form the scalars after k_sys_tiles_st
};
// k_sys_tiles output: per individual NT(NT-1)/2 off-diagonal tiles (I > J, t = I(I-1)/2 + J) of
// 128 x 128 int16 counts, in the order the off-diagonal kernel's lanes read them:
// [column block ib][row block cb][lane][4].  Exact while n_T <= 8191 (counts <= 4 n_T).
constexpr int64_t KC_TILE = (int64_t)TILE * TILE;
constexpr int64_t KD_TILE = (int64_t)NPACK * BLKD;   // diagonal tile counts: the 36 lower 16x16 blocks
constexpr int64_t KC_MAX_NT = 8191;
// workgroup trace record (profiling only): {start, end, kind << 56 | I << 40 | b, J},
// s_memrealtime ticks (100 MHz); kinds below
constexpr int WGT_REC = 4;
// a diagonal launch's records are followed by DTR_RECS records holding the phase stamps of
// its workgroup 0 (8 waves x 64 uint64), written as kind-0 records
constexpr int DTR_RECS = 8 * 64 / WGT_REC;
enum { WGT_DIAG = 1, WGT_TILE = 2, WGT_PREP = 3, WGT_KJJ = 4, WGT_SYS = 5, WGT_PART = 6, WGT_DPREP = 9, WGT_EPART = 10 };   // 7 / 8: the chained solve (k_solve.hip)
// Work units of the off-diagonal launch of column J, per individual (k_chol.hip):
//   nI  T-units: tiles (I, J), I > J
//   nP  x nrs P-units (ahead schedule): partial sums K - sum_{L<J} of tiles (I, J+1), I >= J+2, in
//       nrs row slices -- launch J+1's T-units then start from them (ahead_cur) and sum one L
//   nds D-units: the diagonal tile J+1's partial sum over L < J (1 or 2 block slices)
//   n_kd K_JJ workgroups (column 0 of the kernel form only)
//   ndd: the D-units run in the DIAGONAL launch J instead (whole, one per individual; nds = 0), on
//   the CUs its B workgroups leave idle -- they need only the columns L < J, complete before it
//   ne  E-units, also in the DIAGONAL launch J (after its D-units), one per CU still idle: the GEMM1
//       term L = Ls0 (Ls0 = J-1 after an ahead launch, else 0) of column J's tiles e < ne in
//       I-major order (tile (J+1 + e / B, J) of individual e % B), into the partial-sum slot J&1;
//       such a tile's T-unit starts from that partial and sums from Ls0 + 1 (its MFMA chains
//       unchanged: bit-identical)
struct OffPlan {
  int nI, nP, nrs, nds, ahead_cur;
  int ndd;
  int64_t n_kd;
  int64_t ne;
  __host__ __device__ int64_t units() const { return (int64_t)nP * nrs + nds + nI; }
};
// Schedule policy (host, per chunk: a function of B and the system shape only, so the results
// are bit-identical for any policy -- every accumulator keeps its MFMA chain):
//   ahead: -1 auto (launch j ahead when B * (NT - 2 - j) < AHEAD_SLOTS; measured at config 2 against
//   the classic schedule: +14% at B = 32, +2.3% at B = 128, even at 256; a whole-chunk B < 64 rule
//   and thresholds 512 / 1024 were slower at 128), 0 never, 1 always; nrs: 0 auto (fill >= 2 units per CU
//   slot pair), else fixed 1 / 2 / 4; without k_sys_tiles counts (int8 K in-tile) nrs = 1
constexpr int64_t AHEAD_SLOTS = 256;
// diag_d: D-units in the diagonal launch, -1 auto (DD_MIN_B < B <= DD_MAX_B and J <= DD_MAX_J), 0 never,
// 1 always.  Measured (config 2, A/B): pop 128 +2.4% (off-diagonal -49 us, diagonal +11 us per step);
// pop 64 -0.8%, pop 32 -1.5% (their off-diagonal launches are bound by other units, and the diagonal
// launches still grow); every J (TBLUP_DIAG_D=1): diagonal +100 us at pop 128
constexpr int64_t DD_MIN_B = 64;
constexpr int64_t DD_MAX_B = 128;
#ifndef TBLUP_AB_DD_MAX_J   // A/B builds only (tools/ab_build_defs.sh)
#define TBLUP_AB_DD_MAX_J 3
#endif
constexpr int DD_MAX_J = TBLUP_AB_DD_MAX_J;
// diag_e: E-units in the diagonal launch, -1 auto (one per CU the launch's other workgroups leave
// idle, ncu - B (1 + ndd), up to the column's tiles; so none at B >= ncu), 0 never, 1 every tile of
// the column (tests), 2 only columns covered whole
OffPlan off_plan(int64_t B, int NT, int J, bool sys_tiles, int ahead, int nrs, int64_t slots = AHEAD_SLOTS,
                 int diag_d = 0, int dd_maxj = DD_MAX_J, int diag_e = 0, int64_t ncu = 0);
// multiprocessor count of the current device (256 when the query fails)
int cu_count();
inline int64_t offdiag_grid(const OffPlan& p, int64_t B) { return p.nI > 0 ? B * p.units() + p.n_kd : 0; }
// Fused GRM + tile Cholesky, column by column (k_chol.hip): diagonal tile J (k_chol_diag),
// then the off-diagonal tiles (I > J, J) plus the preparation of diagonal tile J+1.
hipError_t launch_chol_diag(const CholLaunch& c, int J, const OffPlan& p, hipStream_t s);
hipError_t launch_chol_offdiag(const CholLaunch& c, int J, const OffPlan& p, hipStream_t s);
// all diagonal GRM tiles K_JJ of the batch (one launch, before the column loop)
hipError_t launch_diag_grm(const CholLaunch& c, hipStream_t s);
// kernel form, shared fold counts: A_R A_R^T of every individual (FoldTab::gsh) from fold 0's panels
hipError_t launch_gshare(const CholLaunch& c, hipStream_t s);
// SNP form: every (I >= J) system tile of the batch on FP4 MFMA in one launch -- off-diagonal
// counts into c.kc, diagonal tiles' counts into c.kd (replaces launch_diag_grm and the int8 phase
// of the off-diagonal tiles)
hipError_t launch_sys_tiles(const CholLaunch& c, hipStream_t s);
// its grid: > 0 the persistent super-tile kernel's workgroups (k_sys_tiles_st), else minus the
// per-tile kernel's
int64_t sys_tiles_grid(const CholLaunch& c);
constexpr int SP_ROWTAB = 4096;   // k_sys_tiles_st: rows of its LDS row table (ns <= SP_ROWTAB)
// the same for a fold-fused chunk whose folds share their train + valid rows (FoldTab::share):
// C_{R_f} = C_{T_all} - C_{V_f}, one workgroup per (individual, tile) for all F folds
hipError_t launch_sys_tiles_folds(const CholLaunch& c, hipStream_t s);
// Back substitution, prediction and fitness.  ch == null: one workgroup per individual
// (k_solve); else (SNP form) the chained solve (k_solve_chain): an individual's block rows and
// tile products spread over the chip, handing beta_J and the partial products on through
// per-call flags (SolveChain).
struct SolveChain {
  int32_t* flags;   // [B][chain_flags(NT)], compared with seq (never reset)
  double* beta;     // [B][nt][ns]: beta_J, published by the pull units (flags [0, NT) of an individual)
  double* cpart;    // [B][NT (row I)][NT (tile J)][nt][128]: L_JI^T beta_J
  double* epart;    // [B][NT][nt][nV]: block J's share of X_V beta
  double* mbpart;   // [B][NT][nt]: block J's share of sum_a s_a beta_a
  int32_t* err;     // this call's slot of the expiry ring (CHAIN_ERR_RING words, slot seq % CHAIN_ERR_RING):
                    // = seq once a wait of the call gave up -- the call's later waits give up at once,
                    // and the host entries read it to re-run that chunk's solve through k_solve
  int32_t* expired; // device entries: the context's sticky solve-status word (set to 1 by a unit whose
                    // wait gave up; tblup_solve_error / tblup_status_async); host entries: a scratch
                    // word (they recover from their own ring slot instead)
  int32_t seq;      // this call's flag value
  int32_t mode;     // TBLUP_CHAIN_SYNC (k_solve.hip)
  int32_t spin_max; // polls before a wait gives up (CHAIN_SPIN_MAX; lowered only by the debug knob)
  int32_t pull;     // 1: pull units (block column J: beta_K, K > J, and the tiles (K, J)); 0: push units
  int32_t delay;    // debug knob only: U(0, NT-1) sleeps this many s_sleep(127) rounds before
                    // publishing, so its consumers' waits expire (0 in production)
};
// Bound on a hand-off wait: 2^20 polls (an sc1 load round trip each plus s_sleep 2: ~0.5-1 s).
// Progress does not need the bound (see k_solve.hip); it turns a broken dispatch assumption into
// an error the host reports instead of a hang.
constexpr int32_t CHAIN_SPIN_MAX = 1 << 20;
// expiry records, one slot per call sequence number modulo the ring size (after the flags)
constexpr int CHAIN_ERR_RING = 64;
// the context's device status words (tblup_index_error / tblup_solve_error / tblup_status_async)
enum { ST_INDEX = 0, ST_SOLVE = 1, ST_WORDS = 2 };
__host__ __device__ inline int64_t chain_flags(int NT) { return (int64_t)NT * (NT + 2); }
hipError_t launch_solve(const CholLaunch& c, const SolveChain* ch, double* fitness, double* ebv, hipStream_t s);

// ---- launcher (k_decode.hip): RandomKey genome decode, top-k of each key row ----
hipError_t launch_decode_topk(const double* keys, int64_t B, int64_t d, int64_t ld, const int64_t* off, int64_t* out,
                              hipStream_t s);

// ---- launcher (k_de.hip): one DE generation (mutation + binary crossover + clip) per individual ----
hipError_t launch_de_step(const uint32_t* key, int pos0, const uint32_t* polys, int end_jump, int end_s, int end_pos,
                          const double* parent, int64_t ldp, const int32_t* donors, const int64_t* fixed, int strategy,
                          double F, double cr, int clip, double hi, int64_t L, int pop, double* child, int64_t ldc,
                          uint32_t* key_out, int32_t* pos_out, hipStream_t s, const int32_t* strat_i = nullptr,
                          const double* F_i = nullptr, const double* cr_i = nullptr, uint32_t* scratch = nullptr);
// scratch (null: one launch, k_de_step): DE_SEQ_SCRATCH words for the base sequence + pop x 624 for
// the workgroups' windows -- the three-launch form for large populations (k_de.hip)
constexpr int64_t DE_SEQ_SCRATCH = 624 + 19937 + 624 + 64;

// ---- launcher (k_de.hip): rows from scattered device rows into one matrix (up to ROWPTRS rows
//      per launch, source pointers in the kernel arguments) ----
constexpr int ROWPTRS = 128;
struct RowPtrs {
  const double* p[ROWPTRS];
};
hipError_t launch_gather_rows(double* dst, int64_t ldd, int64_t L, const RowPtrs& src, int nr, hipStream_t s);

// ---- launcher (k_scan.hip): per-SNP sums over a set of animals (seeder GWAS metric) ----
hipError_t launch_snp_scan(const int8_t* geno_sm, int64_t n, int64_t P, const int32_t* rows, int64_t nr,
                           const double* yc, int64_t* sx, int64_t* sxx, double* sxy, hipStream_t s);

// XCD-aware bijective remap of a 1-D block id (blocks b and b+8 share an XCD
// under the observed round-robin placement; speed only, never correctness).
__device__ __forceinline__ int64_t xcd_remap(int64_t orig, int64_t nwg) {
  if (nwg <= 8) return orig;
  int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  int64_t base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

}  // namespace tblup
