// Batched left-looking tile Cholesky of (K_TT + lambda I), fp64, 128x128 tiles,
// with the GRM tiles from exact integer counts (K is never stored in fp64).
//
// Replaces the reference's per-individual dense solves
//   gblup:    G_inv = np.linalg.inv(G_TT + lambda I)          (tblup/evaluator.py:280-284)
//   snp_blup: Ridge(alpha).fit -> scipy.linalg.solve(assume_a="pos") (evaluator.py:311-312,
//             scikit-learn 1.7.2 _ridge.py _solve_cholesky[_kernel])
// by one Cholesky factorisation per individual, batched over the population.
// For each tile column J:
//   k_chol_diag    (one WG per individual): K_JJ (int8 MFMA) - sum_L L_JL L_JL^T (fp64 MFMA
//                  SYRK on the lower blocks), blocked 16x16 factorisation, blocked inverse
//                  X_J = L_JJ^{-1}, forward-substitution block z_J = X_J (y_J - mu - w_J)
//   k_chol_offdiag (one WG per individual x tile row I > J), all transposes in registers:
//                  T^T = K_JI - sum_L L_JL L_IL^T  (int8 MFMA for K, fp64 MFMA, acc = T^T)
//                  L_IJ^T = X_J T^T               (acc of T^T is the B operand directly)
//                  w_I += L_IJ z_J                (forward-substitution partial sums)
//
// Storage of L ("Lt"): tile-contiguous and transposed.  Tile (I, J), I >= J, of matrix b
// is 128x128 doubles at L + ((b*NT + I)*NT + J)*128*128 with Lt[j][i] = L[128I+i][128J+j],
// so a 16-k-row stage of any operand is 16 KiB contiguous and every tile write coalesces.
//
// MFMA layouts (verified on gfx950 by tools/mfma_probe*.hip):
//   f64 16x16x4 : A[i=l&15][k=l>>4], B[k=l>>4][j=l&15], C row=(l>>4)+4r, col=l&15
//   i8 16x16x64 : A row l&15, B col l&15, 16 B of k per lane, C row=4(l>>4)+r, col=l&15
//   i8 32x32x32 : C row=(r&3)+8(r>>2)+4(l>>5), col=l&31
// Reading the i8 16x16x64 A rows through the permutation pi(rho) = (rho>>2) + 4(rho&3)
// makes its accumulator land in the f64 C layout, so the exact integer GRM counts
// become the fp64 accumulators of the Cholesky GEMM without any data movement.
#include "i8_tile.h"
#include "k_stats.h"
#include <algorithm>
#include <type_traits>

namespace tblup {

namespace {

constexpr int BKD = 16;                // k rows per fp64 stage
constexpr int LTS = BKD * TILE;        // doubles in one 16-row stage of an Lt tile (16 KiB)
constexpr int TT = TILE * TILE;        // doubles per tile

__device__ __forceinline__ v4d mfma64(double a, double b, v4d c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// c - a*b: for f64 MFMA the BLGP field is the operand-negate mask (neg:[1,0,0] = -A)
__device__ __forceinline__ v4d mfma64_nega(double a, double b, v4d c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);
}

constexpr int NSLOT = TBLUP_NSLOT;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// (glds16_asm, the stage rings' LDS-DMA as inline asm: tblup_internal.h)
#ifndef TBLUP_AB_ASM_SYRK   // A/B builds only (tools/ab_build_defs.sh): the SYRK ring's DMA as inline asm
#define TBLUP_AB_ASM_SYRK 1
#endif
#ifndef TBLUP_AB_ASM_GEMM1   // the GEMM1 ring's DMA as inline asm
#define TBLUP_AB_ASM_GEMM1 1
#endif
// Non-temporal result stores (round 5): the L tiles of the T-units, the partial sums (P- / E-units),
// the diagonal targets S and last terms Q -- each read by a later launch, none by this one (the
// last-term read-back aside), and every line a kernel leaves dirty in L2 is written back at its
// end (the kernel boundary).  Interleaved A/B at config 2 (profiles/r05_nt_store_ab.txt): both on
// +0.9% at pop 256 (off-diagonal 1.611 -> 1.594 ms), +1.0% at 128, +0.9% at 64 (the L tiles alone:
// -0.3% at 64).  TBLUP_AB_NT_*: A/B builds only (tools/ab_build_defs.sh).
#ifndef TBLUP_AB_NT_L
#define TBLUP_AB_NT_L 1
#endif
#ifndef TBLUP_AB_NT_PART
#define TBLUP_AB_NT_PART 1
#endif
#ifndef TBLUP_AB_NT_X   // the diagonal kernel's X_J (Dinv) stores
#define TBLUP_AB_NT_X 0
#endif
#ifndef TBLUP_AB_NT_PLD   // the partial sums' and S's loads non-temporal (each read once; A/B:
#define TBLUP_AB_NT_PLD 1    // +0.7% at pop 128, +0.15% at 256, profiles/r05_nt_store_ab.txt)
#endif
#ifndef TBLUP_AB_NT_KD   // the K_JJ + lambda I tiles J < 2 of the system-tile epilogue
#define TBLUP_AB_NT_KD 0
#endif
template <bool NT>
__device__ __forceinline__ void st64(double* p, double v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}
#ifndef TBLUP_AB_ASM_I8   // the integer-count rings' DMA (int8 / packed tiles, per-tile system tiles) as inline asm
#define TBLUP_AB_ASM_I8 1
#endif
// one ring DMA: inline asm (A) or the builtin
template <bool A>
__device__ __forceinline__ void ring_glds(const void* g, void* lds) {
  if constexpr (A)
    glds16_asm(g, lds);
  else
    __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)lds, 16, 0, 0);
}

// Stage image [16 k][128 x] of an Lt tile: 16-B chunk p of row k holds source chunk
// p ^ 8(k&1), so the fragment pattern (16 x in one k row, the next k in lanes 16-31)
// covers all 64 banks.  One LDS-DMA instruction moves one 1 KiB k row.
__device__ __forceinline__ int lt_off(int k, int x) { return k * TILE + 2 * ((x >> 1) ^ (8 * (k & 1))) + (x & 1); }

// ---- int8 GRM tile in the f64 accumulator layout (offdiag) ----
// cnt[cb][ib] = sum_s A[16cb + pi-row][s] B[32w + 16ib + col][s] with A = panel rows of tile J
// (c) and B = panel rows of tile I (i).  Panel tiles [128 rows][64 B]; A chunk swizzle
// (row>>2)&3 and B chunk swizzle (row>>2)&2 keep both ds_read_b128 patterns conflict-free.
__device__ __forceinline__ int i8off_a(int row, int c) { return row * 64 + 16 * (c ^ ((row >> 2) & 3)); }
__device__ __forceinline__ int i8off_b(int row, int c) { return row * 64 + 16 * (c ^ ((row >> 2) & 2)); }

// ---- SYRK restricted to the 36 lower 16x16 blocks (diag kernel), A = Lt tiles (J, L) ----
__host__ __device__ constexpr int tri_q(int e) {
  int q = 0;
  while ((q + 1) * (q + 2) / 2 <= e) ++q;
  return q;
}
__host__ __device__ constexpr int tri_s(int e) { return e - tri_q(e) * (tri_q(e) + 1) / 2; }
// runtime row of packed lower block e (e < 36)
__device__ __forceinline__ int tri_q_rt(int e) {
  int q = (int)((__builtin_sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  if ((q + 1) * (q + 2) / 2 <= e) ++q;
  if (q * (q + 1) / 2 > e) --q;
  return q;
}


// acc (16x16, f64 MFMA C layout) += A(16x16) * B(16x16)^T, both blocks in LDS
__device__ __forceinline__ v4d mma_abt(const double* A, const double* Bt, v4d acc, int l) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int k = 4 * kk + (l >> 4);
    acc = mfma64(A[bo(l & 15, k)], Bt[bo(l & 15, k)], acc);
  }
  return acc;
}

// Factor the 16x16 SPD block D with ONE wave (no barriers): X <- L^{-1} (lower, zeros above),
// and L into D's lower triangle on the debug path.  Right-looking elimination with unscaled
// pivots; E = L'^{-1} is built by row operations on I alongside (L = L' D^{1/2}, X = D^{-1/2} E):
//   c > j : T_ic -= (T_ij / piv_j) T_jc
//   i > j : E_ic -= (T_ij / piv_j) E_jc (c < j),  E_ij = -T_ij / piv_j
// Column scaling by 1/sqrt(piv) is deferred to the end.
__device__ __forceinline__ double recip(double p) {
  double r = __builtin_amdgcn_rcp(p);
  double e = __builtin_fma(-p, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-p, r, 1.0);
  return __builtin_fma(r, e, r);
}

__device__ __forceinline__ double rdlane(double x, int lane) {
  const long long bits = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)bits, lane);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// x += x[lane J of this 16-lane row] * m in one instruction (DPP64 row_newbcast on src0).  The
// compiler does not see inside asm, so hazards are handled here: NOP = the DPP read-after-VALU-
// write wait for a register the previous instruction may have written (the next pivot's
// column); the others are volatile so they keep their order, in which no fmac reads a
// register the one before it wrote.  That the compiler places no other VALU write of an fmac's
// src0 within 2 wait states of it is checked on the built library by tools/check_dpp_hazards.py
// (tests/test_abi.py); an s_nop on every fmac instead would lengthen factor16's pivot chain.
template <int J, bool NOP>
__device__ __forceinline__ void fmac_row(double& x, double m) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "+v"(x) : "v"(m), "i"(J));
  else
    asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(m), "i"(J));
}

// Rows 0 and 2 of the wave to rows 1 and 3 (v_permlane16_swap on each 32-bit half).
__device__ __forceinline__ double even_rows_to_odd(double x) {
  const long long bits = __double_as_longlong(x);
  const unsigned lo = (unsigned)bits, hi = (unsigned)(bits >> 32);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __longlong_as_double(((long long)b[0] << 32) | (unsigned)a[0]);
}

// v on lanes whose row (lane & 15) is below J, +0 elsewhere: the lane mask is a constant in
// SGPRs (no compare on the pivot chain)
template <int J>
__device__ __forceinline__ double rows_below(double v) {
  constexpr unsigned long long r = (0xFFFFull << (J + 1)) & 0xFFFFull;
  constexpr unsigned long long msk = r | (r << 16) | (r << 32) | (r << 48);
  const long long bits = __double_as_longlong(v);
  int lo = (int)bits, hi = (int)(bits >> 32);
  asm("v_cndmask_b32_e64 %0, 0, %0, %2\n\tv_cndmask_b32_e64 %1, 0, %1, %2" : "+v"(lo), "+v"(hi) : "s"(msk));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// 16x16 factor and inverse.  Lane l = i + 16 g: even groups hold row i of T in x[0..15]
// (column c in register c), odd groups row i of E (the Gauss-Jordan inverse, starting at I)
// with column c in register 15 - c.  Pivot j: T_jj by v_readlane, l_i = T_ij / T_jj from the
// lane's own register j (zero for i <= j), handed from the T rows to the E rows by a
// permlane16 swap, then every register the two halves still need -- T columns > j, E columns
// <= j, the same registers thanks to E's reversed order -- takes x += x[row j] * (-l_i) in one
// DPP64 fmac.  Registers outside those sets only ever receive x += 0 or hold finished columns,
// so no per-element masks.  The next pivot's column goes first; for j < 7 it is an E column
// above the diagonal (E_jc = 0) for the odd groups, so it takes the multiplier before the swap
// and the swap leaves the pivot chain.  Same operations in the same order per element as the
// factor / elimination T_ic -= l_i T_jc, E_ic -= l_i E_jc, so the factor and its inverse are
// unchanged.  Row i of T is final after pivot i - 1 (later multipliers are 0 there), so T_ii,
// the pivot, is still in register i at the end.
template <int J, int R>
__device__ __forceinline__ void f16_upd(double (&x)[NB], double m) {
  if constexpr (R < NB) {
    if constexpr (R != J + 1) fmac_row<J, false>(x[R], m);
    f16_upd<J, R + 1>(x, m);
  }
}

template <int J, bool WL>
__device__ __forceinline__ void f16_steps(double (&x)[NB], double (&ls)[NB]) {
  if constexpr (J + 1 < NB) {
    const double piv = rdlane(x[J], J);
    if constexpr (WL) ls[J] = x[J];
    const double mt = rows_below<J>(-(x[J] * recip(piv)));
    const double m = even_rows_to_odd(mt);
    fmac_row<J, true>(x[J + 1], (J < 7) ? mt : m);   // next pivot's column first
    constexpr int R0 = (J + 1 < NB - 1 - J) ? J + 1 : NB - 1 - J;
    f16_upd<J, R0>(x, m);
    f16_steps<J + 1, WL>(x, ls);
  } else if constexpr (WL) {
    ls[J] = x[J];
  }
}

template <int C>
__device__ __forceinline__ void f16_store_l(double* D, const double (&ls)[NB], double rs_own, int l) {
  if constexpr (C < NB) {
    const double rc = __builtin_amdgcn_mov_dpp(rs_own, 0x150 + C, 0xF, 0xF, true);  // lane C's 1/sqrt(piv_C)
    if (l < 16 && l >= C) D[bo(l, C)] = ls[C] * rc;
    f16_store_l<C + 1>(D, ls, rs_own, l);
  }
}

__device__ __forceinline__ void fstamp(uint64_t* st, int slot) {
  if (st && (threadIdx.x & 63) == 0) st[slot] = __builtin_amdgcn_s_memrealtime();
}

// D: symmetric 16x16 block (both triangles) -> X = L^{-1} (and, WL, L into D's lower triangle;
// the diagonal L blocks are read back only by the debug path).  X must hold the reversed
// identity (X_{i,15-i} = 1) on entry: the E rows load it as their starting point.
template <bool WL>
__device__ __forceinline__ void factor16(double* D, double* X, int l, uint64_t* st) {
  const int i = l & 15;
  fstamp(st, 50);
  const bool t_row = ((l >> 4) & 1) == 0;
  const double* src = t_row ? D : X;
  double x[NB], ls[NB];
#pragma unroll
  for (int k = 0; k < NB / 2; ++k) {
    const v2d v = *reinterpret_cast<const v2d*>(src + bo(i, 2 * k));
    x[2 * k] = v[0];
    x[2 * k + 1] = v[1];
  }
  fstamp(st, 51);
  f16_steps<0, WL>(x, ls);
  fstamp(st, 52);
  // the pivot of row i from register i of the T rows, to the E rows by the same swap
  double own = x[0];
#pragma unroll
  for (int c = 1; c < NB; ++c) own = (i == c) ? x[c] : own;
  own = even_rows_to_odd(own);
  // deferred scaling: X_ic = E_ic / sqrt(piv_i) (E_ic = +0 above the diagonal); L_ic = T_ic / sqrt(piv_c)
  const double rs_own = 1.0 / sqrt(own);
  if (l >= 16 && l < 32) {
#pragma unroll
    for (int k = 0; k < NB / 2; ++k)
      *reinterpret_cast<v2d*>(X + bo(i, 2 * k)) = v2d{x[NB - 1 - 2 * k] * rs_own, x[NB - 2 - 2 * k] * rs_own};
  }
  if constexpr (WL) f16_store_l<0>(D, ls, rs_own, l);
  fstamp(st, 53);
}


}  // namespace

// Per-launch arguments shared by the two Cholesky kernels.
struct CholArgs {
  double* L;                // Lt tiles [B][NT][NT][128*128]
  double* Dinv;             // [B][NT][36 packed 16x16 blocks] X = L_JJ^{-1}
  double* z;                // [B][nt][ns]
  double* w;                // [B][nt][ns] forward-substitution partial sums
  double* S;                // [B][2][36*256] K_JJ - sum_{L<J-1} L_JL L_JL^T, slot J&1
  double* Kd;               // [B][NT][36*256] GRM diagonal tiles (k_diag_grm)
  const double* yT;         // [nt][ytp] dual right-hand sides (y_T - mu, on the fly)
  const double* rhs;        // [B][nt][ns] primal right-hand sides
  const uint8_t* panel;     // [B] x pstride: kernel form, prow packed animal rows of pstride / prow bytes
  int64_t pstride;
  const double* u;          // [B][prow]
  const double* scal;       // [B][SCAL]
  int64_t ns, prow;         // padded system size, panel rows per contraction block
  int form;
  // primal form: rows read in place from the split's 2-bit packed SNP-major matrix
  // (row P is zero; ft.gpk of the system's split)
  const int64_t* idx;
  const int64_t* off;
  int64_t gs_row, P;
  int64_t ytp;              // yT stride (nTp)
  int nt;                   // traits (right-hand sides)
  int NT, J;
  int skip;                 // diagnostic ablation mask (TBLUP_DBG_SKIP); 0 in production
  uint64_t* wgt;            // workgroup trace records (TBLUP_WG_TRACE), null in production
  uint64_t* dtr;            // diagonal launch: phase timestamps of workgroup 0 (TBLUP_WG_TRACE), else null
  const int16_t* kc;        // off-diagonal system-tile counts (k_sys_tiles, either form), else null
  double* part;             // [2][B][NT][128*128] off-diagonal partial sums K - sum_{L<J-1} (acc layout), slot J&1
  double* q;                // last-term mode: [B][NPACK*BLKD] L_{J,J-1} L_{J,J-1}^T, from launch J-1's tile (J, J-1)
  int64_t B;                // individuals in the chunk
  FoldTab ft;               // each system's split (ymu, packed rows)
  int padskip;              // contractions over block column 0 skip the leading padding rows (SNP form)
  int padfirst;             // SNP form: padding rows lead (SC_PAD = ns - k)
  int16_t* kd;              // with k_sys_tiles: the diagonal tiles' exact counts for J >= 2 (KD_TILE
                            // each; the D-units form K_JJ + lambda I where they read it, kd_block); Kd then
                            // holds J < 2 only (the diagonal kernel's direct reads)
};

// K_JJ + lambda I (identity on padding rows) of packed lower block e of individual b's diagonal tile J,
// from its exact counts (k_sys_tiles), minus sub (may be null), into the packed-block image dst: the
// f64 MFMA C layout, element (16 q + (l >> 4) + 4 r, 16 s + (l & 15)) of the tile at
// dst[pk(q, s) + bo((l >> 4) + 4 r, l & 15)], q / s the block's row / column.  cv: the block's
// counts (int2 load issued by the caller).  (v - 0.0 == v exactly, so sub = 0 stores K itself.)
__device__ __forceinline__ void kd_block(const CholArgs& a, int64_t b, int J, int e, int2 cv, v4d sub,
                                         double* dst) {
  const int l = threadIdx.x & 63;
  const double* sc = a.scal + b * SCAL;
  const double sa = sc[SC_SA], cN = sc[SC_CN], invd = sc[SC_INVD], lam = sc[SC_LAM], sm = sc[SC_SM];
  const int64_t nrow = (int64_t)sc[SC_NROW], pad = (int64_t)sc[SC_PAD];
  int q = 0;
  while ((q + 1) * (q + 2) / 2 <= e) ++q;
  const int sb = e - q * (q + 1) / 2;
  const int64_t j0 = (int64_t)J * TILE;
  const double* ub = a.u + b * a.prow + j0;
  const int il = 16 * sb + (l & 15);
  const int64_t gj = j0 + il;
  const double uj = ub[il];
  const int32_t c4[4] = {(int32_t)(int16_t)(cv.x & 0xffff), (int32_t)(int16_t)(cv.x >> 16),
                         (int32_t)(int16_t)(cv.y & 0xffff), (int32_t)(int16_t)(cv.y >> 16)};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int cl = 16 * q + (l >> 4) + 4 * r;
    const int64_t gi = j0 + cl;
    const double kv = grm_value(c4[r], ub[cl], uj, sa, cN, invd, sm);
    const double v = (sys_real(gi, pad, nrow) && sys_real(gj, pad, nrow)) ? kv + ((gi == gj) ? lam : 0.0)
                                                                         : ((gi == gj) ? 1.0 : 0.0);
    st64<TBLUP_AB_NT_PART>(dst + pk(q, sb) + bo((l >> 4) + 4 * r, l & 15), v - sub[r]);
  }
}
// The exact count tiles are written once (k_sys_tiles) and read once (the unit that forms their K):
// non-temporal accesses, so that 235 MB of them a step do not push the Lt tiles out of the caches
__device__ __forceinline__ int2 nt_load2(const int16_t* p) {
  const long long v = __builtin_nontemporal_load(reinterpret_cast<const long long*>(p));
  return int2{(int)(unsigned)(v & 0xffffffffll), (int)(v >> 32)};
}
__device__ __forceinline__ void nt_store2(int16_t* p, int2 v) {
  __builtin_nontemporal_store((long long)(((unsigned long long)(unsigned)v.y << 32) | (unsigned)v.x),
                              reinterpret_cast<long long*>(p));
}
__device__ __forceinline__ int2 kd_load(const CholArgs& a, int64_t b, int J, int e) {
  const int l = threadIdx.x & 63;
  return nt_load2(a.kd + ((b * a.NT + J) * KD_TILE) + (e * 64 + l) * 4);
}

// Leading contraction rows of block column 0 that a GEMM1 / SYRK run starting at L = 0 skips:
// individual b's leading padding rows (SC_PAD), rounded down to the MFMA's 4-row k-step.
__device__ __forceinline__ int skip_rows(const CholArgs& a, int64_t b) {
  return a.padskip ? ((int)a.scal[b * SCAL + SC_PAD] & ~3) : 0;
}

// st: profiling only (phase stamps of one factorisation in diagonal workgroup 0), else null
__device__ __forceinline__ void factor16_any(const CholArgs& a, double* D, double* X, int l, uint64_t* st = nullptr) {
  if (a.skip & FLAG_WRITE_LJJ)
    factor16<true>(D, X, l, st);
  else
    factor16<false>(D, X, l, st);
}

// Profiling only: lane 0 of each wave of diagonal workgroup 0 stamps phase boundaries
// (s_memrealtime) into dtr[wave * 64 + slot].
__device__ __forceinline__ void dstamp(const CholArgs& a, int slot) {
  if (a.dtr && blockIdx.x == 0 && (threadIdx.x & 63) == 0)
    a.dtr[(threadIdx.x >> 6) * 64 + slot] = __builtin_amdgcn_s_memrealtime();
}

// Profiling only: workgroup start / end timestamps (s_memrealtime, 100 MHz) of a launch.
struct WgTrace {
  uint64_t* rec;
  uint64_t t0;
  uint64_t ph;   // up to three phase marks of wave 0 (10-ns ticks from the start, 16 bits each)
  __device__ __forceinline__ explicit WgTrace(uint64_t* base) : rec(nullptr), t0(0), ph(0) {
    if (base) {
      rec = base + (int64_t)blockIdx.x * WGT_REC;
      t0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ void mark(int k) {
    if (!rec) return;
    const uint64_t d = __builtin_amdgcn_s_memrealtime() - t0;
    ph |= (d < 0xffff ? d : 0xffff) << (16 * k);
  }
  __device__ __forceinline__ void done(int kind, int J, int I, int64_t b) {
    if (!rec) return;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
      rec[0] = t0;
      rec[1] = t1;
      rec[2] = ((uint64_t)kind << 56) | ((uint64_t)I << 40) | (uint64_t)b;
      rec[3] = (uint64_t)J | (ph << 16);
    }
  }
};

// Packed panel row of system row r of individual b (kernel form: the gathered animal rows,
// dual_pk_row = pstride / prow bytes each; stage kb at + 16 kb, as row_packed's)
__device__ __forceinline__ const uint8_t* row_dpk(const CholArgs& a, int64_t b, int64_t r) {
  return a.panel + b * a.pstride + r * (a.pstride / a.prow);
}
// Packed split row of system row r (primal: row r holds selected SNP r - pad; padding rows -> the
// zero row P; stage kb at + 16 kb).
__device__ __forceinline__ const uint8_t* row_packed(const CholArgs& a, int64_t b, int64_t r) {
  const int64_t o0 = a.off[b], k = a.off[b + 1] - o0;
  const int64_t pad = a.padfirst ? a.ns - k : 0;   // = SC_PAD, without a dependent scal load
  int64_t p = a.P;
  if (sys_real(r, pad, k)) {
    p = snp_col(a.idx[o0 + r - pad], a.P);
  }
  return a.ft.gpk[fold_of(a.ft, b)] + p * a.gs_row;
}

// Kernel form, folds sharing one animal set (FoldTab::gsh): the exact count A_r . A_c of system
// rows r, c (< n_Tp) of system s, from its individual's A_R A_R^T (k_gshare); padding rows count 0,
// as their zero panel rows do
__device__ __forceinline__ int32_t gsh_count(const CholArgs& a, int64_t s, int64_t r, int64_t c) {
  const FoldTab& ft = a.ft;
  const int32_t* mp = ft.gmap + (int64_t)fold_of(ft, s) * ft.gmap_ld;
  const int32_t mr = mp[r], mc = mp[c];
  return (mr >= 0 && mc >= 0) ? ft.gsh[((s % ft.bpf) * ft.gsh_ld + mr) * ft.gsh_ld + mc] : 0;
}

// ---------------------------------------------------------------------------
// Diagonal tile T_J = K_JJ - sum_{L<J} L_JL L_JL^T is assembled from pieces that are
// computed OFF the column-to-column critical path:
//   K_JJ            k_diag_grm, all J of the batch in one launch up front
//   L < J-1 terms   extra workgroups of the off-diagonal launch of column J-1
//   L = J-1 term    k_diag_prep right before the diagonal kernel (split over k)
// Each piece is written in the packed block layout the diagonal kernel factorises in,
// so the diagonal kernel sums them with a linear sweep.
// ---------------------------------------------------------------------------
constexpr int DW = 8;            // waves per diagonal workgroup
constexpr int DTHR = 64 * DW;
static_assert(DTHR == 4 * TILE, "diag z: four lanes per row");

// ===========================================================================
// Off-diagonal launch, 8 waves (512 threads) per workgroup, two workgroups per CU:
// wave w owns the 16 columns i in [16w, 16w+16) of its tile; 16 waves per CU hide the
// operand latency better than 8 (GEMM1 microbenchmark: 62 vs 58 TFLOP/s).
// ===========================================================================
constexpr int OW = 8;            // waves per off-diagonal workgroup
constexpr int OTH = 64 * OW;     // threads

// Packed rows (the SNP form's split rows, the kernel form's gathered panel), 64-B stages: stage st
// = 256 contraction elements = 64 B of each packed row (rows of 4 swizzled 16-B chunks; every
// 128-B line of a row is consumed by two consecutive stages).
// Lane (rho, ch) reads one 16-B chunk = 4 packed dwords and feeds dword s to k-step s, so
// the four lane groups x four k-steps cover the 16 dwords once (animal order inside a
// stage is immaterial to the counts; A and B use the same order).  A stage past the
// training block (nblk = 64-animal blocks, nblk % 4 != 0) zeroes chunks ch >= nblk % 4.
template <int D, int WCL = -1>
__device__ __forceinline__ void i8_tt8_pk64(const uint8_t* sa, const uint8_t* sb, int64_t nblk, uint8_t* lds,
                                            v4i (&cnt)[8]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wc = (WCL < 0) ? w : WCL;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) cnt[cb] = v4i{0, 0, 0, 0};
  if (nblk <= 0) return;
  const int64_t nst = (nblk + 3) >> 2;
  constexpr int TB = TILE * 64;
  auto issue = [&](int64_t st) {
    uint8_t* slot = lds + (int)(st % D) * 2 * TB;
    ring_glds<TBLUP_AB_ASM_I8>(sa + st * 64, slot + w * 1024);
    ring_glds<TBLUP_AB_ASM_I8>(sb + st * 64, slot + TB + w * 1024);
  };
  for (int64_t st = 0; st < D - 1 && st < nst; ++st) issue(st);
  const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
  const int tail_ch = (int)(nblk & 3);
  for (int64_t st = 0; st < nst; ++st) {
    if (st + D - 2 < nst) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 2) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (st + D - 1 < nst) issue(st + D - 1);
    const uint8_t* As = lds + (int)(st % D) * 2 * TB;
    const uint8_t* Bs = As + TB;
    uint4 bq = *reinterpret_cast<const uint4*>(Bs + i8off_b(16 * wc + rho, ch));
    if (st == nst - 1 && tail_ch != 0 && ch >= tail_ch) bq = uint4{0u, 0u, 0u, 0u};
    uint4 aq[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
      if (cb >= WCL) aq[cb] = *reinterpret_cast<const uint4*>(As + i8off_a(16 * cb + prow, ch));
    const uint32_t bw[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const v4i bv = unpack16(bw[s4]);
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        if (cb >= WCL) {
          const uint32_t aw = s4 == 0 ? aq[cb].x : s4 == 1 ? aq[cb].y : s4 == 2 ? aq[cb].z : aq[cb].w;
          cnt[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(unpack16(aw), bv, cnt[cb], 0, 0, 0);
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// Off-diagonal SNP-form tile with a 2-D wave split: the stages are loaded exactly as in
// i8_tt8_pk64, but wave w = (wr, wc) = (w >> 2, w & 3) computes row blocks 4wr..4wr+3 x
// column blocks 2wc, 2wc+1, so each k-step unpacks 4 A + 2 B dwords for 8 MFMAs (instead of
// 8 + 1).  The counts then go through LDS (64 blocks x 1 KiB, lane-linear 16-B slots) so
// that wave w ends up with column block w for all 8 row blocks -- the layout GEMM1/GEMM2 use
// (the MFMA lane mapping inside a block is the same in both layouts).
template <int D>
__device__ __forceinline__ void i8_tt2d_pk64(const uint8_t* sa, const uint8_t* sb, int64_t nblk, uint8_t* lds,
                                             v4i (&cnt)[8]) {
  // D is unused: two 128-B super-stages (each = two of i8_tt8_pk64's 64-B stages, 32 KiB)
  // alternate in the 64 KiB ring, one barrier per 512 animals
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  v4i c2[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) c2[m][ib] = v4i{0, 0, 0, 0};
  if (nblk > 0) {
    const int64_t nh = (nblk + 3) >> 2;   // 64-B half stages
    const int64_t nst = (nh + 1) >> 1;
    constexpr int TB = TILE * 64;
    auto issue = [&](int64_t st) {
      uint8_t* slot = lds + (int)(st & 1) * 4 * TB;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t hs = 2 * st + h;
        if (hs < nh) {
          ring_glds<TBLUP_AB_ASM_I8>(sa + hs * 64, slot + h * 2 * TB + w * 1024);
          ring_glds<TBLUP_AB_ASM_I8>(sb + hs * 64, slot + h * 2 * TB + TB + w * 1024);
        }
      }
    };
    issue(0);
    const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
    const int tail_ch = (int)(nblk & 3);
    for (int64_t st = 0; st < nst; ++st) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (st + 1 < nst) issue(st + 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t hs = 2 * st + h;
        if (hs < nh) {
          const uint8_t* As = lds + (int)(st & 1) * 4 * TB + h * 2 * TB;
          const uint8_t* Bs = As + TB;
          const bool ztail = (hs == nh - 1 && tail_ch != 0 && ch >= tail_ch);
          uint4 bq[2], aq[4];
#pragma unroll
          for (int ib = 0; ib < 2; ++ib) {
            bq[ib] = *reinterpret_cast<const uint4*>(Bs + i8off_b(16 * (2 * wc + ib) + rho, ch));
            if (ztail) bq[ib] = uint4{0u, 0u, 0u, 0u};
          }
#pragma unroll
          for (int m = 0; m < 4; ++m)
            aq[m] = *reinterpret_cast<const uint4*>(As + i8off_a(16 * (4 * wr + m) + prow, ch));
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            v4i bv[2];
#pragma unroll
            for (int ib = 0; ib < 2; ++ib)
              bv[ib] = unpack16(s4 == 0 ? bq[ib].x : s4 == 1 ? bq[ib].y : s4 == 2 ? bq[ib].z : bq[ib].w);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
              const v4i av = unpack16(s4 == 0 ? aq[m].x : s4 == 1 ? aq[m].y : s4 == 2 ? aq[m].z : aq[m].w);
#pragma unroll
              for (int ib = 0; ib < 2; ++ib)
                c2[m][ib] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv[ib], c2[m][ib], 0, 0, 0);
            }
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // exchange: block (row cb, column ib) at slot ib * 8 + cb, lane l's 16 B at l
  v4i* xs = reinterpret_cast<v4i*>(lds);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) xs[((2 * wc + ib) * 8 + 4 * wr + m) * 64 + l] = c2[m][ib];
  __syncthreads();
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) cnt[cb] = xs[(w * 8 + cb) * 64 + l];
  __syncthreads();
}

// GEMM1: acc[cb] -= sum_k L_J[c][k] L_I[i][k] over the nL Lt tiles starting at ltJ / ltI (k < 128 nL)
// for the wave's 16 columns i and the NCB row blocks cb0 .. cb0+NCB-1, on 32-row stages: only A
// (the Lt_J stage every wave reads) goes through the LDS ring (2 x 32 KiB); each wave's B operand
// (its own 16 columns of Lt_I) is loaded straight into registers one stage ahead.  (A 16-row A+B
// ring has twice the barriers and measured 2% slower.)  Every accumulator element's chain of MFMAs
// is the same whatever NCB / cb0 and wherever the L range is split, so partial sums handed from
// one launch to the next reproduce the one-workgroup result bit for bit.
//
// r0 (a multiple of 4): leading contraction rows skipped -- the SNP form's leading padding rows,
// whose columns of block column 0 are exact zeros (sys_real), so only a range that starts at L = 0
// passes r0 > 0: whole 32-row stages, then the first stage computed from k-step (r0 & 31) / 4 (a
// peeled stage: the main loop stays the branch-free one; a short LAST stage instead, or a per-k-step
// bound inside the loop, made the compiler spill or split the MFMA chains).  The MFMAs skipped would
// only have added exact zeros, so the result is the same bit for bit.
template <int NCB>
__device__ __forceinline__ void gemm1_a32(const double* __restrict__ ltJ, const double* __restrict__ ltI, int nL,
                                          int cb0, double* lds, v4d (&acc)[NCB], int r0 = 0) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int AS = 32 * TILE;   // doubles per 32-row stage
  const int s0 = r0 >> 5;         // whole leading stages skipped
  const int kf = (r0 & 31) >> 2;  // leading k-steps skipped in the first stage computed
  const int nst = 4 * nL;
  if (nst <= s0) return;
  auto src_of = [&](int s) { return (int64_t)(s >> 2) * TT + (s & 3) * AS; };
  auto issue_a = [&](int s) {
    double* slot = lds + (s & 1) * AS;
    const int64_t src = src_of(s);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * w + e;
      if constexpr (TBLUP_AB_ASM_GEMM1)
        glds16_asm(ltJ + src + k * TILE + 2 * (l ^ (8 * (k & 1))), slot + k * TILE);
      else
        __builtin_amdgcn_global_load_lds(ltJ + src + k * TILE + 2 * (l ^ (8 * (k & 1))), (lds_ptr_t)(slot + k * TILE),
                                         16, 0, 0);
    }
  };
  const double* bcol = ltI + 16 * w + (l & 15) + (l >> 4) * TILE;
  double bc[8];
  issue_a(s0);
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) bc[kk] = bcol[src_of(s0) + 4 * kk * TILE];
  int s = s0;
  if (kf > 0) {   // the first stage from k-step kf
    // the next stage's A issued before this short stage's wait, not after it (its 4 LDS-DMA ops
    // stay outstanding: vmcnt(4))
    const bool more = s + 1 < nst;
    if (more) {
      issue_a(s + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const double* bs = bcol + src_of(more ? s + 1 : s);
    const double* As = lds + (s & 1) * AS;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = 4 * kk + (l >> 4);
      if (kk >= kf) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          acc[cb] = mfma64_nega(As[lt_off(k, 16 * (cb0 + cb) + (l & 15))], bc[kk], acc[cb]);
      }
      if (more) bc[kk] = bs[4 * kk * TILE];
    }
    ++s;
  }
  for (; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bool more = s + 1 < nst;
    if (more) issue_a(s + 1);
    const double* bs = bcol + src_of(more ? s + 1 : s);
    const double* As = lds + (s & 1) * AS;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = 4 * kk + (l >> 4);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        acc[cb] = mfma64_nega(As[lt_off(k, 16 * (cb0 + cb) + (l & 15))], bc[kk], acc[cb]);
      // B of the next stage into the register this k-step has consumed
      if (more) bc[kk] = bs[4 * kk * TILE];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// The 36 lower blocks over 8 waves, by block-row pairs (q, 7 - q), q = W & 3: the pair's 9 blocks
// (7-q, 0 .. 7-q), (q, 0 .. q) in that order, the first 5 to wave q, the other 4 to wave q + 4 -- a
// wave's blocks share their rows, so it reads 4-6 of the 8 A fragments per k-step instead of all 8
// (round 4: the D-units' LDS reads per MFMA 1.78 -> 1.08; each block keeps its MFMA chain, so the
// sums are unchanged bit for bit).  syrk_e(W, i): packed index of wave W's i-th block, i < syrk_nb(W).
__host__ __device__ constexpr int syrk_nb(int W) { return W < 4 ? 5 : 4; }
__host__ __device__ constexpr int syrk_e(int W, int i) {
  const int q = W & 3, j = (W < 4) ? i : 5 + i, r1 = 8 - q;   // r1: blocks in row 7 - q
  return (j < r1) ? (7 - q) * (8 - q) / 2 + j : q * (q + 1) / 2 + (j - r1);
}
// every lower block exactly once
constexpr bool syrk_map_ok() {
  int seen[NPACK] = {};
  for (int W = 0; W < 8; ++W)
    for (int i = 0; i < syrk_nb(W); ++i) {
      const int e = syrk_e(W, i);
      if (e < 0 || e >= NPACK || seen[e]++) return false;
    }
  for (int e = 0; e < NPACK; ++e)
    if (seen[e] != 1) return false;
  return true;
}
static_assert(syrk_map_ok(), "SYRK block map must cover the 36 lower blocks once");

// SYRK of Lt stages restricted to the 36 lower blocks, 8 waves: wave W takes blocks syrk_e(W, i),
// i < syrk_nb(W); only the i in MASK (a diagonal-target slice).
// PART: from k-step ks on (the first stage of a run that starts past padding rows).
template <int W, int MASK, bool PART = false>
__device__ __forceinline__ void syrk_stage8(const double* As, v4d (&acc)[5], int l, int ks = 0) {
  constexpr int NBW = syrk_nb(W);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    if (PART && kk < ks) continue;
    const int k = 4 * kk + (l >> 4);
    double a8[8];   // the fragments no block of this wave uses are never loaded (dead)
#pragma unroll
    for (int q = 0; q < 8; ++q) a8[q] = As[lt_off(k, 16 * q + (l & 15))];
#pragma unroll
    for (int i = 0; i < NBW; ++i)
      if ((MASK >> i) & 1) acc[i] = mfma64(a8[tri_q(syrk_e(W, i))], a8[tri_s(syrk_e(W, i))], acc[i]);
  }
}

// block masks of the diagonal-target slices: all blocks; even i; odd i
__host__ __device__ constexpr int slice_mask(int sl) { return sl == 0 ? 0x1F : sl == 1 ? 0x15 : 0x0A; }

// SYRK of Lt rows restricted to the 36 lower blocks, 8 waves (wave W takes blocks syrk_e(W, i), i in
// slice_mask(sl)), on 32-row stages through a 2 x 32 KiB LDS-DMA ring: one barrier per 32 k rows.
// r0 (a multiple of 4): leading rows skipped, as in gemm1_a32 (zero padding columns of block
// column 0): whole stages, then the first stage computed from k-step (r0 & 31) / 4.
__device__ __forceinline__ void syrk_lower8_32(const double* __restrict__ src, int nst16, double* lds, v4d (&acc)[5],
                                               int sl = 0, int r0 = 0) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int AS = 32 * TILE;
  const int nst = nst16 >> 1;   // 8 x (number of Lt tiles): always even
  const int s0 = r0 >> 5, kf = (r0 & 31) >> 2;
  if (nst <= s0) return;
  auto issue = [&](int s) {
    double* slot = lds + (s & 1) * AS;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * w + e;
      if constexpr (TBLUP_AB_ASM_SYRK)
        glds16_asm(src + (int64_t)s * AS + k * TILE + 2 * (l ^ (8 * (k & 1))), slot + k * TILE);
      else
        __builtin_amdgcn_global_load_lds(src + (int64_t)s * AS + k * TILE + 2 * (l ^ (8 * (k & 1))),
                                         (lds_ptr_t)(slot + k * TILE), 16, 0, 0);
    }
  };
  issue(s0);
  const int ws = w + 8 * sl;   // wave-uniform (wave, slice) instantiation
#define SYRK_CASE(W, SL)                                    \
  case W + 8 * SL:                                          \
    syrk_stage8<W, slice_mask(SL)>(As, acc, l);             \
    syrk_stage8<W, slice_mask(SL)>(As + LTS, acc, l);       \
    break;
#define SYRK_PCASE(W, SL)                                                             \
  case W + 8 * SL:                                                                    \
    if (kf < 4) syrk_stage8<W, slice_mask(SL), true>(As, acc, l, kf);                 \
    syrk_stage8<W, slice_mask(SL), true>(As + LTS, acc, l, kf < 4 ? 0 : kf - 4);      \
    break;
#define SYRK_CASES(C, SL) C(0, SL) C(1, SL) C(2, SL) C(3, SL) C(4, SL) C(5, SL) C(6, SL) C(7, SL)
  int s = s0;
  if (kf > 0) {   // the next stage issued before this short stage's wait (as in gemm1_a32)
    if (s + 1 < nst) {
      issue(s + 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const double* As = lds + (s & 1) * AS;
    switch (ws) {
      SYRK_CASES(SYRK_PCASE, 0)
      SYRK_CASES(SYRK_PCASE, 1)
      SYRK_CASES(SYRK_PCASE, 2)
      default: break;
    }
    ++s;
  }
  for (; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nst) issue(s + 1);
    const double* As = lds + (s & 1) * AS;
    switch (ws) {
      SYRK_CASES(SYRK_CASE, 0)
      SYRK_CASES(SYRK_CASE, 1)
      SYRK_CASES(SYRK_CASE, 2)
      default: break;
    }
  }
#undef SYRK_CASES
#undef SYRK_PCASE
#undef SYRK_CASE
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// Packed-block store of a wave's SYRK accumulators (blocks W + 8i, i in the slice):
// dst[o] = base[o] - acc (base null: dst[o] = acc).
__device__ __forceinline__ void store_syrk_blocks(double* dst, const double* base, const v4d (&acc)[5], int sl) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int e = syrk_e(w, i);
    if (i < syrk_nb(w) && ((slice_mask(sl) >> i) & 1)) {
      const int q = tri_q_rt(e), sb = e - q * (q + 1) / 2;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = pk(q, sb) + bo((l >> 4) + 4 * r, l & 15);
        st64<TBLUP_AB_NT_PART>(dst + o, base ? base[o] - acc[i][r] : acc[i][r]);
      }
    }
  }
}

// S[b][Jt&1] = K_{Jt,Jt} - sum_{L < nterm} L_{Jt,L} L_{Jt,L}^T (packed blocks; the blocks of slice
// sl only), 8 waves: the diagonal target's partial sum.  K_{Jt,Jt} from Kd, or formed from the
// exact counts (kd: their loads issued before the SYRK, whose first wait covers them).
__device__ __forceinline__ void syrk_partial8(const CholArgs& a, int64_t b, int Jt, int nterm, double* lds, int sl) {
  const int w = threadIdx.x >> 6;
  v4d acc[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) acc[i] = v4d{0.0, 0.0, 0.0, 0.0};
  int2 kv[5];
  if (a.kd) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int e = syrk_e(w, i);
      kv[i] = (i < syrk_nb(w) && ((slice_mask(sl) >> i) & 1)) ? kd_load(a, b, Jt, e) : int2{0, 0};
    }
  }
  if (!(a.skip & 2)) syrk_lower8_32(a.L + b * l_stride(a.NT) + (int64_t)Jt * a.NT * TT, 8 * nterm, lds, acc, sl, skip_rows(a, b));
  double* dst = a.S + (b * NSLOT + (Jt & 1)) * (int64_t)NPACK * BLKD;
  if (!a.kd) {
    store_syrk_blocks(dst, a.Kd + (b * a.NT + Jt) * (int64_t)NPACK * BLKD, acc, sl);
    return;
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int e = syrk_e(w, i);
    if (i < syrk_nb(w) && ((slice_mask(sl) >> i) & 1)) kd_block(a, b, Jt, e, kv[i], acc[i], dst);
  }
}

// ---------------------------------------------------------------------------
// diagonal tile
//   A. T = K_JJ - sum_{L<J} L_JL L_JL^T = Kd + partials; r = y_J - mu - w_J
//   C. for panel p: one wave factors T_pp (-> L_pp, X_pp = L_pp^{-1});
//      all waves: L_qp = T_qp X_pp^T (q > p); T_qs -= L_qp L_sp^T (q >= s > p)   [MFMA]
//   D. blocked inverse X = L^{-1}: X_{j+d,j} = -X_{j+d,j+d} sum_{l=j}^{j+d-1} L_{j+d,l} X_{l,j}
//      (off-diagonal X blocks written to / re-read from Dinv, diagonal ones stay in LDS)
//   E. write L_JJ^T (Lt tile), X_J^T (Dinv, zeros below its diagonal), z_J = X_J r
// ---------------------------------------------------------------------------
// X block (q, jb), q > jb, of X = L^{-1}: X_{q,jb} = -X_qq sum_{lb=jb}^{q-1} L_{q,lb} X_{lb,jb}
// (needs L row q and X rows jb..q-1, X_qq); one wave.
__device__ __forceinline__ void xinv_block(const double* Tp, double* Xp, int q, int jb, int l) {
  // two independent MFMA chains (even / odd lb) halve the dependent-accumulator latency
  v4d s0 = {0.0, 0.0, 0.0, 0.0}, s1 = {0.0, 0.0, 0.0, 0.0};
  int lb = jb;
  for (; lb + 1 < q; lb += 2) {
    const double* A0 = Tp + pk(q, lb);
    const double* B0 = Xp + pk(lb, jb);
    const double* A1 = Tp + pk(q, lb + 1);
    const double* B1 = Xp + pk(lb + 1, jb);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * kk + (l >> 4);
      s0 = mfma64(A0[bo(l & 15, k)], B0[bo(k, l & 15)], s0);
      s1 = mfma64(A1[bo(l & 15, k)], B1[bo(k, l & 15)], s1);
    }
  }
  if (lb < q) {
    const double* A0 = Tp + pk(q, lb);
    const double* B0 = Xp + pk(lb, jb);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * kk + (l >> 4);
      s0 = mfma64(A0[bo(l & 15, k)], B0[bo(k, l & 15)], s0);
    }
  }
  const v4d sacc = s0 + s1;
  v4d xo = {0.0, 0.0, 0.0, 0.0};
  const double* Xqq = Xp + pk(q, q);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) xo = mfma64_nega(Xqq[bo(l & 15, 4 * kk + (l >> 4))], sacc[kk], xo);
  double* dst = Xp + pk(q, jb);
#pragma unroll
  for (int r = 0; r < 4; ++r) dst[bo((l >> 4) + 4 * r, l & 15)] = xo[r];
}

// z_J[i] = sum_{c <= i} X[i][c] r[c] for the NTR right-hand sides: four lanes per row
// (c = q mod 4), shuffle-reduced.
template <int NTR>
__device__ __forceinline__ void diag_z(const CholArgs& a, const double* Xp, const double (*rsh)[TILE], int64_t b,
                                       int64_t j0) {
  const int t = threadIdx.x, i = t >> 2, q = t & 3;
  const int qi = i >> 4, ii = i & 15;
  double acc[NTR];
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) acc[tr] = 0.0;
  for (int c = q; c <= i; c += 4) {
    const double xc = Xp[pk(qi, c >> 4) + bo(ii, c & 15)];
#pragma unroll
    for (int tr = 0; tr < NTR; ++tr) acc[tr] += xc * rsh[tr][c];
  }
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) {
    double v = acc[tr];
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    if (q == 0) a.z[(b * NTR + tr) * a.ns + j0 + i] = v;
  }
}

// Diagonal tile J of individual b.  T = S - sum_{L0 <= L < J} L_JL L_JL^T where S is
// K_JJ - sum_{L < L0} (the buffer slot J&1 left by an earlier off-diagonal launch) when
// L0 > 0, else k_diag_grm's K_JJ.
// LDS (lds >= 2 * NPACK * BLKD doubles = 144 KiB): Tp = T -> L (packed lower 16x16 blocks),
// Xp = X = L^{-1} in the same packed layout; before the factorisation Xp's space is the
// 64 KiB SYRK stage ring.  X never round-trips through global memory: Dinv receives X^T
// once, at the end.
__device__ __forceinline__ void diag_tile(const CholArgs& a, int64_t b, int J, int L0, double* lds,
                                          double (*rsh)[TILE]) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int64_t ns = a.ns;
  const int NT = a.NT;
  const int64_t j0 = (int64_t)J * TILE;
  const double* sc = a.scal + b * SCAL;
  const double muf = sc[SC_MUF];
  const int64_t nrow = (int64_t)sc[SC_NROW], pad = (int64_t)sc[SC_PAD];
  const int nt = a.nt;
  double* Tp = lds;
  double* Xp = lds + NPACK * BLKD;
  dstamp(a, 0);

  // forward-substitution right-hand side r = rhs_J - w_J: loads issued first so that their
  // latency overlaps the S load and the SYRK
  double rv[MAXT] = {0.0, 0.0, 0.0, 0.0};
  const int64_t gi = j0 + t;
  if (t < TILE) {
#pragma unroll
    for (int tr = 0; tr < MAXT; ++tr) {
      if (tr < nt) {
        const int64_t o = (b * nt + tr) * ns + gi;
        const double wv = (J > 0) ? a.w[o] : 0.0;
        const int fo = fold_of(a.ft, b);   // the system's split (fold-fused batches)
        rv[tr] = ((a.form == FORM_PRIMAL) ? a.rhs[o] : a.ft.yT[fo][tr * a.ytp + gi] - muf * a.ft.ymu[fo][tr]) - wv;
      }
    }
  }

  // T = S - sum_{L0 <= L < J} L_JL L_JL^T: S by LDS-DMA, the SYRK through the stage ring.
  // (Streaming the whole Lt tile in one burst, or 4 stages in flight, measured slower: the
  // launch's loads are HBM-bound and the SYRK at 2 waves per SIMD then runs after them.)
  const double* src = (L0 == 0) ? a.Kd + (b * NT + J) * (int64_t)NPACK * BLKD
                                : a.S + (b * NSLOT + (J & 1)) * (int64_t)NPACK * BLKD;
  {
#pragma unroll
    for (int e = 0; e < NPACK * BLKD / 2 / DTHR; ++e) {   // 9 x 16 B per thread
      const int chunk = (e * DW + w) * 64;
      __builtin_amdgcn_global_load_lds(src + 2 * (chunk + l), (lds_ptr_t)(Tp + 2 * chunk), 16, 0, TBLUP_AB_NT_PLD ? 2 : 0);
    }
    if (J > L0 && a.q != nullptr) {
      // last-term mode: Q = L_{J,J-1} L_{J,J-1}^T came with launch J-1's tile (J, J-1)
      const double* qg = a.q + b * (int64_t)NPACK * BLKD;
#pragma unroll
      for (int e = 0; e < NPACK * BLKD / 2 / DTHR; ++e) {
        const int chunk = (e * DW + w) * 64;
        __builtin_amdgcn_global_load_lds(qg + 2 * (chunk + l), (lds_ptr_t)(Xp + 2 * chunk), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int e = t; e < NPACK * BLKD; e += DTHR) Tp[e] -= Xp[e];
      __syncthreads();
    } else if (J > L0 && !(a.skip & 2)) {
      v4d acc[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) acc[i] = v4d{0.0, 0.0, 0.0, 0.0};
      // waits for all its stages (and the older S loads) and ends in a barrier
      // (no padding skip here: at J = 1 only, and it keeps the peeled stage out of this kernel)
      syrk_lower8_32(a.L + b * l_stride(NT) + ((int64_t)J * NT + L0) * TT, 8 * (J - L0), Xp, acc);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int e = syrk_e(w, i);
        if (i < syrk_nb(w)) {
          const int q = tri_q_rt(e);
          double* blk = Tp + pk(q, e - q * (q + 1) / 2);
#pragma unroll
          for (int r = 0; r < 4; ++r) blk[bo((l >> 4) + 4 * r, l & 15)] -= acc[i][r];
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // X's diagonal blocks start as the reversed identity (factor16's inverse rows load it); the
  // SYRK ring that shared their space is drained
#pragma unroll
  for (int e = t; e < NBLK * BLKD; e += DTHR) {
    const int p = e >> 8, o = e & 255, r = o >> 4;
    const int c = 2 * (((o & 15) >> 1) ^ ((r >> 1) & 7)) + (o & 1);   // bo(r, c) == o
    Xp[pk(p, p) + o] = (c == NB - 1 - r) ? 1.0 : 0.0;
  }
  if (t < TILE) {
#pragma unroll
    for (int tr = 0; tr < MAXT; ++tr) rsh[tr][t] = (tr < nt && sys_real(gi, pad, nrow)) ? rv[tr] : 0.0;
  }
  dstamp(a, 1);
  __syncthreads();
  dstamp(a, 2);

  // C. blocked right-looking factorisation over 16-column panels, with a one-block
  //    look-ahead: wave 0 updates diagonal block p+1 first and factors it while waves 1-3
  //    finish the rest of step p's trailing update.
  if (!(a.skip & 4)) {
    if (w == 0 && !(a.skip & 256)) factor16_any(a, Tp + pk(0, 0), Xp + pk(0, 0), l);
    __syncthreads();
  }
  for (int p = 0; p < ((a.skip & 4) ? 0 : NBLK); ++p) {
    for (int q = p + 1 + w; q < ((a.skip & 512) ? 0 : NBLK); q += DW) {
      v4d x = {0.0, 0.0, 0.0, 0.0};
      x = mma_abt(Tp + pk(q, p), Xp + pk(p, p), x, l);
#pragma unroll
      for (int r = 0; r < 4; ++r) Tp[pk(q, p) + bo((l >> 4) + 4 * r, l & 15)] = x[r];
    }
    dstamp(a, 3 + 3 * p);
    __syncthreads();
    if (p + 1 == NBLK) break;
    const int nb = NBLK - 1 - p;
    if (w == 0) {
      uint64_t* st = (a.dtr && blockIdx.x == 0 && p == 3) ? a.dtr : nullptr;
      fstamp(st, 54);
      if (!(a.skip & 512)) {
        v4d x = {0.0, 0.0, 0.0, 0.0};
        x = mma_abt(Tp + pk(p + 1, p), Tp + pk(p + 1, p), x, l);
        double* dst = Tp + pk(p + 1, p + 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[bo((l >> 4) + 4 * r, l & 15)] -= x[r];
      }
      if (!(a.skip & 256)) factor16_any(a, Tp + pk(p + 1, p + 1), Xp + pk(p + 1, p + 1), l, st);
    } else {
      // trailing blocks e = 1 .. nb(nb+1)/2 - 1 (e = 0 is block (p+1, p+1)) over waves 1 .. DW-1
      // (wave DW/2 shares wave 0's SIMD; factor16 leaves it enough issue slots)
      const int wi = w - 1;   // 0 .. DW-2
      constexpr int NTW = DW - 1;
      // two blocks per pass: independent MFMA chains and LDS traffic overlap
      const int ne = (a.skip & 512) ? 0 : nb * (nb + 1) / 2;
      for (int e = wi + 1; e < ne; e += 2 * NTW) {
        const int e2 = e + NTW;
        int qq = 0;
        while ((qq + 1) * (qq + 2) / 2 <= e) ++qq;
        const int q = p + 1 + qq, sb = p + 1 + (e - qq * (qq + 1) / 2);
        const bool two = e2 < ne;
        int qq2 = qq;
        while ((qq2 + 1) * (qq2 + 2) / 2 <= e2) ++qq2;
        const int q2 = two ? p + 1 + qq2 : q, sb2 = two ? p + 1 + (e2 - qq2 * (qq2 + 1) / 2) : sb;
        const double* A = Tp + pk(q, p);
        const double* B = Tp + pk(sb, p);
        const double* A2 = Tp + pk(q2, p);
        const double* B2 = Tp + pk(sb2, p);
        v4d x = {0.0, 0.0, 0.0, 0.0}, x2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = 4 * kk + (l >> 4);
          x = mfma64(A[bo(l & 15, k)], B[bo(l & 15, k)], x);
          x2 = mfma64(A2[bo(l & 15, k)], B2[bo(l & 15, k)], x2);
        }
        double* dst = Tp + pk(q, sb);
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[bo((l >> 4) + 4 * r, l & 15)] -= x[r];
        if (two) {
          double* dst2 = Tp + pk(q2, sb2);
#pragma unroll
          for (int r = 0; r < 4; ++r) dst2[bo((l >> 4) + 4 * r, l & 15)] -= x2[r];
        }
      }
      // D (overlapped). block row p of X = L^{-1}: L row p and X rows < p are final and
      // X_pp came out of the previous window's factor16
      if (!(a.skip & 8) && wi < p) xinv_block(Tp, Xp, p, wi, l);
    }
    dstamp(a, 4 + 3 * p);
    __syncthreads();
    dstamp(a, 5 + 3 * p);
  }
  if (a.skip & 16) return;

  // D. last block row of X (rows < NBLK-1 were built inside the factorisation windows)
  if (!(a.skip & 4) && !(a.skip & 8)) {
    if (w < NBLK - 1) xinv_block(Tp, Xp, NBLK - 1, w, l);
    dstamp(a, 26);
    __syncthreads();
    dstamp(a, 27);
  }

  // E. X into Dinv as packed lower blocks, each block transposed (block (q, jb) holds
  //    X_{q,jb}^T in the bo() layout), z_J = X r, and L_JJ^T only for the debug readback.
  {
    // coalesced: thread writes the 16-B pair at g = 2k of Dinv, i.e. elements (r, c0), (r, c0+1)
    // of block blk's transpose, read from X at bo(c0, r), bo(c0 + 1, r)
    double* Xg = a.Dinv + (b * NT + J) * (int64_t)NPACK * BLKD;
    for (int k = t; k < ((a.skip & (1 << 14)) ? 0 : NPACK * BLKD / 2); k += DTHR) {
      const int g = 2 * k, blk = g >> 8, o = g & 255, r = o >> 4;
      const int c0 = 2 * (((o & 15) >> 1) ^ ((r >> 1) & 7));
      const double* xb = Xp + blk * BLKD;
      if constexpr (TBLUP_AB_NT_X)
        __builtin_nontemporal_store(v2d{xb[bo(c0, r)], xb[bo(c0 + 1, r)]}, reinterpret_cast<v2d*>(Xg + g));
      else
        *reinterpret_cast<v2d*>(Xg + g) = v2d{xb[bo(c0, r)], xb[bo(c0 + 1, r)]};
    }
  }
  if (a.skip & FLAG_WRITE_LJJ) {
    double* Ld = a.L + b * l_stride(NT) + ((int64_t)J * NT + J) * TT;
    for (int e = t; e < TT; e += DTHR) {
      const int rr = e >> 7, cc = e & 127;
      Ld[e] = (cc >= rr) ? Tp[pk(cc >> 4, rr >> 4) + bo(cc & 15, rr & 15)] : 0.0;
    }
  }
  dstamp(a, 28);
  // z_J[i] = sum_{c <= i} X[i][c] r[c]: four lanes per row (c = q mod 4), shuffle-reduced
  if (!(a.skip & (1 << 15))) {
    switch (nt) {
      case 1: diag_z<1>(a, Xp, rsh, b, j0); break;
      case 2: diag_z<2>(a, Xp, rsh, b, j0); break;
      case 3: diag_z<3>(a, Xp, rsh, b, j0); break;
      default: diag_z<4>(a, Xp, rsh, b, j0); break;
    }
  }
  dstamp(a, 29);
}

// ---------------------------------------------------------------------------
// Off-diagonal launch of column J: one 8-wave workgroup per unit, two per CU (LDS <= 72 KiB).
//   T-unit, tile (I, J), I > J:
//     0. acc = K_JI in the f64 accumulator layout: from k_sys_tiles' counts (either form) or int8
//        MFMA here (rows permuted so the counts land in the f64 layout) -- or, when launch J-1 ran
//        ahead, its partial sum K_JI - sum_{L<J-1} L_JL L_IL^T
//     1. acc -= sum_{L} L_JL L_IL^T over the L < J not summed yet   (acc = T^T, wave w: its 16 i)
//     2. out^T[jb] = sum_{cb<=jb} X[jb][cb] T^T[cb]   (X = inv(L_JJ); acc is the B operand)
//        -> Lt tile (I, J); w_I += L_IJ z_J
//   P-unit (ahead), tile (I, J+1), I >= J+2, row blocks of slice rs: acc = K - sum_{L<J} (steps 0-1
//     of launch J+1's T-unit, which continues the same MFMA chains: bit-identical results)
//   D-unit, diagonal tile J+1, block slice: S = K - sum_{L<J} L_{J+1,L} L_{J+1,L}^T (packed blocks)
// ---------------------------------------------------------------------------

// K_{I,Jt} (the T^T layout of tile (I, Jt)) for the NCB row blocks from cb0: exact counts of
// k_sys_tiles (loads issued by kc_issue) or, NCB = 8 only, the int8 tile here.
template <int NCB>
__device__ __forceinline__ void kc_issue(const CholArgs& a, int64_t b, int I, int Jt, int cb0, int2 (&kcv)[NCB]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int NT = a.NT;
  const int16_t* kt = a.kc + ((b * (NT * (NT - 1) / 2)) + I * (I - 1) / 2 + Jt) * KC_TILE + w * 8 * 64 * 4;
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) kcv[cb] = nt_load2(kt + ((cb0 + cb) * 64 + l) * 4);
}

// K_ij = (c - (u_i + u_j) sa - u_i u_j sm + cN) / d regrouped around the column j: c / d + P_j u_i +
// Q_j, P_j = -(sa + sm u_j) / d, Q_j = (cN - sa u_j) / d, with P_j = Q_j = 0 on padding columns (whose
// counts are 0): per element an LDS pair, a conversion and two fmas, where the plain formula took
// seven fp64 ops and a 64-bit compare -- an fp64 VALU op waits for the matrix pipe while the CU's
// other waves stream MFMAs (gfx950 does not dual-issue them).  Only the off-diagonal tiles' K comes
// from here (T-, P- and E-units alike), so every schedule agrees.  k_stage (threads t < TILE, before
// the unit's barrier): the column pairs of tile Jt and the row sums u_i of tile I.
__device__ __forceinline__ void k_stage(const CholArgs& a, int64_t b, int64_t i0, int64_t j0, double* pq_sh,
                                        double* ui_sh) {
  const int t = threadIdx.x;
  if (t < TILE) {
    const double* sc = a.scal + b * SCAL;
    const double sa = sc[SC_SA], cN = sc[SC_CN], invd = sc[SC_INVD], sm = sc[SC_SM];
    const int64_t nrow = (int64_t)sc[SC_NROW], pad = (int64_t)sc[SC_PAD];
    const double uj = a.u[b * a.prow + j0 + t];
    const bool rj = sys_real(j0 + t, pad, nrow);
    reinterpret_cast<v2d*>(pq_sh)[t] = rj ? v2d{-invd * (sa + sm * uj), invd * (cN - sa * uj)} : v2d{0.0, 0.0};
    ui_sh[t] = a.u[b * a.prow + i0 + t];
  }
}

// GSH: the kernel-form path may read shared fold counts (FoldTab::gsh); the diagonal kernel's E-units
// are built without it (E-units are not planned for such chunks: run_chunk), which keeps that
// latency-bound kernel's code as it was
template <int NCB, bool GSH = true>
__device__ __forceinline__ void k_acc(const CholArgs& a, int64_t b, int I, int Jt, int cb0, const int2 (&kcv)[NCB],
                                      uint8_t* lds8, const double* pq_sh, const double* ui_sh, v4d (&acc)[NCB]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)Jt * TILE;
  const double* sc = a.scal + b * SCAL;
  const double invd = sc[SC_INVD];
  const int64_t nrow = (int64_t)sc[SC_NROW], pad = (int64_t)sc[SC_PAD];
  const int il = 16 * w + (l & 15);
  const bool ireal = sys_real(i0 + il, pad, nrow);
  const double ui = ui_sh[il];
  const v2d* pq = reinterpret_cast<const v2d*>(pq_sh);
  if (a.kc) {
    // counts issued before the u / z loads landed; exact ints -> fp64 K
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      const int32_t c4[4] = {(int32_t)(int16_t)(kcv[cb].x & 0xffff), (int32_t)(int16_t)(kcv[cb].x >> 16),
                             (int32_t)(int16_t)(kcv[cb].y & 0xffff), (int32_t)(int16_t)(kcv[cb].y >> 16)};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = 16 * (cb0 + cb) + (l >> 4) + 4 * r;
        const v2d q = pq[cl];
        const double v = __builtin_fma((double)c4[r], invd, __builtin_fma(q[0], ui, q[1]));
        acc[cb][r] = ireal ? v : 0.0;
      }
    }
    return;
  }
  if constexpr (NCB == 8) {
    v4i cnt[8];
    const int64_t nblk = (int64_t)sc[SC_CBLK];
    if (GSH && !(a.skip & 32) && a.form != FORM_PRIMAL && a.ft.gsh) {
      // kernel-form folds: the counts of the individual's shared A_R A_R^T (same integers)
#pragma unroll
      for (int cb = 0; cb < 8; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) cnt[cb][r] = gsh_count(a, b, j0 + 16 * cb + (l >> 4) + 4 * r, i0 + il);
    } else if (!(a.skip & 32)) {
      // 2-bit packed rows of either form: the SNP form's split rows, the kernel form's gathered panel
      const int row = 16 * w + (l >> 2), pos = l & 3;
      const bool pf = a.form == FORM_PRIMAL;
      const uint8_t* sa = (pf ? row_packed(a, b, j0 + row) : row_dpk(a, b, j0 + row)) + 16 * (pos ^ ((row >> 2) & 3));
      const uint8_t* sb = (pf ? row_packed(a, b, i0 + row) : row_dpk(a, b, i0 + row)) + 16 * (pos ^ ((row >> 2) & 2));
      i8_tt2d_pk64<4>(sa, sb, nblk, lds8, cnt);
    } else {
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) cnt[cb] = v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = 16 * cb + (l >> 4) + 4 * r;
        const v2d q = pq[cl];
        const double v = __builtin_fma((double)cnt[cb][r], invd, __builtin_fma(q[0], ui, q[1]));
        acc[cb][r] = ireal ? v : 0.0;
      }
    }
  }
}

// Partial sums of launch J+1's tiles, acc layout: [slot Jt&1][b][I][wave][cb][lane][4]
__device__ __forceinline__ double* part_ptr(const CholArgs& a, int64_t b, int I, int Jt) {
  return a.part + (((int64_t)(Jt & 1) * a.B + b) * a.NT + I) * TT + (threadIdx.x >> 6) * 8 * 64 * 4;
}

// P-unit: acc = K_{I,J+1} - sum_{L<J} L_{J+1,L} L_{I,L}^T for row blocks [cb0, cb0 + NCB).
template <int NCB>
__device__ __forceinline__ void part_unit(const CholArgs& a, int64_t b, int I, int rs, double* lds, double* uj_sh,
                                          double* ui_sh) {
  const int t = threadIdx.x, l = t & 63;
  const int J = a.J, Jt = J + 1, NT = a.NT, cb0 = rs * NCB;
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)Jt * TILE;
  int2 kcv[NCB];
  if (a.kc) kc_issue<NCB>(a, b, I, Jt, cb0, kcv);
  k_stage(a, b, i0, j0, uj_sh, ui_sh);
  __syncthreads();
  v4d acc[NCB];
  k_acc<NCB>(a, b, I, Jt, cb0, kcv, reinterpret_cast<uint8_t*>(lds), uj_sh, ui_sh, acc);
  const double* Lb = a.L + b * l_stride(NT);
  if (!(a.skip & 64))
    gemm1_a32<NCB>(Lb + (int64_t)Jt * NT * TT, Lb + (int64_t)I * NT * TT, J, cb0, lds, acc, skip_rows(a, b));
  double* pd = part_ptr(a, b, I, Jt);
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    v2d* d = reinterpret_cast<v2d*>(pd + ((cb0 + cb) * 64 + l) * 4);
    if constexpr (TBLUP_AB_NT_PART) {
      __builtin_nontemporal_store(v2d{acc[cb][0], acc[cb][1]}, d);
      __builtin_nontemporal_store(v2d{acc[cb][2], acc[cb][3]}, d + 1);
    } else {
      d[0] = v2d{acc[cb][0], acc[cb][1]};
      d[1] = v2d{acc[cb][2], acc[cb][3]};
    }
  }
}

// T-unit: tile (I, J).
template <int NTR>   // traits the w update runs over: 1, or MAXT (the zero traits' FMAs wait on the matrix pipe too)
__device__ __forceinline__ void tile_unit(const CholArgs& a, int64_t b, int I, int ahead_cur, int edone, double* lds,
                                          double* uj_sh, double* ui_sh, double (*zj_sh)[TILE], WgTrace& tr) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int J = a.J, NT = a.NT;
  const int64_t ns = a.ns;
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)J * TILE;
  const double* Lb = a.L + b * l_stride(NT);
  v4d acc[8];
  int2 kcv[8];
  const bool from_part = ahead_cur || edone;
  if (from_part) {
    const double* pd = part_ptr(a, b, I, J);
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
      const v2d* s2 = reinterpret_cast<const v2d*>(pd + (cb * 64 + l) * 4);
      const v2d lo = TBLUP_AB_NT_PLD ? __builtin_nontemporal_load(s2) : s2[0];
      const v2d hi = TBLUP_AB_NT_PLD ? __builtin_nontemporal_load(s2 + 1) : s2[1];
      acc[cb] = v4d{lo[0], lo[1], hi[0], hi[1]};
    }
  } else if (a.kc) {
    kc_issue<8>(a, b, I, J, 0, kcv);
  }
  if (!from_part) k_stage(a, b, i0, j0, uj_sh, ui_sh);
  if (t < TILE) {
#pragma unroll
    for (int tr = 0; tr < MAXT; ++tr)
      zj_sh[tr][t] = (tr < a.nt) ? a.z[(b * a.nt + tr) * ns + j0 + t] : 0.0;
  }
  __syncthreads();
  if (!from_part) k_acc<8>(a, b, I, J, 0, kcv, reinterpret_cast<uint8_t*>(lds), uj_sh, ui_sh, acc);
  tr.mark(0);

  // 1. T^T = K_JI - sum_L L_JL L_IL^T over the L not summed by launch J-1 or this tile's E-unit
  const int Ls = (ahead_cur ? J - 1 : 0) + edone;
  if (J > Ls && !(a.skip & 64))
    gemm1_a32<8>(Lb + (int64_t)J * NT * TT + (int64_t)Ls * TT, Lb + (int64_t)I * NT * TT + (int64_t)Ls * TT, J - Ls, 0,
                 lds, acc, Ls == 0 ? skip_rows(a, b) : 0);
  tr.mark(1);

  // 2. L_IJ^T = X T^T by 16-row blocks of X (X[j][c] = 0 for c > j).  Dinv holds X in the
  //    packed block layout (blocks transposed): all 36 blocks (72 KiB) land in LDS in one
  //    LDS-DMA burst, then the 8 block rows run without further waits.
  double* Lout = const_cast<double*>(Lb) + ((int64_t)I * NT + J) * TT;
  double* xl = lds;
  {
    const double* Xg = a.Dinv + (b * NT + J) * (int64_t)NPACK * BLKD;
#pragma unroll
    for (int e = 0; e < NPACK * BLKD / 2 / OTH; ++e) {   // 9 x 16 B per thread
      const int chunk = (e * OW + w) * 64;
      __builtin_amdgcn_global_load_lds(Xg + 2 * (chunk + l), (lds_ptr_t)(xl + 2 * chunk), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  tr.mark(2);
  double wacc[MAXT] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
  for (int jb = 0; jb < NBLK; ++jb) {
    v4d o = {0.0, 0.0, 0.0, 0.0};
    if (!(a.skip & 128)) {
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        if (cb <= jb) {
          const double* xb = xl + pk(jb, cb);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) o = mfma64(xb[bo(4 * kk + (l >> 4), l & 15)], acc[cb][kk], o);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int jl = 16 * jb + (l >> 4) + 4 * r, il = 16 * w + (l & 15);
      st64<TBLUP_AB_NT_L>(Lout + jl * TILE + il, o[r]);
#pragma unroll
      for (int tr = 0; tr < NTR; ++tr) wacc[tr] += o[r] * zj_sh[tr][jl];
    }
  }
  // w_I[i] += sum_j L_IJ[i][j] z_J[j]: reduce the 4 lane groups that share a column i
#pragma unroll
  for (int tr = 0; tr < NTR; ++tr) {
    if (tr < a.nt) {
      double v = wacc[tr];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if ((l >> 4) == 0) {
        const int64_t gi = (b * a.nt + tr) * ns + i0 + 16 * w + l;
        a.w[gi] = (J == 0) ? v : a.w[gi] + v;
      }
    }
  }
  // last-term mode: the diagonal tile J+1's last SYRK term L_{J+1,J} L_{J+1,J}^T from the tile
  // just stored (read back through the same stage ring and MFMA chains the diagonal kernel would
  // run, so its T = S - Q is bit-identical)
  if (a.q != nullptr && I == J + 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    v4d qa[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) qa[i] = v4d{0.0, 0.0, 0.0, 0.0};
    syrk_lower8_32(Lout, 8, lds, qa, 0, J == 0 ? skip_rows(a, b) : 0);
    store_syrk_blocks(a.q + b * (int64_t)NPACK * BLKD, nullptr, qa, 0);
  }
}

// E-unit (diagonal launch J, on a CU its other workgroups leave idle): the GEMM1 term L = ls0 of tile
// (I, J) -- from K_JI (ls0 = 0) or from launch J-1's partial over L < J-1 (ls0 = J-1) -- into the
// partial-sum slot J&1, where launch J's T-unit picks it up (OffPlan::ne).  The same k_acc start and
// gemm1_a32 MFMA chains as the T-unit, split after the term: bit-identical.
__device__ __forceinline__ void e_unit(const CholArgs& a, int64_t b, int I, int ls0, double* lds) {
  const int t = threadIdx.x, l = t & 63;
  const int J = a.J, NT = a.NT;
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)J * TILE;
  double* uj_sh = lds + NPACK * BLKD;   // past the GEMM1 ring (2 x 32 KiB) and k_acc's int8 ring
  double* ui_sh = uj_sh + 2 * TILE;
  double* pd = part_ptr(a, b, I, J);
  v4d acc[8];
  if (ls0 > 0) {
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
      const v2d* s2 = reinterpret_cast<const v2d*>(pd + (cb * 64 + l) * 4);
      const v2d lo = TBLUP_AB_NT_PLD ? __builtin_nontemporal_load(s2) : s2[0];
      const v2d hi = TBLUP_AB_NT_PLD ? __builtin_nontemporal_load(s2 + 1) : s2[1];
      acc[cb] = v4d{lo[0], lo[1], hi[0], hi[1]};
    }
  } else {
    int2 kcv[8];
    if (a.kc) kc_issue<8>(a, b, I, J, 0, kcv);
    k_stage(a, b, i0, j0, uj_sh, ui_sh);
    __syncthreads();
    k_acc<8, false>(a, b, I, J, 0, kcv, reinterpret_cast<uint8_t*>(lds), uj_sh, ui_sh, acc);
  }
  const double* Lb = a.L + b * l_stride(NT);
  if (!(a.skip & 64))
    gemm1_a32<8>(Lb + (int64_t)J * NT * TT + (int64_t)ls0 * TT, Lb + (int64_t)I * NT * TT + (int64_t)ls0 * TT, 1, 0, lds,
                 acc, ls0 == 0 ? skip_rows(a, b) : 0);
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) {
    v2d* d = reinterpret_cast<v2d*>(pd + (cb * 64 + l) * 4);
    if constexpr (TBLUP_AB_NT_PART) {
      __builtin_nontemporal_store(v2d{acc[cb][0], acc[cb][1]}, d);
      __builtin_nontemporal_store(v2d{acc[cb][2], acc[cb][3]}, d + 1);
    } else {
      d[0] = v2d{acc[cb][0], acc[cb][1]};
      d[1] = v2d{acc[cb][2], acc[cb][3]};
    }
  }
}

// Diagonal tile J of every individual: for J >= 2 the previous off-diagonal launch left
// K_JJ - sum_{L < J-1} in S[J&1], and the L = J-1 term is subtracted here.  Grid: the B diagonal
// workgroups, then nd D-units, then ne E-units (OffPlan).
__global__ __launch_bounds__(DTHR) void k_chol_diag(CholArgs a, int64_t ne, int ls0) {
  __shared__ __attribute__((aligned(16))) double lds[2 * NPACK * BLKD];   // 144 KiB: T/L and X
  __shared__ double rsh[MAXT][TILE];
  WgTrace tr(a.wgt);
  if ((int64_t)blockIdx.x >= a.B) {
    const int64_t x = blockIdx.x - a.B, nd = gridDim.x - a.B - ne;
    if (x < nd) {
      // OffPlan::ndd: the D-unit of diagonal target J+1 (S = K - sum_{L<J}), on a CU the diagonal
      // workgroups (dispatched first) leave idle; blocks B + x and x share an XCD when 8 | B
      const int64_t b = xcd_remap(x, nd);
      syrk_partial8(a, b, a.J + 1, a.J, lds, 0);
      tr.done(WGT_DPREP, a.J, a.J + 1, b);
    } else {
      const int64_t lg = xcd_remap(x - nd, ne);
      const int64_t b = lg % a.B;
      const int I = a.J + 1 + (int)(lg / a.B);
      e_unit(a, b, I, ls0, lds);
      tr.done(WGT_EPART, a.J, I, b);
    }
    return;
  }
  // individual b on the XCD that runs its off-diagonal tiles (same L2 for L, S, X, w)
  const int64_t b = xcd_remap(blockIdx.x, a.B);
  diag_tile(a, b, a.J, a.J >= 2 ? a.J - 1 : 0, lds, rsh);
  tr.done(WGT_DIAG, a.J, a.J, b);
}

// K_JJ for every (individual, J) with the off-diagonal kernel's 8-wave int8 tile (A = B =
// the rows of tile J, output in the f64 accumulator layout: a wave holds the 16 columns of
// one column block, MFMAs only for the lower row blocks), exact counts + fp64 centring,
// + lambda I, identity on padded rows; packed lower 16x16 blocks into Kd[b][J].  J = 0, 1 run in
// k_diag_grm8 before the column loop; J >= 2 are extra workgroups at the end of the column-0
// off-diagonal launch (they fill its last round; the first reader is column 1's preparation).
__device__ __forceinline__ void diag_grm_tile(const CholArgs& a, int64_t b, int J, uint8_t* lds, double* u_sh) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int NT = a.NT;
  const int64_t j0 = (int64_t)J * TILE;
  const double* sc = a.scal + b * SCAL;
  const double sa = sc[SC_SA], cN = sc[SC_CN], invd = sc[SC_INVD], lam = sc[SC_LAM], sm = sc[SC_SM];
  const int64_t nrow = (int64_t)sc[SC_NROW], nblk = (int64_t)sc[SC_CBLK], pad = (int64_t)sc[SC_PAD];
  if (t < TILE) u_sh[t] = a.u[b * a.prow + j0 + t];
  double* Kd = a.Kd + (b * NT + J) * (int64_t)NPACK * BLKD;
  v4i cnt[8];
  const int row = 16 * w + (l >> 2), pos = l & 3;
  // lower blocks only; waves w and w+4 share a SIMD, so they take column blocks w and 7-w
  // (8-w and w+1 row blocks: 9 per SIMD)
  const int wc = (w < 4) ? w : 11 - w;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) cnt[cb] = v4i{0, 0, 0, 0};
  if (a.skip & 1) {
    __syncthreads();
  } else if (a.ft.gsh) {
    // kernel-form folds: the lower blocks' counts from the individual's shared A_R A_R^T
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
      if (cb >= wc)
#pragma unroll
        for (int r = 0; r < 4; ++r) cnt[cb][r] = gsh_count(a, b, j0 + 16 * cb + (l >> 4) + 4 * r, j0 + 16 * wc + (l & 15));
  } else {
    // 2-bit packed rows: the SNP form's split rows, the kernel form's gathered panel
    const uint8_t* rp = a.form == FORM_PRIMAL ? row_packed(a, b, j0 + row) : row_dpk(a, b, j0 + row);
    const uint8_t* sa = rp + 16 * (pos ^ ((row >> 2) & 3));
    const uint8_t* sb = rp + 16 * (pos ^ ((row >> 2) & 2));
    switch (wc) {   // wave-uniform: one instantiation per column block
      case 0: i8_tt8_pk64<4, 0>(sa, sb, nblk, lds, cnt); break;
      case 1: i8_tt8_pk64<4, 1>(sa, sb, nblk, lds, cnt); break;
      case 2: i8_tt8_pk64<4, 2>(sa, sb, nblk, lds, cnt); break;
      case 3: i8_tt8_pk64<4, 3>(sa, sb, nblk, lds, cnt); break;
      case 4: i8_tt8_pk64<4, 4>(sa, sb, nblk, lds, cnt); break;
      case 5: i8_tt8_pk64<4, 5>(sa, sb, nblk, lds, cnt); break;
      case 6: i8_tt8_pk64<4, 6>(sa, sb, nblk, lds, cnt); break;
      default: i8_tt8_pk64<4, 7>(sa, sb, nblk, lds, cnt); break;
    }
  }
  __syncthreads();
  const int il = 16 * wc + (l & 15);
  const int64_t gj = j0 + il;
  const double uj = u_sh[il];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) {
    if (cb >= wc) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = 16 * cb + (l >> 4) + 4 * r;
        const int64_t gi = j0 + cl;
        const double kv = grm_value(cnt[cb][r], u_sh[cl], uj, sa, cN, invd, sm);
        const double v = (sys_real(gi, pad, nrow) && sys_real(gj, pad, nrow)) ? kv + ((gi == gj) ? lam : 0.0)
                                                                              : ((gi == gj) ? 1.0 : 0.0);
        Kd[pk(cb, wc) + bo(cl & 15, il & 15)] = v;
      }
    }
  }
}

// Off-diagonal launch of column J (see OffPlan).  The grid holds the unit classes longest first
// -- every P-unit, then every D-unit, then every T-unit (a class's units dispatched after
// another class's have started cannot hide behind them: with the D-units after the T-units of
// their own individual, as one list per individual, the launches ran 9% longer) -- each class
// XCD-remapped so that one XCD's L2 serves an individual's Lt block rows; and, column 0 of the
// kernel form only, the K_JJ workgroups for J >= 2 at the end.
// NTRK: the traits the T-units' w update runs over (1, or MAXT for several traits) -- one kernel per
// case, so the single-trait kernel's registers are allocated for its own path
template <int NTRK>
__global__ __launch_bounds__(OTH, 4) void k_chol_offdiag(CholArgs a, OffPlan p) {
  __shared__ __attribute__((aligned(16))) double lds[NPACK * BLKD];   // 72 KiB: rings, then packed X
  __shared__ __attribute__((aligned(16))) double uj_sh[2 * TILE];   // k_stage's column pairs (P_j, Q_j)
  __shared__ double ui_sh[TILE], zj_sh[MAXT][TILE];
  const int64_t npu = (int64_t)p.nP * p.nrs;
  const int64_t n_p = a.B * npu, n_d = a.B * p.nds, n_t = a.B * p.nI;
  int64_t bid = blockIdx.x;
  WgTrace tr(a.wgt);
  if (bid < n_p) {
    const int64_t lg = xcd_remap(bid, n_p);
    const int64_t b = lg / npu;
    const int u = (int)(lg % npu);
    const int I = a.J + 2 + u / p.nrs, rs = u % p.nrs;
    switch (p.nrs) {
      case 1: part_unit<8>(a, b, I, rs, lds, uj_sh, ui_sh); break;
      case 2: part_unit<4>(a, b, I, rs, lds, uj_sh, ui_sh); break;
      default: part_unit<2>(a, b, I, rs, lds, uj_sh, ui_sh); break;
    }
    tr.done(WGT_PART, a.J, I, b);
    return;
  }
  bid -= n_p;
  if (bid < n_d) {
    const int64_t lg = xcd_remap(bid, n_d);
    const int64_t b = lg / p.nds;
    const int u = (int)(lg % p.nds);
    syrk_partial8(a, b, a.J + 1, a.J, lds, p.nds == 1 ? 0 : 1 + u);
    tr.done(WGT_PREP, a.J, a.J + 1, b);
    return;
  }
  bid -= n_d;
  if (bid < n_t) {
    int64_t b;
    int I;
    if (a.q != nullptr) {   // last-term mode: the B tiles (J+1, J) first, then the rest
      if (bid < a.B) {
        b = xcd_remap(bid, a.B);
        I = a.J + 1;
      } else {
        const int64_t lg = xcd_remap(bid - a.B, n_t - a.B);
        b = lg / (p.nI - 1);
        I = a.J + 2 + (int)(lg % (p.nI - 1));
      }
    } else if (p.ne > 0 && p.ne < n_t) {
      // some tiles started by E-units: the others first, those last (with the dispatcher's
      // round-robin a CU then pairs a whole tile with a shortened one or with a lighter class),
      // each class in the E-units' own order (tile e, I-major: its E-unit's XCD)
      const int64_t nne = n_t - p.ne;
      const int64_t e = bid < nne ? p.ne + xcd_remap(bid, nne) : xcd_remap(bid - nne, p.ne);
      b = e % a.B;
      I = a.J + 1 + (int)(e / a.B);
    } else {
      const int64_t lg = xcd_remap(bid, n_t);
      b = lg / p.nI;
      I = a.J + 1 + (int)(lg % p.nI);
    }
    // an E-unit of the diagonal launch summed the term L = Ls0 of the first ne tiles (I-major)
    const int ed = (int64_t)(I - a.J - 1) * a.B + b < p.ne ? 1 : 0;
    tile_unit<NTRK>(a, b, I, p.ahead_cur, ed, lds, uj_sh, ui_sh, zj_sh, tr);
    tr.done(WGT_TILE, a.J, I, b);
    return;
  }
  // column 0, kernel form: K_JJ for J >= 2
  const int64_t lg = xcd_remap(bid - n_t, p.n_kd);
  const int nJ = a.NT - 2;
  diag_grm_tile(a, lg / nJ, 2 + (int)(lg % nJ), reinterpret_cast<uint8_t*>(lds), uj_sh);
  tr.done(WGT_KJJ, a.J, 2 + (int)(lg % nJ), lg / nJ);
}

// ===========================================================================
// SNP form: every system tile (I >= J) of the batch in one launch, before the column loop:
// C = A B^T over the n_T train animals on FP4 MFMA (16x16x128, e2m1 operands, fp32 accumulate),
// 2-bit packed split rows read in place.  Genotype code g read as an e2m1 nibble is g / 2 (0, 0.5,
// 1.0), so a packed dword's even fields become nibbles by x & 0x33333333 and its odd fields by
// (x >> 2) & 0x33333333 -- 3 VALU ops per 16 animals into 2 operand dwords (the int8 form spent 7
// per 16 animals) -- and both operands carry the E8M0 scale 2.0; the counts (<= 4 n_T < 2^24)
// accumulate exactly in fp32 at twice the int8 rate.  The animals' order inside k is the same for A and B, so A B^T is unchanged.
// 4 waves per workgroup; wave (qr, qc) computes a 64 x 64 quadrant = 4 x 4 blocks; 256-animal
// stages through a 3-deep LDS-DMA ring (48 KiB, three workgroups per CU).  A rows are read
// through pi(rho) so the counts land in the f64 accumulator layout.  Off-diagonal tiles store
// the exact counts as int16 where the off-diagonal kernel's lanes read them (kc, see
// tblup_internal.h); diagonal tiles store the exact counts of their 36 lower blocks the same way
// (kd: 18 KiB a tile instead of 72 KiB of fp64 K_JJ + lambda I -- the diagonal kernel and the
// D-units form those values where they read them, kd_block).  (Rows stored as nibbles -- twice the
// bytes, no unpack -- measured no faster: those loads then bound the launch.)
// ===========================================================================
constexpr int STW = 4;   // waves per system-tile workgroup

// K_JJ + lambda I (identity on padding rows) from a diagonal tile's accumulators (exact counts in
// fp32) as packed fp64 blocks into Kd: the tiles J < 2, which the diagonal kernel reads directly
// (sc / ub: the system's scalars and tile J's centring sums -- scal / u, or their LDS copies)
__device__ __forceinline__ void sys_diag_epilogue_src(const CholArgs& a, const v4f (&cnt)[4][4], int64_t b, int J, int qr,
                                                      int qc, int l, const double* sc, const double* ub) {
  const int64_t j0 = (int64_t)J * TILE;
  const double sa_ = sc[SC_SA], cN = sc[SC_CN], invd = sc[SC_INVD], lam = sc[SC_LAM], sm = sc[SC_SM];
  const int64_t nrow = (int64_t)sc[SC_NROW], pad = (int64_t)sc[SC_PAD];
  double* Kd = a.Kd + (b * a.NT + J) * (int64_t)NPACK * BLKD;
  // every centring sum this lane needs, loaded before the first store (Kd and u are both double
  // pointers: loads interleaved with the stores were issued one after another, ~47 us a launch)
  double ur[4][4], uc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) ur[m][r] = ub[16 * (4 * qr + m) + (l >> 4) + 4 * r];
#pragma unroll
  for (int n = 0; n < 4; ++n) uc[n] = ub[16 * (4 * qc + n) + (l & 15)];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int cb = 4 * qr + m, ib = 4 * qc + n;
      if (cb < ib) continue;
      const int il = 16 * ib + (l & 15);
      const int64_t gj = j0 + il;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = 16 * cb + (l >> 4) + 4 * r;
        const int64_t gi = j0 + cl;
        const double kv = grm_value((int32_t)cnt[m][n][r], ur[m][r], uc[n], sa_, cN, invd, sm);
        const double v = (sys_real(gi, pad, nrow) && sys_real(gj, pad, nrow)) ? kv + ((gi == gj) ? lam : 0.0)
                                                                              : ((gi == gj) ? 1.0 : 0.0);
        st64<TBLUP_AB_NT_KD>(Kd + pk(cb, ib) + bo(cl & 15, il & 15), v);
      }
    }
}
__device__ __forceinline__ void sys_diag_epilogue_inl(const CholArgs& a, const v4f (&cnt)[4][4], int64_t b, int J, int qr,
                                                      int qc, int l) {
  sys_diag_epilogue_src(a, cnt, b, J, qr, qc, l, a.scal + b * SCAL, a.u + b * a.prow + (int64_t)J * TILE);
}
__device__ void sys_diag_epilogue(const CholArgs& a, const v4f (&cnt)[4][4], int64_t b, int J, int qr, int qc, int l);

// a diagonal tile's counts as int16 (diag): its 36 lower blocks (cb >= ib) only, packed block
// e = cb (cb + 1) / 2 + ib, lane order of the f64 C layout (kd_load / kd_block read them); an
// off-diagonal tile's: store_counts16's layout
// The super-tile kernel's counted ring waits (k_sys_tiles_st) leave the VMEM ops younger than the
// stage they wait for outstanding: ST_STAGE_OPS LDS-DMA loads per lane for each later stage (issue():
// two rows x A and B) and, after a unit of two off-diagonal tiles, this function's stores -- one 8-B
// store per 16 x 16 block of the wave's 4 x 4 quadrant (all 16 off the diagonal: addresses 512 B
// apart within a lane, never merged).  A count above the real number only waits for more.
constexpr int ST_STAGE_OPS = 4;
constexpr int ST_TILE_STORES = 4 * 4;
constexpr int ST_UNIT_STORES = 2 * ST_TILE_STORES;
static_assert(2 * ST_STAGE_OPS + ST_UNIT_STORES < 64, "vmcnt holds 6 bits");
__device__ __forceinline__ void store_counts16_any(int16_t* kt, const v4f (&cnt)[4][4], int qr, int qc, int l,
                                                   bool diag) {
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int cb = 4 * qr + m, ib = 4 * qc + n;
      if (diag && cb < ib) continue;
      const v4f c = cnt[m][n];
      const int2 packed = {(int)((uint32_t)((int)c[0] & 0xffff) | ((uint32_t)(int)c[1] << 16)),
                           (int)((uint32_t)((int)c[2] & 0xffff) | ((uint32_t)(int)c[3] << 16))};
      nt_store2(kt + ((diag ? cb * (cb + 1) / 2 + ib : ib * 8 + cb) * 64 + l) * 4, packed);
    }
}

// two packed dwords (32 animals) -> one fp4 MFMA operand (even fields, odd fields of each): the
// 2-bit code g lands in the low half of a nibble, e2m1 value g / 2 (0, 0.5 subnormal, 1.0), and
// the E8M0 operand scales 2.0 (128) restore g -- 3 VALU ops per packed dword instead of 4
__device__ __forceinline__ v4i fp4_operand(uint32_t x0, uint32_t x1) {
  constexpr uint32_t M = 0x33333333u;
  return v4i{(int)(x0 & M), (int)((x0 >> 2) & M), (int)(x1 & M), (int)((x1 >> 2) & M)};
}
// the scaled f8f6f4 MFMA with fp4 operands in 4 VGPRs each (the clang builtin types them as 8 VGPRs,
// the upper half unused by fp4 -- 32 more VGPRs and a zeroing move per operand)
__device__ v4f mfma_fp4_16x16x128(v4i a, v4i b, v4f c, int cbsz, int blgp, int opsel_a, int scale_a, int opsel_b,
                                  int scale_b) __asm("llvm.amdgcn.mfma.scale.f32.16x16x128.f8f6f4.v4i32.v4i32");

template <bool DUAL>   // kernel form: the gathered panel's packed animal rows
__global__ __launch_bounds__(64 * STW, 2) void k_sys_tiles(CholArgs a, int16_t* kc, int ntri) {
  constexpr int D = 3;                 // 64-B stages (256 animals) in the LDS ring (48 KiB: 3 workgroups per CU)
  constexpr int TB = TILE * 64;        // one operand image of a stage: 8 KiB
  __shared__ __attribute__((aligned(16))) uint8_t lds[D * 2 * TB];   // 64 KiB
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, qr = w >> 1, qc = w & 1;
  WgTrace tr(a.wgt);
  const int64_t lg = xcd_remap(blockIdx.x, gridDim.x);   // an individual's tiles on one XCD
  const int64_t b = lg / ntri;
  const int t = (int)(lg % ntri);
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  const int J = t - I * (I + 1) / 2;
  const bool compute = (I != J) || (qr >= qc);   // diagonal tile: the upper quadrant is never read
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)J * TILE;
  const double* sc = a.scal + b * SCAL;
  const int64_t nblk = (int64_t)sc[SC_CBLK];
  const int64_t nst = (nblk + 3) >> 2;
  const int tail_ch = (int)(nblk & 3);
  // loader: wave w fills rows 16 (2w + h) + (l >> 2), h = 0, 1, of both operand images
  const uint8_t* sa[2];
  const uint8_t* sb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 16 * (2 * w + h) + (l >> 2), pos = l & 3;
    sa[h] = (DUAL ? row_dpk(a, b, j0 + row) : row_packed(a, b, j0 + row)) + 16 * (pos ^ ((row >> 2) & 3));
    sb[h] = (DUAL ? row_dpk(a, b, i0 + row) : row_packed(a, b, i0 + row)) + 16 * (pos ^ ((row >> 2) & 2));
  }
  auto issue = [&](int64_t st) {
    uint8_t* slot = lds + (int)(st % D) * 2 * TB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ring_glds<TBLUP_AB_ASM_I8>(sa[h] + st * 64, slot + (2 * w + h) * 1024);
      ring_glds<TBLUP_AB_ASM_I8>(sb[h] + st * 64, slot + TB + (2 * w + h) * 1024);
    }
  };
  v4f cnt[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) cnt[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int64_t st = 0; st < D - 1 && st < nst; ++st) issue(st);
  const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
  for (int64_t st = 0; st < nst; ++st) {
    if (st + D - 2 < nst) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 4) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (st + D - 1 < nst) issue(st + D - 1);
    if (compute && !(a.skip & (1 << 18))) {
      const uint8_t* As = lds + (int)(st % D) * 2 * TB;
      const uint8_t* Bs = As + TB;
      const bool ztail = (st == nst - 1 && tail_ch != 0 && ch >= tail_ch);   // past the training animals
      uint4 aq[4], bq[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        aq[m] = *reinterpret_cast<const uint4*>(As + i8off_a(16 * (4 * qr + m) + prow, ch));
        bq[m] = *reinterpret_cast<const uint4*>(Bs + i8off_b(16 * (4 * qc + m) + rho, ch));
        if (ztail) bq[m] = uint4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        v4i av[4], bv[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          av[m] = s2 == 0 ? fp4_operand(aq[m].x, aq[m].y) : fp4_operand(aq[m].z, aq[m].w);
          bv[m] = s2 == 0 ? fp4_operand(bq[m].x, bq[m].y) : fp4_operand(bq[m].z, bq[m].w);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n)   // cbsz = blgp = 4: A, B in fp4; E8M0 scales 128 = 2.0
            cnt[m][n] = mfma_fp4_16x16x128(av[m], bv[n], cnt[m][n], 4, 4, 0, 128, 0, 128);
      }
    }
  }
  if (compute && I == J && J < 2 && !(a.skip & (1 << 17)))
    sys_diag_epilogue(a, cnt, b, J, qr, qc, l);   // read directly by the diagonal kernel
  else if (compute && !(a.skip & (I != J ? 1 << 16 : 1 << 17)))
    store_counts16_any(I != J ? kc + ((b * (a.NT * (a.NT - 1) / 2)) + I * (I - 1) / 2 + J) * KC_TILE
                              : a.kd + (b * a.NT + J) * KD_TILE,
                       cnt, qr, qc, l, I == J);
  tr.done(WGT_SYS, J, I, b);
}

// Persistent super-tile form of k_sys_tiles (large batches, sys_tiles_grid): one 8-wave workgroup
// per CU walks a contiguous run of units, a unit being a 256 x 256 super-tile = the 2 x 2 tiles
// (I0 + ti, J0 + tj), I0 = 2 SI, J0 = 2 SJ, SI >= SJ, of one individual (10 units at NT = 8 instead
// of 36 tile workgroups).  Per 256-animal stage a unit loads 2 x 256 rows (32 KiB: half the bytes
// per tile of the single-tile form) and runs 64 MFMAs per wave: wave (tj, qr, qc) accumulates
// quadrant (qr, qc) of tiles (I0, J0 + tj) and (I0 + 1, J0 + tj) (A fragments shared).  The
// 3-deep LDS-DMA ring runs on across unit boundaries (the next unit's first stages load while
// this one's last stage computes and its counts are stored), so the per-tile prologue and store
// latency of 36 short workgroups is paid once per run.  Row addresses come from a per-individual
// row table in LDS (no global load whose use would drain the ring).  The same exact fp32 counts as
// k_sys_tiles (every partial sum an integer below 2^24), stored to the same places.
constexpr int SPW = 8;                 // waves per super-tile workgroup
constexpr int SP_MAXIND = 64;          // individuals in one workgroup's run (sys_tiles_grid checks)

#ifndef TBLUP_AB_SYS_ST_MIN   // A/B builds only (tools/ab_build_defs.sh)
#define TBLUP_AB_SYS_ST_MIN 4
#endif
#ifndef TBLUP_AB_SP_D
#define TBLUP_AB_SP_D 3
#endif
static_assert(TBLUP_AB_SP_D >= 3 && TBLUP_AB_SP_D <= 4, "ring waits are written for 1-2 stages ahead");
constexpr int64_t SYS_ST_MIN = TBLUP_AB_SYS_ST_MIN;   // auto: at least this many units per CU

template <bool DUAL>   // kernel form: the gathered panel's packed animal rows
__global__ __launch_bounds__(64 * SPW, 1) void k_sys_tiles_st(CholArgs a, int16_t* kc, int nsu, int nunits) {
  constexpr int D = TBLUP_AB_SP_D;     // stages in the ring
  constexpr int TB2 = 2 * TILE * 64;   // one 256-row operand image of a stage: 16 KiB
  __shared__ __attribute__((aligned(16))) uint8_t lds[D * 2 * TB2];   // 96 KiB at D = 3
  __shared__ int32_t rowtab[SP_ROWTAB];
  __shared__ int32_t cblk_tab[SP_MAXIND];   // contraction blocks of the run's individuals (SNP form:
                                            // n_Tp / 64 each, SC_CBLK -- not read from scal, so this
                                            // launch may precede the scalars' k_stats_diag_counts)
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int tj = w >> 2, qr = (w >> 1) & 1, qc = w & 1;
  const int NT = a.NT;
  WgTrace tr(a.wgt);
  const int u0 = (int)((int64_t)blockIdx.x * nunits / gridDim.x), u1 = (int)((int64_t)(blockIdx.x + 1) * nunits / gridDim.x);
  const int b_first = u0 / nsu;
  const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
  const int pos = l & 3;
  // super-tile s of the lower triangle (row-major): SI, SJ
  auto unit_tiles = [&](int u, int& b, int& I0, int& J0) __attribute__((always_inline)) {
    b = __builtin_amdgcn_readfirstlane(u / nsu);
    const int s = __builtin_amdgcn_readfirstlane(u % nsu);
    int SI = 0;
    while ((SI + 1) * (SI + 2) / 2 <= s) ++SI;
    I0 = 2 * SI;
    J0 = 2 * (s - SI * (SI + 1) / 2);
  };
  // the row table of individual b: packed row index of each of its ns system rows (row P: zero)
  int tab_b = -1;
  auto load_rowtab = [&](int b) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int64_t o0 = a.off[b], k = a.off[b + 1] - o0;
    const int64_t pad = a.padfirst ? a.ns - k : 0;
    const int nrt = 2 * TILE * ((NT + 1) / 2);   // rows a super-tile reads (ns rounded up to 256)
    if constexpr (!DUAL) {
      for (int r = t; r < nrt; r += 64 * SPW)
        rowtab[r] = (int32_t)(r < a.ns && sys_real(r, pad, k) ? snp_col(a.idx[o0 + r - pad], a.P) : a.P);
    } else {   // kernel form: the panel's own rows (past ns: any row -- those tiles are not stored)
      for (int r = t; r < nrt; r += 64 * SPW) rowtab[r] = r < a.ns ? r : 0;
    }
    __syncthreads();
    tab_b = b;
  };
  // issue cursor: the unit and stage whose loads go out next, and its row pointers
  int iu = u0, ib = 0;
  int ist = 0, inst = 0;
  int ra[2], rb[2];                    // packed rows of this lane's A / B loads (h = 0, 1)
  const uint8_t* gbase = nullptr;
  const int64_t gsr = DUAL ? a.pstride / a.prow : a.gs_row;   // packed row bytes
  const int offa[2] = {16 * (pos ^ (((l >> 2) >> 2) & 3)), 16 * (pos ^ (((16 + (l >> 2)) >> 2) & 3))};
  const int offb[2] = {16 * (pos ^ (((l >> 2) >> 2) & 2)), 16 * (pos ^ (((16 + (l >> 2)) >> 2) & 2))};
  auto setup_issue = [&]() __attribute__((always_inline)) {
    int I0, J0;
    unit_tiles(iu, ib, I0, J0);
    if (ib != tab_b) load_rowtab(ib);
    inst = (cblk_tab[ib - b_first] + 3) >> 2;
    gbase = DUAL ? a.panel + ib * a.pstride : a.ft.gpk[fold_of(a.ft, ib)];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 16 * (2 * w + h) + (l >> 2);
      ra[h] = rowtab[J0 * TILE + row];
      rb[h] = rowtab[I0 * TILE + row];
    }
    ist = 0;
  };
  // issue one stage into ring slot g % D and advance the cursor (false: nothing left)
  auto issue = [&](int g) __attribute__((always_inline)) {
    if (iu >= u1) return;
    uint8_t* slot = lds + (g % D) * 2 * TB2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      glds16_asm(gbase + (int64_t)ra[h] * gsr + (offa[h] + ist * 64), slot + (2 * w + h) * 1024);
      glds16_asm(gbase + (int64_t)rb[h] * gsr + (offb[h] + ist * 64), slot + TB2 + (2 * w + h) * 1024);
    }
    if (++ist == inst && ++iu < u1) setup_issue();
  };
  if (u0 >= u1) return;
  const int nind = (u1 - 1) / nsu - b_first + 1;
  if (t < nind) {   // kernel form: the individual's k SNPs
    const int64_t bt = b_first + t;
    cblk_tab[t] = (int32_t)(DUAL ? (a.off[bt + 1] - a.off[bt] + KBLK - 1) / KBLK : a.ytp / KBLK);
  }
  __syncthreads();
  setup_issue();
  // total stages of the run (the units of one individual share its stage count)
  int nstages = 0;
  for (int u = u0; u < u1;) {
    const int b = u / nsu, ue = min(u1, (b + 1) * nsu);
    nstages += (ue - u) * ((cblk_tab[b - b_first] + 3) >> 2);
    u = ue;
  }
  for (int g = 0; g < D - 1; ++g) issue(g);

  v4f cnt[2][4][4];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) cnt[ti][m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  // compute cursor
  int cu = u0, cb_ = 0;
  int cI0 = 0, cJ0 = 0, cst = 0;
  unit_tiles(cu, cb_, cI0, cJ0);
  int cnblk = cblk_tab[cb_ - b_first];
  int cnst = (int)((cnblk + 3) >> 2);
  bool stored_full = false;   // the previous stage ended a unit whose every wave stored 32 count pairs
  for (int g = 0; g < nstages; ++g) {
    // stage g's loads done: the younger ops are the 4 loads of each stage issued after it (up to
    // D - 2) and the stores of the unit that ended last stage (32 per wave after a full
    // off-diagonal super-tile: 16 8-B stores per tile whose addresses lie 512 B apart within a
    // lane, so none can be merged; any other unit: waited for)
    const int ahead = min(D - 2, nstages - 1 - g);   // stages issued after stage g
    if (ahead >= 2) {
      if (stored_full)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * ST_STAGE_OPS + ST_UNIT_STORES) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * ST_STAGE_OPS) : "memory");
    } else if (ahead == 1) {
      if (stored_full)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(ST_STAGE_OPS + ST_UNIT_STORES) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(ST_STAGE_OPS) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    issue(g + D - 1);
    const int J0t = cJ0 + tj;
    bool comp[2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti) {
      const int I = cI0 + ti;
      comp[ti] = I < NT && J0t < NT && (I > J0t || (I == J0t && qr >= qc));
    }
    if ((comp[0] || comp[1]) && !(a.skip & (1 << 18))) {
      const uint8_t* As = lds + (g % D) * 2 * TB2;
      const uint8_t* Bs = As + TB2;
      const int tail_ch = (int)(cnblk & 3);
      const bool ztail = (cst == cnst - 1 && tail_ch != 0 && ch >= tail_ch);   // past the training animals
      uint4 aq[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) aq[m] = *reinterpret_cast<const uint4*>(As + i8off_a(TILE * tj + 16 * (4 * qr + m) + prow, ch));
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        if (!comp[ti]) continue;
        uint4 bq[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          bq[n] = *reinterpret_cast<const uint4*>(Bs + i8off_b(TILE * ti + 16 * (4 * qc + n) + rho, ch));
          if (ztail) bq[n] = uint4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          v4i av[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) av[m] = s2 == 0 ? fp4_operand(aq[m].x, aq[m].y) : fp4_operand(aq[m].z, aq[m].w);
#pragma unroll
          for (int n = 0; n < 4; ++n) {
            const v4i bv = s2 == 0 ? fp4_operand(bq[n].x, bq[n].y) : fp4_operand(bq[n].z, bq[n].w);
#pragma unroll
            for (int m = 0; m < 4; ++m)   // cbsz = blgp = 4: A, B in fp4; E8M0 scales 128 = 2.0
              cnt[ti][m][n] = mfma_fp4_16x16x128(av[m], bv, cnt[ti][m][n], 4, 4, 0, 128, 0, 128);
          }
        }
      }
    }
    stored_full = false;
    if (++cst == cnst) {
      // the unit's epilogue: its tiles' counts (diagonal tiles J < 2 too: k_sys_diag_counts forms
      // their K_JJ + lambda I afterwards -- the fp64 epilogue here would spill the accumulators)
      stored_full = cI0 != cJ0 && cI0 + 1 < NT && !(a.skip & (1 << 16));
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        const int I = cI0 + ti;
        if (!comp[ti]) continue;
        if (!(a.skip & (I != J0t ? 1 << 16 : 1 << 17))) {
          store_counts16_any(I != J0t ? kc + ((int64_t)cb_ * (NT * (NT - 1) / 2) + I * (I - 1) / 2 + J0t) * KC_TILE
                                      : a.kd + ((int64_t)cb_ * NT + J0t) * KD_TILE,
                             cnt[ti], qr, qc, l, I == J0t);
        }
      }
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) cnt[ti][m][n] = v4f{0.f, 0.f, 0.f, 0.f};
      if (++cu < u1) {
        unit_tiles(cu, cb_, cI0, cJ0);
        cnblk = cblk_tab[cb_ - b_first];
        cnst = (int)((cnblk + 3) >> 2);
      }
      cst = 0;
    }
  }
  tr.done(WGT_SYS, 0, 0, u0 / nsu);
}

// Fold-fused evaluation with shared counts (IntraGCV's folds, tblup_eval_folds*): when every fold's
// training rows R_f and validation rows V_f make up the same multiset T_all, C_{R_f} = C_{T_all} -
// C_{V_f}.  One workgroup per (individual b, tile) accumulates C_{T_all} over fold 0's rows
// [0, nRp) (train, zero padding, validation, zero padding), then for f = 0 .. F-1 adds C_{V_{f-1}}
// back (f > 0) and subtracts C_{V_f} -- the A operand negated through the e2m1 sign bits -- and
// stores system f * B + b's tile after each subtraction.  The stage sequence runs through one
// 3-deep LDS-DMA ring across these segments.  Every partial sum is an exact integer in fp32, so
// the tiles equal k_sys_tiles' per-fold ones bit for bit; contraction (nRp + (2F - 1) nVp) / (F nTp)
// of the per-fold launch's (config 2, 5 folds of 256: 14 stages of 256 animals instead of 20).
__global__ __launch_bounds__(64 * STW, 2) void k_sys_tiles_folds(CholArgs a, int16_t* kc, int ntri) {
  constexpr int D = 3;
  constexpr int TB = TILE * 64;
  __shared__ __attribute__((aligned(16))) uint8_t lds[D * 2 * TB];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, qr = w >> 1, qc = w & 1;
  WgTrace tr(a.wgt);
  const int64_t lg = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t b = lg / ntri;   // individual: system b of fold 0
  const int t = (int)(lg % ntri);
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  const int J = t - I * (I + 1) / 2;
  const bool compute = (I != J) || (qr >= qc);
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)J * TILE;
  const int F = a.ft.nf;
  const int64_t bpf = a.ft.bpf;
  const int64_t vbyte = a.ytp / 4;                           // validation rows start (nTp animals)
  const int64_t nblkA = a.gs_row / 16, nsA = (nblkA + 3) >> 2;   // all nRp animals, 64 per block
  const int64_t nblkV = nblkA - a.ytp / 64, nsV = (nblkV + 3) >> 2;
  const int64_t nst = nsA + (2 * F - 1) * nsV;
  // the same SNP rows in every fold's layout: per-lane row offsets, fold bases per stage
  int64_t oa[2], ob[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 16 * (2 * w + h) + (l >> 2), pos = l & 3;
    oa[h] = (row_packed(a, b, j0 + row) - a.ft.gpk[0]) + 16 * (pos ^ ((row >> 2) & 3));
    ob[h] = (row_packed(a, b, i0 + row) - a.ft.gpk[0]) + 16 * (pos ^ ((row >> 2) & 2));
  }
  // stage g -> segment k (0: T_all of fold 0, 2f + 1: minus V_f, 2f + 2: plus V_f) and its stage
  auto seg_of = [&](int64_t g, int& k, int64_t& st) {
    if (g < nsA) {
      k = 0;
      st = g;
    } else {
      k = 1 + (int)((g - nsA) / nsV);
      st = (g - nsA) % nsV;
    }
  };
  auto issue = [&](int64_t g) __attribute__((always_inline)) {
    int k;
    int64_t st;
    seg_of(g, k, st);
    const uint8_t* base = a.ft.gpk[k == 0 ? 0 : (k - 1) >> 1] + (k == 0 ? 0 : vbyte) + st * 64;
    uint8_t* slot = lds + (int)(g % D) * 2 * TB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      ring_glds<TBLUP_AB_ASM_I8>(base + oa[h], slot + (2 * w + h) * 1024);
      ring_glds<TBLUP_AB_ASM_I8>(base + ob[h], slot + TB + (2 * w + h) * 1024);
    }
  };
  v4f cnt[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) cnt[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int64_t g = 0; g < D - 1 && g < nst; ++g) issue(g);
  const int rho = l & 15, prow = (rho >> 2) + 4 * (rho & 3), ch = l >> 4;
  int64_t g = 0;
  for (int k = 0; k < 2 * F; ++k) {
    const int64_t ns_k = k == 0 ? nsA : nsV;
    const int tail_ch = (int)((k == 0 ? nblkA : nblkV) & 3);
    const int neg = (k & 1) ? (int)0x88888888u : 0;   // e2m1 sign bits: subtract this segment
    for (int64_t st = 0; st < ns_k; ++st, ++g) {
      if (g + D - 2 < nst) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 4) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (g + D - 1 < nst) issue(g + D - 1);
      if (compute) {
        const uint8_t* As = lds + (int)(g % D) * 2 * TB;
        const uint8_t* Bs = As + TB;
        const bool ztail = (st == ns_k - 1 && tail_ch != 0 && ch >= tail_ch);   // past the segment's rows
        uint4 aq[4], bq[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          aq[m] = *reinterpret_cast<const uint4*>(As + i8off_a(16 * (4 * qr + m) + prow, ch));
          bq[m] = *reinterpret_cast<const uint4*>(Bs + i8off_b(16 * (4 * qc + m) + rho, ch));
          if (ztail) bq[m] = uint4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          v4i av[4], bv[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            av[m] = s2 == 0 ? fp4_operand(aq[m].x, aq[m].y) : fp4_operand(aq[m].z, aq[m].w);
            av[m] |= neg;
            bv[m] = s2 == 0 ? fp4_operand(bq[m].x, bq[m].y) : fp4_operand(bq[m].z, bq[m].w);
          }
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
              cnt[m][n] = mfma_fp4_16x16x128(av[m], bv[n], cnt[m][n], 4, 4, 0, 128, 0, 128);
        }
      }
    }
    if (!(k & 1) || !compute) continue;
    const int64_t s = (int64_t)((k - 1) >> 1) * bpf + b;   // C_{T_all} - C_{V_f}: system f * B + b
    store_counts16_any(I != J ? kc + ((s * (a.NT * (a.NT - 1) / 2)) + I * (I - 1) / 2 + J) * KC_TILE
                              : a.kd + (s * a.NT + J) * KD_TILE,
                       cnt, qr, qc, l, I == J);
  }
  tr.done(WGT_SYS, J, I, b);
}


__device__ void sys_diag_epilogue(const CholArgs& a, const v4f (&cnt)[4][4], int64_t b, int J, int qr, int qc,
                                  int l) {
  sys_diag_epilogue_inl(a, cnt, b, J, qr, qc, l);
}

// fold-fused chunks (k_sys_tiles_folds stores every diagonal tile's counts): K_JJ + lambda I of the
// tiles J < 2 into Kd, one 4-wave workgroup per (system, J)
__global__ __launch_bounds__(64 * STW) void k_sys_diag_counts(CholArgs a) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, qr = w >> 1, qc = w & 1;
  const int64_t s = blockIdx.x >> 1;
  const int J = (int)(blockIdx.x & 1);
  if (qr < qc || J >= a.NT) return;   // the upper quadrant is never read
  const int16_t* kt = a.kd + (s * a.NT + J) * KD_TILE;
  v4f cnt[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int cb = 4 * qr + m, ib = 4 * qc + n;
      int2 p = {0, 0};
      if (cb >= ib) p = *reinterpret_cast<const int2*>(kt + ((cb * (cb + 1) / 2 + ib) * 64 + l) * 4);
      cnt[m][n] = v4f{(float)(int16_t)(p.x & 0xffff), (float)(int16_t)(p.x >> 16), (float)(int16_t)(p.y & 0xffff),
                      (float)(int16_t)(p.y >> 16)};
    }
  sys_diag_epilogue_inl(a, cnt, s, J, qr, qc, l);
}

// k_sys_tiles_st chunks: k_sys_diag_counts with the per-individual scalars formed here (the same
// stats_wg code as k_indiv_stats) instead of in a launch before the system tiles -- one launch less
// on the chain.  Workgroup (b, J < 2): stats_wg (workgroup J = 0 also stores scal), tile
// J's centring sums into LDS, then the epilogue from the LDS copies; the u / rhs rows are split
// between the two workgroups.
__global__ __launch_bounds__(64 * STW) void k_stats_diag_counts(CholArgs a, StatsFuse x) {
  static_assert(64 * STW == STATS_THREADS, "stats_wg runs on the workgroup's 256 threads");
  __shared__ StatsShared sh;
  __shared__ double u_sh[TILE];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, qr = w >> 1, qc = w & 1;
  const int64_t b = blockIdx.x >> 1;
  const int J = (int)(blockIdx.x & 1);
  const bool tile = qr >= qc && J < a.NT;   // the upper quadrant is never read
  // the counts first: their loads overlap the scalars' reduction
  v4f cnt[4][4];
  const int16_t* kt = a.kd + (b * a.NT + J) * KD_TILE;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int cb = 4 * qr + m, ib = 4 * qc + n;
      int2 p = {0, 0};
      if (tile && cb >= ib) p = *reinterpret_cast<const int2*>(kt + ((cb * (cb + 1) / 2 + ib) * 64 + l) * 4);
      cnt[m][n] = v4f{(float)(int16_t)(p.x & 0xffff), (float)(int16_t)(p.x >> 16), (float)(int16_t)(p.y & 0xffff),
                      (float)(int16_t)(p.y >> 16)};
    }
  // u_a = s_a of tile J's rows (stats_wg's u values, gathered here before its reduction so that
  // these loads overlap it)
  if (t < TILE) {
    const int64_t o0 = a.off[b], k = a.off[b + 1] - o0;
    const int64_t pad = a.padfirst ? a.ns - k : 0;
    const int64_t r = (int64_t)J * TILE + t;
    const int32_t* csT = a.ft.csT[fold_of(a.ft, b)];
    u_sh[t] = (r < a.ns && sys_real(r, pad, k)) ? (double)csT[snp_col(a.idx[o0 + r - pad], a.P)] : 0.0;
  }
  // (stats_wg's barriers also publish u_sh)
  stats_wg(a.idx, a.off, a.ft, x.csA, x.n, x.nT, a.ytp, a.P, a.form, a.ns, a.padfirst, a.nt, x.branch, x.h2, b,
           J == 0 ? x.scal : nullptr, x.err, sh);
  if (tile) sys_diag_epilogue_src(a, cnt, b, J, qr, qc, l, sh.sc, u_sh);
  // then the u / rhs rows, split between the individual's two workgroups (their stores overlap the
  // epilogue's)
  const int64_t half = (a.ns / 2 + 63) & ~(int64_t)63;
  stats_rows(a.idx, a.off, a.ft, a.P, a.ns, a.padfirst, a.nt, b, x.u, x.rhs, sh, J == 0 ? 0 : half,
             J == 0 ? half : a.ns);
}

static CholArgs make_args(const CholLaunch& c, int J) {
  CholArgs a{c.L, c.Dinv, c.z, c.w, c.S, c.Kd, c.yT, c.rhs, c.panel, c.pstride, c.u, c.scal, c.sd.ns,
             c.sd.prow, c.sd.form, c.idx, c.off, c.gpk_row, c.d.P, c.d.nTp, c.d.nt, c.sd.NT, J, c.skip,
             c.wgt, nullptr, c.kc, c.part, c.q, c.B, c.ft, c.padskip,
             (c.sd.form == FORM_PRIMAL && c.sd.pad_first) ? 1 : 0, c.kd};
  return a;
}

int cu_count() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

int64_t sys_tiles_grid(const CholLaunch& c) {
  const int64_t ntri = (int64_t)c.sd.NT * (c.sd.NT + 1) / 2;
  const int64_t NS = (c.sd.NT + 1) / 2, units = c.B * (NS * (NS + 1) / 2);
  const int64_t cus = cu_count();
  const bool st = c.sys_st > 0 || (c.sys_st < 0 && units >= SYS_ST_MIN * cus);
  const int64_t grid = std::min(units, cus);
  const int64_t nsu = NS * (NS + 1) / 2, per = (units + grid - 1) / grid;
  if (!st || c.sd.ns > SP_ROWTAB || per / nsu + 2 > SP_MAXIND) return -(c.B * ntri);
  return grid;
}

hipError_t launch_sys_tiles(const CholLaunch& c, hipStream_t s) {
  CholArgs a = make_args(c, 0);
  const int ntri = c.sd.NT * (c.sd.NT + 1) / 2;
  const int64_t grid = sys_tiles_grid(c);
  if (grid > 0) {
    const int NS = (c.sd.NT + 1) / 2;
    if (c.sd.form == FORM_PRIMAL)
      hipLaunchKernelGGL(k_sys_tiles_st<false>, dim3((unsigned)grid), dim3(64 * SPW), 0, s, a, c.kc, NS * (NS + 1) / 2,
                         (int)(c.B * (NS * (NS + 1) / 2)));
    else
      hipLaunchKernelGGL(k_sys_tiles_st<true>, dim3((unsigned)grid), dim3(64 * SPW), 0, s, a, c.kc, NS * (NS + 1) / 2,
                         (int)(c.B * (NS * (NS + 1) / 2)));
    if (hipError_t e = hipGetLastError()) return e;
    a.wgt = nullptr;
    if (c.stats)
      hipLaunchKernelGGL(k_stats_diag_counts, dim3((unsigned)(c.B * 2)), dim3(64 * STW), 0, s, a, *c.stats);
    else
      hipLaunchKernelGGL(k_sys_diag_counts, dim3((unsigned)(c.B * 2)), dim3(64 * STW), 0, s, a);
  } else {
    if (c.stats) return hipErrorInvalidValue;   // the per-tile kernel reads the scalars
    if (c.sd.form == FORM_PRIMAL)
      hipLaunchKernelGGL(k_sys_tiles<false>, dim3((unsigned)(c.B * ntri)), dim3(64 * STW), 0, s, a, c.kc, ntri);
    else
      hipLaunchKernelGGL(k_sys_tiles<true>, dim3((unsigned)(c.B * ntri)), dim3(64 * STW), 0, s, a, c.kc, ntri);
  }
  return hipGetLastError();
}

hipError_t launch_sys_tiles_folds(const CholLaunch& c, hipStream_t s) {
  CholArgs a = make_args(c, 0);
  const int ntri = c.sd.NT * (c.sd.NT + 1) / 2;
  hipLaunchKernelGGL(k_sys_tiles_folds, dim3((unsigned)(c.ft.bpf * ntri)), dim3(64 * STW), 0, s, a, c.kc, ntri);
  if (hipError_t e = hipGetLastError()) return e;
  a.wgt = nullptr;
  if (c.stats)   // k_sys_tiles_folds reads no scalar either
    hipLaunchKernelGGL(k_stats_diag_counts, dim3((unsigned)(c.B * 2)), dim3(64 * STW), 0, s, a, *c.stats);
  else
    hipLaunchKernelGGL(k_sys_diag_counts, dim3((unsigned)(c.B * 2)), dim3(64 * STW), 0, s, a);
  return hipGetLastError();
}

__global__ __launch_bounds__(OTH, 2) void k_diag_grm8(CholArgs a, int nJ) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * TILE * 64];
  __shared__ double u_sh[TILE];
  const int64_t lg = xcd_remap(blockIdx.x, gridDim.x);   // an individual's tiles on one XCD
  diag_grm_tile(a, lg / nJ, (int)(lg % nJ), lds, u_sh);
}

hipError_t launch_diag_grm(const CholLaunch& c, hipStream_t s) {
  CholArgs a = make_args(c, 0);
  a.wgt = nullptr;
  const int nJ = std::min(c.sd.NT, 2);
  hipLaunchKernelGGL(k_diag_grm8, dim3((unsigned)(c.B * nJ)), dim3(OTH), 0, s, a, nJ);
  return hipGetLastError();
}

// Kernel-form folds sharing one animal set: A_R A_R^T of individual b over fold 0's split rows (its
// panel, system b), every 128 x 128 tile pair I >= J of the n_Rp rows on int8 MFMA from the packed
// rows (i8_tt8_pk64), stored both ways into a full n_Rp x n_Rp int32 matrix (FoldTab::gsh)
__global__ __launch_bounds__(OTH, 2) void k_gshare(CholArgs a, int NR) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * TILE * 64];
  const int64_t ntp = (int64_t)NR * (NR + 1) / 2;
  const int64_t lg = xcd_remap(blockIdx.x, gridDim.x);   // an individual's tiles on one XCD
  const int64_t b = lg / ntp;
  const int tp = (int)(lg % ntp);
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= tp) ++I;
  const int J = tp - I * (I + 1) / 2;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i0 = (int64_t)I * TILE, j0 = (int64_t)J * TILE;
  const int row = 16 * w + (l >> 2), pos = l & 3;
  const int64_t nblk = (int64_t)a.scal[b * SCAL + SC_CBLK];
  v4i cnt[8];
  i8_tt8_pk64<4>(row_dpk(a, b, j0 + row) + 16 * (pos ^ ((row >> 2) & 3)),
                 row_dpk(a, b, i0 + row) + 16 * (pos ^ ((row >> 2) & 2)), nblk, lds, cnt);
  const int64_t ld = a.ft.gsh_ld;
  int32_t* G = a.ft.gsh + b * ld * ld;
  const int64_t ic = i0 + 16 * w + (l & 15);
#pragma unroll
  for (int cb = 0; cb < 8; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t jr = j0 + 16 * cb + (l >> 4) + 4 * r;
      G[jr * ld + ic] = cnt[cb][r];
      G[ic * ld + jr] = cnt[cb][r];
    }
}

hipError_t launch_gshare(const CholLaunch& c, hipStream_t s) {
  const FoldTab& ft = c.ft;
  if (!ft.gsh || c.sd.form != FORM_DUAL || c.d.nRp % TILE) return hipErrorInvalidValue;
  CholArgs a = make_args(c, 0);
  a.wgt = nullptr;
  const int NR = (int)(c.d.nRp / TILE);
  hipLaunchKernelGGL(k_gshare, dim3((unsigned)(ft.bpf * NR * (NR + 1) / 2)), dim3(OTH), 0, s, a, NR);
  return hipGetLastError();
}

hipError_t launch_chol_diag(const CholLaunch& c, int J, const OffPlan& p, hipStream_t s) {
  CholArgs a = make_args(c, J);
  const int64_t nwg = c.B * (1 + p.ndd) + p.ne;
  // E-units need the partial-sum slots and a tile below the diagonal, and are built without the
  // shared fold counts (k_acc<8, false>)
  if (p.ne > 0 && (c.part == nullptr || J < 1 || p.ne > c.B * p.nI || c.ft.gsh)) return hipErrorInvalidValue;
  // profiling: the phase stamps of this launch follow its workgroup records
  if (c.wgt) a.dtr = c.wgt + nwg * WGT_REC;
  hipLaunchKernelGGL(k_chol_diag, dim3((unsigned)nwg), dim3(DTHR), 0, s, a, p.ne, p.ahead_cur ? J - 1 : 0);
  return hipGetLastError();
}

hipError_t launch_chol_offdiag(const CholLaunch& c, int J, const OffPlan& p, hipStream_t s) {
  if (p.nI <= 0) return hipSuccess;
  CholArgs a = make_args(c, J);
  if (c.d.nt == 1)
    hipLaunchKernelGGL(k_chol_offdiag<1>, dim3((unsigned)offdiag_grid(p, c.B)), dim3(OTH), 0, s, a, p);
  else
    hipLaunchKernelGGL(k_chol_offdiag<MAXT>, dim3((unsigned)offdiag_grid(p, c.B)), dim3(OTH), 0, s, a, p);
  return hipGetLastError();
}

}  // namespace tblup
