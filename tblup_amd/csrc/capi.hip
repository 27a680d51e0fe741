// C ABI of libtblup_gpu.so (see include/tblup_gpu.h): context, splits, workspace,
// batched evaluation pipeline and per-kernel-class event timing.
//
// Pipeline per chunk of B individuals (one HIP stream, no host syncs inside):
//   k_indiv_stats -> k_gather -> k_grm -> for J: (k_chol_diag, k_chol_offdiag) -> k_solve
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "capi_ctx.h"
#include "mt_jump.h"

using namespace tblup;

namespace tblup_capi {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

void clear_error() { g_err.clear(); }

int dev_alloc(tblup_ctx* c, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return 0;
  if (b.p) c->mem_in_use -= (int64_t)b.bytes;
  b.release();
  if (bytes == 0) return 0;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) {
    b.p = nullptr;
    return fail(TBLUP_ERR_OOM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
  }
  b.bytes = bytes;
  c->mem_in_use += (int64_t)bytes;
  return 0;
}

void dev_free(tblup_ctx* c, DevBuf& b) {
  if (b.p) c->mem_in_use -= (int64_t)b.bytes;
  b.release();
}

int check_ctx(tblup_ctx* c) {
  if (!c) return fail(TBLUP_ERR_ARG, "null context");
  return 0;
}

}  // namespace tblup_capi

using namespace tblup_capi;

namespace {

hipEvent_t get_event(tblup_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

int drain_events(tblup_ctx* c) {
  for (auto& p : c->pending) {
    HIPCHK(hipEventSynchronize(p.b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
    c->ms[p.cls] += ms;
    c->event_pool.push_back(p.a);
    c->event_pool.push_back(p.b);
  }
  c->pending.clear();
  return 0;
}

// Launch wrapper: records an event pair around the launch when profiling.
template <typename F>
int timed(tblup_ctx* c, hipStream_t s, int cls, double flops, double bytes, F&& launch) {
  hipEvent_t a = nullptr, b = nullptr;
  if (c->profiling) {
    a = get_event(c);
    b = get_event(c);
    if (a) (void)hipEventRecord(a, s);
  }
  hipError_t e = launch();
  if (e != hipSuccess) return fail(TBLUP_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
  if (c->profiling && a && b) {
    (void)hipEventRecord(b, s);
    c->pending.push_back({cls, a, b});
    c->launches[cls] += 1;
    c->flops[cls] += flops;
    c->bytes[cls] += bytes;
  }
  return 0;
}

struct Carve {
  char* base;
  size_t used = 0;
  template <typename T>
  T* take(size_t count) {
    used = round_up((int64_t)used, 256);
    T* p = reinterpret_cast<T*>(base + used);
    used += count * sizeof(T);
    return p;
  }
};

// TBLUP_DBG_SKIP (phase ablation, results wrong when set): honoured by diagnostic builds only
// (tools/ab_build_defs.sh 'diag=-DTBLUP_DIAG_BUILD'); the production library ignores it
inline int dbg_skip(const tblup_ctx* c) {
#ifdef TBLUP_DIAG_BUILD
  return c->dbg_skip;
#else
  (void)c;
  return 0;
#endif
}

// The batched system-tile launch (k_sys_tiles) builds every exact tile up front; int16 counts stay
// exact while the contraction -- n_T animals (SNP form), k SNPs (kernel form: every k <= 64 cblk) --
// is <= KC_MAX_NT (beyond it, and for one-tile systems, the in-tile int8 products of the
// off-diagonal kernel).  Kernel form: TBLUP_DUAL_ST=0 keeps the in-tile products (A/B timing).
bool sys_tiles(const tblup_ctx* c, const EvalDims& d, const SysDims& sd) {
  if (sd.NT < 2) return false;
  if (sd.form == FORM_PRIMAL) return d.nT <= KC_MAX_NT;
  return c->dual_st && sd.cblk * KBLK <= KC_MAX_NT;
}

}  // namespace

// Makespan of greedy list scheduling, in order, of classes {duration, count} on `slots` identical
// slots (slot free times kept as {time: free slots} groups).
static double list_makespan(std::initializer_list<std::pair<double, int64_t>> classes, int64_t slots) {
  std::map<double, int64_t> fr{{0.0, slots}};
  double end = 0.0;
  for (const auto& cl : classes) {
    int64_t n = cl.second;
    while (n > 0) {
      auto it = fr.begin();
      const double t = it->first;
      const int64_t use = std::min(n, it->second);
      if ((it->second -= use) == 0) fr.erase(it);
      fr[t + cl.first] += use;
      end = std::max(end, t + cl.first);
      n -= use;
    }
  }
  return end;
}

OffPlan tblup::off_plan(int64_t B, int NT, int J, bool st, int ahead, int nrs_pol, int64_t slots, int diag_d,
                        int dd_maxj, int diag_e, int64_t ncu) {
  OffPlan p{};
  p.nI = NT - J - 1;
  if (p.nI <= 0) {
    p.nI = 0;
    return p;
  }
  // launch j computes the partial sums of column j + 1's tiles; auto: when the launch's P-units
  // (B x (NT - 2 - j)) fit in AHEAD_SLOTS workgroup slots, i.e. run beside its T-units in one wave
  auto ahead_at = [&](int j) {
#ifdef TBLUP_AB_AHEAD_MASK   // A/B builds only (tools/ab_build_defs.sh): launches ahead by bit j
    const bool on = ahead == 1 || (ahead < 0 && (B * (NT - 2 - j) < slots || ((TBLUP_AB_AHEAD_MASK >> j) & 1)));
#else
    const bool on = ahead == 1 || (ahead < 0 && B * (NT - 2 - j) < slots);
#endif
    return on && j >= 1 && j + 2 <= NT - 1;
  };
  p.nP = ahead_at(J) ? NT - 2 - J : 0;
  p.ahead_cur = (J >= 2 && ahead_at(J - 1)) ? 1 : 0;
  int dt = (J >= 1 && J + 1 < NT) ? 1 : 0;   // diagonal target J + 1 (its partial over L < J)
  // small batches: the D-units in the diagonal launch J (its B workgroups leave 256 - B CUs idle
  // for ~45 us; a D-unit alone on a CU sums J / 2 SYRK terms, so J <= DD_MAX_J keeps it shorter)
  if (dt && (diag_d == 1 || (diag_d < 0 && B > DD_MIN_B && B <= DD_MAX_B && J <= dd_maxj))) {
    p.ndd = 1;
    dt = 0;
  }
  // E-units: column J's GEMM1 term L = Ls0 of its first tiles, on the CUs the diagonal launch J
  // leaves idle (its B diagonal workgroups and D-units take one CU each: 144 KiB of LDS).  One term
  // (29 us alone on a CU, measured) ends inside the ~45 us diagonal launch.  Auto: one per idle CU.
  // The off-diagonal launch dispatches the tiles they started last, so that (the dispatcher filling
  // every CU's first slot, then its second) a CU pairs a whole tile with a shortened one or with a
  // lighter unit class -- an off-diagonal launch of one round lasts as long as its busiest CU.  (In
  // the tiles' plain order, columns covered only in part gained nothing: A/B, profiles/r05_epol_ab.txt,
  // r05_eord_ab.txt -- with the order pop 96 +1.9%, 160 +0.3%, 128 +0.2%.)  2: only whole columns.
  if (J >= 1 && (diag_e == 1 || (diag_e != 0 && ncu > 0))) {
    const int64_t idle = std::max<int64_t>(0, ncu - B * (1 + p.ndd));
    p.ne = diag_e == 1 ? B * p.nI : std::min<int64_t>(B * p.nI, idle);
    if (diag_e == 2 && p.ne < B * p.nI) p.ne = 0;
  }
  p.nrs = 1;
  p.nds = dt;
  // Row slices of the P-units (they need k_sys_tiles' counts: the int8 K is a whole-tile
  // product) and block slices of the D-unit: the pair whose greedy list schedule -- grid order
  // P, D, T on 512 slots (two workgroups per CU), unit work in 2*128^3-flop GEMM units plus a
  // fixed 0.25 -- ends first (ties: fewer units).  T-unit: the GEMM1 terms it still sums (1 after
  // an ahead launch, else J) + 0.5 (GEMM2); P-unit: J / nrs; D-unit: J / 2 / nds.
  // A slicing other than (1, 1) must gain 10%: the model ignores that tiles sharing a CU with
  // tiles (not with the lighter D-units) slow each other down (round 2: D split in two at pop 256
  // measured slower although such a model predicted -90 us).
  const double jt = J, tw = (p.ahead_cur ? 1.0 : jt) + 0.5, c0 = 0.25;
  const int64_t nT = B * p.nI;
  auto span = [&](int nrs, int nds) {
    return list_makespan({{c0 + jt / nrs, B * p.nP * nrs}, {c0 + 0.5 * jt / nds, B * dt * nds}, {c0 + tw, nT}}, 512);
  };
  const bool slice_p = p.nP > 0 && st;
  double best = (nrs_pol > 1 && slice_p) ? 1e300 : 0.9 * span(1, 1);
  for (int nrs : {1, 2, 4}) {
    if (nrs > 1 && !slice_p) break;
    if (nrs_pol > 0 && nrs != nrs_pol && slice_p) continue;
    for (int nds = 1; nds <= (dt ? 2 : 1); ++nds) {
      if (nrs == 1 && nds == 1) continue;
      const double ms = span(nrs, nds);
      if (ms < best) {
        best = ms;
        p.nrs = slice_p ? nrs : 1;
        p.nds = dt * nds;
      }
    }
  }
  p.n_kd = (J == 0 && NT > 2 && !st) ? B * (NT - 2) : 0;
  return p;
}

namespace {

OffPlan plan_of(const tblup_ctx* c, int64_t B, int NT, int J, bool st) {
  return off_plan(B, NT, J, st, c->ahead, c->nrs, AHEAD_SLOTS, c->diag_d, DD_MAX_J, c->diag_e, cu_count());
}

// the chunk's launches hand partial sums of off-diagonal tiles on (P-units or E-units)
bool uses_part(const tblup_ctx* c, int64_t B, int NT, bool st) {
  for (int J = 0; J < NT; ++J) {
    const OffPlan p = plan_of(c, B, NT, J, st);
    if (p.nP > 0 || p.ne > 0) return true;
  }
  return false;
}

// SNP-form solve: the chained kernel up to CHAIN_MAX_B individuals (measured at config 2: solve
// 0.175 -> 0.071 ms at B = 32, 0.184 -> 0.092 at 64, 0.199 -> 0.151 at 128 (round 4's block-row
// units; round 3's tile units: 0.078 / 0.102 / 0.162), even at 192 (round 3), 0.238 -> 0.274 at
// 256, where one workgroup per individual already streams L near the HBM rate).  Round 5's pull
// units (one trait; profiles/r05_solve_pull_ab.txt): 0.061 -> 0.049 ms at 32, 0.079 -> 0.068 at 64,
// 0.128 -> 0.125 at 128, even at 160, 0.188 (k_solve) -> 0.180 at 192, even at 256 -- bound 192
constexpr int64_t CHAIN_MAX_B = 160;
constexpr int64_t CHAIN_PULL_MAX_B = 192;
bool use_chain(const tblup_ctx* c, const SysDims& sd, int64_t B, int64_t nt) {
  const bool pull = c->solve_pull == 1 || (c->solve_pull < 0 && nt == 1);
  return sd.form == FORM_PRIMAL &&
         (c->solve_chain == 1 || (c->solve_chain < 0 && B <= (pull ? CHAIN_PULL_MAX_B : CHAIN_MAX_B)));
}

// Last-term mode: the diagonal tile's last SYRK term computed by the previous launch's tile
// (J, J-1) workgroup (dispatched first) instead of inside the diagonal launch, where one
// workgroup per individual runs it on one CU.  Bit-identical either way.  Measured (config 2,
// A/B): the diagonal launches lose ~8 us each at every B (0.349 -> 0.282 ms per step at B = 32,
// 0.394 -> 0.331 at 256) but the off-diagonal launches gain 42 (B = 32) to 97 us (256): +3.3% at
// 32, +2.0% at 64, -1.3% at 128, -1% at 192 and 256.
// Per diagonal launch (bit J: diagonal J takes its last term from launch J-1), round 5: at
// 64 < B <= 160 only diagonal launches 1 and 3 -- the workgroup traces of round 4 (pop 128,
// profiles/r04_wg_trace_pop128_auto.txt / _lastterm.txt) give, per launch, the off-diagonal launch's
// extra time against the next diagonal launch's saving: J = 0: -1.1 / -9.1 us, J = 2: +0.5 / -5.6;
// every other launch loses.  Late in round 5 (pull-unit solve, non-temporal stores; traces
// profiles/r05i_wg_trace_pop128.txt: tiles (7, 6) and (6, 5) done 20 / 40 us before their launches
// end) diagonal launches 6 and 7 too up to 128: pop 128 +0.8%, 96 +1.5%, 112 even, 160 -0.2%
// (profiles/r05_lt_mask4_ab.txt).
constexpr int64_t LT_MAX_B = 64;
constexpr int64_t LT_LATE_MAX_B = 128;
constexpr int64_t LT_PART_MAX_B = 160;
uint32_t last_term_mask(const tblup_ctx* c, const SysDims& sd, int64_t B) {
  if (sd.NT < 2 || c->last_term == 0) return 0;
  if (c->lt_mask >= 0) return (uint32_t)c->lt_mask;
  if (c->last_term == 1 || B <= LT_MAX_B) return ~1u;   // every diagonal launch J >= 1
  if (B <= LT_LATE_MAX_B) return (1u << 1) | (1u << 3) | (1u << 6) | (1u << 7);
  return B <= LT_PART_MAX_B ? (1u << 1) | (1u << 3) : 0u;
}
bool use_last_term(const tblup_ctx* c, const SysDims& sd, int64_t B) { return last_term_mask(c, sd, B) != 0; }
// bit J of a last-term mask; a kernel-form system can have NT > 32 tile columns (n_T > 4096), and
// there the all-launches mask (~1u, J >= 1) keeps its meaning while a sparse mask names none
inline bool lt_bit(uint32_t m, int J) { return J < 32 ? ((m >> J) & 1u) != 0 : m == ~1u; }

size_t chunk_bytes(const tblup_ctx* c, const EvalDims& d, const SysDims& sd, int64_t B, int64_t sum_k,
                   bool with_ebv) {
  size_t s = 0;
  auto add = [&](size_t x) { s = (size_t)round_up((int64_t)(s + x), 256); };
  add(sd.form == FORM_DUAL ? (size_t)B * sd.prow * dual_pk_row(sd) : 0);   // packed panel (dual only)
  add((size_t)B * sd.prow * 8);                                 // u
  add((size_t)B * SCAL * 8);                                    // scal
  add((size_t)B * l_stride(sd.NT) * 8);                         // L (Lt tiles)
  add((size_t)B * sd.NT * NPACK * BLKD * 8);                    // Dinv (packed X)
  add((size_t)B * d.nt * sd.ns * 8);                            // z
  add((size_t)B * d.nt * sd.ns * 8);                            // w
  add((size_t)B * d.nt * sd.ns * 8);                            // rhs
  add((size_t)B * TBLUP_NSLOT * 36 * 256 * 8);                  // next diagonal tile (minus its last SYRK term)
  add((size_t)B * sd.NT * NPACK * BLKD * 8);                    // diagonal GRM tiles
  add(sys_tiles(c, d, sd) ? (size_t)B * sd.NT * KD_TILE * 2 : 0);  // their int16 counts (k_sys_tiles)
  add(sys_tiles(c, d, sd) ? (size_t)B * sd.NT * (sd.NT - 1) / 2 * KC_TILE * 2 : 0);   // off-diagonal counts
  add(uses_part(c, B, sd.NT, sys_tiles(c, d, sd)) ? (size_t)2 * B * sd.NT * TILE * TILE * 8 : 0);   // partial sums
  if (use_chain(c, sd, B, d.nt)) {                                    // chained solve: beta, c_{J->I}, EBV shares
    add((size_t)B * d.nt * sd.ns * 8);
    add((size_t)B * sd.NT * sd.NT * d.nt * TILE * 8);
    add((size_t)B * sd.NT * d.nt * d.nV * 8);
    add((size_t)B * sd.NT * d.nt * 8);
  }
  add(use_last_term(c, sd, B) ? (size_t)B * NPACK * BLKD * 8 : 0);   // diagonal tiles' last SYRK terms
  add((size_t)B * 8);                                           // fitness
  add(with_ebv ? (size_t)B * d.nt * d.nV * 8 : 0);              // ebv
  add((size_t)sum_k * 8 + (size_t)(B + 1) * 8);                 // idx, off
  return s + 4096;
}

// Form of the per-individual system for a batch.  The SNP-space (primal) form is what
// sklearn's Ridge solves when k <= n_T (_ridge.py _solve_cholesky: X^T X + alpha I); it is
// used when every individual takes the snp branch and it gives no more 128-row tiles than the
// kernel form.  pref: 0 auto, 1 force dual, 2 force primal (snp batches only).
SysDims choose_sys(const tblup_ctx* c, const EvalDims& d, const int64_t* h_off, int64_t B, int branch, int pref);

EvalDims dims_of(const tblup_ctx* c, const Split& sp) {
  EvalDims d;
  d.n = c->n;
  d.P = c->P;
  d.nT = sp.nT;
  d.nV = sp.nV;
  d.nTp = sp.nTp;
  d.nVp = sp.nVp;
  d.nRp = sp.nRp;
  d.NT = (int)(sp.nTp / TILE);
  d.NR = (int)(sp.nRp / TILE);
  d.nt = c->nt;
  return d;
}

SysDims choose_sys(const tblup_ctx* c, const EvalDims& d, const int64_t* h_off, int64_t B, int branch, int pref) {
  int64_t max_k = 1;
  bool all_snp = true;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t k = h_off[b + 1] - h_off[b];
    max_k = std::max(max_k, k);
    const int mode = branch ? branch : (k > c->n ? 1 : 2);   // evaluator.py:257
    if (mode != 2) all_snp = false;
  }
  const int64_t kp = round_up(max_k, TILE);
  // equal tile counts (kp == nTp, e.g. k = 1000 against a 1024-animal CV fold) also take the SNP
  // form: its system tiles come from k_sys_tiles' FP4 counts instead of the in-tile int8 products
  const bool primal = all_snp && pref != 1 && (pref == 2 || kp <= d.nTp);
  SysDims sd;
  if (primal) {
    sd.form = FORM_PRIMAL;
    sd.pad_first = c->pad_first;
    sd.ns = kp;
    sd.prow = kp;
    sd.cblk = d.nRp / KBLK;
  } else {
    sd.form = FORM_DUAL;
    sd.ns = d.nTp;
    sd.prow = d.nRp;
    sd.cblk = round_up(max_k, KBLK) / KBLK;
  }
  sd.NT = (int)(sd.ns / TILE);
  return sd;
}

// Every buffer carved so far lies inside the workspace (checked before the launches that use
// them: a sizing mistake fails the call instead of faulting the GPU)
int ws_check(const tblup_ctx* c, const Carve& cv) {
  if (cv.base >= (char*)c->ws.p && cv.base + cv.used <= (char*)c->ws.p + c->ws.bytes) return 0;
  return fail(TBLUP_ERR_STATE, "internal error: workspace carve of " + std::to_string(cv.used) +
                                   " bytes overruns the " + std::to_string(c->ws.bytes) + "-byte workspace");
}

FoldTab single_fold(const Split& sp, int64_t B) {
  FoldTab ft{};
  ft.bpf = std::max<int64_t>(B, 1);
  ft.nf = 1;
  ft.gpk[0] = (const uint8_t*)sp.gpk.p;
  ft.csT[0] = (const int32_t*)sp.colsumT.p;
  ft.xty[0] = (const double*)sp.xty.p;
  ft.yV[0] = (const double*)sp.yV.p;
  ft.yT[0] = (const double*)sp.yT.p;
  ft.ymu[0] = (const double*)sp.ymu.p;
  return ft;
}

// Enqueue the full pipeline for one chunk whose idx/off already sit in device memory.  ftp: the
// systems' splits when they are not all sp (fold-fused evaluation; sp is then fold 0).
// stop_stage: 0 the whole pipeline; 1 / 2 debug readbacks (K, L); 3 the solve only, through the
// one-workgroup k_solve, on the factor an earlier run_chunk of the same chunk left in the same
// carve (host entries, after that run's chained solve gave up a wait: bit-identical results);
// 4 the whole pipeline with the one-workgroup k_solve instead of the chained solve (a per-call
// choice: the context's policy is not touched).
int run_chunk(tblup_ctx* c, const Split& sp, const EvalDims& d, const SysDims& sd, hipStream_t s,
              const int64_t* d_idx, const int64_t* d_off, const int64_t* h_off, int64_t B, double h2,
              int branch, Carve& cv, double* d_fit, double* d_ebv, int stop_stage, double** K_out,
              double** z_out, const FoldTab* ftp = nullptr) {
  const FoldTab ft = ftp ? *ftp : single_fold(sp, B);
  const bool redo = stop_stage == 3;
  const bool chain = stop_stage != 4 && use_chain(c, sd, B, d.nt);
  c->last_chain_seq = 0;
  double grm_flops = 0.0, gather_bytes = 0.0, stats_bytes = 0.0;
  const double tri = (double)d.nT * (d.nT + 1) / 2.0 + (double)d.nV * d.nT;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t k = h_off[b + 1] - h_off[b];
    grm_flops += 2.0 * (double)k * tri;
    gather_bytes += 0.5 * (double)k * (double)(d.nT + d.nV);   // 2-bit split rows in, 2-bit rows out
    stats_bytes += 16.0 * (double)k;
  }
  const int64_t pk_row = (sd.form == FORM_DUAL) ? dual_pk_row(sd) : 0;
  const int64_t pstride = sd.prow * pk_row;
  uint8_t* panel = cv.take<uint8_t>((size_t)B * pstride);
  double* u = cv.take<double>((size_t)B * sd.prow);
  double* scal = cv.take<double>((size_t)B * SCAL);
  double* L = cv.take<double>((size_t)B * l_stride(sd.NT));
  double* Dinv = cv.take<double>((size_t)B * sd.NT * NPACK * BLKD);
  double* z = cv.take<double>((size_t)B * d.nt * sd.ns);
  double* wv = cv.take<double>((size_t)B * d.nt * sd.ns);
  double* rhs = cv.take<double>((size_t)B * d.nt * sd.ns);
  double* Sp = cv.take<double>((size_t)B * TBLUP_NSLOT * 36 * 256);
  // (kernel-form fold chunks read their counts from the shared A_R A_R^T instead)
  const bool use_st = sys_tiles(c, d, sd) && stop_stage != 1 && !ft.gsh;
  // diagonal system tiles: fp64 K_JJ + lambda I (with k_sys_tiles: J < 2 only, the diagonal
  // kernel's direct reads) and, with k_sys_tiles, the exact int16 counts of J >= 2 (the D-units')
  double* Kdg = cv.take<double>((size_t)B * sd.NT * NPACK * BLKD);
  int16_t* kdb = use_st ? cv.take<int16_t>((size_t)B * sd.NT * KD_TILE) : nullptr;
  int16_t* kcb = use_st ? cv.take<int16_t>((size_t)B * sd.NT * (sd.NT - 1) / 2 * KC_TILE) : nullptr;
  double* Pp = uses_part(c, B, sd.NT, sys_tiles(c, d, sd)) ? cv.take<double>((size_t)2 * B * sd.NT * TILE * TILE) : nullptr;
  double* Qb = use_last_term(c, sd, B) ? cv.take<double>((size_t)B * NPACK * BLKD) : nullptr;
  const bool fold_share = use_st && sd.form == FORM_PRIMAL && ft.nf > 1 && ft.share;   // k_sys_tiles_folds
  if (int rc = ws_check(c, cv)) return rc;
  std::vector<OffPlan> plan(sd.NT);
  for (int J = 0; J < sd.NT; ++J) {
    plan[J] = plan_of(c, B, sd.NT, J, use_st);
    if (ft.gsh) plan[J].ne = 0;   // the diagonal kernel's E-units do not read shared fold counts
  }
  const int32_t* csA = (const int32_t*)c->colsum_all.p;
  // the scalars formed after k_sys_tiles_st / k_sys_tiles_folds, in their K_JJ epilogue launch (one
  // launch less; neither reads a scalar), else by k_indiv_stats first
  CholLaunch probe{};
  probe.B = B;
  probe.sd = sd;
  probe.sys_st = c->sys_st;
  const bool fuse_stats = !redo && use_st && sd.form == FORM_PRIMAL && (fold_share || sys_tiles_grid(probe) > 0);
  const StatsFuse sf{csA, d.n, d.nT, branch, h2, (int32_t*)c->status.p + ST_INDEX, scal, u, rhs};
  int rc = 0;
  if (!redo && !fuse_stats)
    rc = timed(c, s, KC_STATS, 2.0 * (double)h_off[B], stats_bytes, [&] {
      return launch_indiv_stats(d_idx, d_off, B, ft, csA, d, sd, branch, h2, scal, u, rhs,
                                (int32_t*)c->status.p + ST_INDEX, s);
    });
  if (rc) return rc;
  if (sd.form == FORM_DUAL && !redo) {
    // primal rows are read in place from the split matrix: no gather
    rc = timed(c, s, KC_GATHER, 0.0, gather_bytes, [&] {
      return launch_gather(ft, d_idx, d_off, pstride, B, csA, scal, d, pk_row, panel, u, s);
    });
    if (rc) return rc;
  }
  if (z_out) *z_out = z;
  if (stop_stage == 1) {
    // parity readback only: the full K_{R,T} block of the unified form (k_grm); the
    // production path never materialises K (the Cholesky kernels rebuild each tile)
    double* K = cv.take<double>((size_t)B * d.nRp * d.nTp);
    if (int rc2 = ws_check(c, cv)) return rc2;
    if (K_out) *K_out = K;
    const double kbytes = (double)B * ((double)d.nT * d.nT / 2.0 + (double)d.nV * d.nT) * 8.0;
    return timed(c, s, KC_GRM, grm_flops, kbytes + gather_bytes / 2.0,
                 [&] { return launch_grm(panel, pstride, pk_row, d_off, u, scal, d, B, K, s); });
  }
  if (K_out) *K_out = L;
  CholLaunch cl{d, sd, B, L, Dinv, z, wv, rhs, Sp, Kdg, (const double*)sp.yT.p, panel, pstride, d_off, d_idx,
                d.nRp, d.nRp / 4, ft, u, scal, dbg_skip(c) | (stop_stage == 2 ? FLAG_WRITE_LJJ : 0), nullptr, kcb,
                Pp, Qb};
  cl.kd = kdb;
  cl.sys_st = c->sys_st;
  cl.padskip = (sd.form == FORM_PRIMAL && sd.pad_first) ? 1 : 0;
  const double T3 = (double)TILE * TILE * TILE;
  // profiling only: room for one record per Cholesky workgroup of this chunk
  uint64_t* wgt = nullptr;
  if (c->wg_trace && !redo) {
    int64_t nwg = 0;
    for (int J = 0; J < sd.NT; ++J) nwg += B * (1 + plan[J].ndd) + plan[J].ne + DTR_RECS + offdiag_grid(plan[J], B);
    if (use_st) nwg += B * sd.NT * (sd.NT + 1) / 2;
    if (chain) nwg += B * sd.NT;   // chained solve units
    if (int rc = dev_alloc(c, c->wgt, (size_t)nwg * WGT_REC * 8)) return rc;
    HIPCHK(hipMemsetAsync(c->wgt.p, 0, (size_t)nwg * WGT_REC * 8, s));
    wgt = (uint64_t*)c->wgt.p;
    c->wgt_used = 0;
  }
  const double kbar = B > 0 ? (double)h_off[B] / (double)B : 0.0;
  const double cbar = (sd.form == FORM_PRIMAL) ? (double)d.nT : kbar;   // contraction length
  if (redo) {
  } else if (use_st) {
    // every system tile (I >= J) in one int8 launch: int ops 2 x 128^2 x n_T per tile
    const double ntri = (double)sd.NT * (sd.NT + 1) / 2.0;
    const double fg = (double)B * ntri * 2.0 * 128.0 * 128.0 * cbar;
    const double nd8 = std::min(sd.NT, 2);   // diagonal tiles stored as fp64 (the rest as int16 counts)
    const double bg = (double)B * ((ntri - sd.NT) * KC_TILE * 2.0 + (sd.NT - nd8) * KD_TILE * 2.0 + nd8 * KD_TILE * 8.0);
    if (wgt) {
      cl.wgt = wgt + c->wgt_used * WGT_REC;
      const int64_t sg = fold_share ? -(B * sd.NT * (sd.NT + 1) / 2) : sys_tiles_grid(cl);
      c->wgt_used += sg > 0 ? sg : -sg;
    }
    cl.stats = fuse_stats ? &sf : nullptr;
    rc = timed(c, s, KC_GRM, fg, bg + (fuse_stats ? stats_bytes : 0.0), [&] {
      return fold_share ? launch_sys_tiles_folds(cl, s) : launch_sys_tiles(cl, s);
    });
    cl.stats = nullptr;
    if (rc) return rc;
  } else {
    if (ft.gsh) {
      // kernel-form folds: every individual's A_R A_R^T once (int ops 2 x nRp^2 x k / 2 + the diagonal tiles)
      const double NR = (double)(d.nRp / TILE);
      const double fgs = (double)ft.bpf * NR * (NR + 1) / 2.0 * 2.0 * 128.0 * 128.0 * kbar;
      rc = timed(c, s, KC_GRM, fgs, (double)ft.bpf * d.nRp * d.nRp * 4.0, [&] { return launch_gshare(cl, s); });
      if (rc) return rc;
    }
    // int ops of the diagonal GRM tiles J < 2 (J >= 2 run inside the column-0 off-diagonal launch)
    const double nJ = (double)std::min(sd.NT, 2);
    const double fg = (double)B * nJ * 128.0 * 129.0 * cbar;
    rc = timed(c, s, KC_GRM, fg, (double)B * nJ * 36 * 256 * 8.0, [&] { return launch_diag_grm(cl, s); });
    if (rc) return rc;
  }
  // Column loop.  (A look-ahead schedule -- tile (J+1, J) and diagonal tile J+1 on a
  // high-priority stream beside the rest of column J -- measured slower on MI355X: the
  // chip is already full during the off-diagonal launches, and sharing CUs slows the
  // critical path more than it hides.)
  const double Bd = (double)B;
  const uint32_t ltm = last_term_mask(c, sd, B);
  for (int J = 0; !redo && J < sd.NT; ++J) {
    const double jt = (double)J;
    const OffPlan& p = plan[J];
    // algorithmic fp64 work: the L = J-1 SYRK term of the diagonal tile, potrf + trtri,
    // forward-substitution GEMV (the exact system tiles are counted under KC_GRM)
    const bool qd = Qb && lt_bit(ltm, J), qo = Qb && lt_bit(ltm, J + 1);
    const double lt_d = qd ? 0.0 : std::min(jt, 1.0);   // the last SYRK term's share of this launch
    // (+ the D-units when they run in this launch: 128^3 per L < J, as in the off-diagonal launch)
    // (+ the E-units: one 2*128^3 GEMM1 term each, moved out of launch J's T-units)
    const double fd = Bd * (T3 * lt_d + 2.0 * T3 / 3.0 + 2.0 * TILE * TILE * jt) + (p.ndd ? Bd * T3 * jt : 0.0) +
                      (double)p.ne * 2.0 * T3;
    const double bd = Bd * (TILE * TILE * lt_d * 8.0 + 2.0 * TILE * TILE * 8.0) +
                      (p.ndd ? 2.0 * Bd * TILE * TILE * jt * 8.0 : 0.0) + (double)p.ne * 3.0 * TILE * TILE * 8.0;
    if (wgt) {
      cl.wgt = wgt + c->wgt_used * WGT_REC;
      c->wgt_used += B * (1 + p.ndd) + p.ne + DTR_RECS;
    }
    cl.q = qd ? Qb : nullptr;   // diagonal J: its last term from launch J-1
    rc = timed(c, s, KC_DIAG, fd, bd, [&] { return launch_chol_diag(cl, J, p, s); });
    cl.q = qo ? Qb : nullptr;   // off-diagonal J: the last term of diagonal J+1
    if (rc) return rc;
    if (p.nI > 0) {
      // T-units: GEMM1 over the L not summed ahead (2*128^3 each) + the triangular solve 128^3;
      // P-units: 2*128^3 per L < J; D-unit: 128^3 per L < J (lower half); the fused int8 GRM
      // tiles' int-ops are excluded
      const double lt = p.ahead_cur ? 1.0 : jt;
      const double fo = Bd * p.nI * (2.0 * T3 * lt + T3) + Bd * p.nP * 2.0 * T3 * jt + (p.nds ? Bd * T3 * jt : 0.0) +
                        (qo ? Bd * T3 : 0.0) - (double)p.ne * 2.0 * T3;
      const double bo = Bd * p.nI * (TILE * TILE * lt * 8.0 + TILE * TILE * 8.0) +
                        Bd * p.nP * (2.0 * TILE * TILE * jt * 8.0 + TILE * TILE * 8.0) +
                        (p.nds ? 2.0 * Bd * TILE * TILE * jt * 8.0 : 0.0);
      if (wgt) {
        cl.wgt = wgt + c->wgt_used * WGT_REC;
        c->wgt_used += offdiag_grid(p, B);
      }
      rc = timed(c, s, KC_OFFDIAG, fo, bo, [&] { return launch_chol_offdiag(cl, J, p, s); });
      if (rc) return rc;
    }
  }
  if (stop_stage == 2) return 0;
  const double fs = (double)B * (2.0 * (double)sd.ns * sd.ns / 2.0 + 2.0 * kbar * (double)(d.nT + d.nV) + 10.0 * d.nV);
  const double bs = (double)B * (((double)sd.ns * sd.ns / 2.0 + (double)sd.NT * TILE * TILE) * 8.0 +
                                 kbar * (double)(d.nT + d.nV));
  SolveChain ch{};
  const SolveChain* chp = nullptr;
  if (!redo && chain) {
    const size_t fbytes = ((size_t)B * chain_flags(sd.NT) + CHAIN_ERR_RING + 1) * 4;
    if (c->chain.bytes < fbytes || c->chain_seq >= INT32_MAX - 1) {
      HIPCHK(hipStreamSynchronize(s));   // the flags may still be read by an earlier chained solve
      if (int rc2 = dev_alloc(c, c->chain, fbytes)) return rc2;
      HIPCHK(hipMemsetAsync(c->chain.p, 0, c->chain.bytes, s));
      c->chain_seq = 0;
    }
    ch.flags = (int32_t*)c->chain.p;
    int32_t* ring = ch.flags + (c->chain.bytes / 4 - CHAIN_ERR_RING - 1);
    ch.beta = cv.take<double>((size_t)B * d.nt * sd.ns);
    ch.cpart = cv.take<double>((size_t)B * sd.NT * sd.NT * d.nt * TILE);
    ch.epart = cv.take<double>((size_t)B * sd.NT * d.nt * d.nV);
    ch.mbpart = cv.take<double>((size_t)B * sd.NT * d.nt);
    if (int rc2 = ws_check(c, cv)) return rc2;
    ch.seq = ++c->chain_seq;
    ch.err = ring + ch.seq % CHAIN_ERR_RING;
    // host entries recover from their ring slot (chain_expired); device entries raise the status word
    ch.expired = c->host_entry ? ring + CHAIN_ERR_RING : (int32_t*)c->status.p + ST_SOLVE;
    c->last_chain_seq = ch.seq;
    ch.mode = c->chain_sync;
    // pull units for one trait (several traits: their registers spill at two units per CU)
    ch.pull = c->solve_pull == 1 || (c->solve_pull < 0 && d.nt == 1);
    ch.spin_max = CHAIN_SPIN_MAX;
    ch.delay = 0;
    if (c->chain_dbg_shots > 0) {
      --c->chain_dbg_shots;
      ch.spin_max = c->chain_dbg_spin;
      ch.delay = c->chain_dbg_delay;
    }
    chp = &ch;
    if (wgt) {
      cl.wgt = wgt + c->wgt_used * WGT_REC;
      c->wgt_used += B * sd.NT;
    }
  }
  rc = timed(c, s, KC_SOLVE, fs, bs, [&] { return launch_solve(cl, chp, d_fit, d_ebv, s); });
  return rc;
}

// Host entries, after the chunk's stream synchronisation: whether the chained solve `seq` (0: none)
// gave up a wait.  Its ring slot holds seq exactly then (slots of other calls hold their own seqs).
int chain_expired(tblup_ctx* c, int32_t seq, bool* out) {
  *out = false;
  if (seq <= 0 || !c->chain.p) return 0;
  const int32_t* ring = (const int32_t*)c->chain.p + (c->chain.bytes / 4 - CHAIN_ERR_RING - 1);
  int32_t v = 0;
  HIPCHK(hipMemcpyAsync(&v, ring + seq % CHAIN_ERR_RING, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *out = v == seq;
  return 0;
}

// Marks a synchronous entry for its duration: its chained solves write their expiry to the ring
// only (the entry re-runs the affected chunk's solve through k_solve and counts it), not to the
// context's sticky status word that the device entries' callers read.
struct HostEntry {
  tblup_ctx* c;
  explicit HostEntry(tblup_ctx* cc) : c(cc) { c->host_entry = true; }
  ~HostEntry() { c->host_entry = false; }
};

Split* find_split(tblup_ctx* c, int id) {
  auto it = c->splits.find(id);
  return it == c->splits.end() ? nullptr : it->second.get();
}

}  // namespace

extern "C" {

const char* tblup_last_error(void) { return tblup_capi::g_err.c_str(); }

const char* tblup_version(void) { return "tblup_gpu 0.1.0 (gfx950)"; }

int tblup_device_count(int* out) {
  if (!out) return fail(TBLUP_ERR_ARG, "null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *out = n;
  return 0;
}

int tblup_ctx_create(const int8_t* geno, int64_t n, int64_t P, int layout, const double* pheno, int device,
                     tblup_ctx** out) {
  g_err.clear();
  if (!out) return fail(TBLUP_ERR_ARG, "null out_ctx");
  *out = nullptr;
  const bool panel = geno || pheno || n || P;   // (NULL, 0, 0, NULL): DE / decode-only context
  if (panel && (!geno || !pheno || n < 2 || P < 1)) return fail(TBLUP_ERR_ARG, "bad genotype/phenotype arguments");
  if (layout != TBLUP_LAYOUT_ANIMAL_MAJOR && layout != TBLUP_LAYOUT_SNP_MAJOR) return fail(TBLUP_ERR_ARG, "bad layout");
  if (n > (int64_t)1 << 30) return fail(TBLUP_ERR_ARG, "too many animals");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(TBLUP_ERR_HIP, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(TBLUP_ERR_ARG, "device id out of range");
  HIPCHK(hipSetDevice(device));
  std::unique_ptr<tblup_ctx> c(new tblup_ctx());
  c->device = device;
  c->n = n;
  c->P = P;
  if (panel) c->pheno.assign(pheno, pheno + n);
  c->nt = 1;
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  const char* env = getenv("TBLUP_WORKSPACE_MB");
  c->budget = (size_t)(env ? atoll(env) : 32768) << 20;
#ifdef TBLUP_DIAG_BUILD
  const char* dbg = getenv("TBLUP_DBG_SKIP");
  c->dbg_skip = dbg ? atoi(dbg) : 0;
#endif
  const char* wt = getenv("TBLUP_WG_TRACE");
  c->wg_trace = wt && atoi(wt) != 0;
  const char* fp = getenv("TBLUP_FORM");
  c->form_pref = fp ? std::max(0, std::min(2, atoi(fp))) : 0;
  if (const char* e = getenv("TBLUP_AHEAD")) c->ahead = std::max(-1, std::min(1, atoi(e)));
  if (const char* e = getenv("TBLUP_SOLVE_CHAIN")) c->solve_chain = std::max(-1, std::min(1, atoi(e)));
  if (const char* e = getenv("TBLUP_SOLVE_PULL")) c->solve_pull = std::max(-1, std::min(1, atoi(e)));
  if (const char* e = getenv("TBLUP_CHAIN_SYNC")) c->chain_sync = atoi(e);
  if (const char* e = getenv("TBLUP_LAST_TERM")) c->last_term = std::max(-1, std::min(1, atoi(e)));
  if (const char* e = getenv("TBLUP_LT_MASK")) c->lt_mask = (int)strtol(e, nullptr, 0);
  if (const char* e = getenv("TBLUP_FOLD_FUSE")) c->fold_fuse = atoi(e) != 0;
  if (const char* e = getenv("TBLUP_FOLD_SHARE")) c->fold_share = atoi(e) != 0;
  if (const char* e = getenv("TBLUP_SYS_ST")) c->sys_st = std::max(-1, std::min(1, atoi(e)));
  if (const char* e = getenv("TBLUP_FOLD_GSHARE")) c->fold_gshare = atoi(e) != 0;
  if (const char* e = getenv("TBLUP_DUAL_ST")) c->dual_st = atoi(e) != 0;
  if (const char* e = getenv("TBLUP_DIAG_D")) c->diag_d = std::max(-1, std::min(1, atoi(e)));
  if (const char* e = getenv("TBLUP_DIAG_E")) c->diag_e = std::max(-1, std::min(2, atoi(e)));
  if (const char* e = getenv("TBLUP_PAD_FIRST")) c->pad_first = atoi(e) != 0;
  if (const char* e = getenv("TBLUP_NRS")) c->nrs = (atoi(e) == 1 || atoi(e) == 2 || atoi(e) == 4) ? atoi(e) : 0;
  if (const char* e = getenv("TBLUP_CHAIN_DEBUG")) {
    int sp = 0, dl = 0, sh = 0;
    if (sscanf(e, "%d,%d,%d", &sp, &dl, &sh) == 3 && sp > 0 && dl >= 0 && sh > 0) {
      c->chain_dbg_spin = sp;
      c->chain_dbg_delay = dl;
      c->chain_dbg_shots = sh;
    }
  }
  if (!panel) {
    *out = c.release();
    return 0;
  }
  const size_t gbytes = (size_t)n * (size_t)P;
  if (int rc = dev_alloc(c.get(), c->geno_sm, gbytes)) return rc;
  if (int rc = dev_alloc(c.get(), c->colsum_all, (size_t)P * 4)) return rc;
  if (int rc = dev_alloc(c.get(), c->status, ST_WORDS * 4)) return rc;
  HIPCHK(hipMemsetAsync(c->status.p, 0, ST_WORDS * 4, c->stream));
  if (layout == TBLUP_LAYOUT_SNP_MAJOR) {
    HIPCHK(hipMemcpyAsync(c->geno_sm.p, geno, gbytes, hipMemcpyHostToDevice, c->stream));
  } else {
    if (int rc = dev_alloc(c.get(), c->scratch, gbytes)) return rc;
    HIPCHK(hipMemcpyAsync(c->scratch.p, geno, gbytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_transpose_geno((const int8_t*)c->scratch.p, (int8_t*)c->geno_sm.p, n, P, c->stream));
  }
  HIPCHK(launch_colsum_all((const int8_t*)c->geno_sm.p, (int32_t*)c->colsum_all.p, n, P, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  dev_free(c.get(), c->scratch);
  *out = c.release();
  return 0;
}

int tblup_ctx_destroy(tblup_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& p : c->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  for (auto& kv : c->splits) {
    kv.second->gpk.release();
    kv.second->colsumT.release();
    kv.second->xty.release();
    kv.second->yT.release();
    kv.second->yV.release();
    kv.second->ymu.release();
  }
  c->geno_sm.release();
  c->colsum_all.release();
  c->status.release();
  c->scratch.release();
  c->ws.release();
  c->wgt.release();
  c->chain.release();
  c->dec_keys.release();
  c->dec_idx.release();
  c->de_polys.release();
  c->de_small.release();
  c->de_par.release();
  c->de_chi.release();
  if (c->de_ev) (void)hipEventDestroy(c->de_ev);
  if (c->de_host) (void)hipHostFree(c->de_host);
  if (c->de_stage) (void)hipHostFree(c->de_stage);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int tblup_set_split(tblup_ctx* c, int split_id, const int64_t* train, int64_t nT, const int64_t* valid,
                    int64_t nV) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (c->n == 0) return fail(TBLUP_ERR_STATE, "context has no genotype panel (DE / decode-only context)");
  if (!train || !valid || nT < 1 || nV < 2) return fail(TBLUP_ERR_ARG, "split needs >= 1 train and >= 2 valid rows");
  for (int64_t i = 0; i < nT; ++i)
    if (train[i] < 0 || train[i] >= c->n) return fail(TBLUP_ERR_ARG, "train index out of range");
  for (int64_t i = 0; i < nV; ++i)
    if (valid[i] < 0 || valid[i] >= c->n) return fail(TBLUP_ERR_ARG, "valid index out of range");
  HIPCHK(hipSetDevice(c->device));
  auto sp = std::make_unique<Split>();
  sp->nT = nT;
  sp->nV = nV;
  sp->nTp = round_up(nT, TILE);
  sp->nVp = round_up(nV, TILE);
  sp->nRp = sp->nTp + sp->nVp;
  sp->rows.assign(train, train + nT);
  sp->rows.insert(sp->rows.end(), valid, valid + nV);
  sp->train.assign(train, train + nT);
  sp->valid.assign(valid, valid + nV);
  std::sort(sp->rows.begin(), sp->rows.end());
  std::vector<int32_t> rowmap(sp->nRp, -1);
  for (int64_t i = 0; i < nT; ++i) rowmap[i] = (int32_t)train[i];
  for (int64_t i = 0; i < nV; ++i) rowmap[sp->nTp + i] = (int32_t)valid[i];
  const int nt = c->nt;
  std::vector<double> yT((size_t)nt * sp->nTp, 0.0), yV((size_t)nt * nV);
  sp->meanyT.assign(nt, 0.0);
  for (int t = 0; t < nt; ++t) {
    // mean(y_T) as numpy computes it for Ridge's y_offset (pairwise summation differs only in rounding)
    long double acc = 0.0L;
    for (int64_t i = 0; i < nT; ++i) {
      const double y = c->pheno[train[i] * nt + t];
      yT[t * sp->nTp + i] = y;
      acc += y;
    }
    sp->meanyT[t] = (double)(acc / (long double)nT);
    for (int64_t i = 0; i < nV; ++i) yV[t * nV + i] = c->pheno[valid[i] * nt + t];
  }
  if (int rc = dev_alloc(c, sp->gpk, (size_t)(c->P + 1) * (sp->nRp / 4) + 64)) return rc;
  if (int rc = dev_alloc(c, sp->colsumT, (size_t)c->P * 4)) return rc;
  if (int rc = dev_alloc(c, sp->xty, (size_t)nt * c->P * 8)) return rc;
  if (int rc = dev_alloc(c, sp->yT, yT.size() * 8)) return rc;
  if (int rc = dev_alloc(c, sp->yV, yV.size() * 8)) return rc;
  if (int rc = dev_alloc(c, sp->ymu, (size_t)nt * 8)) return rc;
  DevBuf rm;
  if (int rc = dev_alloc(c, rm, rowmap.size() * 4)) return rc;
  HIPCHK(hipMemcpyAsync(rm.p, rowmap.data(), rowmap.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(sp->yT.p, yT.data(), yT.size() * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(sp->yV.p, yV.data(), yV.size() * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(sp->ymu.p, sp->meanyT.data(), (size_t)nt * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(launch_build_split((const int8_t*)c->geno_sm.p, c->n, c->P, (const int32_t*)rm.p, sp->nRp, nT,
                            (const double*)sp->yT.p, (const double*)sp->ymu.p, nt, (uint8_t*)sp->gpk.p, (int32_t*)sp->colsumT.p, (double*)sp->xty.p, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  dev_free(c, rm);
  auto it = c->splits.find(split_id);
  if (it != c->splits.end()) {
  dev_free(c, it->second->gpk);
    dev_free(c, it->second->colsumT);
    dev_free(c, it->second->xty);
    dev_free(c, it->second->yT);
    dev_free(c, it->second->yV);
    dev_free(c, it->second->ymu);
  }
  c->splits[split_id] = std::move(sp);
  return 0;
}

int tblup_set_traits(tblup_ctx* c, const double* pheno, int64_t n_traits) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (c->n == 0) return fail(TBLUP_ERR_STATE, "context has no genotype panel (DE / decode-only context)");
  if (!pheno || n_traits < 1 || n_traits > MAXT) return fail(TBLUP_ERR_ARG, "need 1 <= n_traits <= 4 and phenotypes");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (auto& kv : c->splits) {   // splits hold per-trait phenotype vectors
    dev_free(c, kv.second->gpk);
    dev_free(c, kv.second->colsumT);
    dev_free(c, kv.second->xty);
    dev_free(c, kv.second->yT);
    dev_free(c, kv.second->yV);
    dev_free(c, kv.second->ymu);
  }
  c->splits.clear();
  c->nt = (int)n_traits;
  c->pheno.assign(pheno, pheno + c->n * n_traits);
  return 0;
}

int tblup_get_traits(tblup_ctx* c, int64_t* n_traits) {
  if (int rc = check_ctx(c)) return rc;
  if (n_traits) *n_traits = c->nt;
  return 0;
}

int tblup_drop_split(tblup_ctx* c, int split_id) {
  if (int rc = check_ctx(c)) return rc;
  auto it = c->splits.find(split_id);
  if (it == c->splits.end()) return fail(TBLUP_ERR_ARG, "unknown split id");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  dev_free(c, it->second->gpk);
  dev_free(c, it->second->colsumT);
  dev_free(c, it->second->xty);
  dev_free(c, it->second->yT);
  dev_free(c, it->second->yV);
  dev_free(c, it->second->ymu);
  c->splits.erase(it);
  return 0;
}

// numpy's fancy-index bound (the reference's data[:, indices], evaluator.py:275/298):
// -P <= i < P is valid (negatives wrap, on the device); anything else is numpy's IndexError.
static int check_indices(const tblup_ctx* c, const int64_t* idx, int64_t count) {
  for (int64_t i = 0; i < count; ++i)
    if (idx[i] < -c->P || idx[i] >= c->P)
      return fail(TBLUP_ERR_INDEX, "index " + std::to_string(idx[i]) + " is out of bounds for axis 1 with size " +
                                       std::to_string(c->P));
  return 0;
}

static int validate_batch(tblup_ctx* c, int branch, double h2, const int64_t* offsets, int64_t batch) {
  if (branch < 0 || branch > 2) return fail(TBLUP_ERR_ARG, "bad branch");
  if (!(h2 > 0.0) || !(h2 <= 1.0)) return fail(TBLUP_ERR_ARG, "h2 must be in (0, 1]");
  if (batch < 0) return fail(TBLUP_ERR_ARG, "negative batch");
  if (batch > 0 && !offsets) return fail(TBLUP_ERR_ARG, "null offsets");
  for (int64_t b = 0; b < batch; ++b)
    if (offsets[b + 1] - offsets[b] < 1) return fail(TBLUP_ERR_ARG, "every individual needs k >= 1 indices");
  if (batch > 0 && offsets[0] != 0) return fail(TBLUP_ERR_ARG, "offsets[0] must be 0");
  (void)c;
  return 0;
}

int tblup_eval_batch(tblup_ctx* c, int split_id, const int64_t* idx, const int64_t* offsets, int64_t batch,
                     double h2, int branch, double* fitness, double* ebv) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (int rc = validate_batch(c, branch, h2, offsets, batch)) return rc;
  if (batch == 0) return 0;
  if (!idx || !fitness) return fail(TBLUP_ERR_ARG, "null idx/fitness");
  Split* sp = find_split(c, split_id);
  if (!sp) return fail(TBLUP_ERR_ARG, "unknown split id");
  if (int rc = check_indices(c, idx, offsets[batch])) return rc;
  HIPCHK(hipSetDevice(c->device));
  HostEntry he(c);
  const EvalDims d = dims_of(c, *sp);
  const bool want_ebv = ebv != nullptr;
  const SysDims sd = choose_sys(c, d, offsets, batch, branch, c->form_pref);
  int64_t b0 = 0;
  while (b0 < batch) {
    // grow the chunk while it fits the workspace budget
    int64_t b1 = b0, sum_k = 0;
    while (b1 < batch) {
      const int64_t k = offsets[b1 + 1] - offsets[b1];
      if (b1 > b0 && chunk_bytes(c, d, sd, b1 + 1 - b0, sum_k + k, want_ebv) > c->budget) break;
      if (b1 - b0 >= 65535) break;
      sum_k += k;
      ++b1;
    }
    const int64_t B = b1 - b0;
    const size_t need = chunk_bytes(c, d, sd, B, sum_k, want_ebv);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (int rc = dev_alloc(c, c->ws, need)) return rc;
    Carve cv{(char*)c->ws.p};
    int64_t* d_idx = cv.take<int64_t>((size_t)sum_k);
    int64_t* d_off = cv.take<int64_t>((size_t)B + 1);
    double* d_fit = cv.take<double>((size_t)B);
    double* d_ebv = want_ebv ? cv.take<double>((size_t)B * d.nt * d.nV) : nullptr;
    std::vector<int64_t> hoff(B + 1);
    for (int64_t b = 0; b <= B; ++b) hoff[b] = offsets[b0 + b] - offsets[b0];
    HIPCHK(hipMemcpyAsync(d_idx, idx + offsets[b0], (size_t)sum_k * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_off, hoff.data(), (size_t)(B + 1) * 8, hipMemcpyHostToDevice, c->stream));
    const Carve cv0 = cv;
    for (int pass = 0;; ++pass) {
      // pass 1: the chained solve of pass 0 gave up a wait -- the same factor, solved by k_solve
      Carve cvp = cv0;
      if (int rc = run_chunk(c, *sp, d, sd, c->stream, d_idx, d_off, hoff.data(), B, h2, branch, cvp, d_fit, d_ebv,
                             pass ? 3 : 0, nullptr, nullptr))
        return rc;
      const int32_t seq = c->last_chain_seq;
      HIPCHK(hipMemcpyAsync(fitness + b0, d_fit, (size_t)B * 8, hipMemcpyDeviceToHost, c->stream));
      if (want_ebv)
        HIPCHK(hipMemcpyAsync(ebv + b0 * d.nt * d.nV, d_ebv, (size_t)B * d.nt * d.nV * 8, hipMemcpyDeviceToHost,
                              c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      bool expired = false;
      if (int rc = chain_expired(c, seq, &expired)) return rc;
      if (!expired) break;
      ++c->chain_recoveries;
    }
    b0 = b1;
  }
  if (c->profiling) return drain_events(c);
  return 0;
}

int tblup_eval_batch_device(tblup_ctx* c, int split_id, const int64_t* d_idx, const int64_t* d_offsets,
                            const int64_t* h_offsets, int64_t batch, double h2, int branch, double* d_fitness,
                            double* d_ebv, void* stream) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (int rc = validate_batch(c, branch, h2, h_offsets, batch)) return rc;
  if (batch == 0) return 0;
  if (!d_idx || !d_offsets || !d_fitness) return fail(TBLUP_ERR_ARG, "null device pointers");
  if (batch > 65535) return fail(TBLUP_ERR_ARG, "device batch limited to 65535 individuals per call");
  Split* sp = find_split(c, split_id);
  if (!sp) return fail(TBLUP_ERR_ARG, "unknown split id");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  const EvalDims d = dims_of(c, *sp);
  const SysDims sd = choose_sys(c, d, h_offsets, batch, branch, c->form_pref);
  const size_t need = chunk_bytes(c, d, sd, batch, 0, false);
  if (need > c->ws.bytes) {
    // the workspace may still be in use by earlier work on either stream
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (int rc = dev_alloc(c, c->ws, need)) return rc;
  }
  Carve cv{(char*)c->ws.p};
  return run_chunk(c, *sp, d, sd, s, d_idx, d_offsets, h_offsets, batch, h2, branch, cv, d_fitness, d_ebv, 0, nullptr,
                   nullptr);
}

// IntraGCV's k folds (evaluator.py:509-537) or any set of splits: every individual against every
// split in one call, one host round trip for the whole set.  Fold-fused (the default whenever
// the splits have equal dimensions and the batch takes the SNP form with k_sys_tiles): the
// F x B systems (s = f * B + b: individual b against split f) run as ONE batch through one
// launch sequence -- 18 launches instead of 18 F, each filling the chip F times over, the
// system's split picked per workgroup from the FoldTab.  Otherwise the folds' batches run back to
// back on one stream, reusing one workspace in stream order.  Results are bit-identical either
// way (every system's arithmetic is independent of the batch it runs in).

// Fused layout of a chunk: the F splits of equal dimensions in the SNP form with system tiles
// (otherwise 0).  sd: the common system shape.
static bool fold_fusable(const tblup_ctx* c, const std::vector<Split*>& sps, const int64_t* h_off, int64_t B,
                         int branch, SysDims& sd) {
  const int64_t F = (int64_t)sps.size();
  if (!c->fold_fuse || F < 2 || F > MAXF || F * B > 65535 || B < 1) return false;
  for (const Split* sp : sps)
    if (sp->nT != sps[0]->nT || sp->nV != sps[0]->nV || sp->nTp != sps[0]->nTp || sp->nRp != sps[0]->nRp) return false;
  const EvalDims d = dims_of(c, *sps[0]);
  sd = choose_sys(c, d, h_off, B, branch, c->form_pref);
  return true;   // either form: every system reads its own split through the FoldTab
}

// Kernel form, folds partitioning one animal set (IntraGCV): the systems' int8 counts come from one
// A_R A_R^T per individual over fold 0's split rows (k_gshare; FoldTab::gsh) -- the fold systems'
// training rows are all rows of fold 0's split -- instead of one int8 GEMM per system.  The counts
// are the same exact integers, so the results are bit-identical (TBLUP_FOLD_GSHARE=0 for A/B).
// (only where the systems would form their counts in-tile: FP4 system tiles per fold system beat the
// shared int32 counts' row-mapped reads -- config-4-shaped 5 folds 21.9 vs 22.5 ms)
static bool fold_gshare(const tblup_ctx* c, const std::vector<Split*>& sps, const SysDims& sd) {
  if (sd.form != FORM_DUAL || !c->fold_share || !c->fold_gshare || sps.size() < 2) return false;
  if (sys_tiles(c, dims_of(c, *sps[0]), sd)) return false;
  for (const Split* sp : sps)
    if (sp->rows != sps[0]->rows || (int64_t)sp->train.size() != sp->nT || (int64_t)sp->valid.size() != sp->nV)
      return false;
  return true;
}
static size_t gshare_bytes(const std::vector<Split*>& sps, int64_t B) {
  const int64_t nRp = sps[0]->nRp, nTp = sps[0]->nTp, F = (int64_t)sps.size();
  return (size_t)round_up(B * nRp * nRp * 4, 256) + (size_t)round_up(F * nTp * 4, 256) + 512;
}

// The fused chunk: the index lists replicated per fold (F x sum_k, device to device), the fused
// offsets built on the device, then run_chunk over F x B systems.
static int run_folds_fused(tblup_ctx* c, const std::vector<Split*>& sps, const SysDims& sd, hipStream_t s,
                           const int64_t* d_idx, const int64_t* d_off, const int64_t* h_off, int64_t B, double h2, int branch, Carve& cv,
                           double* d_fit, int stop_stage = 0) {
  const int64_t F = (int64_t)sps.size(), FB = F * B, sum_k = h_off[B];
  const EvalDims d = dims_of(c, *sps[0]);
  int64_t* idx_f = cv.take<int64_t>((size_t)(F * sum_k));
  int64_t* off_f = cv.take<int64_t>((size_t)FB + 1);
  std::vector<int64_t>& ho = c->fold_hoff;   // host copy (run_chunk's work accounting and shapes)
  ho.assign((size_t)FB + 1, 0);
  for (int64_t f = 0; f < F; ++f)
    for (int64_t b = 0; b < B; ++b) ho[f * B + b] = f * sum_k + h_off[b];
  ho[FB] = F * sum_k;
  for (int64_t f = 0; f < F; ++f)
    HIPCHK(hipMemcpyAsync(idx_f + f * sum_k, d_idx, (size_t)sum_k * 8, hipMemcpyDeviceToDevice, s));
  HIPCHK(launch_fold_offsets(d_off, B, F, sum_k, off_f, s));
  FoldTab ft{};
  ft.bpf = B;
  ft.nf = (int)F;
  ft.share = c->fold_share;
  for (int64_t f = 1; f < F; ++f) ft.share = ft.share && sps[f]->rows == sps[0]->rows;
  if (fold_gshare(c, sps, sd) && stop_stage != 3) {
    // the fold row maps: system row r of fold f -> fold 0's split row of the same animal
    const int64_t nRp = sps[0]->nRp, nTp = sps[0]->nTp, nT = sps[0]->nT;
    std::unordered_map<int64_t, int32_t> pos0;
    pos0.reserve((size_t)(sps[0]->nT + sps[0]->nV) * 2);
    for (int64_t i = 0; i < sps[0]->nT; ++i) pos0[sps[0]->train[i]] = (int32_t)i;
    for (int64_t j = 0; j < sps[0]->nV; ++j) pos0[sps[0]->valid[j]] = (int32_t)(nTp + j);
    std::vector<int32_t>& hm = c->gmap_host;
    HIPCHK(hipStreamSynchronize(s));   // the previous chunk's map copy may still read hm
    hm.assign((size_t)(F * nTp), -1);
    for (int64_t f = 0; f < F; ++f)
      for (int64_t r = 0; r < nT; ++r) {
        const auto it = pos0.find(sps[f]->train[r]);
        if (it == pos0.end()) return fail(TBLUP_ERR_STATE, "internal error: fold rows are not one animal set");
        hm[(size_t)(f * nTp + r)] = it->second;
      }
    ft.gsh = cv.take<int32_t>((size_t)(B * nRp * nRp));
    int32_t* dmap = cv.take<int32_t>((size_t)(F * nTp));
    if (int rc = ws_check(c, cv)) return rc;
    HIPCHK(hipMemcpyAsync(dmap, hm.data(), hm.size() * 4, hipMemcpyHostToDevice, s));
    ft.gmap = dmap;
    ft.gsh_ld = nRp;
    ft.gmap_ld = nTp;
  } else if (fold_gshare(c, sps, sd)) {
    // the solve-only re-run: the counts are not read again, but the carve must match the first pass
    const int64_t nRp = sps[0]->nRp, nTp = sps[0]->nTp;
    cv.take<int32_t>((size_t)(B * nRp * nRp));
    cv.take<int32_t>((size_t)(F * nTp));
  }
  for (int64_t f = 0; f < F; ++f) {
    ft.gpk[f] = (const uint8_t*)sps[f]->gpk.p;
    ft.csT[f] = (const int32_t*)sps[f]->colsumT.p;
    ft.xty[f] = (const double*)sps[f]->xty.p;
    ft.yV[f] = (const double*)sps[f]->yV.p;
    ft.yT[f] = (const double*)sps[f]->yT.p;
    ft.ymu[f] = (const double*)sps[f]->ymu.p;
  }
  return run_chunk(c, *sps[0], d, sd, s, idx_f, off_f, ho.data(), FB, h2, branch, cv, d_fit, nullptr, stop_stage,
                   nullptr, nullptr, &ft);
}

// workspace of a fused chunk: its replicated index lists and the diagonal tiles' counts included,
// plus room for the host entry's own copy of the chunk's index list and offsets ahead of it
static size_t fused_bytes(const tblup_ctx* c, const std::vector<Split*>& sps, const SysDims& sd, int64_t B,
                          int64_t sum_k) {
  const int64_t F = (int64_t)sps.size();
  return chunk_bytes(c, dims_of(c, *sps[0]), sd, F * B, F * sum_k, false) + (size_t)(sum_k + B + 1) * 8 + 1024 +
         (fold_gshare(c, sps, sd) ? gshare_bytes(sps, B) : 0);
}

static int validate_splits(tblup_ctx* c, const int* split_ids, int n_splits, std::vector<Split*>& sps) {
  if (!split_ids || n_splits < 1) return fail(TBLUP_ERR_ARG, "need n_splits >= 1 split ids");
  sps.resize(n_splits);
  for (int f = 0; f < n_splits; ++f) {
    sps[f] = find_split(c, split_ids[f]);
    if (!sps[f]) return fail(TBLUP_ERR_ARG, "unknown split id " + std::to_string(split_ids[f]));
  }
  return 0;
}

int tblup_eval_folds_device(tblup_ctx* c, const int* split_ids, int n_splits, const int64_t* d_idx,
                            const int64_t* d_offsets, const int64_t* h_offsets, int64_t batch, double h2, int branch,
                            double* d_fitness, void* stream) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (int rc = validate_batch(c, branch, h2, h_offsets, batch)) return rc;
  std::vector<Split*> sps;
  if (int rc = validate_splits(c, split_ids, n_splits, sps)) return rc;
  if (batch == 0) return 0;
  if (!d_idx || !d_offsets || !d_fitness) return fail(TBLUP_ERR_ARG, "null device pointers");
  if (batch > 65535) return fail(TBLUP_ERR_ARG, "device batch limited to 65535 individuals per call");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  SysDims fsd{};
  const bool fused = fold_fusable(c, sps, h_offsets, batch, branch, fsd) &&
                     fused_bytes(c, sps, fsd, batch, h_offsets[batch]) <= c->budget;
  size_t need = 0;
  if (fused) {
    need = fused_bytes(c, sps, fsd, batch, h_offsets[batch]);
  } else {
    for (int f = 0; f < n_splits; ++f) {
      const EvalDims d = dims_of(c, *sps[f]);
      need = std::max(need, chunk_bytes(c, d, choose_sys(c, d, h_offsets, batch, branch, c->form_pref), batch, 0, false));
    }
  }
  if (need > c->ws.bytes) {
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (int rc = dev_alloc(c, c->ws, need)) return rc;
  }
  if (fused) {
    Carve cv{(char*)c->ws.p};
    return run_folds_fused(c, sps, fsd, s, d_idx, d_offsets, h_offsets, batch, h2, branch, cv, d_fitness);
  }
  for (int f = 0; f < n_splits; ++f) {
    const EvalDims d = dims_of(c, *sps[f]);
    const SysDims sd = choose_sys(c, d, h_offsets, batch, branch, c->form_pref);
    Carve cv{(char*)c->ws.p};
    if (int rc = run_chunk(c, *sps[f], d, sd, s, d_idx, d_offsets, h_offsets, batch, h2, branch, cv,
                           d_fitness + (int64_t)f * batch, nullptr, 0, nullptr, nullptr))
      return rc;
  }
  return 0;
}

int tblup_eval_folds(tblup_ctx* c, const int* split_ids, int n_splits, const int64_t* idx, const int64_t* offsets,
                     int64_t batch, double h2, int branch, double* fitness) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (int rc = validate_batch(c, branch, h2, offsets, batch)) return rc;
  std::vector<Split*> sps;
  if (int rc = validate_splits(c, split_ids, n_splits, sps)) return rc;
  if (batch == 0) return 0;
  if (!idx || !fitness) return fail(TBLUP_ERR_ARG, "null idx/fitness");
  if (int rc = check_indices(c, idx, offsets[batch])) return rc;
  HIPCHK(hipSetDevice(c->device));
  HostEntry he(c);
  std::vector<EvalDims> ds(n_splits);
  for (int f = 0; f < n_splits; ++f) ds[f] = dims_of(c, *sps[f]);
  auto fold_bytes = [&](const int64_t* off, int64_t B, int64_t sum_k) {
    size_t m = 0;
    for (int f = 0; f < n_splits; ++f)
      m = std::max(m, chunk_bytes(c, ds[f], choose_sys(c, ds[f], off, B, branch, c->form_pref), B, sum_k, false));
    SysDims fsd{};
    if (fold_fusable(c, sps, off, B, branch, fsd)) m = std::max(m, fused_bytes(c, sps, fsd, B, sum_k));
    return m + (size_t)n_splits * B * 8 + 256;
  };
  int64_t b0 = 0;
  while (b0 < batch) {
    int64_t b1 = b0, sum_k = 0;
    std::vector<int64_t> hoff(1, 0);
    while (b1 < batch) {
      const int64_t k = offsets[b1 + 1] - offsets[b1];
      hoff.push_back(hoff.back() + k);
      if (b1 > b0 && fold_bytes(hoff.data(), b1 + 1 - b0, sum_k + k) > c->budget) {
        hoff.pop_back();
        break;
      }
      if (b1 - b0 >= 65535) {
        hoff.pop_back();
        break;
      }
      sum_k += k;
      ++b1;
    }
    const int64_t B = b1 - b0;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (int rc = dev_alloc(c, c->ws, fold_bytes(hoff.data(), B, sum_k))) return rc;
    Carve head{(char*)c->ws.p};
    int64_t* d_idx = head.take<int64_t>((size_t)sum_k);
    int64_t* d_off = head.take<int64_t>((size_t)B + 1);
    double* d_fit = head.take<double>((size_t)n_splits * B);
    HIPCHK(hipMemcpyAsync(d_idx, idx + offsets[b0], (size_t)sum_k * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_off, hoff.data(), (size_t)(B + 1) * 8, hipMemcpyHostToDevice, c->stream));
    SysDims fsd{};
    const bool fused = fold_fusable(c, sps, hoff.data(), B, branch, fsd);
    for (int pass = 0;; ++pass) {
      // pass 1 after a chained solve gave up a wait: fused, the same factor solved by k_solve; split
      // by split (the folds reuse one workspace, so the earlier folds' factors are gone), every fold
      // again with the chained solve off -- bit-identical either way
      std::vector<int32_t> seqs;
      if (fused) {
        Carve cv = head;
        if (int rc = run_folds_fused(c, sps, fsd, c->stream, d_idx, d_off, hoff.data(), B, h2, branch, cv, d_fit,
                                     pass ? 3 : 0))
          return rc;
        seqs.push_back(c->last_chain_seq);
      } else {
        for (int f = 0; f < n_splits; ++f) {
          Carve cv = head;   // every fold reuses the same workspace after the inputs, in stream order
          const SysDims sd = choose_sys(c, ds[f], hoff.data(), B, branch, c->form_pref);
          // the recovery pass runs every fold with k_solve (stop_stage 4: a per-call choice)
          if (int rc = run_chunk(c, *sps[f], ds[f], sd, c->stream, d_idx, d_off, hoff.data(), B, h2, branch, cv,
                                 d_fit + (int64_t)f * B, nullptr, pass ? 4 : 0, nullptr, nullptr))
            return rc;
          seqs.push_back(c->last_chain_seq);
        }
      }
      for (int f = 0; f < n_splits; ++f)
        HIPCHK(hipMemcpyAsync(fitness + (int64_t)f * batch + b0, d_fit + (int64_t)f * B, (size_t)B * 8,
                              hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      bool any = false;
      for (int32_t q : seqs) {
        bool e = false;
        if (int rc = chain_expired(c, q, &e)) return rc;
        any = any || e;
      }
      if (!any) break;
      ++c->chain_recoveries;
    }
    b0 = b1;
  }
  if (c->profiling) return drain_events(c);
  return 0;
}

int tblup_set_profiling(tblup_ctx* c, int enable) {
  if (int rc = check_ctx(c)) return rc;
  c->profiling = enable != 0;
  return 0;
}

int tblup_get_profile(tblup_ctx* c, double* ms, int64_t* launches, double* flops, double* bytes) {
  if (int rc = check_ctx(c)) return rc;
  HIPCHK(hipSetDevice(c->device));
  if (int rc = drain_events(c)) return rc;
  for (int i = 0; i < TBLUP_N_KCLASS; ++i) {
    if (ms) ms[i] = c->ms[i];
    if (launches) launches[i] = c->launches[i];
    if (flops) flops[i] = c->flops[i];
    if (bytes) bytes[i] = c->bytes[i];
  }
  return 0;
}

int tblup_reset_profile(tblup_ctx* c) {
  if (int rc = check_ctx(c)) return rc;
  if (int rc = drain_events(c)) return rc;
  for (int i = 0; i < TBLUP_N_KCLASS; ++i) {
    c->ms[i] = 0;
    c->launches[i] = 0;
    c->flops[i] = 0;
    c->bytes[i] = 0;
  }
  return 0;
}

int tblup_debug_grm(tblup_ctx* c, int split_id, const int64_t* idx, int64_t k, double h2, int branch, int stage,
                    double* out, double* z_out) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (!idx || k < 1 || !out) return fail(TBLUP_ERR_ARG, "bad debug arguments");
  if (stage != 1 && stage != 2) return fail(TBLUP_ERR_ARG, "stage must be 1 or 2");
  int64_t offs[2] = {0, k};
  if (int rc = validate_batch(c, branch, h2, offs, 1)) return rc;
  if (int rc = check_indices(c, idx, k)) return rc;
  Split* sp = find_split(c, split_id);
  if (!sp) return fail(TBLUP_ERR_ARG, "unknown split id");
  HIPCHK(hipSetDevice(c->device));
  const EvalDims d = dims_of(c, *sp);
  const SysDims sd = choose_sys(c, d, offs, 1, branch, 1);   // readback is of the kernel (dual) form
  HIPCHK(hipStreamSynchronize(c->stream));
  if (int rc = dev_alloc(c, c->ws, chunk_bytes(c, d, sd, 1, k, false) + (size_t)d.nRp * d.nTp * 8 + 4096)) return rc;
  Carve cv{(char*)c->ws.p};
  int64_t* d_idx = cv.take<int64_t>((size_t)k);
  int64_t* d_off = cv.take<int64_t>(2);
  double* d_fit = cv.take<double>(1);
  HIPCHK(hipMemcpyAsync(d_idx, idx, (size_t)k * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(d_off, offs, 16, hipMemcpyHostToDevice, c->stream));
  double *K = nullptr, *z = nullptr;
  if (int rc = run_chunk(c, *sp, d, sd, c->stream, d_idx, d_off, offs, 1, h2, branch, cv, d_fit, nullptr, stage,
                         &K, &z))
    return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  const int64_t rows = (stage == 1) ? d.nRp : d.nTp;
  std::vector<double> full((size_t)rows * d.nTp);
  HIPCHK(hipMemcpy(full.data(), K, full.size() * 8, hipMemcpyDeviceToHost));
  const int64_t nR = d.nT + d.nV;
  if (stage == 2) {
    // Lt tiles: tile (I, J) at ((I*NT + J) * 128*128), element [j][i] = L[128I+i][128J+j]
    std::memset(out, 0, (size_t)nR * d.nT * 8);   // upper triangle and V rows are zero
    const int64_t TT = (int64_t)TILE * TILE;
    for (int64_t r = 0; r < d.nT; ++r)
      for (int64_t cc = 0; cc <= r; ++cc) {
        const int64_t I = r / TILE, Jt = cc / TILE;
        out[r * d.nT + cc] = full[(I * d.NT + Jt) * TT + (cc % TILE) * TILE + (r % TILE)];
      }
  } else {
    for (int64_t r = 0; r < nR; ++r) {
      const int64_t src = r < d.nT ? r : d.nTp + (r - d.nT);
      std::memcpy(out + r * d.nT, full.data() + src * d.nTp, (size_t)d.nT * 8);
    }
  }
  if (z_out) {
    std::vector<double> zz(d.nTp);   // trait 0
    HIPCHK(hipMemcpy(zz.data(), z, (size_t)d.nTp * 8, hipMemcpyDeviceToHost));
    std::memcpy(z_out, zz.data(), (size_t)d.nT * 8);
  }
  if (c->profiling) return drain_events(c);
  return 0;
}

int tblup_grm(tblup_ctx* c, const int64_t* idx, int64_t k, double* G) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (c->n == 0) return fail(TBLUP_ERR_STATE, "context has no genotype panel");
  if (!idx || k < 1 || !G) return fail(TBLUP_ERR_ARG, "bad grm arguments");
  const int64_t n = c->n;
  // G = K_TT of the gblup-branch kernel form with T = every animal (p over all rows, as
  // make_grm) and lambda = 0 (h2 = 1); V is a placeholder the solve never reaches
  std::vector<int64_t> T(n);
  for (int64_t i = 0; i < n; ++i) T[i] = i;
  const int64_t V[2] = {0, 1};
  const int sid = -0x7ffffff0;   // reserved id, dropped before returning
  if (int rc = tblup_set_split(c, sid, T.data(), n, V, 2)) return rc;
  std::vector<double> K((size_t)(n + 2) * n);
  const int rc = tblup_debug_grm(c, sid, idx, k, 1.0, TBLUP_BRANCH_GBLUP, 1, K.data(), nullptr);
  const std::string err = g_err;
  tblup_drop_split(c, sid);
  if (rc) return fail(rc, err);
  for (int64_t r = 0; r < n; ++r)   // lower-triangle tiles are computed; mirror the upper triangle
    for (int64_t cc = 0; cc < n; ++cc) G[r * n + cc] = cc <= r ? K[(size_t)r * n + cc] : K[(size_t)cc * n + r];
  return 0;
}

int tblup_get_wg_trace(tblup_ctx* c, uint64_t* out, int64_t cap, int64_t* n_records) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (!n_records) return fail(TBLUP_ERR_ARG, "null n_records");
  *n_records = c->wg_trace ? c->wgt_used : 0;
  if (!c->wg_trace || !out || cap <= 0) return 0;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipDeviceSynchronize());
  const int64_t n = std::min(cap, c->wgt_used);
  HIPCHK(hipMemcpy(out, c->wgt.p, (size_t)n * WGT_REC * 8, hipMemcpyDeviceToHost));
  return 0;
}

static int read_status_word(tblup_ctx* c, void* stream, int* flag, int word) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (!flag) return fail(TBLUP_ERR_ARG, "null flag");
  *flag = 0;
  if (!c->status.p) return 0;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  int32_t h = 0;
  int32_t* w = (int32_t*)c->status.p + word;
  HIPCHK(hipMemcpyAsync(&h, w, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemsetAsync(w, 0, 4, s));
  HIPCHK(hipStreamSynchronize(s));
  *flag = h != 0;
  return 0;
}

int tblup_index_error(tblup_ctx* c, void* stream, int* flag) { return read_status_word(c, stream, flag, ST_INDEX); }

int tblup_solve_error(tblup_ctx* c, void* stream, int* flag) { return read_status_word(c, stream, flag, ST_SOLVE); }

int tblup_status_async(tblup_ctx* c, void* stream, int32_t* host_status) {
  g_err.clear();
  if (int rc = check_ctx(c)) return rc;
  if (!host_status) return fail(TBLUP_ERR_ARG, "null host_status");
  if (!c->status.p) return fail(TBLUP_ERR_STATE, "context has no genotype panel");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  HIPCHK(hipMemcpyAsync(host_status, c->status.p, ST_WORDS * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemsetAsync(c->status.p, 0, ST_WORDS * 4, s));
  return 0;
}

int tblup_chain_recoveries(tblup_ctx* c, int64_t* count) {
  if (int rc = check_ctx(c)) return rc;
  if (!count) return fail(TBLUP_ERR_ARG, "null count");
  *count = c->chain_recoveries;
  return 0;
}

int tblup_mem_info(tblup_ctx* c, int64_t* bytes) {
  if (int rc = check_ctx(c)) return rc;
  if (bytes) *bytes = c->mem_in_use;
  return 0;
}

}  // extern "C"
