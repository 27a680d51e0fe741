// Internal to libtblup_gpu.so's C-ABI translation units (capi.hip, capi_aux.hip): the context
// (struct tblup_ctx of include/tblup_gpu.h), its device buffers and the error / allocation helpers.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/tblup_gpu.h"
#include "tblup_internal.h"

namespace tblup_capi {

int fail(int code, const std::string& msg);   // sets the calling thread's tblup_last_error()

#define HIPCHK(expr)                                                                                      \
  do {                                                                                                    \
    hipError_t e_ = (expr);                                                                               \
    if (e_ != hipSuccess) return fail(TBLUP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

struct Split {
  int64_t nT = 0, nV = 0, nTp = 0, nVp = 0, nRp = 0;
  std::vector<int64_t> rows;   // train + valid animals, sorted (fold sets: shared counts)
  std::vector<int64_t> train, valid;   // the split's animal lists in system-row order
  std::vector<double> meanyT;   // [nt]
  DevBuf gpk, colsumT, xty, yT, yV, ymu;
};

enum { KC_STATS = 0, KC_GATHER, KC_GRM, KC_DIAG, KC_OFFDIAG, KC_SOLVE };

struct EventPair {
  int cls;
  hipEvent_t a, b;
};

}  // namespace tblup_capi

using tblup_capi::DevBuf;
using tblup_capi::EventPair;
using tblup_capi::Split;

struct tblup_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t n = 0, P = 0;
  DevBuf geno_sm, colsum_all, scratch;
  DevBuf status;               // int32 [ST_WORDS] device status words: ST_INDEX an index outside
                               // [-P, P) reached k_indiv_stats; ST_SOLVE a chained-solve wait expired
  std::vector<double> pheno;   // [n][nt] animal-major
  int nt = 1;                  // traits (tblup_set_traits)
  std::map<int, std::unique_ptr<Split>> splits;
  DevBuf ws;
  DevBuf dec_keys, dec_idx;   // host-pointer decode staging
  DevBuf de_polys, de_small, de_par, de_chi;   // DE step: jump polynomials, per-call args, host-path staging
  int64_t de_L = -1, de_pop = -1;              // (L, pop) of the uploaded polynomials
  bool de_end_jump = false;
  uint32_t* de_host = nullptr;   // page-locked: the MT state after the last step (624 words + pos)
  char* de_stage = nullptr;      // page-locked: the per-call arguments on their way to de_small
  size_t de_stage_bytes = 0;
  hipEvent_t de_ev = nullptr;    // recorded behind that state's copy
  bool de_pending = false;       // tblup_de_step_device_async issued, tblup_de_state_wait not yet called
  size_t budget = 0;
  // profiling
  bool profiling = false;
  std::vector<EventPair> pending;
  std::vector<hipEvent_t> event_pool;
  double ms[TBLUP_N_KCLASS] = {0};
  int64_t launches[TBLUP_N_KCLASS] = {0};
  double flops[TBLUP_N_KCLASS] = {0};
  double bytes[TBLUP_N_KCLASS] = {0};
  int64_t mem_in_use = 0;

  // TBLUP_WG_TRACE: per-workgroup start/end records of the Cholesky launches of the last chunk
  bool wg_trace = false;
  DevBuf wgt;
  int64_t wgt_used = 0;
  int dbg_skip = 0;   // TBLUP_DBG_SKIP, read only by diagnostic builds (-DTBLUP_DIAG_BUILD): phase
                      // ablation, results wrong when set; the production library never reads it
  int form_pref = 0;  // TBLUP_FORM: 0 auto, 1 kernel (dual) form only, 2 SNP (primal) form for snp batches
  // Cholesky schedule (results are bit-identical under every setting; see OffPlan):
  int ahead = -1;     // TBLUP_AHEAD: -1 auto (per launch: B * (NT - 2 - j) < AHEAD_SLOTS), 0 never, 1 always
  int nrs = 0;        // TBLUP_NRS: partial-sum row slices, 0 auto, else 1 / 2 / 4
  int diag_d = -1;    // TBLUP_DIAG_D: D-units in the diagonal launch (-1 auto, 0 never, 1 always)
  int diag_e = -1;    // TBLUP_DIAG_E: E-units in the diagonal launch (-1 auto, 0 never, 1 every tile)
  int chain_sync = 0;    // TBLUP_CHAIN_SYNC (k_solve.hip)
  int last_term = -1;    // TBLUP_LAST_TERM: -1 auto (last_term_mask), 0 never, 1 always (see use_last_term)
  int lt_mask = -1;      // TBLUP_LT_MASK: the diagonal launches in last-term mode by bit (A/B timing; -1 auto)
  int solve_chain = -1;  // TBLUP_SOLVE_CHAIN: SNP-form back substitution spread over the chip (k_solve_chain):
                         // -1 auto (B <= CHAIN_MAX_B), 0 never, 1 always -- bit-identical results either way
  int solve_pull = -1;   // TBLUP_SOLVE_PULL: the chained solve's units pull beta_K and the tiles of their block
                         // column (1; -1 auto: one trait) or push the tile products of their block row (0)
                         // -- the same bits
  int fold_fuse = 1;     // TBLUP_FOLD_FUSE: 0 evaluates a fold set split by split (A/B timing)
  int fold_share = 1;    // TBLUP_FOLD_SHARE: 0 builds every fold's system tiles from its own rows
  int fold_gshare = 1;   // TBLUP_FOLD_GSHARE: kernel-form folds read their counts from one A_R A_R^T
  int dual_st = 1;       // TBLUP_DUAL_ST: kernel-form system tiles from k_sys_tiles (0: in-tile products)
  std::vector<int32_t> gmap_host;   // the fold row maps of the last fused kernel-form chunk (H2D source)
  int sys_st = -1;       // TBLUP_SYS_ST: system tiles by the persistent super-tile kernel (k_sys_tiles_st):
                         // -1 auto (sys_tiles_grid), 0 never, 1 whenever it applies -- the same exact counts
  // SNP form: the padding rows (ns - k) lead the system, so the contractions over block column 0
  // skip them (TBLUP_PAD_FIRST=0: trailing padding, equal up to rounding -- a test knob).
  int pad_first = 1;
  std::vector<int64_t> fold_hoff;   // host offsets of the last fold-fused chunk (host-side shapes only)
  DevBuf chain;          // its flags [B][chain_flags(NT)], the expiry ring [CHAIN_ERR_RING] and one
                         // scratch word (zeroed when allocated)
  int32_t chain_seq = 0; // flag value of the last chained solve
  int32_t last_chain_seq = 0;   // seq of the chained solve the last run_chunk enqueued, 0 if none
  bool host_entry = false;      // a synchronous entry is running: its chained solves recover on expiry
  int64_t chain_recoveries = 0; // chunks whose expired chained solve was re-run through k_solve
  // debug knob (TBLUP_CHAIN_DEBUG="spin,delay,shots"): the next `shots` chained solves poll at
  // most `spin` times and delay one producer by `delay` sleep rounds -- forces an expiry (tests)
  int32_t chain_dbg_spin = 0, chain_dbg_delay = 0, chain_dbg_shots = 0;
};

namespace tblup_capi {
int dev_alloc(tblup_ctx* c, DevBuf& b, size_t bytes);
void dev_free(tblup_ctx* c, DevBuf& b);
int check_ctx(tblup_ctx* c);
void clear_error();
}  // namespace tblup_capi
