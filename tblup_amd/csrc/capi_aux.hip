// C ABI of libtblup_gpu.so, the entry points beside the evaluation pipeline (include/tblup_gpu.h):
// RandomKey genome decode, the seeder's SNP scan, the GPU DE generation step (numpy's MT19937
// stream jumped per individual, mt_jump.cpp) and its helpers, host memory registration.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "capi_ctx.h"
#include "mt_jump.h"

using namespace tblup;
using namespace tblup_capi;

extern "C" {

static int validate_decode(int64_t batch, int64_t d, const int64_t* offsets) {
  if (batch < 0 || d < 1 || d > 0x7fffffff) return fail(TBLUP_ERR_ARG, "decode needs batch >= 0, 1 <= d < 2^31");
  if (batch > 0 && (!offsets || offsets[0] != 0)) return fail(TBLUP_ERR_ARG, "offsets must start at 0");
  for (int64_t b = 0; b < batch; ++b) {
    const int64_t k = offsets[b + 1] - offsets[b];
    if (k < 1 || k > d || k > 8192) return fail(TBLUP_ERR_ARG, "every k must be in [1, min(d, 8192)]");
  }
  return 0;
}

int tblup_decode_topk_device(tblup_ctx* c, const double* d_keys, int64_t batch, int64_t d, int64_t ld,
                             const int64_t* d_offsets, const int64_t* h_offsets, int64_t* d_idx_out, void* stream) {
  clear_error();
  if (int rc = check_ctx(c)) return rc;
  if (int rc = validate_decode(batch, d, h_offsets)) return rc;
  if (ld < d) return fail(TBLUP_ERR_ARG, "ld < d");
  if (batch == 0) return 0;
  if (!d_keys || !d_offsets || !d_idx_out) return fail(TBLUP_ERR_ARG, "null device pointers");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  HIPCHK(launch_decode_topk(d_keys, batch, d, ld, d_offsets, d_idx_out, s));
  return 0;
}

int tblup_decode_topk(tblup_ctx* c, const double* keys, int64_t batch, int64_t d, const int64_t* offsets,
                      int64_t* idx_out) {
  clear_error();
  if (int rc = check_ctx(c)) return rc;
  if (int rc = validate_decode(batch, d, offsets)) return rc;
  if (batch == 0) return 0;
  if (!keys || !idx_out) return fail(TBLUP_ERR_ARG, "null keys/idx_out");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int64_t total = offsets[batch];
  if (int rc = dev_alloc(c, c->dec_keys, (size_t)batch * d * 8)) return rc;
  if (int rc = dev_alloc(c, c->dec_idx, (size_t)(total + batch + 1) * 8)) return rc;
  int64_t* d_idx = (int64_t*)c->dec_idx.p;
  int64_t* d_off = d_idx + total;
  HIPCHK(hipMemcpyAsync(c->dec_keys.p, keys, (size_t)batch * d * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(d_off, offsets, (size_t)(batch + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(launch_decode_topk((const double*)c->dec_keys.p, batch, d, d, d_off, d_idx, c->stream));
  HIPCHK(hipMemcpyAsync(idx_out, d_idx, (size_t)total * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int tblup_snp_scan(tblup_ctx* c, const int64_t* rows, int64_t n_rows, const double* yc, int64_t* sx, int64_t* sxx,
                   double* sxy) {
  clear_error();
  if (int rc = check_ctx(c)) return rc;
  if (c->n == 0) return fail(TBLUP_ERR_STATE, "context has no genotype panel");
  if (!rows || n_rows < 1 || !yc || !sx || !sxx || !sxy) return fail(TBLUP_ERR_ARG, "bad scan arguments");
  std::vector<int32_t> r32((size_t)n_rows);
  for (int64_t i = 0; i < n_rows; ++i) {
    if (rows[i] < 0 || rows[i] >= c->n) return fail(TBLUP_ERR_ARG, "animal row out of range");
    r32[i] = (int32_t)rows[i];
  }
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const size_t P = (size_t)c->P;
  DevBuf buf;
  const size_t o_y = round_up(4 * (size_t)n_rows, 16), o_sx = o_y + 8 * (size_t)n_rows, o_sxx = o_sx + 8 * P,
               o_sxy = o_sxx + 8 * P, bytes = o_sxy + 8 * P;
  if (int rc = dev_alloc(c, buf, bytes)) return rc;
  char* b = (char*)buf.p;
  int rc = 0;
  auto run = [&]() -> int {
    HIPCHK(hipMemcpyAsync(b, r32.data(), 4 * (size_t)n_rows, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_y, yc, 8 * (size_t)n_rows, hipMemcpyHostToDevice, c->stream));
    HIPCHK(launch_snp_scan((const int8_t*)c->geno_sm.p, c->n, c->P, (const int32_t*)b, n_rows,
                           (const double*)(b + o_y), (int64_t*)(b + o_sx), (int64_t*)(b + o_sxx),
                           (double*)(b + o_sxy), c->stream));
    HIPCHK(hipMemcpyAsync(sx, b + o_sx, 8 * P, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(sxx, b + o_sxx, 8 * P, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(sxy, b + o_sxy, 8 * P, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
  };
  rc = run();
  dev_free(c, buf);
  return rc;
}

// ---- differential-evolution step (k_de.hip; jump polynomials from mt_jump.cpp) ----

int tblup_mt19937_jump(const uint32_t* key, int32_t pos, uint64_t n_words, uint32_t* key_out, int32_t* pos_out) {
  clear_error();
  if (!key || !key_out || !pos_out) return fail(TBLUP_ERR_ARG, "null key/key_out/pos_out");
  if (pos < 0 || pos > 624) return fail(TBLUP_ERR_ARG, "pos must be in [0, 624]");
  int po = 0;
  tblup_mt::jump_state(key, pos, n_words, key_out, &po);
  *pos_out = po;
  return 0;
}

int tblup_de_donors(int strategy, int64_t pop, int64_t L, int32_t best, uint32_t* py_mt, int32_t* py_index,
                    int32_t* donors, int64_t* fixed) {
  clear_error();
  if (strategy != TBLUP_DE_RAND_1 && strategy != TBLUP_DE_CURRENT_TO_BEST_1)
    return fail(TBLUP_ERR_ARG, "unknown DE strategy");
  if (pop < 4 || pop > 65535 || L < 1 || L >= ((int64_t)1 << 32))
    return fail(TBLUP_ERR_ARG, "need 4 <= pop <= 65535 and 1 <= L < 2^32");
  if (!py_mt || !py_index || !donors || !fixed) return fail(TBLUP_ERR_ARG, "null py_mt/py_index/donors/fixed");
  if (*py_index < 0 || *py_index > 624) return fail(TBLUP_ERR_ARG, "py_index must be in [0, 624]");
  if (strategy == TBLUP_DE_CURRENT_TO_BEST_1 ? (best < 0 || best >= pop) : best != -1)
    return fail(TBLUP_ERR_ARG, "best must be in [0, pop) for current-to-best/1 and -1 for rand/1");
  tblup_mt::py_random_donors(py_mt, py_index, pop, L, best, donors, fixed);
  return 0;
}

static int validate_de(int strategy, int64_t pop, int64_t L, const int32_t* donors, const int64_t* fixed, double cr,
                       const uint32_t* mt_key, const int32_t* mt_pos) {
  if (strategy != TBLUP_DE_RAND_1 && strategy != TBLUP_DE_CURRENT_TO_BEST_1)
    return fail(TBLUP_ERR_ARG, "unknown DE strategy");
  if (pop < 1 || pop > 65535 || L < 1 || L > ((int64_t)1 << 31)) return fail(TBLUP_ERR_ARG, "need 1 <= pop <= 65535, 1 <= L <= 2^31");
  if (!donors || !fixed || !mt_key || !mt_pos) return fail(TBLUP_ERR_ARG, "null donors/fixed/mt_key/mt_pos");
  if (*mt_pos < 0 || *mt_pos > 624) return fail(TBLUP_ERR_ARG, "mt_pos must be in [0, 624]");
  if (!(cr == cr)) return fail(TBLUP_ERR_ARG, "crossover rate is NaN");
  for (int64_t i = 0; i < 3 * pop; ++i)
    if (donors[i] < 0 || donors[i] >= pop) return fail(TBLUP_ERR_ARG, "donor index out of range");
  for (int64_t i = 0; i < pop; ++i)
    if (fixed[i] < 0 || fixed[i] >= L) return fail(TBLUP_ERR_ARG, "fixed crossover position out of range");
  return 0;
}

// The asynchronous step, with optional per-individual strategies / F / crossover rates (host
// arrays of pop; null: the scalars).
static int de_step_async(tblup_ctx* c, int strategy, const int32_t* strat_i, const double* F_i, const double* cr_i,
                         const double* d_parents, int64_t pop, int64_t L, int64_t ld, const int32_t* donors,
                         const int64_t* fixed, double F, double cr, int clip, double clip_hi, const uint32_t* mt_key,
                         int32_t mt_pos, double* d_children, int64_t ldc, void* stream) {
  clear_error();
  if (int rc = check_ctx(c)) return rc;
  if (c->de_pending) return fail(TBLUP_ERR_STATE, "the previous DE step's state was not fetched (tblup_de_state_wait)");
  int32_t* const mt_pos_in = &mt_pos;
  if (int rc = validate_de(strategy, pop, L, donors, fixed, cr, mt_key, mt_pos_in)) return rc;
  for (int64_t i = 0; strat_i && i < pop; ++i)
    if (strat_i[i] != TBLUP_DE_RAND_1 && strat_i[i] != TBLUP_DE_CURRENT_TO_BEST_1)
      return fail(TBLUP_ERR_ARG, "unknown DE strategy");
  for (int64_t i = 0; cr_i && i < pop; ++i)
    if (!(cr_i[i] == cr_i[i])) return fail(TBLUP_ERR_ARG, "crossover rate is NaN");
  if (ld < L || ldc < L) return fail(TBLUP_ERR_ARG, "ld/ldc < L");
  if (!d_parents || !d_children) return fail(TBLUP_ERR_ARG, "null device pointers");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (c->de_L != L || c->de_pop != pop) {
    const tblup_mt::DePolys dp = tblup_mt::de_polys(L, pop);
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (int rc = dev_alloc(c, c->de_polys, dp.words.size() * 4)) return rc;
    HIPCHK(hipMemcpy(c->de_polys.p, dp.words.data(), dp.words.size() * 4, hipMemcpyHostToDevice));
    c->de_L = L;
    c->de_pop = pop;
    c->de_end_jump = dp.end_jump;
  }
  // per-call arguments: key in, key out, pos out, donors, fixed
  const size_t o_keyo = 624 * 4, o_pos = 2 * 624 * 4, o_don = o_pos + 16, o_fix = o_don + (size_t)round_up(12 * pop, 16);
  const size_t o_str = o_fix + 8 * (size_t)pop, o_F = o_str + (size_t)round_up(4 * pop, 16), o_cr = o_F + 8 * (size_t)pop;
  const size_t small = o_cr + 8 * (size_t)pop;
  // device-only scratch of the three-launch form (large populations): base sequence + windows
  // (from more individuals than CUs: both forms need a second round of jump workgroups there, and the
  // split form's mask and stream run several per CU; TBLUP_DE_SPLIT = the smallest split population)
  static const int64_t split_min = getenv("TBLUP_DE_SPLIT") ? atoll(getenv("TBLUP_DE_SPLIT")) : cu_count() + 1;
  const bool split = pop >= split_min;
  const size_t o_scr = (size_t)round_up((int64_t)small, 256);
  const size_t need = split ? o_scr + 4 * (size_t)(DE_SEQ_SCRATCH + 624 * pop) : small;
  if (need > c->de_small.bytes) {
    HIPCHK(hipStreamSynchronize(s));
    if (int rc = dev_alloc(c, c->de_small, need)) return rc;
  }
  char* base = (char*)c->de_small.p;
  // page-locked staging that outlives this call (the copy is asynchronous); the previous call's
  // copy from it finished before that call's state was fetched (one step pending at a time)
  if (small > c->de_stage_bytes) {
    HIPCHK(hipStreamSynchronize(s));
    if (c->de_stage) HIPCHK(hipHostFree(c->de_stage));
    c->de_stage = nullptr;
    c->de_stage_bytes = 0;
    HIPCHK(hipHostMalloc((void**)&c->de_stage, small, hipHostMallocDefault));
    c->de_stage_bytes = small;
  }
  char* stage = c->de_stage;
  std::memcpy(stage, mt_key, 624 * 4);
  std::memcpy(stage + o_don, donors, 12 * pop);
  std::memcpy(stage + o_fix, fixed, 8 * pop);
  if (strat_i) std::memcpy(stage + o_str, strat_i, 4 * pop);
  if (F_i) std::memcpy(stage + o_F, F_i, 8 * pop);
  if (cr_i) std::memcpy(stage + o_cr, cr_i, 8 * pop);
  HIPCHK(hipMemcpyAsync(base, stage, small, hipMemcpyHostToDevice, s));
  const tblup_mt::EndState e = tblup_mt::end_state(mt_pos, 2 * (uint64_t)L * (uint64_t)pop);
  HIPCHK(launch_de_step((const uint32_t*)base, mt_pos, (const uint32_t*)c->de_polys.p, c->de_end_jump ? 1 : 0, e.s,
                        e.pos, d_parents, ld, (const int32_t*)(base + o_don), (const int64_t*)(base + o_fix), strategy,
                        F, cr, clip ? 1 : 0, clip_hi, L, (int)pop, d_children, ldc, (uint32_t*)(base + o_keyo),
                        (int32_t*)(base + o_pos), s, strat_i ? (const int32_t*)(base + o_str) : nullptr,
                        F_i ? (const double*)(base + o_F) : nullptr, cr_i ? (const double*)(base + o_cr) : nullptr,
                        split ? (uint32_t*)(base + o_scr) : nullptr));
  if (!c->de_host) HIPCHK(hipHostMalloc((void**)&c->de_host, 625 * 4, hipHostMallocDefault));
  if (!c->de_ev) HIPCHK(hipEventCreateWithFlags(&c->de_ev, hipEventDisableTiming));
  HIPCHK(hipMemcpyAsync(c->de_host, base + o_keyo, 624 * 4 + 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(c->de_ev, s));
  c->de_pending = true;
  return 0;
}

int tblup_de_step_device_async(tblup_ctx* c, int strategy, const double* d_parents, int64_t pop, int64_t L,
                               int64_t ld, const int32_t* donors, const int64_t* fixed, double F, double cr, int clip,
                               double clip_hi, const uint32_t* mt_key, int32_t mt_pos, double* d_children,
                               int64_t ldc, void* stream) {
  return de_step_async(c, strategy, nullptr, nullptr, nullptr, d_parents, pop, L, ld, donors, fixed, F, cr, clip,
                       clip_hi, mt_key, mt_pos, d_children, ldc, stream);
}

int tblup_de_step_device_async_mix(tblup_ctx* c, const int32_t* strategies, const double* F, const double* cr,
                                   const double* d_parents, int64_t pop, int64_t L, int64_t ld, const int32_t* donors,
                                   const int64_t* fixed, int clip, double clip_hi, const uint32_t* mt_key,
                                   int32_t mt_pos, double* d_children, int64_t ldc, void* stream) {
  if (!strategies || !F || !cr) {
    clear_error();
    return fail(TBLUP_ERR_ARG, "null strategies/F/cr");
  }
  // element 0 is read only for a non-empty population (validate_de rejects pop < 1); the scalar
  // slots are placeholders when per-individual arrays are given
  const bool any = pop >= 1;
  return de_step_async(c, any ? strategies[0] : TBLUP_DE_RAND_1, strategies, F, cr, d_parents, pop, L, ld, donors,
                       fixed, any ? F[0] : 0.0, any ? cr[0] : 0.0, clip, clip_hi, mt_key, mt_pos, d_children, ldc,
                       stream);
}

int tblup_de_state_wait(tblup_ctx* c, uint32_t* mt_key, int32_t* mt_pos) {
  clear_error();
  if (int rc = check_ctx(c)) return rc;
  if (!mt_key || !mt_pos) return fail(TBLUP_ERR_ARG, "null mt_key/mt_pos");
  if (!c->de_pending) return fail(TBLUP_ERR_STATE, "no DE step pending (tblup_de_step_device_async)");
  HIPCHK(hipSetDevice(c->device));
  c->de_pending = false;
  HIPCHK(hipEventSynchronize(c->de_ev));
  std::memcpy(mt_key, c->de_host, 624 * 4);
  std::memcpy(mt_pos, c->de_host + 624, 4);
  return 0;
}

int tblup_de_step_device(tblup_ctx* c, int strategy, const double* d_parents, int64_t pop, int64_t L, int64_t ld,
                         const int32_t* donors, const int64_t* fixed, double F, double cr, int clip, double clip_hi,
                         uint32_t* mt_key, int32_t* mt_pos, double* d_children, int64_t ldc, void* stream) {
  if (!mt_key || !mt_pos) {
    clear_error();
    return fail(TBLUP_ERR_ARG, "null donors/fixed/mt_key/mt_pos");
  }
  if (int rc = tblup_de_step_device_async(c, strategy, d_parents, pop, L, ld, donors, fixed, F, cr, clip, clip_hi,
                                          mt_key, *mt_pos, d_children, ldc, stream))
    return rc;
  return tblup_de_state_wait(c, mt_key, mt_pos);
}

int tblup_de_step(tblup_ctx* c, int strategy, const double* parents, int64_t pop, int64_t L, const int32_t* donors,
                  const int64_t* fixed, double F, double cr, int clip, double clip_hi, uint32_t* mt_key,
                  int32_t* mt_pos, double* children) {
  clear_error();
  if (int rc = check_ctx(c)) return rc;
  if (int rc = validate_de(strategy, pop, L, donors, fixed, cr, mt_key, mt_pos)) return rc;
  if (!parents || !children) return fail(TBLUP_ERR_ARG, "null parents/children");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const size_t bytes = (size_t)pop * L * 8;
  if (int rc = dev_alloc(c, c->de_par, bytes)) return rc;
  if (int rc = dev_alloc(c, c->de_chi, bytes)) return rc;
  HIPCHK(hipMemcpyAsync(c->de_par.p, parents, bytes, hipMemcpyHostToDevice, c->stream));
  if (int rc = tblup_de_step_device(c, strategy, (const double*)c->de_par.p, pop, L, L, donors, fixed, F, cr, clip,
                                    clip_hi, mt_key, mt_pos, (double*)c->de_chi.p, L, nullptr))
    return rc;
  HIPCHK(hipMemcpy(children, c->de_chi.p, bytes, hipMemcpyDeviceToHost));
  return 0;
}

int tblup_gather_rows(tblup_ctx* c, double* d_dst, int64_t n, int64_t L, int64_t ldd, const double* const* d_src_rows,
                      void* stream) {
  clear_error();
  if (int rc = check_ctx(c)) return rc;
  if (n < 0 || L < 0 || ldd < L) return fail(TBLUP_ERR_ARG, "need n >= 0, 0 <= L <= ldd");
  if (n == 0 || L == 0) return 0;
  if (!d_dst || !d_src_rows) return fail(TBLUP_ERR_ARG, "null destination / source table");
  for (int64_t i = 0; i < n; ++i)
    if (!d_src_rows[i]) return fail(TBLUP_ERR_ARG, "null source row");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  for (int64_t r0 = 0; r0 < n; r0 += ROWPTRS) {
    const int nr = (int)std::min<int64_t>(ROWPTRS, n - r0);
    RowPtrs t{};
    for (int k = 0; k < nr; ++k) t.p[k] = d_src_rows[r0 + k];
    HIPCHK(launch_gather_rows(d_dst + r0 * ldd, ldd, L, t, nr, s));
  }
  return 0;
}

int tblup_host_register(void* ptr, int64_t bytes) {
  clear_error();
  if (!ptr || bytes <= 0) return fail(TBLUP_ERR_ARG, "null pointer or non-positive size");
  HIPCHK(hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault));
  return 0;
}

int tblup_host_unregister(void* ptr) {
  clear_error();
  if (!ptr) return fail(TBLUP_ERR_ARG, "null pointer");
  HIPCHK(hipHostUnregister(ptr));
  return 0;
}

}  // extern "C"
