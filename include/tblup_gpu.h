/*
 * tblup_gpu.h — C ABI of the MI355X GBLUP fitness evaluator (libtblup_gpu.so).
 *
 * Drop-in boundary for the reference's fitness-evaluation hot path
 * (ianwhale/tblup).  The reference has no native FFI; its boundary is the
 * Python evaluator plugin API, whose compute leg is the multiprocessing
 * worker pool:
 *
 *   ParallelEvaluator.__enter__/__exit__   tblup/evaluator.py:120-135  -> tblup_ctx_create / tblup_ctx_destroy
 *   BlupParallelEvaluator.__init__ split   tblup/evaluator.py:188-203  -> tblup_set_split
 *   worker() + enqueue() + blup()          tblup/evaluator.py:205-263  -> tblup_eval_batch
 *     gblup()    evaluator.py:265-286   (branch TBLUP_BRANCH_GBLUP)
 *     snp_blup() evaluator.py:288-314   (branch TBLUP_BRANCH_SNP)
 *     dispatch   evaluator.py:257       (branch TBLUP_BRANCH_AUTO: k > n -> gblup)
 *   make_grm()                             tblup/utils.py:7-18          -> tblup_debug_grm (block readback)
 *
 * The ctypes binding a maintainer adds on the reference side is shown in
 * INTEGRATION.md.  All functions return 0 on success and a negative status
 * otherwise; tblup_last_error() returns a thread-local message.  Host buffers
 * are borrowed for the duration of the call only.  A NaN fitness (constant
 * prediction, degenerate panel) is returned as NaN, never raised.
 */
#ifndef TBLUP_GPU_H
#define TBLUP_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tblup_ctx tblup_ctx;

enum {
  TBLUP_OK = 0,
  TBLUP_ERR_ARG = -1,      /* invalid argument (shape, index range, unknown split) */
  TBLUP_ERR_HIP = -2,      /* HIP runtime error (no device, launch or copy failure) */
  TBLUP_ERR_OOM = -3,      /* device allocation failed */
  TBLUP_ERR_STATE = -4,    /* call out of order */
  TBLUP_ERR_INDEX = -5     /* SNP index outside [-n_snps, n_snps): numpy's IndexError for data[:, indices] */
};

enum {
  TBLUP_BRANCH_AUTO = 0,   /* evaluator.py:257: len(indices) > n_animals -> GBLUP else SNP-BLUP */
  TBLUP_BRANCH_GBLUP = 1,  /* evaluator.py:265-286: p over all n animals, no phenotype centring */
  TBLUP_BRANCH_SNP = 2     /* evaluator.py:288-314: p over train animals, ridge intercept = mean(y_T) */
};

enum {
  TBLUP_LAYOUT_ANIMAL_MAJOR = 0, /* n_animals x n_snps, row-major (the .npy the reference loads) */
  TBLUP_LAYOUT_SNP_MAJOR = 1     /* n_snps x n_animals, row-major */
};

/* Last error message of the calling thread ("" if none). */
const char* tblup_last_error(void);

/* Library version string. */
const char* tblup_version(void);

/* Number of visible HIP devices (0 when none). */
int tblup_device_count(int* out_count);

/*
 * Create a context on HIP device `device`: uploads the {0,1,2} genotype
 * matrix (int8) and the phenotype vector (float64, length n_animals).
 * Replaces the per-worker np.load of evaluator.py:215-216.
 * tblup_ctx_create(NULL, 0, 0, layout, NULL, device, &ctx) creates a context
 * without a panel, for the DE step and genome decode only (no split can be set).
 */
int tblup_ctx_create(const int8_t* geno, int64_t n_animals, int64_t n_snps, int layout,
                     const double* pheno, int device, tblup_ctx** out_ctx);

int tblup_ctx_destroy(tblup_ctx* ctx);

/*
 * Register a train/validation split under `split_id` (replacing any split
 * with that id).  train/valid are animal row ids in the reference's order
 * (evaluator.py:196-203, 316-322, 485-491, 555-561, 413).
 */
int tblup_set_split(tblup_ctx* ctx, int split_id, const int64_t* train, int64_t n_train,
                    const int64_t* valid, int64_t n_valid);

int tblup_drop_split(tblup_ctx* ctx, int split_id);

/*
 * Multi-trait evaluation (BASELINE config 5; build-defined, the reference is
 * single-trait): replace the context's phenotypes with an n_animals x n_traits
 * row-major matrix, 1 <= n_traits <= TBLUP_MAX_TRAITS.  Independent traits with
 * a shared G decouple (G (x) I + lambda I), so one Cholesky per individual
 * serves every trait's right-hand side; each trait's EBVs are exactly the
 * single-trait blup() of that phenotype column (evaluator.py:244-314), and
 * fitness = mean over traits of |pearson(EBV_V,t, y_V,t)|; ebv outputs become
 * batch x n_traits x n_valid.  Drops every registered split (they hold
 * per-trait phenotype vectors): call tblup_set_split again afterwards.
 */
#define TBLUP_MAX_TRAITS 4
int tblup_set_traits(tblup_ctx* ctx, const double* pheno, int64_t n_traits);
int tblup_get_traits(tblup_ctx* ctx, int64_t* n_traits);

/*
 * Evaluate `batch` individuals (one blup() call each, evaluator.py:244-314).
 *   idx      : concatenated selected SNP column indices (duplicates allowed,
 *              any order), length offsets[batch].  numpy fancy-index rules, as the
 *              reference's data[:, indices] (evaluator.py:275/298) applies them to an
 *              IndexIndividual genome (individual.py:93-95, unclipped DE can go
 *              negative): -n_snps <= i < 0 addresses column i + n_snps; any index
 *              outside [-n_snps, n_snps) fails the whole call with TBLUP_ERR_INDEX
 *   offsets  : batch+1 prefix offsets into idx; an individual may have k >= 1
 *   h2       : heritability, lambda = (1-h2)/h2
 *   branch   : TBLUP_BRANCH_*
 *   fitness  : out, batch doubles, |pearson(EBV_V, y_V)| (NaN when undefined)
 *   ebv      : optional out (may be NULL), batch x n_valid predicted breeding values
 *              (batch x n_traits x n_valid after tblup_set_traits)
 * Synchronous; host pointers.  A chained solve (SNP form, small chunks) whose bounded hand-off
 * wait expires does not fail the call: the chunk's factor is solved again by the one-workgroup
 * back substitution, bit-identical to an unexpired run, and counted (tblup_chain_recoveries).
 */
int tblup_eval_batch(tblup_ctx* ctx, int split_id, const int64_t* idx, const int64_t* offsets,
                     int64_t batch, double h2, int branch, double* fitness, double* ebv);

/*
 * Same computation on device-resident inputs/outputs, enqueued on `stream`
 * (a hipStream_t; NULL = the context's own stream) without synchronising.
 * d_idx / d_offsets / d_fitness / d_ebv are device pointers on the
 * context's device; h_offsets is the same batch+1 offsets on the host (used
 * for workspace sizing).  The workspace is shared with other calls on the
 * context: calls must be serialised on one stream.  Negative indices wrap as in
 * tblup_eval_batch; an individual with an index outside [-n_snps, n_snps) gets a NaN
 * fitness and raises the context's index-error flag (read it with tblup_index_error).
 */
int tblup_eval_batch_device(tblup_ctx* ctx, int split_id, const int64_t* d_idx,
                            const int64_t* d_offsets, const int64_t* h_offsets, int64_t batch,
                            double h2, int branch, double* d_fitness, double* d_ebv, void* stream);

/*
 * Every individual against each of n_splits registered splits (IntraGCVBlupParallelEvaluator's
 * k folds, tblup/evaluator.py:509-537, whose fitness is the mean over folds; or any split set):
 * fitness is n_splits x batch row-major (row f = split_ids[f]).  The splits' evaluations are
 * enqueued back to back on one stream with one upload of the index lists and one
 * synchronisation, instead of one tblup_eval_batch round trip per fold.  When the splits partition
 * one animal set (IntraGCV's folds), the exact genotype products are shared: in the SNP-space form
 * C_{T_f} = C_{T_all} - C_{V_f}, in the kernel (GRM) form one A_R A_R^T per individual that every
 * fold's system reads its counts from.  Same numbers as tblup_eval_batch per split, bit for bit.
 * Host pointers, synchronous.
 */
int tblup_eval_folds(tblup_ctx* ctx, const int* split_ids, int n_splits, const int64_t* idx, const int64_t* offsets,
                     int64_t batch, double h2, int branch, double* fitness);

/* Same on device-resident inputs / outputs (d_fitness: n_splits x batch), enqueued on `stream`
 * (NULL = the context's stream) without synchronising; h_offsets as in tblup_eval_batch_device. */
int tblup_eval_folds_device(tblup_ctx* ctx, const int* split_ids, int n_splits, const int64_t* d_idx,
                            const int64_t* d_offsets, const int64_t* h_offsets, int64_t batch, double h2, int branch,
                            double* d_fitness, void* stream);

/*
 * RandomKeyIndividual / CoevolutionIndividual genome decode
 * (tblup/individual.py:154-156, `np.argsort(keys)[-int(length):]`): for each of
 * `batch` key rows of length d, the indices of its k_b = offsets[b+1]-offsets[b]
 * largest keys in ascending key order, written to idx_out[offsets[b] ...] — the
 * (idx, offsets) pair tblup_eval_batch takes.  Equal keys are ordered by index (a
 * stable argsort), so a tie straddling the k-th position selects its largest
 * indices; with continuous keys this is the set numpy's default sort returns.
 * 1 <= k_b <= min(d, 8192).  Host pointers, synchronous.
 */
int tblup_decode_topk(tblup_ctx* ctx, const double* keys, int64_t batch, int64_t d, const int64_t* offsets,
                      int64_t* idx_out);

/*
 * Same on device-resident keys (row stride ld >= d doubles), offsets and output,
 * enqueued on `stream` (NULL = the context's stream); h_offsets is the host copy
 * (validation).  The output feeds tblup_eval_batch_device directly.
 */
int tblup_decode_topk_device(tblup_ctx* ctx, const double* d_keys, int64_t batch, int64_t d, int64_t ld,
                             const int64_t* d_offsets, const int64_t* h_offsets, int64_t* d_idx_out,
                             void* stream);

/*
 * Per-kernel-class timing with HIP events on the launch stream.
 * tblup_set_profiling(ctx, 1) enables recording; tblup_get_profile returns
 * accumulated milliseconds, launch counts and algorithmic flops per class
 * since the last reset (classes: 0 stats, 1 gather, 2 grm, 3 chol_diag,
 * 4 chol_offdiag, 5 solve).  Arrays must hold TBLUP_N_KCLASS entries.
 */
#define TBLUP_N_KCLASS 6
int tblup_set_profiling(tblup_ctx* ctx, int enable);
int tblup_get_profile(tblup_ctx* ctx, double* ms, int64_t* launches, double* flops, double* bytes);
int tblup_reset_profile(tblup_ctx* ctx);

/*
 * Workgroup trace (profiling; enabled by TBLUP_WG_TRACE=1 at tblup_ctx_create): after an
 * evaluation, the Cholesky launches of its last chunk left one record per workgroup,
 * 4 x uint64 {start, end, kind << 56 | I << 40 | individual, J} with s_memrealtime
 * timestamps (100 MHz) and kind 1 diagonal tile, 2 off-diagonal tile (I, J), 3 preparation
 * of diagonal tile I, 4 K_II build.  *n_records = records available; copies min(cap, that).
 */
int tblup_get_wg_trace(tblup_ctx* ctx, uint64_t* out, int64_t cap, int64_t* n_records);

/*
 * Debug / parity readback for ONE individual: runs the pipeline up to
 * `stage` (1 = GRM block K_{RT} incl. lambda on the TT diagonal,
 * 2 = after the tile Cholesky: L in the TT lower triangle) and copies the
 * (n_train + n_valid) x n_train block to `out` (row-major, R = train then
 * valid order), plus z = L^{-1}(y_T - mu) to `z_out` (may be NULL).
 */
int tblup_debug_grm(tblup_ctx* ctx, int split_id, const int64_t* idx, int64_t k, double h2,
                    int branch, int stage, double* out, double* z_out);

/*
 * VanRaden GRM of the selected columns over ALL animals, make_grm(data[:, idx])
 * (tblup/utils.py:7-18): G = W W^T / (2 sum p(1-p)), W = Z - 2p, p = column mean / 2.
 * Exact-integer A A^T on int8 MFMA (2-bit packed rows unpacked into LDS) plus the fp64 rank-1
 * centring (k_grm).  `G` is
 * n_animals x n_animals row-major (host).  Used by the PCA splitter
 * (pca_splitter, evaluator.py:641-663, with idx = every SNP).  Synchronous.
 */
int tblup_grm(tblup_ctx* ctx, const int64_t* idx, int64_t k, double* G);

/*
 * Per-SNP sums over the animal rows `rows` (n_rows ids, any order): sx = sum x,
 * sxx = sum x^2 (exact), sxy = sum x * yc (fp64; yc = the caller's centred phenotypes
 * of those rows), for every SNP of the panel (outputs of length n_snps, host).  The data
 * pass of the seeder's GWAS metric (sklearn f_regression over X[train],
 * tblup/seeder.py:144-160, 202-210).  Synchronous.
 */
int tblup_snp_scan(tblup_ctx* ctx, const int64_t* rows, int64_t n_rows, const double* yc, int64_t* sx,
                   int64_t* sxx, double* sxy);

/*
 * One differential-evolution generation (mutation + binary crossover + clip) for a
 * population of `pop` internal genomes of length L, bit-exact to the reference:
 *   TBLUP_DE_RAND_1            DERandOneEvolver.de_rand_one   tblup/evolver.py:103-138
 *                              donors[i] = (a, b, c):   mutant = a + F (b - c)
 *   TBLUP_DE_CURRENT_TO_BEST_1 DECurrentToBestOneEvolver.de_currenttobest_one  evolver.py:179-221
 *                              donors[i] = (best, a, b): mutant = x + F (best - x) + F (a - b)
 *   crossover (evolver.py:63-82): child_j = mutant_j where u_j < cr or j == fixed[i], else x_j,
 *   u = numpy's legacy np.random.rand(L) for individual i; clip (np.clip(., 0, clip_hi)) when clip.
 * The donors and `fixed` are the caller's python-`random` draws (exclusive_randrange,
 * random.randrange: utils.py:21-36, evolver.py:76).  mt_key / mt_pos hold numpy's global
 * MT19937 state (np.random.get_state()[1:3]) before the generation's first
 * np.random.rand call; on return they hold the state after all pop x 2L outputs, in
 * numpy's own representation (np.random.set_state continues the stream exactly).
 * Host pointers (parents/children: pop x L doubles), synchronous.
 */
enum { TBLUP_DE_RAND_1 = 0, TBLUP_DE_CURRENT_TO_BEST_1 = 1 };
int tblup_de_step(tblup_ctx* ctx, int strategy, const double* parents, int64_t pop, int64_t L,
                  const int32_t* donors, const int64_t* fixed, double F, double cr, int clip, double clip_hi,
                  uint32_t* mt_key, int32_t* mt_pos, double* children);

/* Same with device-resident parents / children (row strides ld, ldc >= L doubles) enqueued on
 * `stream` (NULL = the context's stream); donors, fixed and the MT state are host arrays.
 * Synchronises `stream` before returning (the new MT state is read back). */
int tblup_de_step_device(tblup_ctx* ctx, int strategy, const double* d_parents, int64_t pop, int64_t L, int64_t ld,
                         const int32_t* donors, const int64_t* fixed, double F, double cr, int clip, double clip_hi,
                         uint32_t* mt_key, int32_t* mt_pos, double* d_children, int64_t ldc, void* stream);

/* tblup_de_step_device in two halves: the step and the copy of the new MT state into a
 * page-locked context buffer are enqueued on `stream` without waiting (mt_key is read before
 * returning; mt_pos is passed by value), and tblup_de_state_wait waits for that copy only and
 * writes the state out.  Between the two the caller may enqueue work on the children (the
 * evaluator's decode and evaluation, their copy to the host); one step may be pending at a time.
 * tblup_de_step_device is the two calls back to back. */
int tblup_de_step_device_async(tblup_ctx* ctx, int strategy, const double* d_parents, int64_t pop, int64_t L,
                               int64_t ld, const int32_t* donors, const int64_t* fixed, double F, double cr, int clip,
                               double clip_hi, const uint32_t* mt_key, int32_t mt_pos, double* d_children,
                               int64_t ldc, void* stream);
int tblup_de_state_wait(tblup_ctx* ctx, uint32_t* mt_key, int32_t* mt_pos);

/* tblup_de_step_device_async with a strategy, mutation factor and crossover rate per individual
 * (host arrays of pop): the adaptive evolvers' generation -- SaDE (tblup/evolver.py:407-547) draws
 * each individual's strategy (DE/rand/1 or DE/current-to-best/1, python's random.random() < p)
 * and its crossover rate, with one F per generation.  Same numpy stream layout (one
 * np.random.rand(L) per individual, in order); completed by tblup_de_state_wait. */
int tblup_de_step_device_async_mix(tblup_ctx* ctx, const int32_t* strategies, const double* F, const double* cr,
                                   const double* d_parents, int64_t pop, int64_t L, int64_t ld, const int32_t* donors,
                                   const int64_t* fixed, int clip, double clip_hi, const uint32_t* mt_key,
                                   int32_t mt_pos, double* d_children, int64_t ldc, void* stream);

/* Enqueue dst row i (L doubles, row stride ldd) = the device row d_src_rows[i] (a host array of
 * n device pointers, each to L doubles on this context's device) on `stream` (NULL = the
 * context's stream): one launch per 128 rows.  The DE step's parents gathered from the rows
 * where earlier generations' children still sit on the device (tblup_amd.keystore), as the
 * reference's evolver reads population[i].get_internal_genome() (evolver.py:130-140). */
int tblup_gather_rows(tblup_ctx* ctx, double* d_dst, int64_t n, int64_t L, int64_t ldd, const double* const* d_src_rows,
                      void* stream);

/* Host-only: advance numpy's MT19937 (key[624], pos) state by n_words 32-bit outputs
 * (GF(2) jump-ahead; used to check the DE step's stream arithmetic without a GPU). */
int tblup_mt19937_jump(const uint32_t* key, int32_t pos, uint64_t n_words, uint32_t* key_out, int32_t* pos_out);

/* Host-only: one DE generation's python-`random` draws, the loops of DERandOneEvolver /
 * DECurrentToBestOneEvolver.evolve that feed tblup_de_step: per individual i the donors
 * (exclusive_randrange, utils.py:21-36; rand/1: a, b, c, evolver.py:118-121; current-to-best/1:
 * a, b beside `best`, evolver.py:199-203, donors[i] = (best, a, b)) and then fixed[i] =
 * random.randrange(0, L) (evolver.py:76).  py_mt / py_index hold CPython's MT19937 state
 * (random.getstate()[1]: 624 words, then the index) and are advanced in place exactly as the
 * python loop advances it (random.setstate continues the stream).  best = -1 for rand/1.
 * Needs 4 <= pop (smaller populations raise the reference's assertion: keep those in python). */
int tblup_de_donors(int strategy, int64_t pop, int64_t L, int32_t best, uint32_t* py_mt, int32_t* py_index,
                    int32_t* donors, int64_t* fixed);

/* Index-error flag of the device entry points: synchronises `stream` (NULL = the context's
 * stream), sets *flag = 1 if any individual evaluated since the last call had an index
 * outside [-n_snps, n_snps) (its fitness is NaN), and clears the flag. */
int tblup_index_error(tblup_ctx* ctx, void* stream, int* flag);

/* Solve-error flag: the chained back substitution (SNP form, small batches) hands block rows
 * between workgroups and bounds every wait; a wait that gives up leaves the batch's fitnesses
 * invalid.  The synchronous entries (tblup_eval_batch, tblup_eval_folds) recover by themselves
 * (the chunk's solve re-run through k_solve; tblup_chain_recoveries counts it) and never raise
 * this flag; after device entries read it here: synchronises `stream` (NULL = the context's
 * stream), *flag = 1 if a wait expired since the last read, clears it -- the caller re-evaluates
 * through a synchronous entry (the drop-in evaluator does).  (The reference has no such failure
 * mode -- a dead worker hangs its parent, tblup/evaluator.py:397-398; here it is an error or a
 * recovery, never a silent NaN.) */
int tblup_solve_error(tblup_ctx* ctx, void* stream, int* flag);

/* Number of chunks the synchronous entries re-solved after an expired chained-solve wait since
 * the context was created (each one cost one extra back substitution). */
int tblup_chain_recoveries(tblup_ctx* ctx, int64_t* count);

/* Both status words without synchronising: enqueues on `stream` (NULL = the context's stream) a
 * copy of {index error, solve error} (2 x int32, nonzero = raised) into `host_status`
 * (page-locked host memory) and clears them on the device; valid once the stream has passed
 * that point (the caller's event). */
int tblup_status_async(tblup_ctx* ctx, void* stream, int32_t* host_status);

/* Page-lock `bytes` of existing host memory at `ptr` for DMA (hipHostRegister) / release it.  The
 * multi-rank generation path registers the node-shared memory segments the ranks' shards of the
 * children's genomes are copied into (tblup_amd/shmrows.py), so each rank's device-to-host copy of
 * its shard runs as a DMA straight into the shared rows. */
int tblup_host_register(void* ptr, int64_t bytes);
int tblup_host_unregister(void* ptr);

/* Device memory currently held by the context (bytes). */
int tblup_mem_info(tblup_ctx* ctx, int64_t* bytes_in_use);

#ifdef __cplusplus
}
#endif

#endif /* TBLUP_GPU_H */
