"""Benchmark: GBLUP fitness evals/s on BASELINE config 2 at N = 1 (2000 animals x 50k SNPs,
panel k = 1000, DE population 256 on one GPU) and config 3 at N > 1 (the same panel, DE
population 1024 sharded over the N GPUs: 128 per GPU at N = 8), one process per GPU.

A "step" is one generation's fitness evaluation of the population: for every
individual the exact-integer system tiles (SNP-space form at k < n_T, as sklearn's Ridge
solves it, on FP4 MFMA with genotypes as e2m1 nibbles; kernel/GRM form otherwise, int8
MFMA), the fused fp64 tile
Cholesky, back substitution, prediction and Pearson fitness, plus (N > 1) the RCCL
all-gather of the fp64 fitness vector.  Inputs
(genotypes, split, the population's decoded index sets) are resident in HBM
before timing starts.  Weak scaling: every rank evaluates its own 256
individuals per GPU: with --scaling strong (default) the configuration's population is the
WHOLE job's and every rank evaluates its contiguous shard (tblup_amd.distributed.shard_range);
with --scaling weak it is every rank's own.  Individual i's keys come from its own seed, so the
population -- and the all-gathered fitness vector (`fitness_checksum`) -- is the same for any N.

    python bench.py --gpus N --steps K --warmup W [--config auto|config2|config3|...] [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (n animals, P SNPs, panel k, DE population, n_train, n_valid)
    "config2": (2000, 50_000, 1000, 256, 1280, 320),
    "config3": (2000, 50_000, 1000, 1024, 1280, 320),  # sharded over the node's GPUs (BASELINE config 3)
    "config1": (200, 1000, 100, 32, 128, 32),
    "config4": (5000, 600_000, 5000, 256, 3200, 800),
    "config5": (2000, 50_000, 1000, 256, 1280, 320),   # 3 traits (BASELINE config 5, build-defined)
}
TRAITS = {"config5": 3}

# the bench's own parity bound on the fitness (Pearson r) of every timed individual the CPU
# baseline covered (the parity tests' FIT_ATOL; north_star asks 1e-5 relative on the EBVs)
PARITY_ATOL = 1e-9

# BASELINE.json's metric, verbatim
METRIC = "GBLUP fitness evals/sec (whole node), 2k\u00d750k SNP, DE pop=256; 1/2/4/8 GPUs"

# gfx950 peaks.  "measured": tools/mfma_peak.hip on the box (profiles/r02_mfma_peak.json, again
# profiles/r03c_mfma_peak.json: f64 72.8 TF at 2 waves per SIMD; the
# microarchitecture guide has no fp64 MFMA row): back-to-back MFMAs on independent accumulators,
# 2 waves per SIMD, random operands, at the clock the chip holds under that load (~2.36 GHz).
# "spec": AMD's MI355X dense figures (2.4 GHz).  HBM: the guide's 8 TB/s.
PEAKS = {
    "fp64_mfma_tflops": 72.7, "fp64_mfma_tflops_spec": 78.6,
    "fp32_mfma_tflops": 154.6, "fp32_mfma_tflops_spec": 157.3,
    "int8_mfma_tops": 4140.0, "int8_mfma_tops_spec": 5033.0,
    # FP4 16x16x128 (e2m1 A and B, fp32 accumulate): tools/fp4_probe.hip, 4 waves per SIMD
    # (profiles/r02b_fp4_probe.json, r03c: 8.73 POPS); spec: the guide's ~10 PF dense FP4
    "fp4_mfma_tops": 8811.0, "fp4_mfma_tops_spec": 10066.0,
    "hbm_gbs": 8000.0,
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="auto", choices=["auto"] + sorted(CONFIGS),
                    help="auto: config2 on one GPU, config3 (pop 1024 sharded) on N > 1")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the population is the whole job's, sharded over the ranks; weak: per rank")
    ap.add_argument("--pop", type=int, default=None,
                    help="population (whole job under --scaling strong, per rank under weak; default: the config's)")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--h2", type=float, default=0.4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target wall time of the CPU baseline sample")
    ap.add_argument("--profile-json", default=None, help="write the per-kernel-class event timing here")
    ap.add_argument("--no-events", action="store_true", help="time without per-kernel HIP events (no roofline)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--pmc-mfma-json", default=os.path.join(ROOT, "profiles", "pmc_mfma.json"),
                    help="rocprofv3 MFMA-busy summary (tools/pmc_mfma.py) for the roofline's mfma_busy")
    ap.add_argument("--rocprof-stats", default=os.path.join(ROOT, "profiles", "kernel_stats.csv"),
                    help="rocprofv3 --kernel-trace --stats summary of this bench (config 2): the roofline's "
                         "frac_rocprof from its average duration of the dominant kernel")
    return ap.parse_args()


def make_workload(cfg, seed, lo, hi, traits=1):
    """The panel, split and individuals lo..hi-1 of the population (individual i's RandomKey
    keys from its own seed: the same individuals whatever the sharding)."""
    n, P, k, _, nT, nV = cfg
    rng = np.random.default_rng(seed)
    maf = rng.uniform(0.05, 0.5, size=P)                  # SURVEY.md section 8d synthetic panel
    geno = rng.binomial(2, maf, size=(n, P)).astype(np.int8)
    pheno = rng.standard_normal(n) if traits == 1 else rng.standard_normal((n, traits))
    perm = np.random.default_rng(seed + 1).permutation(n)
    T, V = perm[:nT], perm[nT:nT + nV]
    keys = np.stack([np.random.default_rng((seed, 100, i)).uniform(size=P) for i in range(lo, hi)])
    genomes = np.argsort(keys, axis=1)[:, -k:]            # RandomKeyIndividual decode (individual.py:154-156)
    return geno, pheno, T, V, genomes, keys


# ----------------------------------------------------------------------------- CPU baseline
_CPU = {}


def _cpu_init():
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)


def _cpu_eval(i):
    from oracle.blup_oracle import blup
    d = _CPU
    y = d["pheno"]
    g = d["genomes"][i % len(d["genomes"])]
    if y.ndim == 1:
        return blup(g, d["T"], d["V"], d["data"], y, d["h2"])
    # multi-trait: the reference is single-trait, so one eval = one blup per trait
    return float(np.mean([blup(g, d["T"], d["V"], d["data"], y[:, t], d["h2"]) for t in range(y.shape[1])]))


def cpu_baseline(geno, pheno, T, V, genomes, h2, target_s):
    """The oracle's numpy port of the reference evaluator (same blup dispatch, float64
    genotypes, one single-threaded worker process per core; cf. generate_sbs.py:25
    OMP_NUM_THREADS=1), timed on a bounded sample of the same workload."""
    import multiprocessing as mp
    from threadpoolctl import threadpool_limits
    from oracle.blup_oracle import blup

    host_cpus = len(os.sched_getaffinity(0))
    # at most 16 workers: the GPU box's CPU share per GPU (its affinity mask may show the whole host)
    cores = max(1, min(16, host_cpus))
    _CPU.update(data=geno.astype(np.float64), pheno=pheno, T=T, V=V, genomes=genomes, h2=h2)
    with threadpool_limits(1):
        t0 = time.perf_counter()
        for i in range(2):
            _cpu_eval(i)
        per_eval = (time.perf_counter() - t0) / 2
    count = int(max(cores, min(20_000, target_s * cores / max(per_eval, 1e-6))))
    ctx = mp.get_context("fork")
    with ctx.Pool(cores, initializer=_cpu_init) as pool:
        pool.map(_cpu_eval, range(cores))        # warm the workers
        t0 = time.perf_counter()
        res = pool.map(_cpu_eval, range(count), chunksize=max(1, count // (4 * cores)))
        dt = time.perf_counter() - t0
    _CPU.clear()
    # the oracle fitness of every benchmark individual the sample covered (evaluation i is
    # individual i % pop): the timed GPU fitnesses are checked against these after the timed passes
    oracle_fit = {i: float(res[i]) for i in range(min(count, len(genomes)))}
    return {"value": count / dt, "unit": "evals/s", "cores": cores, "host_cpus_affinity": host_cpus,
            "os_cpu_count": os.cpu_count(), "kind": "port", "_oracle_fit": oracle_fit,
            "sample": f"{count} evaluations of the config workload (k={genomes.shape[1]}"
                      + (f", {pheno.shape[1]} traits: one blup per trait" if pheno.ndim == 2 else "")
                      + ") by the numpy oracle "
                      f"port of BlupParallelEvaluator.blup, {cores} single-threaded worker processes (of {host_cpus} "
                      f"CPUs in this process's affinity mask), {dt:.1f} s"}


def fitness_parity(fit, oracle_fit, pop):
    """Max |GPU - oracle| fitness over the individuals the CPU baseline evaluated (both NaN counts
    as equal -- scipy's pearsonr of a constant prediction; one NaN is a mismatch: inf)."""
    idx_cov = np.array(sorted(oracle_fit), dtype=np.int64)
    ref = np.array([oracle_fit[i] for i in idx_cov], dtype=np.float64)
    got = np.asarray(fit, dtype=np.float64)[idx_cov]
    diff = np.where(np.isnan(ref) & np.isnan(got), 0.0, np.abs(got - ref))
    worst = float(np.max(np.where(np.isnan(diff), np.inf, diff))) if len(diff) else None
    return {"max_abs_fit": worst, "covered": int(len(idx_cov)), "of": int(pop), "atol": PARITY_ATOL,
            "oracle": "oracle/blup_oracle.py blup (float64 numpy), the CPU baseline's own evaluations"}


# ----------------------------------------------------------------------------- main
def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from tblup_amd.distributed import shard_range
    config = args.config if args.config != "auto" else ("config2" if world == 1 else "config3")
    cfg = CONFIGS[config]
    n, P, k, pop_default, nT, nV = cfg
    if args.scaling == "strong":
        total = args.pop or pop_default
        lo, hi = shard_range(total, rank, world)
    else:
        per = args.pop or pop_default
        total, lo, hi = per * world, per * rank, per * (rank + 1)
    pop = hi - lo                                          # this rank's shard
    shard_max = max(b - a for a, b in (shard_range(total, r, world) for r in range(world))) \
        if args.scaling == "strong" else pop

    traits = TRAITS.get(config, 1)
    geno, pheno, T, V, genomes, keys = make_workload(cfg, args.seed, lo, hi, traits)
    if k > 8192:
        keys = None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(geno, pheno, T, V, genomes, args.h2, args.cpu_seconds)

    import torch
    import torch.distributed as dist
    from tblup_amd import distributed as tdist
    # one process per GPU; more ranks than GPUs (a rehearsal of the N > 1 path on a smaller box,
    # TBLUP_DIST_BACKEND=gloo) share them round-robin
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    # the same process-group set-up and all-gather the drop-in evaluator uses
    # (ParallelEvaluator.__enter__ -> init_from_env; _fitness -> allgather)
    os.environ.setdefault("TBLUP_DIST_BACKEND", "nccl")
    owns_group = tdist.init_from_env(device)
    from tblup_amd.engine import GpuBlupEngine, concat_genomes

    eng = GpuBlupEngine(geno, pheno, device=device)
    sid = eng.split_id(T, V)
    idx, off = concat_genomes(list(genomes))
    d_idx = torch.from_numpy(idx).cuda()
    d_off = torch.from_numpy(off).cuda()
    # the all-gather moves equal blocks: shards padded to the largest one
    d_fit = torch.full((shard_max,), float("nan"), dtype=torch.float64, device="cuda")
    full = torch.empty(shard_max * world, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, args.h2, d_fit.data_ptr(),
                            stream_ptr=stream.cuda_stream)
        if world > 1:
            tdist.allgather_device(full, d_fit)

    def timed_steps():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # pass 1: the metric, uninstrumented (per-launch HIP events add ~5% of launch gaps)
    elapsed = timed_steps()
    # pass 2: the same K steps with a HIP event pair around every launch, on the stream each
    # kernel runs on: per-kernel-class time, the roofline's average launch duration
    eng.reset_profile()
    eng.set_profiling(not args.no_events)
    elapsed_events = timed_steps()
    eng.set_profiling(False)
    prof = eng.profile()
    # every timed evaluation must have succeeded: raises for an index error or an expired
    # chained-solve wait (tblup_solve_error), never reports a rate over invalid fitnesses
    eng.check_device_status(stream.cuda_stream)

    # GPU genome decode of the same population (RandomKeyIndividual.genome, individual.py:154-156)
    # from device-resident keys: reported beside the metric, not part of it
    decode_ms = de_ms = None
    if keys is not None:
        d_keys = torch.from_numpy(keys).cuda()
        d_dec = torch.empty(int(off[-1]), dtype=torch.int64, device="cuda")
        for _ in range(2):
            eng.decode_randkey_device(d_keys.data_ptr(), pop, P, P, d_off.data_ptr(), off, d_dec.data_ptr(),
                                      stream.cuda_stream)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(5):
            eng.decode_randkey_device(d_keys.data_ptr(), pop, P, P, d_off.data_ptr(), off, d_dec.data_ptr(),
                                      stream.cuda_stream)
        torch.cuda.synchronize()
        decode_ms = (time.perf_counter() - t1) / 5 * 1e3
        if not np.array_equal(d_dec.cpu().numpy(), idx):
            raise RuntimeError("GPU decode differs from the host argsort decode")
        # GPU DE generation step on the same device-resident keys (tblup_amd.evolver,
        # evolver.py:103-157): DE/rand/1 + binary crossover with numpy's MT19937 stream
        # jumped per individual; reported beside the metric, not part of it
        from tblup_amd.evolver import GpuDEStep
        de = GpuDEStep.get(device)
        drng = np.random.default_rng(args.seed + 7)
        donors = np.stack([drng.choice(pop, 3, replace=False) for _ in range(pop)]).astype(np.int32)
        fixed = drng.integers(0, P, size=pop)
        for _ in range(2):
            de.step_device(0, d_keys, donors, fixed, 0.5, 0.8, False, P - 1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(5):
            de.step_device(0, d_keys, donors, fixed, 0.5, 0.8, False, P - 1)
        torch.cuda.synchronize()
        de_ms = (time.perf_counter() - t1) / 5 * 1e3
        del d_keys, d_dec
    # the same two host steps the reference runs per generation (numpy evolve loop, argsort
    # decode), timed beside them on rank 0 (oracle restatement; reported, not the metric)
    host_ref = None
    if cpu is not None and keys is not None:
        import random as _random
        from oracle import de_oracle
        rows = [keys[i] for i in range(pop)]
        _random.seed(args.seed)
        t1 = time.perf_counter()
        de_oracle.de_generation(rows, [0.0] * pop, 1, "de_rand_1", P, 0.8, 0.5, False)
        t2 = time.perf_counter()
        [np.argsort(r)[-k:] for r in rows]
        t3 = time.perf_counter()
        host_ref = {"de_step_ms": round((t2 - t1) * 1e3, 2), "decode_ms": round((t3 - t2) * 1e3, 2), "cores": 1,
                    "kind": "port", "sample": f"one generation of {pop} x {P} keys (evolver.py:140-157, "
                                              "individual.py:154-156), numpy on one host core"}
    if world > 1:
        fit_all = full.cpu().numpy().reshape(world, shard_max)
        spans = [shard_range(total, r, world) if args.scaling == "strong" else (pop * r, pop * (r + 1))
                 for r in range(world)]
        fit = np.concatenate([fit_all[r, :b - a] for r, (a, b) in enumerate(spans)])
    else:
        fit = d_fit.cpu().numpy()[:pop]
    # the timed fitnesses against the oracle's for every individual the CPU baseline evaluated
    # (evaluator.py:298-314 restated in oracle/blup_oracle.py): the line proves its own results
    parity = None
    if cpu is not None:
        parity = fitness_parity(fit, cpu.pop("_oracle_fit"), pop)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_evals = total * args.steps
    value = total_evals / elapsed

    # roofline of the dominant kernel class, from live HIP-event timing over the timed region.
    # The library counts the flops of the padded 128-row tiles (ns = 1024 at k = 1000); the
    # algorithmic work of the Cholesky classes scales as ns^3, so frac uses (k / ns)^3 of it.
    if args.no_events:
        prof = {c: {"ms": 1e-9, "launches": 0, "flops": 0.0, "bytes": 0.0} for c in prof}
    dom = max(prof, key=lambda c: prof[c]["ms"])
    pd = prof[dom]
    ns = -(-k // 128) * 128 if k < nT else -(-nT // 128) * 128       # SNP-space form at k < n_T (evaluator.py:288-314)
    unpad = (min(k, nT) / ns) ** 3
    peak_spec = None
    if dom in ("chol_diag", "chol_offdiag"):
        bound, unit = "mfma", "TFLOP/s"
        peak, peak_spec = PEAKS["fp64_mfma_tflops"], PEAKS["fp64_mfma_tflops_spec"]
        achieved = pd["flops"] * unpad / (pd["ms"] * 1e-3) / 1e12
    elif dom == "grm":
        bound, unit = "mfma", "TOP/s"
        sys_fmt = "fp4" if k < nT else "int8"
        peak, peak_spec = PEAKS[sys_fmt + "_mfma_tops"], PEAKS[sys_fmt + "_mfma_tops_spec"]
        achieved = pd["flops"] / (pd["ms"] * 1e-3) / 1e12
    else:
        bound, peak, unit, achieved = "hbm", PEAKS["hbm_gbs"], "GB/s", pd["bytes"] / (pd["ms"] * 1e-3) / 1e9
    traffic = None
    if os.path.isfile(args.pmc_json):
        try:
            pmc = json.load(open(args.pmc_json))
            if (pmc.get("config") == config and pmc.get("pop_per_gpu", 256) == shard_max and world == 1
                    and dom in pmc.get("per_launch_bytes", {})):
                traffic = pmc["per_launch_bytes"][dom]
        except (ValueError, OSError):
            traffic = None
    # the same work over rocprofv3's average duration of the dominant kernel (the committed
    # --kernel-trace --stats summary of this bench, config 2): the profiler-timed fraction beside
    # the live HIP-event one
    rocprof = None
    kname = {"chol_offdiag": "k_chol_offdiag", "chol_diag": "k_chol_diag", "solve": "k_solve"}.get(dom)
    # only when the stats file was taken on this workload: its sidecar (<stats>.meta.json, written
    # by tools/collect_evidence.sh) names the config and the per-GPU population it ran
    stats_meta = None
    try:
        stats_meta = json.load(open(os.path.splitext(args.rocprof_stats)[0] + ".meta.json"))
    except (OSError, ValueError):
        stats_meta = None
    stats_match = (stats_meta is not None and stats_meta.get("config") == config
                   and stats_meta.get("pop_per_gpu") == shard_max and world == 1)
    if kname and stats_match and os.path.isfile(args.rocprof_stats) and pd["launches"]:
        import csv
        tot_ns, calls = 0.0, 0   # every instantiation of the kernel (k_chol_offdiag<true> / <false>, ...)
        with open(args.rocprof_stats) as f:
            for row in csv.DictReader(f):
                if "::" + kname + "(" in row["Name"] or "::" + kname + "<" in row["Name"]:
                    tot_ns += float(row["TotalDurationNs"])
                    calls += int(row["Calls"])
        if calls:
            avg_s = tot_ns / calls * 1e-9
            per_launch = (pd["flops"] * unpad if bound == "mfma" else pd["bytes"]) / pd["launches"]
            ach = per_launch / avg_s / (1e12 if bound == "mfma" else 1e9)
            rocprof = {"avg_launch_ms": round(avg_s * 1e3, 4), "achieved": round(ach, 3),
                       "frac": round(ach / peak, 4), "calls": calls,
                       "source": os.path.relpath(args.rocprof_stats, ROOT)}
    mfma_busy = None   # PMC: fraction of SIMD cycles with an MFMA in flight (separate pass)
    if os.path.isfile(args.pmc_mfma_json):
        try:
            pm = json.load(open(args.pmc_mfma_json))
            if (pm.get("config") == config and pm.get("pop_per_gpu", 256) == shard_max and world == 1
                    and dom in pm.get("per_class", {})):
                mfma_busy = pm["per_class"][dom]["mfma_busy"]
        except (ValueError, OSError, KeyError):
            mfma_busy = None
    # Whole-step lower bound of the algorithm run, per GPU: the exact system tiles (lower
    # triangle: k^2 n_T ops; FP4 MFMA in the SNP-space form, int8 in the kernel form), the fp64
    # Cholesky (k^3 / 3), one read of the factor for the back substitution (k^2 / 2 doubles),
    # each at its measured peak.
    m_sys = min(k, nT)
    sys_peak = PEAKS["fp4_mfma_tops"] if k < nT else PEAKS["int8_mfma_tops"]
    t_int8 = pop * float(m_sys) ** 2 * (nT if k < nT else k) / (sys_peak * 1e12)
    t_fp64 = pop * float(m_sys) ** 3 / 3.0 / (PEAKS["fp64_mfma_tflops"] * 1e12)
    t_hbm = pop * float(m_sys) ** 2 / 2.0 * 8.0 / (PEAKS["hbm_gbs"] * 1e9)
    step_bound_ms = (t_int8 + t_fp64 + t_hbm) * 1e3
    # north star: "fraction of the fp32 MFMA roofline" with SURVEY.md 8(d)'s canonical
    # F(k) = 2 k n_T (n_T + n_V) + n_T^3 / 3 + 2 n_T^2 + 2 n_V n_T flops per eval (the dual GRM
    # form in fp32).  The build runs the cheaper exact form (int8 system, k-row fp64 Cholesky),
    # so this ratio can exceed 1: it says how far the canonical algorithm's flop rate is beaten.
    f_canon = 2.0 * k * nT * (nT + nV) + nT ** 3 / 3.0 + 2.0 * nT ** 2 + 2.0 * nV * nT
    roofline = {"bound": bound, "kernel": dom, "achieved": round(achieved, 3), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 4),
                "timing": "hip-events: an event pair around every launch on its stream, timed pass 2",
                "rocprof": rocprof, "traffic": traffic, "mfma_busy": mfma_busy,
                "launches": pd["launches"], "avg_launch_ms": round(pd["ms"] / max(pd["launches"], 1), 4),
                "peak_source": "measured on the box (tools/mfma_peak.hip, profiles/r02_mfma_peak.json, r03c_mfma_peak.json)",
                "peak_spec": peak_spec, "frac_spec": None if peak_spec is None else round(achieved / peak_spec, 4),
                "flops": "algorithmic: library tile count x (k/ns)^3 = %.4f" % unpad,
                "step": {"lower_bound_ms": round(step_bound_ms, 4), "system_tiles_ms": round(t_int8 * 1e3, 4),
                         "system_tiles_mfma": "fp4" if k < nT else "int8",
                         "fp64_ms": round(t_fp64 * 1e3, 4), "hbm_ms": round(t_hbm * 1e3, 4)},
                "canonical_flop_rate_over_fp32_peak": None}
    step_ms = {c: round(prof[c]["ms"] / args.steps, 4) for c in prof}

    if args.profile_json and rank == 0:
        with open(args.profile_json, "w") as f:
            json.dump({"config": config, "steps": args.steps, "profile": prof, "per_step_ms": step_ms,
                       "elapsed_s": elapsed}, f, indent=1)
    roofline["step"]["frac"] = round(roofline["step"]["lower_bound_ms"] / (elapsed / args.steps * 1e3), 4)
    # not a roofline fraction: SURVEY 8(d)'s canonical dual-form fp32 flop count per eval (which the
    # build does not run) times the eval rate, over the fp32 MFMA peak -- above 1 because the
    # build's exact SNP-space form needs ~3.4x fewer flops than the canonical count
    roofline["canonical_flop_rate_over_fp32_peak"] = round(f_canon * value / world / (PEAKS["fp32_mfma_tflops"] * 1e12), 4)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2), "unit": "evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": ("fp4 e2m1 system tiles (exact integer genotype products, fp32 accumulate)" if k < nT else
                      "int8 GRM (exact int32 accumulate)") + " + f64 Cholesky/solve",
            "data": "synthetic (Binomial(2, U(0.05,0.5)) genotypes, N(0,1) phenotype, RandomKey individuals)",
            "config": {"workload": f"{config}: {n} animals x {P} SNPs, panel k={k}, DE pop {total} "
                                   f"({shard_max} per GPU), n_train={nT}, n_valid={nV}, h2={args.h2}"
                                   + (f", {traits} traits (one Cholesky, {traits} RHS)" if traits > 1 else ""),
                       "pop_total": total, "pop_per_gpu": shard_max,
                       "parallelism": f"population sharded over {world} GPU(s) ({args.scaling} scaling)"
                                      + (f", {tdist.backend_name()} fitness all-gather" if world > 1 else "")},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernel_ms_per_step": step_ms,
            "ms_per_step_with_events": round(elapsed_events / args.steps * 1e3, 4),
            "gpu_decode_ms": None if decode_ms is None else round(decode_ms, 4),
            "gpu_de_step_ms": None if de_ms is None else round(de_ms, 4),
            "host_reference_ms": host_ref,
            "fitness_checksum": float(np.nansum(fit)),
            "parity_max_abs_fit": None if parity is None else parity["max_abs_fit"],
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
        if parity is not None and not (parity["max_abs_fit"] is not None and parity["max_abs_fit"] <= PARITY_ATOL):
            print(f"bench: GPU fitness differs from the oracle by {parity['max_abs_fit']} > {PARITY_ATOL}",
                  file=sys.stderr)
            sys.exit(3)
    eng.close()
    if owns_group:
        tdist.destroy()


if __name__ == "__main__":
    main()
