"""The batch shapes the benchmark actually runs, pinned as wholes, and the
chained solve's failure mode.

* Config 5 at pop 256: 3 traits, SNP-space form, B > 160, so the one-workgroup-per-individual
  solve's multi-trait primal branch (k_solve<3>) -- oracle samples per trait at 1e-9 and bit
  identity with the chained solve forced on (TBLUP_SOLVE_CHAIN=1).
* Config 3's per-GPU shard at N = 8 (B = 128 at the config-2 shape) and N = 32 shards (B = 32):
  every automatic small-batch policy at once (ahead P-units with makespan slicing, D-units beside
  the diagonal, last-term mode at B <= 64, the chained solve) -- oracle samples and bit identity
  with every policy off (TBLUP_AHEAD=0 TBLUP_SOLVE_CHAIN=0 TBLUP_DIAG_D=0 TBLUP_LAST_TERM=0
  TBLUP_DIAG_E=0).
* A chained-solve hand-off wait that expires is recovered by the host entries (the chunk's factor
  re-solved through k_solve, same bits) or raises the device status word, which the drop-in
  evaluator's speculative path answers by re-evaluating through the host entry -- never a silent
  NaN -- and the next call on the same context is clean (TBLUP_CHAIN_DEBUG forces expiries: a
  lowered poll bound and a late producer unit).
  Reference behaviour being replaced: a dead worker hangs its parent (tblup/evaluator.py:397-398).
"""
import os

import numpy as np
import pytest

from oracle import blup_oracle as O

pytestmark = pytest.mark.gpu

EBV_RTOL = 1e-9
FIT_ATOL = 1e-9
KNOBS_OFF = {"TBLUP_AHEAD": "0", "TBLUP_SOLVE_CHAIN": "0", "TBLUP_DIAG_D": "0", "TBLUP_LAST_TERM": "0",
             "TBLUP_DIAG_E": "0"}


def _relmax(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


class _env:
    """Temporarily set environment variables (read by tblup_ctx_create)."""

    def __init__(self, env):
        self.env = env

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.env}
        os.environ.update(self.env)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def panel(gpu):
    """BASELINE config-2 panel: 2000 animals x 50k SNPs, T 1280 / V 320, RandomKey genomes k = 1000."""
    rng = np.random.default_rng(2)
    n, P = 2000, 50_000
    geno = O.synth_geno(rng, n, P)
    pheno = rng.standard_normal(n)
    perm = np.random.default_rng(3).permutation(n)
    T, V = perm[:1280], perm[1280:1600]
    keys = np.random.default_rng(4).uniform(size=(256, P))
    genomes = [O.decode_randkeys(k, 1000) for k in keys]
    Y = np.stack([pheno, rng.standard_normal(n), rng.standard_normal(n)], axis=1)
    return dict(geno=geno, pheno=pheno, T=T, V=V, genomes=genomes, Y=Y)


def _run(p, genomes, env=None, traits=False):
    from tblup_amd.engine import GpuBlupEngine
    with _env(env or {}):
        with GpuBlupEngine(p["geno"], p["Y"] if traits else p["pheno"], device=0) as eng:
            return eng.evaluate(genomes, p["T"], p["V"], 0.4, return_ebv=True)


def test_config5_pop256_primal_multitrait_solve(panel):
    """Config 5 as benchmarked: 256 individuals x 3 traits in one batch (k_solve<3>, SNP form)."""
    p = panel
    fit, ebv = _run(p, p["genomes"], traits=True)
    assert ebv.shape == (256, 3, 320)
    for i in (0, 97, 200, 255):
        fs = []
        for tr in range(3):
            f, e = O.blup_grm_form(p["genomes"][i], p["T"], p["V"], p["geno"], p["Y"][:, tr], 0.4)
            assert _relmax(ebv[i, tr], e) <= EBV_RTOL, (i, tr)
            fs.append(f)
        assert abs(fit[i] - np.mean(fs)) <= FIT_ATOL, i
    for pull in ("0", "1"):   # the chained solve's push and pull units
        chained = _run(p, p["genomes"], {"TBLUP_SOLVE_CHAIN": "1", "TBLUP_SOLVE_PULL": pull}, traits=True)
        np.testing.assert_array_equal(chained[0], fit)
        np.testing.assert_array_equal(chained[1], ebv)


@pytest.mark.parametrize("B", [128, 32, 96, 160, 192])
def test_config3_shard_auto_policies(panel, B):
    """B individuals in one batch with every automatic schedule policy at once, against the
    oracle and against every policy switched off, bit for bit.  (96 / 160: E-units covering
    columns in part, their tiles dispatched last; 128: in part and whole; 32: whole; 192: the
    chained solve's pull units at their largest batch.)"""
    p = panel
    genomes = p["genomes"][:B]
    fit, ebv = _run(p, genomes)
    off = _run(p, genomes, KNOBS_OFF)
    np.testing.assert_array_equal(off[0], fit)
    np.testing.assert_array_equal(off[1], ebv)
    for i in sorted({0, B // 2, B - 1}):
        f, e = O.blup_grm_form(genomes[i], p["T"], p["V"], p["geno"], p["pheno"], 0.4)
        assert abs(fit[i] - f) <= FIT_ATOL, i
        assert _relmax(ebv[i], e) <= EBV_RTOL, i


def test_chain_sync_modes_bit_identical(panel):
    """The chained solve's two hand-off protocols (sc1 loads/stores; acquire/release atomics,
    TBLUP_CHAIN_SYNC=1) give the same bits."""
    p = panel
    genomes = p["genomes"][:24]
    a = _run(p, genomes, {"TBLUP_SOLVE_CHAIN": "1", "TBLUP_CHAIN_SYNC": "0"})
    b = _run(p, genomes, {"TBLUP_SOLVE_CHAIN": "1", "TBLUP_CHAIN_SYNC": "1"})
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("pull", ["1", "0"])
def test_chained_solve_expiry_recovers(panel, pull):
    """TBLUP_CHAIN_DEBUG=spin,delay,shots: the next `shots` chained solves poll at most `spin`
    times while one producer sleeps `delay` rounds, so a wait expires.  Host entry: the call
    re-solves the chunk's factor through k_solve and returns the reference bits (counted by
    tblup_chain_recoveries); device entry: the solve-error flag; then the same context is clean.
    Both kinds of chained-solve unit: pull (beta_J hand-offs) and push (tile products)."""
    import torch
    from tblup_amd.engine import GpuBlupEngine, concat_genomes
    p = panel
    genomes = p["genomes"][:8]                  # SNP form, B = 8 <= 160: the chained solve
    ref = _run(p, genomes)
    with _env({"TBLUP_CHAIN_DEBUG": "1000,20000,2", "TBLUP_SOLVE_PULL": pull}):
        eng = GpuBlupEngine(p["geno"], p["pheno"], device=0)
    try:
        fit, ebv = eng.evaluate(genomes, p["T"], p["V"], 0.4, return_ebv=True)   # shot 1: recovered
        np.testing.assert_array_equal(fit, ref[0])
        np.testing.assert_array_equal(ebv, ref[1])
        assert eng.chain_recoveries() == 1
        # device entry (shot 2): no synchronous failure, the status word is raised instead
        sid = eng.split_id(p["T"], p["V"])
        idx, off = concat_genomes(genomes)
        d_idx, d_off = torch.from_numpy(idx).cuda(), torch.from_numpy(off).cuda()
        d_fit = torch.empty(len(genomes), dtype=torch.float64, device="cuda")
        s = torch.cuda.Stream()
        eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr(),
                            stream_ptr=s.cuda_stream)
        assert eng.solve_error(s.cuda_stream)
        assert not eng.solve_error(s.cuda_stream)          # cleared by the read
        # the debug shots are used up: the same context is clean again, host and device entries
        fit, ebv = eng.evaluate(genomes, p["T"], p["V"], 0.4, return_ebv=True)
        np.testing.assert_array_equal(fit, ref[0])
        np.testing.assert_array_equal(ebv, ref[1])
        assert eng.chain_recoveries() == 1
        eng.evaluate_device(sid, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4, d_fit.data_ptr(),
                            stream_ptr=s.cuda_stream)
        eng.check_device_status(s.cuda_stream)
        np.testing.assert_array_equal(d_fit.cpu().numpy(), ref[0])
        # IntraGCV folds (host entry, fused): an expiry there recovers the same way
        folds = [(p["T"][:1024], p["V"]), (p["T"][256:], p["V"])]
        ref_f = eng.evaluate_folds(genomes, folds, 0.4)
    finally:
        eng.close()
    with _env({"TBLUP_CHAIN_DEBUG": "1000,20000,1", "TBLUP_SOLVE_PULL": pull}):
        with GpuBlupEngine(p["geno"], p["pheno"], device=0) as eng:
            np.testing.assert_array_equal(eng.evaluate_folds(genomes, folds, 0.4), ref_f)
            assert eng.chain_recoveries() == 1
    with _env({"TBLUP_CHAIN_DEBUG": "1000,20000,2", "TBLUP_FOLD_FUSE": "0", "TBLUP_SOLVE_PULL": pull}):
        with GpuBlupEngine(p["geno"], p["pheno"], device=0) as eng:   # split by split: both folds again
            np.testing.assert_array_equal(eng.evaluate_folds(genomes, folds, 0.4), ref_f)
            assert eng.chain_recoveries() == 1


def _generations(p, tmp_path, pop, gens, env):
    """Generation 0 (evaluate) and `gens` GPU DE generations (evolve -> speculative evaluate)
    through the drop-in classes on the config-2 panel; returns (fitness per generation,
    chain recoveries, speculative fallbacks)."""
    import random
    from tests.ga_driver import RandomKeyIndividual
    from tests.helpers import Pop
    from tblup_amd.evaluator import BlupParallelEvaluator
    from tblup_amd.evolver import DERandOneEvolver
    gp, pp = str(tmp_path / "g.npy"), str(tmp_path / "y.npy")
    if not os.path.exists(gp):
        np.save(gp, p["geno"])
        np.save(pp, p["pheno"])
    random.seed(5)
    np.random.seed(5)
    rng = np.random.default_rng(6)
    P = p["geno"].shape[1]
    ev = BlupParallelEvaluator(gp, pp, 0.4)
    ev.training_indices, ev.validation_indices = list(p["T"]), list(p["V"])
    inds = [RandomKeyIndividual(1000, P, genome=rng.uniform(size=P)) for _ in range(pop)]
    evo = DERandOneEvolver(P, 0.8, 0.5, False)
    out = []
    with _env(env):
        with ev:
            popn = Pop(inds, 0)
            popn.evaluator = ev
            ev.evaluate(popn, popn, 0)
            out.append([i.fitness for i in popn.population])
            for g in range(1, gens + 1):
                popn.generation = g
                kids = evo.evolve(popn)
                ev.evaluate(popn, kids, g)
                out.append([c.fitness for c in kids])
                popn.population = [c if c.fitness > q.fitness else q for q, c in zip(popn.population, kids)]
            rec = ev.engine.chain_recoveries()
    return np.array(out), rec, ev.spec_fallbacks


def test_evaluator_recovers_from_chain_expiry(panel, tmp_path):
    """The drop-in evaluator under forced chained-solve expiries: generation 0
    goes through the host entry (the chunk re-solved, chain_recoveries = 1), generation 1's
    speculative device-entry evaluation expires too and is dropped (spec_fallbacks = 1): evaluate()
    then evaluates the children through the host entry.  Every fitness equals an undisturbed run's
    bit for bit, where the reference would have hung (tblup/evaluator.py:397-398)."""
    p = panel
    ref, rec0, fb0 = _generations(p, tmp_path, 16, 2, {})
    assert (rec0, fb0) == (0, 0)
    got, rec, fb = _generations(p, tmp_path, 16, 2, {"TBLUP_CHAIN_DEBUG": "1000,20000,2"})
    np.testing.assert_array_equal(got, ref)
    assert (rec, fb) == (1, 1)


def test_kernel_form_folds_fused(panel):
    """IntraGCV's folds in the kernel (GRM) form -- k > n (gblup) and n_T < k <= n (snp branch,
    the kernel form because the fold's n_T = 1024 < k) -- run as ONE fused batch of 5 x B systems
    (each system's panel gathered from its own fold's rows): bit-identical to the folds evaluated
    split by split (TBLUP_FOLD_FUSE=0) and to each fold's own evaluation (SURVEY.md 8 f-2,
    tblup/evaluator.py:509-537)."""
    from tblup_amd.engine import GpuBlupEngine
    from tblup_amd.evaluator import InterGCVBlupParallelEvaluator
    p = panel
    rng = np.random.default_rng(61)
    genomes = [rng.choice(50_000, k, replace=False) for k in (2500, 1100, 2100, 1500, 2400, 1200)]
    folds = InterGCVBlupParallelEvaluator.make_fold_indices(np.asarray(p["T"]), 5)
    with GpuBlupEngine(p["geno"], p["pheno"], device=0) as eng:
        fused = eng.evaluate_folds(genomes, folds, 0.4)
        singles = [eng.evaluate(genomes, t, v, 0.4) for t, v in folds]
    with _env({"TBLUP_FOLD_FUSE": "0"}):
        with GpuBlupEngine(p["geno"], p["pheno"], device=0) as eng:
            unfused = eng.evaluate_folds(genomes, folds, 0.4)
    # round 6: the folds' counts from FP4 system tiles per fold system (default), or -- where the
    # counts are formed in-tile (TBLUP_DUAL_ST=0) -- from one shared A_R A_R^T per individual, or
    # each system's own int8 tiles: the same integers
    runs = []
    for env in ({"TBLUP_DUAL_ST": "0"}, {"TBLUP_DUAL_ST": "0", "TBLUP_FOLD_GSHARE": "0"}):
        with _env(env):
            with GpuBlupEngine(p["geno"], p["pheno"], device=0) as eng:
                runs.append(eng.evaluate_folds(genomes, folds, 0.4))
    np.testing.assert_array_equal(fused, unfused)
    for r in runs:
        np.testing.assert_array_equal(fused, r)
    for f in range(5):
        np.testing.assert_array_equal(fused[f], singles[f])
    for i in (0, 1):
        fo, _ = O.blup_grm_form(genomes[i], folds[2][0], folds[2][1], p["geno"], p["pheno"], 0.4)
        assert abs(fused[2][i] - fo) <= FIT_ATOL


@pytest.mark.parametrize("ks,B", [((2500,), 64), ((300, 1700), 5), ((1150, 2100, 1000), 37), ((1000, 640), 300)])
def test_kernel_form_sys_tiles_bit_identical(panel, ks, B):
    """Kernel form (TBLUP_FORM=1): the system tiles' exact counts from k_sys_tiles on the gathered
    2-bit rows -- the persistent super-tile kernel and the per-tile one -- against the in-tile int8
    products (TBLUP_DUAL_ST=0): the same integers, so bit-identical fitness and EBVs; k from 300 to
    2500 (not multiples of 64 / 256), runs crossing individuals; and the oracle."""
    p = panel
    rng = np.random.default_rng(81 + B)
    genomes = [rng.choice(50_000, ks[i % len(ks)], replace=False) for i in range(B)]
    ref = _run(p, genomes, {"TBLUP_FORM": "1", "TBLUP_DUAL_ST": "0"})
    for env in ({"TBLUP_FORM": "1"}, {"TBLUP_FORM": "1", "TBLUP_SYS_ST": "1"}, {"TBLUP_FORM": "1", "TBLUP_SYS_ST": "0"}):
        got = _run(p, genomes, env)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
    for i in (0, B - 1):
        fo, _ = O.blup_grm_form(genomes[i], p["T"], p["V"], p["geno"], p["pheno"], 0.4)
        assert abs(ref[0][i] - fo) <= FIT_ATOL


@pytest.mark.parametrize("ks,B", [((1000,), 256), ((100, 300), 3), ((1150, 700, 1000), 37), ((1000, 640), 300)])
def test_sys_tiles_persistent_bit_identical(panel, ks, B):
    """The persistent super-tile system-tile kernel (k_sys_tiles_st: 2 x 2 tiles per unit, one
    workgroup per CU walking a run of units, LDS-DMA ring across unit boundaries) against the
    per-tile kernel: every tile count is exact, so the results are bit-identical -- odd and even
    tile counts (NT 1..9), runs that cross individuals (B = 37, 300), B = 256 by default (auto)."""
    p = panel
    rng = np.random.default_rng(71 + B)
    genomes = [rng.choice(50_000, ks[i % len(ks)], replace=False) for i in range(B)]
    st = _run(p, genomes, {"TBLUP_SYS_ST": "1"})
    tile = _run(p, genomes, {"TBLUP_SYS_ST": "0"})
    np.testing.assert_array_equal(st[0], tile[0])
    np.testing.assert_array_equal(st[1], tile[1])
    if B == 256:
        auto = _run(p, genomes)
        np.testing.assert_array_equal(auto[0], tile[0])
    for i in (0, B - 1):
        f, _ = O.blup_grm_form(genomes[i], p["T"], p["V"], p["geno"], p["pheno"], 0.4)
        assert abs(st[0][i] - f) <= FIT_ATOL, i
