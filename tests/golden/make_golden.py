"""Generate golden input/output vectors from the upstream reference (ianwhale/tblup).

Run ONLY in the build container, where the read-only reference is mounted at
/root/reference (it never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference is imported as a library and exercised through its own public
functions (`tblup.utils.make_grm`, `BlupParallelEvaluator.blup/gblup/snp_blup`,
the evaluator classes, the individual decoders, `SNPRemovalHandler`).  Predicted
breeding values (EBVs) are not returned by the reference, so they are captured by
wrapping `tblup.evaluator.pearsonr` (argument order differs per branch:
gblup passes (y_V, pred_V) at evaluator.py:286, snp_blup passes (pred_V, y_V) at
evaluator.py:314).

Outputs are small .npz files next to this script: data only (inputs and expected
outputs), no reference source.
"""
import os
import sys
import random
import tempfile
import hashlib

import numpy as np

REF = os.environ.get("TBLUP_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

# numpy>=1.23 removed np.asscalar, which the reference's monitor/evolver call.
if not hasattr(np, "asscalar"):
    np.asscalar = lambda a: a.item()

import tblup  # noqa: E402  (reference package)
import tblup.evaluator as ref_ev  # noqa: E402
from tblup.utils import make_grm  # noqa: E402


def synth_geno(rng, n, p, maf_lo=0.05, maf_hi=0.5):
    maf = rng.uniform(maf_lo, maf_hi, size=p)
    return rng.binomial(2, maf, size=(n, p)).astype(np.int8)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


class Capture:
    """Wraps scipy.stats.pearsonr inside the reference evaluator to record EBVs."""

    def __init__(self):
        self.orig = ref_ev.pearsonr
        self.calls = []

    def __enter__(self):
        def wrapped(a, b):
            self.calls.append((np.array(a, dtype=np.float64), np.array(b, dtype=np.float64)))
            return self.orig(a, b)
        ref_ev.pearsonr = wrapped
        return self

    def __exit__(self, *exc):
        ref_ev.pearsonr = self.orig


def ref_blup(indices, T, V, data, labels, h2):
    """Calls the reference blup and returns (fitness, ebv_V, branch)."""
    k = len(indices)
    branch = "gblup" if k > data.shape[0] else "snp"
    with Capture() as cap:
        fit = ref_ev.BlupParallelEvaluator.blup(np.asarray(indices), list(T), list(V),
                                               data.copy(), labels, h2)
    a, b = cap.calls[-1]
    ebv = b if branch == "gblup" else a
    return float(fit), ebv, branch


def gen_grm():
    rng = np.random.default_rng(11)
    geno = synth_geno(rng, 64, 200)
    G = make_grm(geno.astype(np.float64))
    # int input too (reference accepts ints for make_grm)
    G_int = make_grm(geno.astype(np.int64))
    np.savez_compressed(os.path.join(HERE, "grm_64x200.npz"), geno=geno, G=G, G_int=G_int)


def make_cases(rng, n, p):
    """Index sets covering both branches, duplicates, boundaries and ragged k."""
    cases = []
    cases.append(("snp_k100", rng.choice(p, 100, replace=False)))
    cases.append(("snp_k100_b", rng.choice(p, 100, replace=False)))
    cases.append(("snp_dup", rng.integers(0, 60, 100)))          # duplicates (IndexIndividual)
    cases.append(("snp_k1", rng.choice(p, 1, replace=False)))
    cases.append(("snp_k2", rng.choice(p, 2, replace=False)))
    cases.append(("snp_k150_kernel", rng.choice(p, 150, replace=False)))  # k > n_T: sklearn kernel solver
    cases.append(("snp_k_eq_n", rng.choice(p, n, replace=False)))  # k == n -> snp branch (strict >)
    cases.append(("gblup_k_n_plus_1", rng.choice(p, n + 1, replace=False)))
    cases.append(("gblup_k300", rng.choice(p, 300, replace=False)))
    cases.append(("gblup_dup", rng.integers(0, p, 350)))
    cases.append(("snp_sorted_desc", np.sort(rng.choice(p, 77, replace=False))[::-1].copy()))
    return cases


def gen_blup_small():
    """200 animals x 1000 SNPs (BASELINE config 1 shape)."""
    rng = np.random.default_rng(2024)
    n, p = 200, 1000
    geno = synth_geno(rng, n, p)
    # a few monomorphic columns (p=0 and p=1) to exercise the p(1-p) terms
    geno[:, 5] = 0
    geno[:, 6] = 2
    pheno = rng.standard_normal(n)
    h2 = 0.4
    data = geno.astype(np.float64)

    # Split exactly as BlupParallelEvaluator.__init__ does (evaluator.py:196-203).
    with tempfile.TemporaryDirectory() as td:
        gp, pp = os.path.join(td, "g.npy"), os.path.join(td, "p.npy")
        np.save(gp, data)
        np.save(pp, pheno)
        random.seed(0)
        np.random.seed(0)
        ev = ref_ev.BlupParallelEvaluator(gp, pp, h2, n_procs=1)
        T, V, X = list(ev.training_indices), list(ev.validation_indices), list(ev.testing_indices)

    out = dict(geno=geno, pheno=pheno, h2=h2, T=np.array(T), V=np.array(V), X=np.array(X))
    names, idx_concat, offs, fits, ebvs, branches = [], [], [0], [], [], []
    TV = T + V
    test_fits, test_ebvs = [], []
    for name, idx in make_cases(rng, n, p):
        idx = np.asarray(idx, dtype=np.int64)
        f, e, br = ref_blup(idx, T, V, data, pheno, h2)
        ft, et, _ = ref_blup(idx, TV, X, data, pheno, h2)
        names.append(name)
        idx_concat.append(idx)
        offs.append(offs[-1] + len(idx))
        fits.append(f)
        ebvs.append(e)
        branches.append(br)
        test_fits.append(ft)
        test_ebvs.append(et)
    out.update(names=np.array(names), idx=np.concatenate(idx_concat), offsets=np.array(offs),
               fitness=np.array(fits), ebv=np.stack(ebvs), branch=np.array(branches),
               test_fitness=np.array(test_fits), test_ebv=np.stack(test_ebvs))

    # Other heritabilities (lambda = (1-h2)/h2) on the first snp and first gblup case.
    h2s = np.array([0.1, 0.25, 0.7, 0.95])
    hf = []
    for h in h2s:
        hf.append([ref_blup(np.asarray(idx_concat[0]), T, V, data, pheno, h)[0],
                   ref_blup(np.asarray(idx_concat[8]), T, V, data, pheno, h)[0]])
    out.update(h2_sweep=h2s, h2_sweep_fitness=np.array(hf))
    np.savez_compressed(os.path.join(HERE, "blup_200x1000.npz"), **out)


def gen_blup_edge():
    """Degenerate inputs: all-monomorphic selections (d == 0), constant phenotype."""
    rng = np.random.default_rng(5)
    n, p = 200, 300
    geno = synth_geno(rng, n, p)
    geno[:, :10] = 1          # monomorphic heterozygous columns -> p = 0.5 (d != 0 but W == 0)
    geno[:, 10:20] = 0        # monomorphic, p = 0 -> d == 0 when selected alone
    pheno = rng.standard_normal(n)
    perm = rng.permutation(n)
    T, V = list(perm[:128]), list(perm[128:160])
    data = geno.astype(np.float64)
    res = {}
    import warnings
    for name, idx in [("mono0_snp", np.arange(10, 20)), ("mono0_gblup", np.tile(np.arange(10, 20), 21)),
                      ("het_snp", np.arange(0, 10))]:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            try:
                f, e, br = ref_blup(idx, T, V, data, pheno, 0.4)
                res[name] = ("value", f)
            except Exception as exc:  # record the reference's failure mode
                res[name] = ("raise", type(exc).__name__)
    np.savez_compressed(os.path.join(HERE, "blup_edge.npz"), geno=geno, pheno=pheno, T=np.array(T),
                        V=np.array(V),
                        names=np.array(list(res.keys())),
                        kind=np.array([v[0] for v in res.values()]),
                        value=np.array([str(v[1]) for v in res.values()]))


def gen_decode():
    """Genome decode per individual type (individual.py:93-95, 154-156, 187-237)."""
    from tblup.individual import (IndexIndividual, RandomKeyIndividual, CoevolutionIndividual,
                                  NullableIndexIndividual)
    rng = np.random.default_rng(9)
    d = 500
    out = {}
    keys = rng.uniform(size=(6, d))
    keys[5, 100:140] = 0.5   # explicit ties in the keys
    rk = [RandomKeyIndividual(37, d, genome=keys[i].copy()).genome for i in range(6)]
    out["rk_keys"] = keys
    out["rk_length"] = 37
    out["rk_genome"] = np.stack(rk)
    # float-length (coevolution lengths are floats after DE)
    ck = CoevolutionIndividual(40, d, genome=keys[0].copy())
    ck.set_internal_genome(np.append(keys[1].copy(), 53.7))
    out["coev_keys"] = keys[1]
    out["coev_length"] = ck.length
    out["coev_genome"] = ck.genome
    ck.set_fitness(0.5)
    out["coev_fitness"] = ck.fitness
    ig = rng.uniform(-20, d + 20, size=80)
    out["index_internal"] = ig
    out["index_genome"] = IndexIndividual(80, d, genome=ig.copy()).genome
    out["nullable_genome"] = NullableIndexIndividual(80, d, genome=ig.copy()).genome
    np.savez_compressed(os.path.join(HERE, "decode.npz"), **out)


def gen_evaluator_flow():
    """Evaluator-level flows on the 200x1000 panel: splits, CV folds, population eval,
    SNP removal and evaluate_testing, all through the reference's own classes."""
    from tblup.individual import RandomKeyIndividual, IndexIndividual
    z = np.load(os.path.join(HERE, "blup_200x1000.npz"))
    geno, pheno = z["geno"], z["pheno"]
    out = {}
    with tempfile.TemporaryDirectory() as td:
        gp, pp = os.path.join(td, "g.npy"), os.path.join(td, "p.npy")
        np.save(gp, geno.astype(np.float64))
        np.save(pp, pheno)

        # --- plain BLUP evaluator, generation-0 population of RandomKey individuals ---
        random.seed(3)
        np.random.seed(3)
        remover = ref_ev.SNPRemovalHandler(100, 0.0, 0.4, False)
        ev = ref_ev.BlupParallelEvaluator(gp, pp, 0.4, n_procs=2, snp_remover=remover)
        pop = [RandomKeyIndividual(100, 1000) for _ in range(32)]
        out["flow_T"], out["flow_V"], out["flow_X"] = (np.array(ev.training_indices),
                                                      np.array(ev.validation_indices),
                                                      np.array(ev.testing_indices))
        out["flow_keys"] = np.stack([i.get_internal_genome() for i in pop])
        with ev:
            ev.evaluate(pop, pop, 0)
            out["flow_fitness"] = np.array([i.fitness for i in pop])
            out["flow_testing"] = np.array(ev.evaluate_testing(pop))

        # --- InterGCV folds + IntraGCV mean fitness ---
        random.seed(4)
        np.random.seed(4)
        remover = ref_ev.SNPRemovalHandler(100, 0.0, 0.4, False)
        iev = ref_ev.IntraGCVBlupParallelEvaluator(gp, pp, 0.4, n_procs=2, n_folds=5, snp_remover=remover)
        out["cv_T"] = np.array(iev.training_indices)
        folds = iev.fold_indices
        out["cv_fold_train"] = np.concatenate([np.array(f[0]) for f in folds])
        out["cv_fold_train_len"] = np.array([len(f[0]) for f in folds])
        out["cv_fold_valid"] = np.concatenate([np.array(f[1]) for f in folds])
        out["cv_fold_valid_len"] = np.array([len(f[1]) for f in folds])
        ipop = [IndexIndividual(80, 1000) for _ in range(8)]
        out["cv_genomes"] = np.stack([i.get_internal_genome() for i in ipop])
        with iev:
            iev.evaluate(ipop, ipop, 0)
            out["cv_intra_fitness"] = np.array([i.fitness for i in ipop])

        # --- MonteCarlo split sequence (numpy global RNG, evaluator.py:555-561) ---
        random.seed(5)
        np.random.seed(5)
        mev = ref_ev.MonteCarloCVBlupParallelEvaluator(gp, pp, 0.4, n_procs=1, snp_remover=remover)
        seq = [mev.train_validation_indices(g) for g in range(3)]
        out["mc_T"] = np.array(mev.training_indices)
        out["mc_V"] = np.array(mev.validation_indices)
        out["mc_split_train"] = np.array([np.array(s[0]) for s in seq])
        out["mc_split_valid"] = np.array([np.array(s[1]) for s in seq])

        # --- SNP removal: threshold 0 forces removal of the best individual's SNPs ---
        random.seed(6)
        np.random.seed(6)
        remover = ref_ev.SNPRemovalHandler(30, -1.0, 0.4, True)   # threshold = sqrt(h2)*0 = 0
        rev = ref_ev.BlupParallelEvaluator(gp, pp, 0.4, n_procs=2, snp_remover=remover)
        prev = [RandomKeyIndividual(60, 1000) for _ in range(10)]
        for i, ind in enumerate(prev):
            ind.set_fitness(0.01 * i)           # individual 9 is "best"
        nxt = [RandomKeyIndividual(60, 1000) for _ in range(10)]
        for i, ind in enumerate(nxt):
            ind.set_fitness(0.02 * ((i * 7) % 10))   # offspring carry a (deep-copied) parent fitness

        class _Mon:
            def log_snp_removal_event(self, g):
                pass

        class _Pop(list):
            monitor = _Mon()

        prev_pop = _Pop(prev)
        out["rm_T"], out["rm_V"], out["rm_X"] = (np.array(rev.training_indices),
                                                np.array(rev.validation_indices),
                                                np.array(rev.testing_indices))
        out["rm_prev_keys"] = np.stack([i.get_internal_genome() for i in prev])
        out["rm_next_keys"] = np.stack([i.get_internal_genome() for i in nxt])
        with rev:
            rev.evaluate(prev_pop, nxt, 1)
            out["rm_removed"] = np.array(remover.removed)
            out["rm_next_fitness"] = np.array([i.fitness for i in nxt])
            out["rm_prev_fitness"] = np.array([i.fitness for i in prev_pop])
            out["rm_testing"] = np.array(rev.evaluate_testing(nxt))
    np.savez_compressed(os.path.join(HERE, "evaluator_flow.npz"), **out)


def gen_blup_config2():
    """Config-2 shape (2000 animals, panel k=1000) on a 4000-SNP synthetic panel.
    The genotype matrix is regenerated in tests from the seed; its sha256 is pinned."""
    seed = 77
    rng = np.random.default_rng(seed)
    n, p = 2000, 4000
    geno = synth_geno(rng, n, p)
    pheno = rng.standard_normal(n)
    perm = np.random.default_rng(seed + 1).permutation(n)
    T, V = perm[:1280], perm[1280:1600]
    data = geno.astype(np.float64)
    sel = np.random.default_rng(seed + 2)
    cases = [sel.choice(p, 1000, replace=False) for _ in range(3)] + [sel.choice(p, 2100, replace=False)]
    fits, ebvs, offs = [], [], [0]
    for idx in cases:
        f, e, _ = ref_blup(idx, T, V, data, pheno, 0.4)
        fits.append(f)
        ebvs.append(e)
        offs.append(offs[-1] + len(idx))
    np.savez_compressed(os.path.join(HERE, "blup_2000x4000.npz"), seed=seed, n=n, p=p,
                        geno_sha256=sha(geno), pheno=pheno, T=T, V=V,
                        idx=np.concatenate(cases), offsets=np.array(offs),
                        fitness=np.array(fits), ebv=np.stack(ebvs[:3]), ebv_gblup=ebvs[3])


class _Pop:
    """The slice of tblup.Population the evolvers read: .population, .generation, [], len."""

    def __init__(self, individuals, generation):
        self.population = individuals
        self.generation = generation

    def __getitem__(self, i):
        return self.population[i]

    def __len__(self):
        return len(self.population)


DE_CASES = [
    # name, individual kind, strategy, d, length, pop, generation, cr, F, clip, pre_draws
    ("rk_rand1", "rk", "de_rand_1", 1000, 50, 8, 1, 0.8, 0.5, False, 0),
    ("rk_rand1_f5", "rk", "de_rand_1", 700, 40, 6, 5, 0.8, 0.5, False, 3),
    ("rk_rand1_clip", "rk", "de_rand_1", 333, 20, 5, 10, 0.9, 0.5, True, 1),
    ("rk_ctb", "rk", "de_currenttobest_1", 300, 30, 6, 3, 0.8, 0.5, False, 7),
    ("coev_rand1", "coev", "de_rand_1", 200, 20, 5, 2, 0.7, 0.6, False, 2),
    ("index_rand1_int", "index", "de_rand_1", 500, 25, 6, 5, 0.8, 0.5, True, 5),
    ("index_ctb", "index", "de_currenttobest_1", 500, 25, 5, 4, 0.5, 0.5, True, 0),
]


def gen_de():
    """One generation of the reference's DE evolvers (evolver.py:86-244) from seeded RNG states:
    parents, fitness, the children's internal genomes and the RNG states afterwards."""
    from tblup.evolver import DERandOneEvolver, DECurrentToBestOneEvolver
    from tblup.individual import RandomKeyIndividual, CoevolutionIndividual, IndexIndividual
    out = {}
    for ci, (name, kind, strat, d, length, pop, gen, cr, F, clip, pre) in enumerate(DE_CASES):
        rng = np.random.default_rng(100 + ci)
        if kind == "index":
            parents = [rng.integers(0, d, size=length) for _ in range(pop)]
            inds = [IndexIndividual(length, d, genome=g.copy()) for g in parents]
        elif kind == "coev":
            keys = rng.uniform(size=(pop, d))
            lens = rng.integers(int(length * 0.9), int(length * 1.1) + 1, size=pop)
            inds = []
            for i in range(pop):
                ind = CoevolutionIndividual(length, d, genome=keys[i].copy())
                ind.length = int(lens[i])
                inds.append(ind)
            parents = [ind.get_internal_genome() for ind in inds]
        else:
            parents = [rng.uniform(size=d) for _ in range(pop)]
            inds = [RandomKeyIndividual(length, d, genome=g.copy()) for g in parents]
        fit = rng.uniform(size=pop)
        for ind, f in zip(inds, fit):
            ind.fitness = float(f)
        random.seed(1000 + ci)
        np.random.seed(2000 + ci)
        np.random.rand(pre)   # move numpy's pos off the block boundary
        ev = (DERandOneEvolver if strat == "de_rand_1" else DECurrentToBestOneEvolver)(d, cr, F, clip)
        kids = ev.evolve(_Pop(inds, gen))
        st = np.random.get_state()
        p = "de_%s_" % name
        out[p + "parents"] = np.stack([np.asarray(g) for g in parents])
        out[p + "fitness"] = fit
        out[p + "children"] = np.stack([np.asarray(k.get_internal_genome()) for k in kids])
        out[p + "children_dtype"] = np.array(str(np.asarray(kids[0].get_internal_genome()).dtype))
        out[p + "mt_key"] = np.asarray(st[1], dtype=np.uint32)
        out[p + "mt_pos"] = np.int64(st[2])
        out[p + "py_next"] = np.float64(random.random())
    # a config-2-sized generation by checksum: pop 32 of d = 50000 RandomKey genomes
    rng = np.random.default_rng(7)
    d, pop = 50000, 32
    keys = rng.uniform(size=(pop, d))
    fit = rng.uniform(size=pop)
    for strat in ("de_rand_1", "de_currenttobest_1"):
        inds = [RandomKeyIndividual(1000, d, genome=keys[i].copy()) for i in range(pop)]
        for ind, f in zip(inds, fit):
            ind.fitness = float(f)
        random.seed(31)
        np.random.seed(32)
        np.random.rand(11)
        ev = (DERandOneEvolver if strat == "de_rand_1" else DECurrentToBestOneEvolver)(d, 0.8, 0.5, False)
        kids = ev.evolve(_Pop(inds, 1))
        st = np.random.get_state()
        p = "big_%s_" % strat
        out[p + "children_sha256"] = np.array(sha(np.stack([k.get_internal_genome() for k in kids])))
        out[p + "children_row0"] = kids[0].get_internal_genome()[:64]
        out[p + "mt_key"] = np.asarray(st[1], dtype=np.uint32)
        out[p + "mt_pos"] = np.int64(st[2])
        out[p + "py_next"] = np.float64(random.random())
    out["big_d"], out["big_pop"] = d, pop
    np.savez_compressed(os.path.join(HERE, "de.npz"), **out)


SADE_CASES = [
    # name, individual kind, d, length, pop, generations, clip
    ("sade_rk", "rk", 150, 15, 8, 56, False),
    ("sade_rk_clip", "rk", 120, 10, 6, 12, True),
    ("sade_index", "index", 200, 20, 6, 12, True),
]


def gen_sade():
    """The reference's SaDE (evolver.py:297-547) over whole runs of generations: each generation's
    children (the first ones whole, then by checksum), the adaptive state after it (cr_m, p, the
    strategy success / failure counts), the parameter CSV it reports (AdaptiveEvolver.report) and the
    RNG states at the end.  The children's fitness comes from a generator of its own (never python's
    `random` or numpy's global one), and selection is DE's greedy replacement (selector.py:27-32), so
    the success counting of count_outcomes sees real uid changes; 56 generations cover the cr
    regenerations (every 5), the cr_m recalculations (25, 50) and the learning period's reset (50)."""
    from tblup.evolver import SaDE
    from tblup.individual import RandomKeyIndividual, IndexIndividual
    out = {}
    for ci, (name, kind, d, length, pop, gens, clip) in enumerate(SADE_CASES):
        rng = np.random.default_rng(300 + ci)
        if kind == "index":
            parents = [rng.integers(0, d, size=length) for _ in range(pop)]
            inds = [IndexIndividual(length, d, genome=g.copy()) for g in parents]
        else:
            parents = [rng.uniform(size=d) for _ in range(pop)]
            inds = [RandomKeyIndividual(length, d, genome=g.copy()) for g in parents]
        fit = rng.uniform(size=pop)
        for ind, f in zip(inds, fit):
            ind.fitness = float(f)
        frng = np.random.default_rng(400 + ci)
        tmp = tempfile.mkdtemp()

        class Mon:
            results_file = os.path.join(tmp, "results.csv")

        random.seed(500 + ci)
        np.random.seed(600 + ci)
        np.random.rand(3 * ci + 1)
        ev = SaDE(d, clip=clip)
        popn = _Pop(inds, 1)
        popn.monitor = Mon
        p = "%s_" % name
        sha_rows, state = [], []
        for g in range(1, gens + 1):
            popn.generation = g
            kids = ev.evolve(popn)
            kg = np.stack([np.asarray(k.get_internal_genome()) for k in kids])
            if g <= 3:
                out[p + "children_g%d" % g] = kg
            sha_rows.append(sha(kg))
            state.append([ev.cr_m, ev.p, ev.ns_1, ev.ns_2, ev.nf_1, ev.nf_2, len(ev.successful_crs)])
            for k, f in zip(kids, frng.uniform(size=pop)):
                k.fitness = float(f)
            popn.population = [k if k.fitness > q.fitness else q for q, k in zip(popn.population, kids)]
        st = np.random.get_state()
        out[p + "parents"] = np.stack([np.asarray(g) for g in parents])
        out[p + "fitness"] = fit
        out[p + "children_sha256"] = np.array(sha_rows)
        out[p + "state"] = np.array(state, dtype=np.float64)
        out[p + "children_dtype"] = np.array(str(kg.dtype))
        out[p + "params_csv"] = np.array(open(os.path.join(tmp, "results_params.csv")).read())
        out[p + "mt_key"] = np.asarray(st[1], dtype=np.uint32)
        out[p + "mt_pos"] = np.int64(st[2])
        out[p + "gauss"] = np.array([st[3], st[4]], dtype=np.float64)
        out[p + "py_next"] = np.float64(random.random())
    np.savez_compressed(os.path.join(HERE, "sade.npz"), **out)


MDE_CASES = [
    # name, individual kind, d, length, pop, generations (g_max), clip
    ("mde_rk", "rk", 150, 15, 12, 8, False),
    ("mde_index", "index", 200, 20, 8, 6, True),
]


def gen_mde():
    """The reference's MDE_pBX (evolver.py:550-687) over whole runs, recorded as gen_sade records
    SaDE (the adaptive state: cr_m, f_m, p)."""
    from tblup.evolver import MDE_pBX
    from tblup.individual import RandomKeyIndividual, IndexIndividual
    out = {}
    for ci, (name, kind, d, length, pop, gens, clip) in enumerate(MDE_CASES):
        rng = np.random.default_rng(700 + ci)
        if kind == "index":
            parents = [rng.integers(0, d, size=length) for _ in range(pop)]
            inds = [IndexIndividual(length, d, genome=g.copy()) for g in parents]
        else:
            parents = [rng.uniform(size=d) for _ in range(pop)]
            inds = [RandomKeyIndividual(length, d, genome=g.copy()) for g in parents]
        fit = rng.uniform(size=pop)
        for ind, f in zip(inds, fit):
            ind.fitness = float(f)
        frng = np.random.default_rng(800 + ci)
        tmp = tempfile.mkdtemp()

        class Mon:
            results_file = os.path.join(tmp, "results.csv")

        random.seed(900 + ci)
        np.random.seed(1000 + ci)
        ev = MDE_pBX(d, gens, clip=clip)
        popn = _Pop(inds, 1)
        popn.monitor = Mon
        p = "%s_" % name
        sha_rows, state = [], []
        for g in range(1, gens + 1):
            popn.generation = g
            kids = ev.evolve(popn)
            kg = np.stack([np.asarray(k.get_internal_genome()) for k in kids])
            if g <= 2:
                out[p + "children_g%d" % g] = kg
            sha_rows.append(sha(kg))
            state.append([ev.cr_m, ev.f_m, ev.p, len(ev.successful_crs), len(ev.successful_fs)])
            for k, f in zip(kids, frng.uniform(size=pop)):
                k.fitness = float(f)
            popn.population = [k if k.fitness > q.fitness else q for q, k in zip(popn.population, kids)]
        st = np.random.get_state()
        out[p + "parents"] = np.stack([np.asarray(g) for g in parents])
        out[p + "fitness"] = fit
        out[p + "children_sha256"] = np.array(sha_rows)
        out[p + "state"] = np.array(state, dtype=np.float64)
        out[p + "params_csv"] = np.array(open(os.path.join(tmp, "results_params.csv")).read())
        out[p + "mt_key"] = np.asarray(st[1], dtype=np.uint32)
        out[p + "mt_pos"] = np.int64(st[2])
        out[p + "py_next"] = np.float64(random.random())
    np.savez_compressed(os.path.join(HERE, "mde.npz"), **out)


def gen_pca():
    """pca_splitter (evaluator.py:641-663) on synthetic panels: n = 200 (sklearn's full SVD)
    and n = 600 (randomized SVD drawing from numpy's global RNG, seeded), both directions."""
    out = {}
    for n, p, seed in ((200, 1000, 3), (600, 1500, 4)):
        geno = synth_geno(np.random.default_rng(seed), n, p)
        out["pca_%d_geno" % n] = geno
        for outl in (False, True):
            np.random.seed(50 + n)
            tr, te = ref_ev.pca_splitter(geno, outliers=outl)
            st = np.random.get_state()
            tag = "pca_%d_%s_" % (n, "out" if outl else "in")
            out[tag + "train"] = np.array(tr)
            out[tag + "test"] = np.array(te)
            out[tag + "mt_key"] = np.asarray(st[1], dtype=np.uint32)
            out[tag + "mt_pos"] = np.int64(st[2])
        out["pca_%d_grm" % n] = make_grm(geno)
    np.savez_compressed(os.path.join(HERE, "pca.npz"), **out)


def gen_seed():
    """The top-SNPs seeder (seeder.py:110-220): sklearn f_regression per fold, the SNP ranking,
    and the first genomes of the RandomKey / Index seeders."""
    from tblup.seeder import TopSNPsSeedStrategy, RandomKeySeeder, IndexSeeder, p_value, f_score
    from sklearn.feature_selection import f_regression
    rng = np.random.default_rng(21)
    n, p = 300, 2000
    geno = synth_geno(rng, n, p)
    geno[:, 7] = 1                       # monomorphic SNP: force_finite path (F = 0, p = 1)
    beta = np.zeros(p)
    qtl = rng.choice(p, 30, replace=False)
    beta[qtl] = rng.standard_normal(30)
    g = geno.astype(np.float64) @ beta
    pheno = g / g.std() * np.sqrt(0.5) + rng.standard_normal(n) * np.sqrt(0.5)
    tmp = tempfile.mkdtemp()
    gp, pp = os.path.join(tmp, "g.npy"), os.path.join(tmp, "y.npy")
    np.save(gp, geno)
    np.save(pp, pheno)
    train = np.sort(rng.choice(n, 192, replace=False))

    class Ev:
        training_indices = list(train)
    strat = TopSNPsSeedStrategy(Ev(), p_value, gp, pp)
    out = {"geno": geno, "pheno": pheno, "training_indices": train, "sorted_indices": strat.indices}
    rows = np.arange(150)
    F, pv = f_regression(geno[rows], pheno[rows].ravel())
    out.update({"f_rows": rows, "f_F": F, "f_p": pv, "f_score": f_score(geno[rows], pheno[rows])})
    np.random.seed(8)
    rk = RandomKeySeeder(strat, 40, p)
    it = iter(rk)
    out["rk_genomes"] = np.stack([next(it) for _ in range(3)])
    ix = IndexSeeder(strat, 900)
    it = iter(ix)
    out["index_genomes"] = np.stack([next(it) for _ in range(2)])
    out["index_random_tail"] = next(it)   # past the end: np.random.choice(indices, 900, replace=False)
    out["mt_key"] = np.asarray(np.random.get_state()[1], dtype=np.uint32)
    np.savez_compressed(os.path.join(HERE, "seed.npz"), **out)


def gen_blup_extra():
    """numpy index semantics and float32 inputs on the 200x1000 panel (blup_extra.npz).

    * IndexIndividual genomes with negative entries (individual.py:93-95 truncates the
      internal floats with astype(int); DE without --clip leaves them negative): the
      reference's data[:, indices] (evaluator.py:275/298) wraps them to i + P.
    * an index >= P: numpy raises IndexError (recorded as the failure mode).
    * float32 genotype panels: snp_blup then computes in float32 in place
      (evaluator.py:298-309) and make_grm in float32 (utils.py:7-18).
    """
    from tblup.individual import IndexIndividual
    z = np.load(os.path.join(HERE, "blup_200x1000.npz"))
    geno, pheno, T, V = z["geno"], z["pheno"], list(z["T"]), list(z["V"])
    n, p = geno.shape
    data = geno.astype(np.float64)
    rng = np.random.default_rng(404)
    out = {}
    neg_cases = []
    for name, k, lo in (("neg_snp", 100, -300.0), ("neg_gblup", 300, -700.0), ("neg_dup", 90, -40.0)):
        internal = rng.uniform(lo, p - 0.01, size=k)
        if name == "neg_dup":
            internal[30:60] = rng.uniform(1.0, p - 0.01, size=30)
            internal[:30] = internal[30:60] - p      # -P + i and i address the same column
        idx = IndexIndividual(k, p, genome=internal.copy()).genome
        assert (idx < 0).any()
        f, e, br = ref_blup(idx, T, V, data, pheno, 0.4)
        neg_cases.append(name)
        out[name + "_internal"] = internal
        out[name + "_idx"] = idx
        out[name + "_fitness"] = f
        out[name + "_ebv"] = e
        out[name + "_branch"] = br
    out["neg_names"] = np.array(neg_cases)
    for name, idx in (("oob_hi", np.array([3, 17, p])), ("oob_lo", np.array([3, -p - 1, 17]))):
        try:
            ref_blup(idx, T, V, data, pheno, 0.4)
            out[name + "_raises"] = np.array("")
        except Exception as exc:  # numpy's fancy-index bound check
            out[name + "_raises"] = np.array(type(exc).__name__)
        out[name + "_idx"] = idx
    data32 = geno.astype(np.float32)
    f32 = []
    for name, k in (("f32_snp", 100), ("f32_snp_kernel", 150), ("f32_gblup", 300)):
        idx = rng.choice(p, k, replace=False)
        f, e, br = ref_blup(idx, T, V, data32, pheno, 0.4)
        f64, e64, _ = ref_blup(idx, T, V, data, pheno, 0.4)
        f32.append(name)
        out[name + "_idx"] = idx
        out[name + "_fitness"] = f
        out[name + "_ebv"] = e
        out[name + "_fitness64"] = f64
        out[name + "_ebv64"] = e64
        out[name + "_branch"] = br
    out["f32_names"] = np.array(f32)
    np.savez_compressed(os.path.join(HERE, "blup_extra.npz"), **out)


# main.py end to end on BASELINE config 1 (200 animals x 1000 SNPs, 100 features, pop 32),
# one worker (-p 1): name -> extra command-line flags
MAIN_CASES = [
    ("rk_rand1", ["--generations", "6"]),
    ("rk_ctb", ["--generations", "4", "--de_strategy", "de_currenttobest_1"]),
    ("index_clip", ["--generations", "4", "--individual", "index", "--clip", "true"]),
    ("coevolve", ["--generations", "3", "--individual", "coevolve"]),
    ("intercv", ["--generations", "3", "--regressor", "intercv_blup"]),
    ("intracv", ["--generations", "3", "--regressor", "intracv_blup"]),
    ("montecv", ["--generations", "3", "--regressor", "montecv_blup"]),
    ("removal_testing_knockout", ["--generations", "4", "--remove_snps", "true", "--removal_r", "20",
                                  "--h2_alpha", "-0.45", "--record_testing", "true", "--local_search", "knockout"]),
    ("stop_h2", ["--generations", "8", "--stop_condition", "h2_max", "--h2_alpha", "-0.3"]),
]
MAIN_BASE = ["-s", "7", "-p", "1", "--population_size", "32", "--features", "100", "--heritability", "0.4"]


def gen_main_runs():
    """The reference's main() (main.py:10-45) run end to end, in-process, per MAIN_CASES: the
    results / testing CSV text, archive and local-search JSON, saved split indices, every
    generation's fitness vector (Monitor.gather_stats wrapped) and the final population's
    decoded genomes (evaluate_testing wrapped).  Writes main_runs.npz."""
    import json
    import signal
    import tblup.monitor as mon
    sys.path.insert(0, REF)
    import main as ref_main
    z = np.load(os.path.join(HERE, "blup_200x1000.npz"))
    out = {"geno": z["geno"], "pheno": z["pheno"], "base_argv": np.array(MAIN_BASE),
           "names": np.array([c[0] for c in MAIN_CASES])}
    rec = {}
    orig_gs = mon.Monitor.gather_stats
    orig_et = ref_ev.BlupParallelEvaluator.evaluate_testing

    def gs(self, population):
        rec["fit"].append([float(i.fitness) for i in population])
        rec["len"].append([float(len(i)) for i in population])
        return orig_gs(self, population)

    def et(self, population):
        rec["genomes"] = [np.asarray(i.genome, dtype=np.int64) for i in population]
        return orig_et(self, population)

    def alarm(*a):
        raise TimeoutError("reference main() did not finish (a worker error hangs it)")

    mon.Monitor.gather_stats = gs
    ref_ev.BlupParallelEvaluator.evaluate_testing = et
    cwd = os.getcwd()
    old = signal.signal(signal.SIGALRM, alarm)
    try:
        for name, extra in MAIN_CASES:
            with tempfile.TemporaryDirectory() as td:
                gp, pp = os.path.join(td, "geno.npy"), os.path.join(td, "pheno.npy")
                np.save(gp, z["geno"].astype(np.float64))
                np.save(pp, z["pheno"])
                os.chdir(td)
                argv = MAIN_BASE + ["--geno", gp, "--pheno", pp, "-o", "run"] + extra
                rec.clear()
                rec.update(fit=[], len=[], genomes=None)
                sys.argv = ["main.py"] + argv
                signal.alarm(900)
                ref_main.main()
                signal.alarm(0)
                rd = os.path.join(td, "results", "run")
                files = sorted(os.listdir(rd))

                def text(fn):
                    f = os.path.join(rd, fn)
                    return open(f).read() if os.path.isfile(f) else ""
                pre = name + "_"
                out[pre + "argv"] = np.array(extra)
                out[pre + "files"] = np.array(files)
                out[pre + "results_csv"] = np.array(text("007_results.csv"))
                out[pre + "testing_csv"] = np.array(text("007_results_testing.csv"))
                out[pre + "archive_json"] = np.array(text("007_archive.json"))
                out[pre + "local_json"] = np.array(text("007_local.json"))
                out[pre + "removals"] = np.array(text("007_removals.csv"))
                for part in ("train", "validation", "testing"):
                    out[pre + part] = np.load(os.path.join(rd, "007_%s_indices.npy" % part))
                out[pre + "gen_fitness"] = np.array(rec["fit"])
                out[pre + "gen_len"] = np.array(rec["len"])
                g = rec["genomes"]
                out[pre + "final_idx"] = np.concatenate(g)
                out[pre + "final_off"] = np.concatenate(([0], np.cumsum([len(x) for x in g])))
                os.chdir(cwd)
                print("main run", name, "generations", len(rec["fit"]) - 1, "archive",
                      list(json.loads(str(out[pre + "archive_json"])).keys()))
    finally:
        os.chdir(cwd)
        signal.signal(signal.SIGALRM, old)
        mon.Monitor.gather_stats = orig_gs
        ref_ev.BlupParallelEvaluator.evaluate_testing = orig_et
    np.savez_compressed(os.path.join(HERE, "main_runs.npz"), **out)


GENERATORS = {
    "grm": gen_grm, "blup": gen_blup_small, "edge": gen_blup_edge, "decode": gen_decode,
    "flow": gen_evaluator_flow, "config2": gen_blup_config2, "de": gen_de, "pca": gen_pca, "seed": gen_seed,
    "extra": gen_blup_extra, "main": gen_main_runs, "sade": gen_sade, "mde": gen_mde,
}

if __name__ == "__main__":
    for key in (sys.argv[1:] or list(GENERATORS)):
        GENERATORS[key]()
    print("golden fixtures written to", HERE)
