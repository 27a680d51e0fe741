"""IntraGCV (k = 5 folds inside every fitness evaluation, evaluator.py:494-537) against one
fold's evaluation on the GPU: config 1 (200 x 1000, k = 100, pop 32), config 2 (2000 x 50k,
k = 1000, pop 256) and a config-4-shaped kernel-form case (5000 x 50k, k = 5000, pop 32; device only).  Per config one JSON line with
  * device-resident genomes (no host decode in the ratio): one fold's evaluate_device and the
    k folds' evaluate_folds_device (tblup_eval_folds_device: fold-fused, the k x pop systems as
    one batch through one launch sequence, system tiles from shared counts; beside it the same
    call with TBLUP_FOLD_SHARE=0 -- every fold's tiles from its own rows --, TBLUP_FOLD_GSHARE=0 (kernel form:
    each system's own int8 tiles instead of one A_R A_R^T per individual) and with
    TBLUP_FOLD_FUSE=0, the folds back to back on one stream), medians over repeats, and ratios;
  * end to end through the drop-in classes: the median time of a fresh population's evaluate()
    for the plain evaluator (one split) and for IntraGCV (one evaluate_folds call).
(A variant with the folds on k contexts driven from k host threads measured slower in round 2:
config 1 1.54 vs 0.91 ms, config 2 35.8 vs 32.3 ms.)"""
import json
import os
import random
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed_evals(ev, make_pop, reps):
    ts = []
    with ev:
        for r in range(reps + 1):
            pop = make_pop()
            t0 = time.perf_counter()
            ev.evaluate(pop, pop, 0)
            if r:
                ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def main():
    import torch  # noqa: F401
    from oracle import blup_oracle as O
    from tests.ga_driver import RandomKeyIndividual
    from tblup_amd import evaluator as E
    cases = (("config1", 200, 1000, 100, 32), ("config2", 2000, 50000, 1000, 256),
             # the kernel (GRM) form: k = 5000 > each fold's n_T = 2560 (BASELINE config 4's animals and
             # panel size on a 50k-SNP panel), device-resident only
             ("config4shape", 5000, 50000, 5000, 32))
    for name, n, p, k, pop in cases:
        rng = np.random.default_rng(3)
        geno = O.synth_geno(rng, n, p)
        tmp = tempfile.mkdtemp()
        gp, pp = os.path.join(tmp, "g.npy"), os.path.join(tmp, "y.npy")
        np.save(gp, geno)
        np.save(pp, rng.standard_normal(n))

        def make_pop():
            return [RandomKeyIndividual(k, p, genome=rng.uniform(size=p)) for _ in range(pop)]
        # device-resident genomes: one fold vs the k folds
        import torch
        from tblup_amd.engine import GpuBlupEngine, concat_genomes
        eng = GpuBlupEngine(geno, np.load(pp), device=0)
        random.seed(1)
        np.random.seed(1)
        ev0 = E.IntraGCVBlupParallelEvaluator(gp, pp, 0.4, n_folds=5)
        splits = [ev0.train_validation_indices(f) for f in range(5)]
        sids = [eng.split_id(t, v) for t, v in splits]
        genomes = [np.argsort(rng.uniform(size=p))[-k:] for _ in range(pop)]
        idx, off = concat_genomes(genomes)
        d_idx, d_off = torch.from_numpy(idx).cuda(), torch.from_numpy(off).cuda()
        d_fit = torch.empty((5, pop), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream()

        def dev_ms(fn, reps=20):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts)) * 1e3
        one_dev = dev_ms(lambda: eng.evaluate_device(sids[0], d_idx.data_ptr(), d_off.data_ptr(), off, 0.4,
                                                     d_fit.data_ptr(), stream_ptr=st.cuda_stream))
        folds_dev = dev_ms(lambda: eng.evaluate_folds_device(sids, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4,
                                                             d_fit.data_ptr(), stream_ptr=st.cuda_stream))
        got = d_fit.cpu().numpy()
        for f in (0, 4):   # the batched folds are each split's own evaluation
            assert np.array_equal(got[f], eng.evaluate(genomes, *splits[f], 0.4))
        eng.close()
        alt = {}
        for var in ("TBLUP_FOLD_SHARE", "TBLUP_FOLD_FUSE", "TBLUP_FOLD_GSHARE"):
            os.environ[var] = "0"   # read at context creation
            eng = GpuBlupEngine(geno, np.load(pp), device=0)
            del os.environ[var]
            sids = [eng.split_id(t, v) for t, v in splits]
            alt[var] = dev_ms(lambda: eng.evaluate_folds_device(sids, d_idx.data_ptr(), d_off.data_ptr(), off, 0.4,
                                                                d_fit.data_ptr(), stream_ptr=st.cuda_stream))
            assert np.array_equal(d_fit.cpu().numpy(), got)
            eng.close()
        seq_dev = alt["TBLUP_FOLD_FUSE"]
        line = {"config": name, "pop": pop, "k": k,
                "device_one_fold_ms": round(one_dev, 3), "device_k_folds_ms": round(folds_dev, 3),
                "device_ratio": round(folds_dev / one_dev, 2),
                "device_k_folds_unshared_ms": round(alt["TBLUP_FOLD_SHARE"], 3),
                # kernel form: the folds' int8 counts from each system's own tiles instead of one
                # shared A_R A_R^T per individual (round 6); the SNP form ignores the knob
                "device_k_folds_own_counts_ms": round(alt["TBLUP_FOLD_GSHARE"], 3),
                "device_k_folds_unfused_ms": round(seq_dev, 3),
                "device_ratio_unfused": round(seq_dev / one_dev, 2)}
        if name == "config4shape":
            print(json.dumps(line), flush=True)
            continue
        random.seed(1)
        np.random.seed(1)
        one = timed_evals(E.BlupParallelEvaluator(gp, pp, 0.4), make_pop, 5)
        random.seed(1)
        np.random.seed(1)
        intra = timed_evals(E.IntraGCVBlupParallelEvaluator(gp, pp, 0.4, n_folds=5), make_pop, 5)
        line.update({"one_split_ms": round(one, 3), "intragcv_ms": round(intra, 3), "ratio": round(intra / one, 2)})
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
