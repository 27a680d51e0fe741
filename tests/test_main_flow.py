"""main.py end to end against the reference's own runs (tests/golden/main_runs.npz).

tests/golden/make_golden.py::gen_main_runs ran the reference's main() on BASELINE config 1
(200 animals x 1000 SNPs, 100 features, pop 32, -p 1, seed 7) for each MAIN_CASES entry:
plain RandomKey DE/rand/1, current-to-best, clipped Index individuals, Coevolution,
Inter/Intra/Monte-Carlo CV, SNP removal + record_testing + knockout local search, and the
h2 stop condition.  tests/ga_driver.py restates main()'s control loop; here it runs

* on the CPU with the tblup_amd evaluator classes over the oracle engine and the oracle
  DE step (pins the restated loop and the evaluator's host logic), and
* on the GPU with the tblup_amd drop-ins themselves (HIP evaluator, GPU DE evolver,
  batched knockout), which must reproduce the reference's run: every generation's
  fitness vector to 1e-9, the results / testing CSV text, archive, removal log, final
  genomes and local-search result exactly.
"""
import os

import numpy as np
import pytest

from tests import ga_driver as D


@pytest.fixture(scope="module")
def runs(golden_dir):
    return np.load(os.path.join(golden_dir, "main_runs.npz"))


def _panel(z, tmp_path):
    gp, pp = str(tmp_path / "geno.npy"), str(tmp_path / "pheno.npy")
    np.save(gp, z["geno"].astype(np.float64))
    np.save(pp, z["pheno"])
    return gp, pp


def _argv(z, name, gp, pp):
    return list(z["base_argv"]) + ["--geno", gp, "--pheno", pp] + list(z[name + "_argv"])


CASES = ["rk_rand1", "rk_ctb", "index_clip", "coevolve", "intercv", "intracv", "montecv",
         "removal_testing_knockout", "stop_h2"]


def test_cases_cover_the_golden(runs):
    assert sorted(CASES) == sorted(str(x) for x in runs["names"])


@pytest.mark.parametrize("name", CASES)
def test_main_flow_oracle(runs, name, tmp_path):
    """CPU: the restated loop + tblup_amd evaluator classes on the oracle engine."""
    from tests.helpers import OracleEngine
    from tblup_amd import evaluator as E
    from tblup_amd import local as LS

    def get_evaluator(args):
        ev = E.get_evaluator(args)
        ev._open_engine = lambda: OracleEngine(np.load(ev.data_path), np.load(ev.labels_path))
        return ev

    gp, pp = _panel(runs, tmp_path)
    run = D.run_main(_argv(runs, name, gp, pp), get_evaluator, D.OracleEvolver, LS.get_local_search)
    D.compare(run, runs, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_main_flow_gpu(runs, name, tmp_path):
    """GPU: the tblup_amd drop-ins (HIP evaluator, GPU DE step, batched knockout)."""
    from tblup_amd import evaluator as E
    from tblup_amd import evolver as EV
    from tblup_amd import local as LS

    gp, pp = _panel(runs, tmp_path)
    run = D.run_main(_argv(runs, name, gp, pp), E.get_evaluator, EV.get_evolver, LS.get_local_search)
    D.compare(run, runs, name)
