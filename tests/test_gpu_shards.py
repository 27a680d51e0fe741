"""BASELINE config 3 on the HIP engine: a pop-1024, 2000 x 50k population sharded over 2 and 4
rank processes, each driving libtblup_gpu.so on its own shard (all on GPU 0 of the box, gloo
backend), through the drop-in evaluator's sharded path -- the fan-out / fan-in the reference
runs through its worker pool (tblup/evaluator.py:120-131, 392-403).  The all-gathered fitness
vector must equal one process's evaluation of the whole population bit for bit and the
oracle's exact form to 1e-9; bench.py's N > 1 path is rehearsed the same way."""
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import blup_oracle as O
from tests.helpers import shard_population

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POP, K = 1024, 1000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def panel(tmp_path_factory):
    d = tmp_path_factory.mktemp("shards")
    rng = np.random.default_rng(42)
    geno = O.synth_geno(rng, 2000, 50_000)
    pheno = rng.standard_normal(2000)
    np.save(d / "geno.npy", geno)
    np.save(d / "pheno.npy", pheno)
    return {"dir": d, "geno": geno, "pheno": pheno, "genomes": shard_population(POP, 50_000, K)}


@pytest.fixture(scope="module")
def single(panel, gpu):
    """One process, the whole population (the reference's single-node result)."""
    d = panel["dir"]
    res = {}
    for world in (2, 4):
        out = d / f"w{world}"
        out.mkdir(exist_ok=True)
        port = _free_port()
        ctx = mp.get_context("spawn")
        from tests import shard_worker
        procs = [ctx.Process(target=shard_worker.run, args=(r, world, port, str(d / "geno.npy"),
                                                             str(d / "pheno.npy"), POP, K, str(out)))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=400)
        for p in procs:
            if p.exitcode is None:
                p.kill()
            assert p.exitcode == 0, f"rank process failed ({p.exitcode})"
        res[world] = out
    meta = json.load(open(res[2] / "rank0.json"))
    from tblup_amd.engine import GpuBlupEngine
    with GpuBlupEngine(panel["geno"], panel["pheno"], device=0) as eng:
        fit = eng.evaluate(panel["genomes"], meta["T"], meta["V"], 0.4)
    return {"out": res, "T": meta["T"], "V": meta["V"], "fit": fit}


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_population_equals_single_process(panel, single, world):
    out = single["out"][world]
    from tblup_amd.distributed import shard_range
    for r in range(world):
        meta = json.load(open(out / f"rank{r}.json"))
        lo, hi = shard_range(POP, r, world)
        assert meta["seen"][0] == hi - lo                 # each rank evaluated only its own shard
        assert meta["group_after"] is False               # the evaluator destroyed the group it made
        assert meta["T"] == single["T"] and meta["V"] == single["V"]
        got = np.load(out / f"fit{r}.npy")
        np.testing.assert_array_equal(got, single["fit"])  # every rank holds the full vector, bit for bit


def test_sharded_population_matches_oracle(panel, single):
    got = np.load(single["out"][4] / "fit0.npy")
    geno = panel["geno"]
    for i in (0, 333, 777, POP - 1):
        f, _ = O.blup_grm_form(panel["genomes"][i], single["T"], single["V"], geno, panel["pheno"], 0.4)
        assert abs(got[i] - f) <= 1e-9, (i, got[i], f)


def test_sharded_testing_pass(panel, single):
    """evaluate_testing's batch shape (train = T u V, the test animals) through the same path,
    with fewer individuals than 2 x ranks + 1 -- uneven and one-element shards."""
    for world in (2, 4):
        out = single["out"][world]
        t0 = np.load(out / "test0.npy")
        assert len(t0) == 2 * world + 1
        for r in range(1, world):
            np.testing.assert_array_equal(np.load(out / f"test{r}.npy"), t0)


def test_bench_multi_rank_rehearsal(gpu, tmp_path):
    """bench.py's N > 1 line (config 3: pop 1024 sharded, strong scaling) from two ranks on this
    one GPU (gloo): the all-gathered population's fitness checksum equals the one-process
    config-3 run, and the line names config 3 with 512 individuals per GPU."""
    env = dict(os.environ, TBLUP_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
            "--no-events"]
    one = subprocess.run(base + ["--config", "config3"], env=env, capture_output=True, text=True, timeout=600)
    assert one.returncode == 0, one.stderr[-3000:]
    port = _free_port()
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port)] + base[1:] + ["--gpus", "2"],
                         env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert two.returncode == 0, two.stderr[-3000:]
    l1 = json.loads([x for x in one.stdout.splitlines() if x.startswith("{")][-1])
    l2 = json.loads([x for x in two.stdout.splitlines() if x.startswith("{")][-1])
    assert l1["config"]["workload"].startswith("config3") and l2["config"]["workload"].startswith("config3")
    assert l2["n_gpus"] == 2 and l2["config"]["pop_total"] == 1024 and l2["config"]["pop_per_gpu"] == 512
    assert l2["scaling"] == "strong"
    assert l1["fitness_checksum"] == l2["fitness_checksum"]


@pytest.mark.parametrize("case", ["rk_rand1", "intercv"])
def test_multi_rank_gpu_generations_reproduce_reference(gpu, golden_dir, tmp_path, case):
    """The GPU generation path at world 2 (gloo, both ranks on this GPU): GPU DE step, each rank
    evaluating ITS shard of the children speculatively while it copies ITS shard of their genomes
    into the node-shared host rows (tblup_amd/shmrows.py), one all-gather per generation -- every
    rank reproduces the reference's single-process main() run (tests/golden/main_runs.npz), and
    the speculative results and the shared rows are the ones used."""
    from tests import shard_worker
    z = np.load(os.path.join(golden_dir, "main_runs.npz"))
    np.save(tmp_path / "geno.npy", z["geno"].astype(np.float64))
    np.save(tmp_path / "pheno.npy", z["pheno"])
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=shard_worker.run_main_gpu, args=(r, 2, port, case, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=400)
    for p in procs:
        if p.exitcode is None:
            p.kill()
        assert p.exitcode == 0, f"rank process failed ({p.exitcode})"
    res = [json.load(open(tmp_path / f"main_gpu_rank{r}.json")) for r in range(2)]
    assert res[0]["taken"] == res[1]["taken"] and sum(res[0]["taken"]) >= 3   # both took the speculative results
    # the children's rows crossed through the node-shared ring (each rank copied its shard)
    assert res[0]["shared"] == res[1]["shared"] and sum(res[0]["shared"]) >= 3


RCCL_SNIPPET = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["TBLUP_ROOT"])
from tblup_amd import distributed as td
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
assert td.backend_name() == "RCCL"
loc = torch.arange(5, dtype=torch.float64, device="cuda") * 0.5
out = torch.empty(5, dtype=torch.float64, device="cuda")
td.allgather_device(out, loc)
torch.cuda.synchronize()
assert torch.equal(out.cpu(), loc.cpu())
full = td.allgather_fitness(np.array([0.25, -1.0, 3.0]), 3, device=0)
assert np.array_equal(full, [0.25, -1.0, 3.0])
td.destroy()
print("rccl ok")
"""


def test_rccl_all_gather_on_device(gpu):
    """The multi-GPU path's collective on this box's GPU: an RCCL (backend "nccl") group of one
    rank, all_gather_into_tensor through `allgather_device` and `allgather_fitness` on device
    memory -- the RCCL library, its device-side init and the collective run on hardware (the 2-
    and 4-rank tests above share one GPU, which RCCL does not allow, so they use gloo)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", TBLUP_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", RCCL_SNIPPET], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "rccl ok" in r.stdout
