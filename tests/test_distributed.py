"""Multi-process population sharding + fitness all-gather (world_size 2, gloo backend on CPU)."""
import json
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from tblup_amd.distributed import shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    for n in (0, 1, 7, 32, 33):
        for ws in (1, 2, 3, 8):
            spans = [shard_range(n, r, ws) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_two_rank_gloo_matches_single_process(golden_dir, tmp_path):
    from tests import dist_worker
    z = np.load(os.path.join(golden_dir, "blup_200x1000.npz"))
    flow = np.load(os.path.join(golden_dir, "evaluator_flow.npz"))
    gp, pp, kp = str(tmp_path / "g.npy"), str(tmp_path / "p.npy"), str(tmp_path / "k.npy")
    np.save(gp, z["geno"].astype(np.float64))
    np.save(pp, z["pheno"])
    keys = flow["flow_keys"][:31]          # odd count: uneven shards
    np.save(kp, keys)
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=dist_worker.run, args=(r, 2, port, gp, pp, kp, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    expect = flow["flow_fitness"][:31]
    for r in range(2):
        np.testing.assert_allclose(res[r]["fitness"], expect, rtol=0, atol=1e-12)
        lo, hi = res[r]["shard"]
        assert res[r]["evaluated"][0] == hi - lo      # each rank computed only its own block
    assert res[0]["testing"] == res[1]["testing"]
    np.testing.assert_allclose(res[0]["testing"], flow["flow_testing"][:31], rtol=0, atol=1e-12)


@pytest.mark.parametrize("case", ["rk_rand1", "removal_testing_knockout", "intracv"])
def test_two_rank_main_flow_without_preinitialised_group(golden_dir, tmp_path, case):
    """torchrun-style main.py run on 2 ranks where nothing but the evaluator creates the
    process group (ParallelEvaluator.__enter__, the reference's worker start-up point,
    evaluator.py:120-131): both ranks reproduce the reference's single-process run, each
    evaluates only its shard of every batch (32 -> 16 + 16), the group exists inside the
    `with evaluator:` block and is gone after it (the knockout search then runs per rank on
    a short-lived context)."""
    from tests import dist_worker
    z = np.load(os.path.join(golden_dir, "main_runs.npz"))
    np.save(tmp_path / "geno.npy", z["geno"].astype(np.float64))
    np.save(tmp_path / "pheno.npy", z["pheno"])
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=dist_worker.run_main_flow, args=(r, 2, port, case, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    res = [json.load(open(tmp_path / f"main_rank{r}.json")) for r in range(2)]
    for r in range(2):
        assert res[r]["group_inside"][0] is True and res[r]["group_after"] is False
        pop_batches = [n for n in res[r]["seen"][:2]]
        assert pop_batches == [16, 16]          # generation 0 and 1: 32 individuals over 2 ranks


def test_rank_failure_raises_on_every_rank(tmp_path):
    """An evaluation that fails on one rank only (an out-of-bounds index in its shard)
    raises the same error on every rank instead of leaving the others in the all-gather; the
    status words of every rank travel in the fitness all-gather (element-wise max)."""
    from tests import dist_worker
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=dist_worker.run_rank_error, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = [json.load(open(tmp_path / f"err_rank{r}.json")) for r in range(2)]
    for r in range(2):
        assert res[r]["status_max"] == [1, 5]
        assert res[r]["full"] == [0.0] * 4 + [1.0] * 3
        assert res[r]["raised"] == "TblupIndexError"
        assert res[r]["raised_other"] == ("ValueError" if r == 0 else "TblupError")
        assert res[r]["clean"] == [0.5] * 4 + [1.5] * 4


def test_two_rank_panel_start_up_is_node_shared(tmp_path):
    """the float64 .npy panel is streamed into int8 once per node (a /dev/shm
    segment both ranks map) instead of loaded whole as float64 by every rank: each rank's peak RSS
    grows by well under the float64 panel's size, both see the same int8 panel, and the segment's
    name is gone once both hold it."""
    from tests import dist_worker
    rng = np.random.default_rng(9)
    n, p = 1000, 40_000
    g = rng.integers(0, 3, size=(n, p)).astype(np.int8)
    path = str(tmp_path / "geno.npy")
    np.save(path, g.astype(np.float64))          # 320 MB of float64, as the reference stores it
    f64 = n * p * 8
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=dist_worker.run_panel_load, args=(r, 2, port, path, str(tmp_path))) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
        assert pr.exitcode == 0
    res = [json.load(open(tmp_path / f"panel_rank{r}.json")) for r in range(2)]
    want = int(g.astype(np.int64).sum())
    print("peak RSS growth per rank (bytes):", [res[r]["grow"] for r in range(2)], "float64 panel:", f64)
    for r in range(2):
        assert res[r]["dtype"] == "int8" and res[r]["shape"] == [n, p] and res[r]["rows"] == n
        assert res[r]["checksum"] == want
        assert res[r]["shared"]
        assert res[r]["grow"] < f64 // 2, (r, res[r]["grow"], f64)
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("tblup_panel_")]


def test_panel_reader_streams_and_validates(tmp_path):
    """tblup_amd.panel.read_panel_int8 (single process): C- and Fortran-ordered .npy panels of any
    integral dtype, chunk boundaries that split the rows unevenly, and the {0,1,2} contract."""
    from tblup_amd.panel import convert_rows, read_panel_int8
    rng = np.random.default_rng(3)
    g = rng.integers(0, 3, size=(257, 1031)).astype(np.float64)
    for arr in (g, np.asfortranarray(g), g.astype(np.float32), g.astype(np.int8), g.astype(np.int64)):
        p = str(tmp_path / "g.npy")
        np.save(p, arr)
        for cb in (1 << 20, 12_345, 1):
            out = read_panel_int8(p, chunk_bytes=cb)
            assert out.dtype == np.int8 and np.array_equal(out, g)
    assert np.array_equal(convert_rows(g, chunk_bytes=4096), g.astype(np.int8))
    for bad in (0.5, 3.0, -1.0):
        h = g.copy()
        h[200, 1000] = bad
        np.save(str(tmp_path / "h.npy"), h)
        with pytest.raises(ValueError):
            read_panel_int8(str(tmp_path / "h.npy"))
