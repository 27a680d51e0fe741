"""Node-shared host rows of a multi-rank generation (tblup_amd/shmrows.py), world size 2 on the
CPU (gloo): every rank sees the rows every rank wrote, the ranks agree on the segment, and a
segment is reused only once no rank holds a row of it any more."""
import json
import multiprocessing as mp
import socket


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_share_and_recycle_segments(tmp_path):
    from tests import shm_worker
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=shm_worker.run, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    logs = [json.load(open(tmp_path / f"shm{r}.json")) for r in range(2)]
    assert logs[0] == logs[1]                       # the same segment on both ranks, every generation
    segs = [e["seg"] for e in logs[0]]
    assert all(e["ok"] for e in logs[0])            # each rank sees both shards
    # 3 segments: gen 1's segment (1) stays held by rank 1 until generation 4, so generations 2-4
    # cycle through the other two only; afterwards segment 1 is free again
    assert segs[:2] == [0, 1]
    assert 1 not in segs[2:5]
    assert segs[2:5] == [2, 0, 2]
