"""Time the GPU DE step (tblup_de_step_device, pop x d on device) against the numpy
oracle of the reference's evolve loop on the host; prints one JSON line."""
import ctypes
import json
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from tblup_amd import _native  # noqa: E402
from tblup_amd.evolver import GpuDEStep  # noqa: E402


def main(pop=256, d=50000, reps=20):
    step = GpuDEStep.get(0)
    lib = _native.load()
    rng = np.random.default_rng(0)
    par = torch.from_numpy(rng.uniform(size=(pop, d))).cuda()
    chi = torch.empty_like(par)
    donors = np.ascontiguousarray(rng.integers(0, pop, size=(pop, 3)), dtype=np.int32)
    fixed = np.ascontiguousarray(rng.integers(0, d, size=pop), dtype=np.int64)
    np.random.seed(0)
    st = np.random.get_state()
    key = np.array(st[1], dtype=np.uint32)
    pos = ctypes.c_int32(int(st[2]))
    U32 = ctypes.POINTER(ctypes.c_uint32)

    def run():
        _native.check("tblup_de_step_device", lib.tblup_de_step_device(
            step._ctx, 0, ctypes.c_void_p(par.data_ptr()), pop, d, d,
            donors.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), fixed.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            0.5, 0.8, 0, float(d - 1), key.ctypes.data_as(U32), ctypes.byref(pos), ctypes.c_void_p(chi.data_ptr()), d,
            None))
    t0 = time.perf_counter()
    run()
    first = time.perf_counter() - t0
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    # host path (tblup_de_step: H2D parents, D2H children)
    hp = par.cpu().numpy()
    t0 = time.perf_counter()
    step.step(0, hp, donors, fixed, 0.5, 0.8, False, d - 1)
    host_path = time.perf_counter() - t0
    # numpy oracle of the reference loop (host)
    from oracle import de_oracle as D
    genomes = [hp[i] for i in range(pop)]
    random.seed(0)
    t0 = time.perf_counter()
    D.de_generation(genomes, [0.0] * pop, 1, "de_rand_1", d, 0.8, 0.5, False)
    cpu = time.perf_counter() - t0
    print(json.dumps({"pop": pop, "d": d, "gpu_de_ms_median": 1e3 * float(np.median(ts)), "gpu_de_ms_min": 1e3 * min(ts),
                      "first_call_ms (incl. jump polynomials)": 1e3 * first, "host_pointer_path_ms": 1e3 * host_path,
                      "numpy_oracle_ms": 1e3 * cpu}))


if __name__ == "__main__":
    main()
