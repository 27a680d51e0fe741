"""Time k_decode_topk on pop x d device-resident random keys (k per individual); one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tblup_amd.evolver import GpuDEStep  # noqa: E402  (panel-less context)
from tblup_amd import _native  # noqa: E402
import ctypes  # noqa: E402


def main(pop=256, d=50000, k=1000, reps=10):
    ctx = GpuDEStep.get(0)
    lib = _native.load()
    keys = torch.from_numpy(np.random.default_rng(0).uniform(size=(pop, d))).cuda()
    off = np.arange(pop + 1, dtype=np.int64) * k
    d_off = torch.from_numpy(off).cuda()
    d_idx = torch.empty(pop * k, dtype=torch.int64, device="cuda")
    P64 = ctypes.POINTER(ctypes.c_int64)

    def run():
        _native.check("decode", lib.tblup_decode_topk_device(ctx._ctx, ctypes.c_void_p(keys.data_ptr()), pop, d, d,
                                                             ctypes.c_void_p(d_off.data_ptr()),
                                                             off.ctypes.data_as(P64),
                                                             ctypes.c_void_p(d_idx.data_ptr()), None))
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    print(json.dumps({"pop": pop, "d": d, "k": k, "decode_ms": (time.perf_counter() - t0) / reps * 1e3,
                      "dbg": os.environ.get("TBLUP_DEC_DBG", "0")}))


if __name__ == "__main__":
    main()
