"""Device decode (k_decode_topk) at config 2: 256 rows of 50k uniform keys, k = 1000; average
kernel time over repeated launches on one stream (HIP events), and the algorithmic bytes
(one read of every key row + the k int64 indices written) per launch."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(B=256, d=50_000, k=1000, reps=50):
    import torch
    from tblup_amd.evolver import GpuDEStep
    step = GpuDEStep.get(0)   # a panel-less context
    keys = torch.rand(B, d, dtype=torch.float64, device="cuda")
    off = np.arange(B + 1, dtype=np.int64) * k
    d_off = torch.from_numpy(off).cuda()
    d_idx = torch.empty(B * k, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    lib, ctx = step._lib, step._ctx
    import ctypes
    from tblup_amd import _native

    def run():
        _native.check("tblup_decode_topk_device", lib.tblup_decode_topk_device(
            ctx, ctypes.c_void_p(keys.data_ptr()), B, d, d, ctypes.c_void_p(d_off.data_ptr()),
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.c_void_p(d_idx.data_ptr()),
            ctypes.c_void_p(s.cuda_stream)))
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    got = d_idx.view(B, k).cpu().numpy()
    ref = np.argsort(keys.cpu().numpy(), axis=1, kind="stable")[:, -k:]
    algo = B * d * 8 + B * k * 8
    print(json.dumps({"B": B, "d": d, "k": k, "ms_per_launch": round(ms, 4), "algorithmic_bytes": algo,
                      "achieved_GBs": round(algo / (ms * 1e-3) / 1e9, 1), "exact": bool((got == ref).all())}))


if __name__ == "__main__":
    main()
