"""tblup_amd — MI355X-native GBLUP fitness evaluator for TBLUP (ianwhale/tblup).

The package mirrors the reference's evaluator plugin API (`tblup.evaluator`)
on top of hand-written gfx950 HIP kernels reached through the C ABI in
include/tblup_gpu.h (libtblup_gpu.so, built in-tree under tblup_amd/lib/).
"""
from .evaluator import (BlupParallelEvaluator, Evaluator, InterGCVBlupParallelEvaluator,
                        IntraGCVBlupParallelEvaluator, MonteCarloCVBlupParallelEvaluator, ParallelEvaluator,
                        SNPRemovalHandler, get_evaluator)

__all__ = [
    "Evaluator", "ParallelEvaluator", "BlupParallelEvaluator", "InterGCVBlupParallelEvaluator",
    "IntraGCVBlupParallelEvaluator", "MonteCarloCVBlupParallelEvaluator", "SNPRemovalHandler", "get_evaluator",
]
__version__ = "0.1.0"
