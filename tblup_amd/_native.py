"""ctypes binding of libtblup_gpu.so (the C ABI declared in include/tblup_gpu.h).

The library is built in-tree by `__graft_entry__.build()` (or `make -C
tblup_amd/csrc`) into `tblup_amd/lib/libtblup_gpu.so`.  There is no CPU
fallback: if the library is missing, `load()` raises ImportError.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TBLUP_GPU_LIB", os.path.join(_HERE, "lib", "libtblup_gpu.so"))

BRANCH = {"auto": 0, "gblup": 1, "snp": 2}
LAYOUT_ANIMAL_MAJOR = 0
LAYOUT_SNP_MAJOR = 1
N_KCLASS = 6
MAX_TRAITS = 4
ERR_STATE = -4   # TBLUP_ERR_STATE: call out of order
ERR_INDEX = -5   # TBLUP_ERR_INDEX: numpy's IndexError for data[:, indices]
KCLASS_NAMES = ("stats", "gather", "grm", "chol_diag", "chol_offdiag", "solve")
CHAIN_EXPIRED = ("chained solve: a block-row hand-off wait expired (CHAIN_SPIN_MAX polls); the affected "
                 "individuals' fitnesses are invalid")

# Every symbol of include/tblup_gpu.h with (restype, argtypes).
_c = ctypes
_P = _c.c_void_p
_I64P = _c.POINTER(_c.c_int64)
_DP = _c.POINTER(_c.c_double)
_I32P = _c.POINTER(_c.c_int32)
_U32P = _c.POINTER(_c.c_uint32)
SIGNATURES = {
    "tblup_last_error": (_c.c_char_p, []),
    "tblup_version": (_c.c_char_p, []),
    "tblup_device_count": (_c.c_int, [_c.POINTER(_c.c_int)]),
    "tblup_ctx_create": (_c.c_int, [_P, _c.c_int64, _c.c_int64, _c.c_int, _DP, _c.c_int, _c.POINTER(_P)]),
    "tblup_ctx_destroy": (_c.c_int, [_P]),
    "tblup_set_split": (_c.c_int, [_P, _c.c_int, _I64P, _c.c_int64, _I64P, _c.c_int64]),
    "tblup_drop_split": (_c.c_int, [_P, _c.c_int]),
    "tblup_set_traits": (_c.c_int, [_P, _DP, _c.c_int64]),
    "tblup_get_traits": (_c.c_int, [_P, _I64P]),
    "tblup_eval_batch": (_c.c_int, [_P, _c.c_int, _I64P, _I64P, _c.c_int64, _c.c_double, _c.c_int, _DP, _DP]),
    "tblup_eval_batch_device": (_c.c_int, [_P, _c.c_int, _P, _P, _I64P, _c.c_int64, _c.c_double, _c.c_int, _P, _P,
                                           _P]),
    "tblup_eval_folds": (_c.c_int, [_P, _I32P, _c.c_int, _I64P, _I64P, _c.c_int64, _c.c_double, _c.c_int, _DP]),
    "tblup_eval_folds_device": (_c.c_int, [_P, _I32P, _c.c_int, _P, _P, _I64P, _c.c_int64, _c.c_double, _c.c_int,
                                           _P, _P]),
    "tblup_set_profiling": (_c.c_int, [_P, _c.c_int]),
    "tblup_get_profile": (_c.c_int, [_P, _DP, _I64P, _DP, _DP]),
    "tblup_reset_profile": (_c.c_int, [_P]),
    "tblup_debug_grm": (_c.c_int, [_P, _c.c_int, _I64P, _c.c_int64, _c.c_double, _c.c_int, _c.c_int, _DP, _DP]),
    "tblup_mem_info": (_c.c_int, [_P, _I64P]),
    "tblup_index_error": (_c.c_int, [_P, _P, _c.POINTER(_c.c_int)]),
    "tblup_solve_error": (_c.c_int, [_P, _P, _c.POINTER(_c.c_int)]),
    "tblup_status_async": (_c.c_int, [_P, _P, _P]),
    "tblup_chain_recoveries": (_c.c_int, [_P, _I64P]),
    "tblup_host_register": (_c.c_int, [_P, _c.c_int64]),
    "tblup_host_unregister": (_c.c_int, [_P]),
    "tblup_get_wg_trace": (_c.c_int, [_P, _c.POINTER(_c.c_uint64), _c.c_int64, _I64P]),
    "tblup_decode_topk": (_c.c_int, [_P, _DP, _c.c_int64, _c.c_int64, _I64P, _I64P]),
    "tblup_decode_topk_device": (_c.c_int, [_P, _P, _c.c_int64, _c.c_int64, _c.c_int64, _P, _I64P, _P, _P]),
    "tblup_de_step": (_c.c_int, [_P, _c.c_int, _DP, _c.c_int64, _c.c_int64, _I32P, _I64P, _c.c_double, _c.c_double,
                                 _c.c_int, _c.c_double, _U32P, _I32P, _DP]),
    "tblup_de_step_device": (_c.c_int, [_P, _c.c_int, _P, _c.c_int64, _c.c_int64, _c.c_int64, _I32P, _I64P,
                                        _c.c_double, _c.c_double, _c.c_int, _c.c_double, _U32P, _I32P, _P,
                                        _c.c_int64, _P]),
    "tblup_de_step_device_async": (_c.c_int, [_P, _c.c_int, _P, _c.c_int64, _c.c_int64, _c.c_int64, _I32P, _I64P,
                                              _c.c_double, _c.c_double, _c.c_int, _c.c_double, _U32P, _c.c_int32,
                                              _P, _c.c_int64, _P]),
    "tblup_de_state_wait": (_c.c_int, [_P, _U32P, _I32P]),
    "tblup_de_step_device_async_mix": (_c.c_int, [_P, _I32P, _DP, _DP, _P, _c.c_int64, _c.c_int64, _c.c_int64, _I32P,
                                                  _I64P, _c.c_int, _c.c_double, _U32P, _c.c_int32, _P, _c.c_int64,
                                                  _P]),
    "tblup_grm": (_c.c_int, [_P, _I64P, _c.c_int64, _DP]),
    "tblup_snp_scan": (_c.c_int, [_P, _I64P, _c.c_int64, _DP, _I64P, _I64P, _DP]),
    "tblup_mt19937_jump": (_c.c_int, [_U32P, _c.c_int32, _c.c_uint64, _U32P, _I32P]),
    "tblup_de_donors": (_c.c_int, [_c.c_int, _c.c_int64, _c.c_int64, _c.c_int32, _U32P, _I32P, _I32P, _I64P]),
    "tblup_gather_rows": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_void_p,
                                     _c.c_void_p]),
}
DE_STRATEGY = {"de_rand_1": 0, "de_currenttobest_1": 1}


class TblupError(RuntimeError):
    """Raised when a C-ABI call returns a non-zero status."""

    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


class TblupIndexError(TblupError, IndexError):
    """A selected-SNP index outside [-P, P): what numpy raises for the reference's
    data[:, indices] (evaluator.py:275/298)."""


_lib = None


def load():
    """Load (once) and return the ctypes library; ImportError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (SONAME
    # libamdhip64.so.7) and loads it by file name, so if /opt/rocm's copy were loaded
    # first (by this library) torch would bring a second runtime and find no GPU.
    # Importing torch first makes this library bind to torch's already-loaded runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.isfile(LIB_PATH):
        raise ImportError(
            f"libtblup_gpu.so not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(fn_name, rc):
    if rc != 0:
        msg = load().tblup_last_error().decode(errors="replace")
        raise (TblupIndexError if rc == ERR_INDEX else TblupError)(fn_name, rc, msg)
    return rc


def device_count():
    n = ctypes.c_int(0)
    check("tblup_device_count", load().tblup_device_count(ctypes.byref(n)))
    return n.value
