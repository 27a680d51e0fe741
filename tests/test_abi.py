"""C-ABI library checks that need no GPU: it loads and exports every declared symbol."""
import ctypes
import os
import re

import pytest

from tblup_amd import _native

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "tblup_gpu.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tblup_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = _native.load()
    names = declared_functions()
    assert len(names) >= 14
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(_native.SIGNATURES), "ctypes signature table out of sync with the header"


def test_version_and_error_strings():
    lib = _native.load()
    assert lib.tblup_version().startswith(b"tblup_gpu")
    assert isinstance(lib.tblup_last_error(), bytes)


def test_device_count_without_gpu_does_not_crash():
    assert _native.device_count() >= 0


def test_bad_arguments_return_status_not_crash():
    lib = _native.load()
    out = ctypes.c_void_p()
    rc = lib.tblup_ctx_create(None, 10, 10, 0, None, 0, ctypes.byref(out))
    assert rc == -1
    assert b"bad" in lib.tblup_last_error()
    assert lib.tblup_ctx_destroy(None) == 0
    assert lib.tblup_set_split(None, 0, None, 0, None, 0) == -1


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError):
        _native.load()


def test_no_dpp_read_after_valu_write_hazard_in_shipped_code():
    """factor16's v_fmac_f64_dpp pivot updates are inline asm the compiler's hazard recognizer
    cannot see into: check the built gfx950 code objects themselves -- no VALU
    write of a DPP instruction's src0 within the 2 wait states the ISA requires."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import check_dpp_hazards as C
    if not os.path.isfile(C.OBJDUMP):
        pytest.skip("llvm-objdump not available")
    n_dpp, bad = C.check(_native.LIB_PATH)
    assert n_dpp >= 500                     # factor16's broadcast-fmacs are in the library
    assert not bad, bad[:3]
    # the checker itself flags the pattern it guards against
    listing = ("v_mov_b32_e32 v65, v34\n\ts_nop 0\n"
               "v_fmac_f64_dpp v[64:65], v[64:65], v[34:35] row_newbcast:0 row_mask:0xf bank_mask:0xf\n")
    assert len(C.check_disassembly(listing)) == 1
    assert not C.check_disassembly(listing.replace("s_nop 0", "s_nop 1"))
