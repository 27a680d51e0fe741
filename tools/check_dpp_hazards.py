"""Static check of the DPP read-after-VALU-write hazard in the shipped gfx950 code objects.

factor16 (k_chol.hip) issues its pivot updates as `v_fmac_f64_dpp` inline asm.  The ISA needs
2 wait states between a VALU write of a VGPR and a DPP read of it (src0 of a DPP instruction);
the compiler's hazard recognizer cannot see into inline asm, so the source guards the one fmac
per pivot whose src0 the previous instruction may have written (`s_nop 1`) and relies on the
compiler not placing a VALU write of the other fmacs' src0 right before them.  This tool checks
that assumption on the ACTUAL library: it pulls every gfx950 code object out of the .so's
offload bundles, disassembles it and, for every DPP instruction, walks back through the
preceding instructions until 2 wait states (s_nop N = N + 1) have passed; any VALU among them
that writes a VGPR of the DPP source is a violation.

    python tools/check_dpp_hazards.py [path/to/libtblup_gpu.so]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
WAIT_STATES = 2

_VREG = re.compile(r"^v(?:\[(\d+):(\d+)\]|(\d+))$")


def code_objects(lib_path):
    """Every gfx950 code object inside the library's offload bundles (bytes)."""
    data = open(lib_path, "rb").read()
    out, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return out
        (num,) = struct.unpack_from("<Q", data, i + len(MAGIC))
        off = i + len(MAGIC) + 8
        for _ in range(num):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode(errors="replace")
            off += tl
            if "gfx950" in triple and sz:
                out.append(data[i + o:i + o + sz])
        pos = i + 1


def _regs(op):
    m = _VREG.match(op.strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def _parse(line):
    """(mnemonic, operands) of one disassembled instruction line, or None."""
    code = line.split("//")[0].strip()
    if not code or code.endswith(":") or code.startswith(("<", ".")):
        return None
    parts = code.split(None, 1)
    mn = parts[0]
    ops = []
    if len(parts) > 1:
        ops = [o.strip() for o in parts[1].split(",")]
        # trailing modifiers (row_newbcast:1 row_mask:...) ride on the last operand
        ops[-1] = ops[-1].split()[0] if ops[-1] else ops[-1]
    return mn, ops


def _vgpr_writes(mn, ops):
    """VGPRs a VALU instruction writes (empty for non-VALU and SGPR-destination VALU)."""
    if not mn.startswith("v_") or not ops:
        return set()
    if mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    w = set(_regs(ops[0]))
    if "permlane" in mn and "swap" in mn and len(ops) > 1:   # both operands are written
        w |= _regs(ops[1])
    return w


def check_disassembly(text):
    """Violations [(index, dpp line, writer line)] in one disassembly listing."""
    insts = []
    for line in text.splitlines():
        p = _parse(line)
        if p is not None:
            insts.append((p[0], p[1], line.strip()))
    bad = []
    for i, (mn, ops, line) in enumerate(insts):
        if not (mn.startswith("v_") and "_dpp" in mn) or len(ops) < 2:
            continue
        src0 = _regs(ops[1])
        waited = 0
        j = i - 1
        while j >= 0 and waited < WAIT_STATES:
            pm, pops, pline = insts[j]
            if pm.startswith(("s_endpgm", "s_branch", "s_cbranch", "s_setpc", "s_swappc")):
                break
            if pm == "s_nop":
                waited += int(pops[0], 0) + 1 if pops else 1
            else:
                if src0 & _vgpr_writes(pm, pops):
                    bad.append((i, line, pline))
                    break
                waited += 1
            j -= 1
    return bad


def check(lib_path=None):
    lib_path = lib_path or os.path.join(ROOT, "tblup_amd", "lib", "libtblup_gpu.so")
    cos = code_objects(lib_path)
    if not cos:
        raise RuntimeError(f"no gfx950 code object in {lib_path}")
    n_dpp, bad = 0, []
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(cos):
            f = os.path.join(td, f"co{k}.o")
            with open(f, "wb") as fh:
                fh.write(co)
            text = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f], check=True, capture_output=True,
                                  text=True).stdout
            n_dpp += sum(1 for line in text.splitlines() if "_dpp" in line.split("//")[0])
            bad += check_disassembly(text)
    return n_dpp, bad


if __name__ == "__main__":
    n, bad = check(sys.argv[1] if len(sys.argv) > 1 else None)
    print(f"{n} DPP instructions checked, {len(bad)} hazard(s)")
    for _, dpp, w in bad:
        print("  writer:", w, "\n  dpp:   ", dpp)
    sys.exit(1 if bad else 0)
