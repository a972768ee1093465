"""Store-data register reuse check over the gfx950 code objects of the build.

A VMEM store of more than 64 bits (buffer/global/flat *_dwordx3 / _dwordx4,
*_b96 / *_b128) reads its data VGPRs after it issues.  On MI355X a VALU
result written into one of those VGPRs right behind the store -- or an LDS
read returning into them -- changed the bytes the store wrote (round 5:
corrupted DP-row bytes of the lane-per-site kernel, DESIGN.md section 5.8;
tools/micro/store_reuse.hip reproduces it).  LLVM inserts the documented
wait state only for stores whose soffset is not an SGPR, so this checker
enforces the stronger rule on every kernel: no instruction among the next
WINDOW issued after such a store writes one of its data VGPRs unless an
``s_nop`` or an ``s_waitcnt vmcnt`` lies between them.

usage: python tools/isa_store_guard.py [objects...]   (default: the build's
trex_amd/csrc/build/*.o); exit 1 and a listing when a violation is found.
Used by tests/test_isa_guard_cpu.py.
"""

from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
WINDOW = 2

_WIDE_STORE = re.compile(r"^(buffer|global|flat)_store_(dwordx[34]|b96|b128)\b")
_VREG = re.compile(r"^v\[(\d+):(\d+)\]$|^v(\d+)$")


def _vregs(tok: str) -> set[int]:
    m = _VREG.match(tok.strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def _writes_vgpr(op: str) -> bool:
    """Instructions whose first operand is a VGPR destination."""
    if op.startswith("v_") and not op.startswith(("v_cmpx", "v_readlane", "v_readfirstlane")):
        return True
    return op.startswith(("ds_read", "ds_load", "buffer_load", "global_load", "flat_load",
                          "scratch_load", "ds_bpermute", "ds_permute", "ds_swizzle"))


def code_object(obj: str, out_dir: str) -> str | None:
    """The gfx950 code object bundled in a host object's .hip_fatbin."""
    fat = os.path.join(out_dir, os.path.basename(obj) + ".fatbin")
    co = os.path.join(out_dir, os.path.basename(obj) + ".co")
    r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj],
                       capture_output=True, text=True)
    if r.returncode != 0 or not os.path.exists(fat):
        return None  # a host-only object (plan.cpp, comm.cpp)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    f"--input={fat}", f"--targets={TARGET}", f"--output={co}"], check=True)
    return co


def scan_disassembly(text: str, window: int = WINDOW) -> list[str]:
    """Violations in llvm-objdump -d output (one string per violation)."""
    bad = []
    func = "?"
    insts: list[tuple[str, str]] = []
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line.strip())
        if m:
            func = m.group(1)
            insts.append(("<func>", func))
            continue
        s = line.strip()
        if not s or s.startswith(("Disassembly", "/")) or s.endswith(":"):
            continue
        s = s.split("//")[0].strip()
        if s:
            insts.append((func, s))
    for i, (fn, s) in enumerate(insts):
        op = s.split()[0]
        if not _WIDE_STORE.match(op):
            continue
        data = _vregs(s.split(None, 1)[1].split(",")[0] if op.startswith("buffer") else
                      s.split(None, 1)[1].split(",")[1])
        for j in range(1, window + 1):
            if i + j >= len(insts):
                break
            fn2, t = insts[i + j]
            if fn2 == "<func>":
                break
            op2 = t.split()[0]
            if op2.startswith("s_nop") or (op2 == "s_waitcnt" and "vmcnt" in t):
                break
            if op2.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                break
            if _writes_vgpr(op2) and len(t.split(None, 1)) > 1:
                dst = _vregs(t.split(None, 1)[1].split(",")[0])
                if dst & data:
                    bad.append(f"{fn}: '{s}' then '{t}' ({j} later)")
    return bad


def scan_objects(objs: list[str], window: int = WINDOW) -> tuple[int, list[str]]:
    n_stores = 0
    bad: list[str] = []
    with tempfile.TemporaryDirectory() as d:
        for obj in objs:
            co = code_object(obj, d)
            if co is None:
                continue
            text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co],
                                  capture_output=True, text=True, check=True).stdout
            n_stores += sum(1 for ln in text.splitlines()
                            if _WIDE_STORE.match(ln.strip().split(" ")[0] if ln.strip() else ""))
            bad += [f"{os.path.basename(obj)}: {b}" for b in scan_disassembly(text, window)]
    return n_stores, bad


def main(argv: list[str]) -> int:
    objs = argv or sorted(glob.glob(os.path.join(ROOT, "trex_amd", "csrc", "build", "*.o")))
    n, bad = scan_objects(objs)
    print(f"{len(objs)} objects, {n} wide VMEM stores, {len(bad)} violations")
    for b in bad[:50]:
        print("  " + b)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
