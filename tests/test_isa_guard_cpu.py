"""Store-data register reuse guard.

Every gfx950 code object of the build is disassembled (llvm-objcopy
--dump-section=.hip_fatbin -> clang-offload-bundler -> llvm-objdump) and no
VMEM store of more than 64 bits may have its data VGPRs overwritten by one
of the next two issued instructions without an s_nop / vmcnt wait between
(tools/isa_store_guard.py).  The checker itself is pinned on the sequence
that corrupted DP-row bytes in round 5 (the pre-fix lane-per-site kernel's
transposed row store) and on its fixed form.
"""

import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_store_guard as guard  # noqa: E402

LLVM_OK = os.path.exists(os.path.join(guard.LLVM, "llvm-objdump"))

# llvm-objdump lines of the pre-fix build (056ab53^, sankoff_site_kernel<1,20>)
_BAD = """
0000000000001000 <_ZN4trex4siteE>:
\tds_write_b128 v70, v[56:59]                                // 000000001000: D9BE0000 0000380F
\tbuffer_store_dwordx4 v[60:63], v71, s[52:55], s8 offen    // 000000001008: E07C1000 08053C47
\tds_read_b128 v[60:63], v70 offset:1024                    // 000000001010: D9FE0400 3C000046
\ts_waitcnt lgkmcnt(0)                                       // 000000001018: BF8CC07F
\tbuffer_store_dwordx4 v[60:63], v75, s[52:55], s8 offen    // 000000001020: E07C1000 08053C4B
\tv_min_f32_e32 v60, v56, v57                                // 000000001028: 1E787338
\ts_endpgm                                                   // 000000001030: BF810000
"""
# the fixed form: the data registers held through an s_nop after the store
_GOOD = """
0000000000001000 <_ZN4trex4siteE>:
\tbuffer_store_dwordx4 v[60:63], v75, s[52:55], s8 offen    // 000000001020: E07C1000 08053C4B
\ts_nop 4                                                    // 000000001028: BF800004
\tv_min_f32_e32 v60, v56, v57                                // 00000000102C: 1E787338
\tglobal_store_dwordx4 v[2:3], v[8:11], off                  // 000000001030: DC7C8000 007D0802
\tv_add_f32_e32 v12, v8, v9                                  // 000000001038: 02181308
\tbuffer_store_dwordx2 v[20:21], v1, s[4:7], 0 offen         // 00000000103C: E0741000 80011401
\tv_mov_b32_e32 v20, 0                                       // 000000001044: 7E280280
\ts_endpgm                                                   // 000000001048: BF810000
"""


def test_guard_flags_the_round5_sequence():
    bad = guard.scan_disassembly(_BAD)
    assert len(bad) == 2, bad
    assert "ds_read_b128 v[60:63]" in bad[0] and "v_min_f32_e32 v60" in bad[1]


def test_guard_accepts_held_registers_and_narrow_stores():
    # s_nop between; a global store whose data (not its address) is read
    # again; a 64-bit store (outside the rule)
    assert guard.scan_disassembly(_GOOD) == []


def test_guard_global_store_data_operand():
    text = ("0000000000000000 <_Zk>:\n"
            "\tglobal_store_dwordx4 v[2:3], v[8:11], off\n"
            "\tv_mov_b32_e32 v9, 0\n")
    assert len(guard.scan_disassembly(text)) == 1
    text2 = ("0000000000000000 <_Zk>:\n"
             "\tglobal_store_dwordx4 v[2:3], v[8:11], off\n"
             "\tv_mov_b32_e32 v2, 0\n")  # the address pair may be reused at once
    assert guard.scan_disassembly(text2) == []


@pytest.mark.skipif(not LLVM_OK, reason="ROCm LLVM tools absent")
def test_build_has_no_store_data_reuse():
    objs = sorted(glob.glob(os.path.join(ROOT, "trex_amd", "csrc", "build", "*.o")))
    if len(objs) < 9:  # not built yet in this checkout: build it (what build() runs)
        subprocess.run(["make", "-j", str(min(8, os.cpu_count() or 1)), "-C",
                        os.path.join(ROOT, "trex_amd", "csrc")], check=True,
                       capture_output=True, timeout=1500)
        objs = sorted(glob.glob(os.path.join(ROOT, "trex_amd", "csrc", "build", "*.o")))
    n, bad = guard.scan_objects(objs)
    assert n > 300, f"only {n} wide VMEM stores found: disassembly not parsed?"
    assert bad == [], "\n".join(bad[:20])
