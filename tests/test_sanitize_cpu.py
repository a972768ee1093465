"""Host code under AddressSanitizer + UBSan (CPU only).

tools/sanitize builds trex_amd/csrc/plan.cpp (the topology planner every
Sankoff launch depends on) and oracle/cpu_port.c (the CPU baseline / checker)
with -fsanitize=address,undefined -fno-sanitize-recover=all and runs a driver
over random, quirky, cyclic and malformed trees.  Any sanitizer report makes
the driver exit non-zero.
"""

from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "sanitize")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_planner_and_cpu_port_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", SAN], check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="2")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(SAN, "build", "driver")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize ok" in r.stdout
