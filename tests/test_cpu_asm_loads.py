"""The LDS walk's record loads are inline asm retired by counted vmcnt waits (csrc/edge_lds.hip):
the compiler does not know they are in flight, so this compiles the file for gfx950 and follows
every path of each kernel (tools/check_asm_loads.py) for an instruction that touches a register
such a load may still be writing. Needs hipcc (this container and the GPU boxes have it)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_no_register_read_while_its_asm_load_is_in_flight():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_loads.py")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "3 kernels scanned, 0 findings" in r.stdout   # the concat walk (two variants) + the head-mean walk
