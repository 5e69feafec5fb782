"""The inline-asm LDS reads (ds_read_b64_tr_b16) are invisible to the compiler's wait insertion: an
MFMA may only read their registers after an explicit `s_waitcnt lgkmcnt`. tools/lds_wait_scan.py
compiles every kernel source to gfx950 assembly and finds such uses (CPU only: hipcc cross-compiles)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc absent")
def test_no_mfma_reads_an_lds_read_in_flight():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "lds_wait_scan.py")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
