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


def _scan(text):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import lds_wait_scan
    return lds_wait_scan.scan(text.strip().splitlines())


def test_scan_flags_straight_line_and_loop_carried_reads():
    straight = """
k:
  ds_read_b128 v[0:3], v10
  v_mfma_f32_16x16x32_bf16 v[20:23], v[0:3], v[4:7], v[20:23]
  s_endpgm
"""
    assert len(_scan(straight)) == 1
    # read issued at the bottom of the loop, consumed at the top after the back-edge
    carried = """
k:
  s_waitcnt lgkmcnt(0)
.LBB0_1:
  v_mfma_f32_16x16x32_bf16 v[20:23], v[0:3], v[4:7], v[20:23]
  ds_read_b128 v[0:3], v10
  s_cbranch_scc1 .LBB0_1
  s_waitcnt lgkmcnt(0)
  s_endpgm
"""
    assert len(_scan(carried)) == 1


def test_scan_ignores_reads_behind_an_unconditional_branch():
    # the block after s_branch is entered only through its label, on whose edges nothing is in flight
    jumped = """
k:
  ds_read_b128 v[0:3], v10
  s_branch .LBB0_2
.LBB0_1:
  v_mfma_f32_16x16x32_bf16 v[20:23], v[0:3], v[4:7], v[20:23]
  s_endpgm
.LBB0_2:
  s_waitcnt lgkmcnt(0)
  s_cbranch_scc1 .LBB0_1
  s_endpgm
"""
    assert _scan(jumped) == []
