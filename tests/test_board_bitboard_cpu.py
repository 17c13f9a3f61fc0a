"""The select descent plays moves with the bitboard play_bb (az_device.h);
this compiles the device header for the host and checks play_bb against the
cell-scan play() -- itself pinned to the reference by the oracle and golden
tests -- on every action of every position of random games over 14 Connect-N
configurations (gravity and not, 1..128 cells, n larger than a side)."""
import os
import subprocess

import pytest

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_play_bb_matches_play(tmp_path):
    exe = tmp_path / "play_bb_check"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-I", os.path.join(R, "custom-alphazero_amd", "csrc"),
                    os.path.join(R, "tests", "native", "play_bb_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout
    assert "(0 also" not in out.stdout  # the one-word Connect-4 form (play_c64) was checked too
