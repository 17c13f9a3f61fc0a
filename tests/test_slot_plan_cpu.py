"""The tower's slot plan, checked on the host against libaz.so
over every board shape 3..11 x 3..11 with a tower tile: each pixel of a full
tile in exactly one slot, the pads filling the rest, every skipped
(block, tap) pair adding exact zeros (each pixel of the block has that tap's
neighbour off its board), and at most a few 2-way LDS bank conflicts.  The
GPU test test_tower_slot_plan_is_bitwise_the_natural_order checks the
kernel's outputs with and without the plan."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "custom-alphazero_amd", "custom_alphazero", "_lib")


@pytest.mark.skipif(not os.path.exists(os.path.join(LIB, "libaz.so")), reason="libaz.so not built")
def test_slot_plan_invariants(tmp_path):
    exe = tmp_path / "slot_plan_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), os.path.join(REPO, "tests", "native", "slot_plan_check.cpp"),
                    os.path.join(LIB, "libaz.so"), f"-Wl,-rpath,{LIB}"], check=True)
    rows = json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)
    planned = [r for r in rows if r["plan"]]
    assert len(planned) >= 20, rows
    for r in planned:
        assert r["dup"] == 0 and r["missing"] == 0 and r["bad"] == 0, r
        assert r["pads"] == r["tile_rows"] - r["boards"] * r["H"] * r["W"], r
        assert r["skipped_block_taps"] >= 6, r
        assert r["conflicts"] <= 4, r
    c4 = next(r for r in rows if (r["H"], r["W"]) == (6, 7) and not r["alt"])
    assert c4["plan"] and c4["skipped_block_taps"] == 12 and c4["conflicts"] <= 2, c4
    # the dual launch's 96-row tiles of two Connect-4 boards (round 6): 12 pads are too few
    # for four border blocks, so top | bottom (the layout measured in profiles/r6/ab_t96.txt)
    c4a = next(r for r in rows if (r["H"], r["W"]) == (6, 7) and r["alt"])
    assert c4a["plan"] and c4a["tile_rows"] == 96 and c4a["skipped_block_taps"] == 6, c4a
    c5 = next(r for r in rows if (r["H"], r["W"]) == (9, 9))
    assert c5["plan"] and c5["tile_rows"] == 192 and c5["skipped_block_taps"] == 12, c5  # two boards: all four edges
