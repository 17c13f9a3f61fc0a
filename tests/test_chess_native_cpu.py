"""The device chess rules (csrc/az_chess.h) compiled for the host under
AddressSanitizer + UBSan and walked over the perft trees of the standard
positions against the oracle (tests/native/chess_legal_check.cpp): no memory
or undefined-behaviour error, two generations per position identical, lists
equal to the oracle's, published perft counts; the chess tower's input planes (full_state4) equal
the oracle's full_state at sampled nodes.  No GPU."""
import os
import subprocess

import pytest

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-C", NATIVE, "_build/chess_legal_check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(NATIVE, "_build", "chess_legal_check")


def test_device_rules_clean_under_asan_ubsan(built):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([built], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
    planes = int(r.stdout.split("input planes checked ")[1].split(",")[0])
    assert planes > 1000, r.stdout  # az_chess.h full_state4 (the tower's chess input) vs the oracle
    assert r.stdout.count("(expected") == 6
    for line in r.stdout.splitlines():
        if line.startswith("perft("):
            got, exp = line.split()[1], line.split("expected ")[1].split(")")[0]
            assert got == exp, line
