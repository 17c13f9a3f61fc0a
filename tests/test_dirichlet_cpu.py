"""The device's Dirichlet root-noise sampler (csrc/az_random.h, built for the
host by tests/native) against numpy's legacy RandomState.dirichlet -- the
draws the reference's get_best_edge_with_noise makes (mcts/mcts.py:70-85).

numpy's gamma sampler calls glibc's log / pow, which are not correctly
rounded (<= 0.52 ULP).  The device restates glibc 2.35's __log_fma /
__pow_fma (their algorithms, their contractions, their tables: az_random.h,
az_libm_tables.h), so every rejection decision and every draw is numpy's bit
for bit: checked here against this host's libm on millions of arguments of
each kind the sampler passes (plus general, near-1, subnormal-argument and
subnormal-result ones), and the whole sampler against
RandomState.dirichlet draw by draw."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "tests", "native", "_build", "dirichlet_check")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "native"), "_build/dirichlet_check"],
                   check=True, timeout=600)
    return EXE


def test_log_pow_are_glibcs_bit_for_bit(exe):
    n = 1_000_000
    out = subprocess.run([exe, "funcs", str(n)], capture_output=True, text=True, check=True,
                         timeout=300).stdout.split()
    bad = [int(v) for v in out]
    # exponential draws' log(1-u), pow(U, 1/alpha), log((1-U)/alpha), pow(1-a+aY, 1/a), general (x, p),
    # near-1 / subnormal / subnormal-result arguments
    assert bad == [0] * 6, bad


@pytest.mark.parametrize("seed,k,alpha", [(0, 7, 0.03), (5, 7, 0.03), (9, 9, 0.03), (7, 25, 0.03),
                                          (3, 4, 0.5), (11, 3, 1.0), (2, 5, 0.003)])
def test_draws_match_numpy_legacy_dirichlet(exe, seed, k, alpha):
    n = 20000
    txt = subprocess.run([exe, "draw", str(seed), str(k), repr(alpha), str(n)], capture_output=True, text=True,
                         check=True).stdout.split()
    got = np.array([float.fromhex(v) for v in txt]).reshape(n, k)
    rs = np.random.RandomState(seed)
    ref = np.stack([rs.dirichlet(np.ones(k) * alpha) for _ in range(n)])
    # every vector is numpy's to the bit (so every rejection decision agreed
    # and the MT19937 stream stayed in step)
    assert (got.view(np.uint64) == ref.view(np.uint64)).all()
