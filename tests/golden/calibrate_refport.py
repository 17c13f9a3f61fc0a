#!/usr/bin/env python3
"""CPU-baseline calibration (dev container only, never on the GPU box):
times the REAL reference self-play (imported from /root/reference with a
torch-CPU stand-in network) against oracle/refport.py on the same seeds,
same core, same network.  Usage: python3 tests/golden/calibrate_refport.py SIMS GAMES
"""
# Calibration (dev container only): reference self-play vs oracle/refport.py,
# same torch-CPU stand-in network, 1 thread, same seeds.  Not committed as a test:
# the reference never leaves this container.
import os, sys, time, types
import numpy as np
REPO = "/root/repo"
sys.path.insert(0, os.path.join(REPO, "oracle")); sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
import torch; torch.set_num_threads(1)
import refport
from custom_alphazero.model.weights import init_weights, weight_spec
W = init_weights(weight_spec(6, 7, 7), seed=0)
net = refport.TorchCPUNet(W, depth=4)
class T:
    def __init__(s, a): s.a = a
    def numpy(s): return s.a
class Stub:
    def __init__(s, input_dim, action_space): pass
    def __call__(s, x):
        b = refport.PortBoard(6, 7, 4, True); b.cells = (x[0][..., 1] - x[0][..., 2]).astype(np.int8)
        p, v = net(b); return T(p[None].astype(np.float32)), T(np.array([[v]], np.float32))
m = types.ModuleType("custom_alphazero.model.tensorflow.model"); m.PolicyValueModel = Stub
gv = types.ModuleType("graphviz"); gv.Digraph = object
sys.modules["graphviz"] = gv
# import the REFERENCE package (shadow our package name)
for k in list(sys.modules):
    if k.startswith("custom_alphazero"): del sys.modules[k]
sys.path.insert(0, "/root/reference")
sys.modules["custom_alphazero.model.tensorflow.model"] = m
os.chdir("/tmp")
from custom_alphazero import config as rc, self_play as rsp
from custom_alphazero.connect_n.board import Board
rc.ConfigGeneral.mono_process = True
S = int(sys.argv[1]); games = int(sys.argv[2])
t0 = time.perf_counter(); exp_ref = 0; plies = 0
import custom_alphazero.mcts.mcts as rm
orig = rm.MCTS.evaluate_and_expand
cnt = [0]
def ce(self, n): cnt[0] += 1; return orig(self, n)
rm.MCTS.evaluate_and_expand = ce
for g in range(games):
    rsp.time.time = lambda g=g: float(1000 + g)
    st, po, rw, _ = rsp.play_game(0, Board.get_all_possible_moves(), S, "x", {})
    plies += len(st)
t_ref = time.perf_counter() - t0
t0 = time.perf_counter(); exp_port = 0; plies_p = 0
for g in range(games):
    r = refport.play_game(6, 7, 4, True, S, 1000 + g, net, cache={})
    exp_port += r["expansions"]; plies_p += r["T"]
t_port = time.perf_counter() - t0
print(f"S={S} games={games}: reference {t_ref:.1f}s ({cnt[0]} exp, {cnt[0]/t_ref:.0f} exp/s, {games/t_ref:.3f} games/s) | "
      f"port {t_port:.1f}s ({exp_port} exp, {exp_port/t_port:.0f} exp/s, {games/t_port:.3f} games/s) | port/ref speed {t_ref/t_port:.2f}x")
