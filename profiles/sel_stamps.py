"""Phase breakdown of select_group_kernel from per-slot wall-clock stamps
(diagnostic build: make EXTRA=-DAZ_SEL_STAMPS, loaded with AZ_LIB_PATH).
bench.py's C4 configuration (4096 slots, 100 sims/move, 2 lanes) after a
warm-up; --synth swaps the network for the synthetic evaluator (no conv
beside the tree kernels).  Stamps (100 MHz s_memrealtime) per slot of the
last select launch of a move: 0 entry, 1 game_id read, 11 root loads done (masks, edge base,
root board), 2 end of descent,
3 after the two per-wave stats atomics, 4 after the eval-queue claim + stores,
5 after the cache probe, 6 end (dedup-table claim for misses); per-level sums: 8 loads, 9 UCB +
reductions, 10 play.
Usage: AZ_LIB_PATH=profiles/ab_libs/selst/libaz.so python profiles/sel_stamps.py [--synth]"""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "custom-alphazero_amd"))
from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402

synth = "--synth" in sys.argv
lib = ctypes.CDLL(os.environ["AZ_LIB_PATH"])
lib.az_diag_sel_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]

spec = weight_spec(6, 7, 7)
eng = az.Engine(6, 7, 4, True, 100, slots=4096, evaluator=az.EVAL_SYNTHETIC if synth else az.EVAL_NETWORK,
                cache_log2=25, compact=True)
if not synth:
    w = init_weights(spec, seed=0)
    eng.set_weights([(n, w[n]) for n, _ in spec])
eng.selfplay_begin(0, 4096 * 40, 0)
for _ in range(40):
    eng.selfplay_step(1)
    eng.selfplay_drain()

buf = np.zeros((16384, 12), np.uint64)
phases = ["dispatch", "game_id", "prologue", "descent", "stats", "queue", "probe", "tail"]
acc = {p: [] for p in phases}
tails = []  # the dedup tail of each move's last select launch: (us from the launch's last slot end, us long, dups)
tail = np.zeros(3, np.uint64)
has_tail = hasattr(lib, "az_diag_sel_tail")
if has_tail:
    lib.az_diag_sel_tail.argtypes = [ctypes.c_void_p]
span, depth_all, per_level = [], [], []
lv_load, lv_reduce, lv_play = [], [], []
for mv in range(6):
    eng.selfplay_step(1)
    eng.selfplay_drain()
    assert lib.az_diag_sel_stamps(buf.ctypes.data, 16384) == 0
    if has_tail:
        assert lib.az_diag_sel_tail(tail.ctypes.data) == 0
    rows = buf[(buf[:, 0] != 0) & (buf[:, 6] != 0)].astype(np.int64)
    rows = rows[np.argsort(rows[:, 0])]
    # launches: the two lanes' last selects run at different times
    cut = np.where(np.diff(rows[:, 0]) > 2000)[0]  # > 20 us apart
    for part in np.split(rows, cut + 1):
        if len(part) < 64:
            continue
        t0 = part[:, 0].min()
        span.append((part[:, 6].max() - t0) / 100.0)
        acc["dispatch"].append((part[:, 0] - t0) / 100.0)
        acc["game_id"].append((part[:, 1] - part[:, 0]) / 100.0)
        acc["prologue"].append((part[:, 11] - part[:, 1]) / 100.0)
        acc["descent"].append((part[:, 2] - part[:, 11]) / 100.0)
        acc["stats"].append((part[:, 3] - part[:, 2]) / 100.0)
        q = part[:, 4] != 0
        acc["queue"].append((part[q, 4] - part[q, 3]) / 100.0)
        p5 = part[:, 5] != 0
        acc["probe"].append((part[p5, 5] - part[p5, 4]) / 100.0)
        acc["tail"].append((part[p5, 6] - part[p5, 5]) / 100.0)
        d = part[:, 7] & 0xFFFF
        depth_all.append(d)
        per_level.append((part[d > 0, 2] - part[d > 0, 11]) / 100.0 / d[d > 0])
        lv_load.append(part[d > 0, 8] / 100.0 / d[d > 0])
        lv_reduce.append(part[d > 0, 9] / 100.0 / d[d > 0])
        lv_play.append(part[d > 0, 10] / 100.0 / d[d > 0])
    if has_tail and len(rows):
        last_end = rows[:, 6].max()
        tails.append(((int(tail[0]) - int(last_end)) / 100.0, (int(tail[1]) - int(tail[0])) / 100.0, int(tail[2])))

print(f"{'synthetic evaluator' if synth else 'network evaluator'}: {len(span)} select launches, "
      f"launch span (first entry -> last end) mean {np.mean(span):.1f} us, max {np.max(span):.1f} us")
for p in phases:
    v = np.concatenate(acc[p])
    print(f"  {p:9s} mean {v.mean():7.2f} us  p50 {np.median(v):7.2f}  p90 {np.percentile(v, 90):7.2f}  "
          f"max {v.max():7.2f}  (n {len(v)})")
d = np.concatenate(depth_all)
lv = np.concatenate(per_level)
print(f"  depth mean {d.mean():.2f} max {d.max()}; descent per level mean {lv.mean():.2f} us p50 {np.median(lv):.2f}")
print(f"  per level (s_waitcnt 0 at each stamp): edge+table loads {np.concatenate(lv_load).mean():.2f} us, "
      f"UCB + first-max + broadcast {np.concatenate(lv_reduce).mean():.2f} us, play {np.concatenate(lv_play).mean():.2f} us")
if tails:
    t = np.array(tails, np.float64)
    print(f"dedup tail (last select launch of each move): starts {t[:, 0].mean():.1f} us after the last slot's end, "
          f"runs {t[:, 1].mean():.1f} us (max {t[:, 1].max():.1f}), {t[:, 2].mean():.0f} duplicates")
