"""Tree kernels without the network: C4 self-play at 4096 slots, S=100, the
synthetic evaluator (one lane / two lanes), for rocprofv3 kernel stats --
select/expand durations when no conv shares the CUs.
Usage: python profiles/tree_iso.py <lanes> <moves>"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "custom-alphazero_amd"))
from custom_alphazero import engine as az  # noqa: E402

lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 1
moves = int(sys.argv[2]) if len(sys.argv) > 2 else 10
eng = az.Engine(6, 7, 4, True, 100, slots=4096, evaluator=az.EVAL_SYNTHETIC, cache_log2=25, lanes=lanes,
                compact=True)
eng.selfplay_begin(0, 4096 * 4, 0)
for _ in range(3):
    eng.selfplay_step(1)
t = time.perf_counter()
for _ in range(moves):
    eng.selfplay_step(1)
dt = time.perf_counter() - t
print(f"lanes {lanes}: {1e3 * dt / moves:.2f} ms per move ({1e6 * dt / moves / 100:.1f} us per simulation)")
