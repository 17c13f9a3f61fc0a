# round 6 copy of profiles/tower_stamps.py: BPW (boards per workgroup) from the environment (2 for the dual launch's 96-row tiles)
"""Phase clocks of tower16_kernel (diagnostic build with -DAZ_T16_STAMPS,
AZ_LIB_PATH): per workgroup wave-0 s_memtime at stem end, each conv's K-loop
end and epilogue end, heads; median over workgroups of the last forward."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
from custom_alphazero import engine as az  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 673
    rng = np.random.RandomState(5)
    w = init_weights(weight_spec(6, 7, 7, depth=4), seed=0, randomize_bn=True)
    eng = az.Engine(6, 7, 4, True, 25, slots=max(nb, 2048), evaluator=az.EVAL_NETWORK, depth=4)
    eng.set_weights(w.items())
    xx = oracle.full_state(rng.randint(-1, 2, (nb, 6, 7)).astype(np.int8))
    for _ in range(30):
        eng.forward(xx)
    buf = np.zeros((4096, 64), np.uint64)
    lib = az.load_library()
    lib.az_t16_stamps.argtypes = [ctypes.c_void_p]
    assert lib.az_t16_stamps(buf.ctypes.data) == 0
    bpw = int(os.environ.get("BPW", "3"))
    nwg = (nb + bpw - 1) // bpw
    s = buf[:nwg].astype(np.int64)
    rel = s - s[:, 0:1]
    clk = (s[:, 19] - s[:, 0]) / np.maximum((s[:, 23] - s[:, 22]) / 100.0, 1)  # cycles per us at 100 MHz
    order = [(0, "start"), (1, "stem mfma"), (21, "stem store")]
    for d in range(4):
        for k, p in enumerate(("c1loop", "c1epi", "c2loop", "c2epi")):
            if not (d == 3 and p == "c2epi"):
                order.append((2 + 4 * d + k, f"b{d}.{p}"))
    order += [(18, "heads1x1"), (19, "end")]
    med = np.median(rel, axis=0)
    prev = 0
    print(f"B={nb} wgs={nwg} clock {np.median(clk):.0f} MHz; total {med[19]:.0f} cycles")
    for i, n in order:
        print(f"  {n:10s} {med[i]:9.0f}  (+{med[i] - prev:7.0f})")
        prev = med[i]
    print(f"  stem: before plan {med[56]:.0f}, MFMAs issued {med[57]:.0f}, DMA landed {med[58]:.0f}, barrier {med[1]:.0f}")
    print("  wave4 1x1: " + " ".join(f"{med[k]:.0f}" for k in range(48, 56)))
    print(f"  heads: pf/vf {med[44]:.0f}, policy {med[45]:.0f}, value {med[46]:.0f}, barrier {med[47]:.0f}, "
          f"end {med[19]:.0f}; last conv2 wave0 {med[16]:.0f} wave4 {med[38]:.0f}; 1x1 done wave0 {med[42]:.0f} "
          f"wave4 {med[43]:.0f}")
    for d in range(4):
        print(f"  b{d}: wave4 c1loop end {med[24 + 4 * d]:.0f} (wave0 {med[2 + 4 * d]:.0f}), after barrier "
              f"{med[40 + d]:.0f}, c1epi end {med[3 + 4 * d]:.0f}; wave4 c2loop end {med[26 + 4 * d]:.0f} "
              f"(wave0 {med[4 + 4 * d]:.0f})")
    if hasattr(lib, "az_t16_wstamps"):
        ws = np.zeros((4096, 8, 5), np.uint64)
        lib.az_t16_wstamps.argtypes = [ctypes.c_void_p]
        assert lib.az_t16_wstamps(ws.ctypes.data) == 0
        ws = ws[:nwg].astype(np.int64)
        t0 = ws[:, :, 0].min(axis=1, keepdims=True)
        simd = (ws[:, :, 4] >> 4) & 3
        print("  block 1 per wave (median over workgroups, cycles from the first wave's conv1 start):")
        for w in range(8):
            c1s, c1e, c2s, c2e = (np.median(ws[:, w, k] - t0[:, 0]) for k in range(4))
            sid = np.bincount(simd[:, w], minlength=4).argmax()
            print(f"    wave {w} simd {sid}: conv1 {c1s:7.0f}..{c1e:7.0f} ({c1e - c1s:6.0f})  "
                  f"conv2 {c2s:7.0f}..{c2e:7.0f} ({c2e - c2s:6.0f})")


if __name__ == "__main__":
    main()
