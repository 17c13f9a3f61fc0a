#!/usr/bin/env python3
"""Summarise a collect_r1.sh run into the markdown committed under profiles/.

Usage: summarize.py <prof_dir> [round]   (prof_dir = gpurun_out/prof_r2, round = r2)
HBM bytes follow MI355X_MICROARCH.md's HBM/rocprofv3 section (FETCH_SIZE x2
on gfx950 for 16 B/lane streams, WRITE_SIZE as is; KiB units)."""
import csv
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:64]


def main():
    d = sys.argv[1]
    st = glob.glob(f"{d}/trace/**/*kernel_stats.csv", recursive=True)[0]
    tr = glob.glob(f"{d}/trace/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(st)))
    rnd = sys.argv[2] if len(sys.argv) > 2 else "r1"
    print("## Kernel time (rocprofv3 --kernel-trace --stats, `bench.py` short window)\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    conv_calls = conv_ns = 0
    for r in rows[:16]:
        n, c, tot, avg, pct = short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]), \
            float(r["AverageNs"]), float(r["Percentage"])
        print(f"| `{n}` | {c} | {tot / 1e6:.1f} | {avg / 1e3:.1f} | {pct:.2f} |")
    for r in rows:
        if "tower16_kernel" in r["Name"] or "tower16_dual_kernel" in r["Name"]:
            conv_calls += int(r["Calls"])
            conv_ns += float(r["TotalDurationNs"])
    print(f"\ntower16_kernel / tower16_dual_kernel (the whole forward): {conv_calls} launches, rocprof average "
          f"{conv_ns / max(conv_calls, 1) / 1e3:.1f} us per launch (whole trace, preroll included)")
    try:
        b = json.loads(open(f"{d}/bench_trace.json").read().strip().splitlines()[-1])
        rf = b["roofline"]
        print(f"same run, bench.py HIP events: avg_launch_ms {rf['avg_launch_ms']} "
              f"({rf['avg_launch_ms'] * 1e3:.1f} us), boards/launch {rf['boards_per_launch']}, "
              f"achieved {rf['achieved']} TFLOP/s algorithmic ({rf['dtype']}), frac {rf['frac']}; "
              f"value {b['value']} games/s under the profiler")
    except Exception as ex:  # noqa: BLE001
        print(f"(bench_trace.json unreadable: {ex})")
    print("\n## GPU occupancy over the last 0.5 s of the trace (profiles/busy.py)\n")
    print("```")
    print(subprocess.run([sys.executable, os.path.join(HERE, "busy.py"), tr, "0.5"],
                         capture_output=True, text=True).stdout.rstrip())
    print("```")
    tj = os.path.join(HERE, rnd, "pmc_conv_traffic.json")
    if os.path.exists(tj):
        t = json.load(open(tj))
        print(f"\n## HBM traffic per board (PMC, profiles/{rnd}/pmc_conv_traffic.json: {t.get('source', '')})\n")
        print("| kernel | HBM KB/board |")
        print("|---|---:|")
        for algo in ("tower16", "f16x2", "direct"):
            for k, v in t.get(algo, {}).get("hbm_bytes_per_board", {}).items():
                print(f"| `{k}` | {v / 1e3:.1f} |")
    sqd = next((p for p in (f"{d}/pmc_conv_4096_0", f"{os.path.dirname(d)}/pmc_conv_4096_0") if os.path.isdir(p)), "")
    sq = glob.glob(f"{sqd}/**/*counter_collection.csv", recursive=True) if sqd else []
    if sq:
        print("\n## SQ counters, tower conv kernels (az_forward, B = 4096)\n")
        print("```")
        print(subprocess.run([sys.executable, os.path.join(HERE, "pmc_summary.py"),
                              sqd, "conv"],
                             capture_output=True, text=True).stdout.rstrip())
        print("```")


if __name__ == "__main__":
    main()
