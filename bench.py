#!/usr/bin/env python3
"""Self-play throughput on MI355X: games/s + MCTS node-expansions/s.

Workload (BASELINE.json configs[1]): Connect-4 6x7, n=4, gravity, 100
simulations per move, 4096 concurrent games per GPU, random-init
128-filter x 4-block policy/value network (Keras defaults, torch seed 0).
A "step" is one move for every game slot: `sims` lockstep simulations
(select -> batched network forward -> expand/backup), a move commit, and
the D2H copy of the games that finished (az_selfplay_drain: a game counts
when its samples are on the host) -- in the timed window the
drain of move m-1 overlaps move m, and the window ends with a synchronize
and a last drain.  Finished games are
replaced by new ones (game g seeded MT19937(g)).

Steady state, whatever --warmup says: all slots start at ply 0 together
and the shared transposition cache (the reference's plays_inferences)
starts empty, so the first moves are not representative.  Untimed moves
run until at least --warmup moves have passed AND the cache is full and has
taken 1.5x its capacity in inserts (least-recently-used eviction, az_tree.h:
its content and hit rate are then stationary, profiles/r6/cache_curve*) --
every one of them real work.  The line states the cache's capacity, fill,
generation, age in moves and the window's hit rate.
value = games drained in the K timed steps, summed over ranks / max-over-
ranks wall time.

Multi-GPU (torchrun, one rank per GPU): games are sharded by global game id
(independent, no data-path collective: scaling "weak"); rank 0's weights
reach the other ranks by one RCCL broadcast over xGMI before timing, and
the games each rank finished in the window are gathered to rank 0 (compact
int8 boards + f64 policies, RCCL) right after it.

The CPU baselines (rank 0, N=1 only) are oracle/refport.py -- the
reference's self-play structure, pinned to the reference by
tests/test_refport.py -- run before the GPU is touched: the reference's
joblib fan-out (one game per worker process, 1-thread torch-CPU network,
plays_inferences shared through a Manager dict, self_play.py:98,
utils.py:38-39) at the benchmark's sims, and BASELINE configs[0] (25
sims/move, one worker, mono-process dict).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

# HIP hardware queues per process, read once at HIP's initialisation (before
# torch or libaz touch the GPU): HIP's default 4 leaves a third lane's stream
# sharing a queue; with 8 the engine's auto lane count runs configs[1] on 3
# lanes, +4.9% games/s (profiles/r5/ab_queues_lanes.txt, ab_lanes_q8.txt)
BENCH_HW_QUEUES = 8
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < BENCH_HW_QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(BENCH_HW_QUEUES)

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E ~8 TB/s
F16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16/fp16 MFMA (no 2:1 sparsity)
MIN_PREROLL = 24                # untimed moves at least (game-completion rate stationary, ~1 game length)
MAX_PREROLL = 4000
WINDOW_EVENT_STRIDE = 1         # the timed window's tower events: every launch of each lane
CACHE_TURNOVER = 1.5            # cache inserts / capacity before the window (full table turned over: stationary)
CACHE_FULL = 0.98               # ... and the table this full


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--game", choices=("connect_n", "chess"), default="connect_n",
                    help="chess: BASELINE configs[4] per-GPU shard (256 games, 800 sims/move)")
    ap.add_argument("--steps", type=int, default=None, help="timed moves (30; chess 3)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed moves at least (5; chess 2)")
    ap.add_argument("--slots", type=int, default=None, help="concurrent games per GPU (4096; chess 256)")
    ap.add_argument("--sims", type=int, default=None, help="sims per move (100; chess 800)")
    ap.add_argument("--height", type=int, default=6)
    ap.add_argument("--width", type=int, default=7)
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-configs0-seconds", type=float, default=10.0,
                    help="BASELINE configs[0] line (C4, 25 sims/move, 1 worker)")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="0 = os.cpu_count() - 1 (self_play.py:98), inside the box's CPU share")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lanes", type=int, default=0, help="slot groups on separate HIP streams (0 = auto)")
    ap.add_argument("--conv-algo", type=int, default=0, help="0 fp16x2 direct (default), 1 fp32 direct")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on MI355X; gloo for rehearsals")
    ap.add_argument("--cache-log2", type=int, default=None,
                    help="transposition cache (the reference's plays_inferences) entries = 2^N (default 26: "
                         "4.6 GB of the 288 GB at configs[1]; chess 0: its cache measured 3-5%% slower in the opening, "
                         "profiles/r6/ab_chess_r5.txt); 0 = off")
    ap.add_argument("--arena-edges", default="bounded",
                    help="tree edges per slot, the average of a lane's pooled halves: 'bounded' (default, "
                         "8*S*A + H*W*A: ~5x the high-water mark measured at configs[1] and configs[3]), "
                         "'proof' (S*H*W*A + A, no game can overflow, capped at 40%% of free HBM) or a number; "
                         "an overflow is a device error, never an overrun")
    ap.add_argument("--rng-skip", type=int, default=None,
                    help="MT19937 words each game's stream discards after its seed (default: the reference "
                         "play_game's model-construction draws, 2*H*W*4; 0: round 4's streams)")
    ap.add_argument("--compact", type=int, default=1,
                    help="1: reclaim the subtrees a game has left after every move (az_config.compact)")
    ap.add_argument("--no-cache-window", action="store_true",
                    help="skip the second timed window with the cache bypassed")
    ap.add_argument("--max-plies", type=int, default=512,
                    help="chess: games stop (as draws) after this many plies (the engine's cap; the reference has none)")
    ap.add_argument("--share-devices", action="store_true",
                    help="rehearsal: allow more ranks than visible GPUs (ranks share devices; "
                         "the line reports shared_devices)")
    args = ap.parse_args()
    chess = args.game == "chess"
    for k, c4, ch in (("steps", 30, 3), ("warmup", 5, 2), ("slots", 4096, 256), ("sims", 100, 800),
                      ("cache_log2", 26, 0)):
        if getattr(args, k) is None:
            setattr(args, k, ch if chess else c4)
    return args


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor()


def cpu_quota():
    """CPUs this job may use: the cgroup CPU quota (cgroup v2 cpu.max, or v1
    cfs_quota/period) and the affinity mask, with where each came from."""
    quota, src = None, "no cgroup CPU quota"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota, src = -(-int(q) // int(per)), f"cgroup v2 cpu.max {q} {per}"
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota, src = -(-q // per), f"cgroup v1 cfs_quota_us {q} / cfs_period_us {per}"
        except (OSError, ValueError):
            pass
    aff = len(os.sched_getaffinity(0))
    return quota, aff, src


def cpu_workers(args):
    """The reference's fan-out is os.cpu_count() - 1 worker processes
    (self_play.py:98).  On a GPU box os.cpu_count() counts the whole machine
    while the job's cgroup grants a share of it, so the pool is
    min(os.cpu_count() - 1, quota - 1, affinity - 1): the reference's rule
    applied to the CPUs this job may actually use."""
    total = os.cpu_count() or 1
    quota, aff, src = cpu_quota()
    ref = max(1, total - 1)
    avail = min(aff, quota) if quota else aff
    w = args.cpu_workers or max(1, min(ref, avail - 1))
    why = (f"reference n_jobs = os.cpu_count() - 1 = {ref}; this job: os.cpu_count() {total}, affinity {aff}, "
           f"{src}" + (f" -> {avail} usable CPUs - 1" if w < ref else ""))
    return w, why


def cpu_baseline(args, weights):
    """Reference-structured CPU self-play, bounded sample (about budget seconds)."""
    import multiprocessing as mp

    import refport
    workers, why = cpu_workers(args)
    job = (args.height, args.width, args.n, True, args.sims, weights, args.depth,
           args.cpu_baseline_seconds)
    ctx = mp.get_context("fork")  # no GPU initialised yet in this process
    with ctx.Manager() as manager:
        shared = manager.dict()  # plays_inferences = Manager().dict() (utils.py:38-39)
        t0 = time.perf_counter()
        with ctx.Pool(workers) as pool:
            res = pool.map(refport.baseline_worker,
                           [job + (10_000_000 + 1000 * i, shared) for i in range(workers)])
        wall = time.perf_counter() - t0
        entries = len(shared)
    games = sum(r[0] for r in res)
    exps = sum(r[1] for r in res)
    busy = [r[2] for r in res]
    # each worker's games over its OWN elapsed time, summed over workers: a
    # worker that finished its last game early does not idle in the
    # denominator (the pool's wall time waits for the slowest straggler)
    rate = sum(r[0] / r[2] for r in res if r[2] > 0)
    erate = sum(r[1] / r[2] for r in res if r[2] > 0)
    return {
        "value": round(rate, 4), "unit": "games/s", "cores": workers,
        "kind": "port", "expansions_per_s": round(erate, 1),
        "basis": "sum over workers of games_i / elapsed_i (each worker plays until the budget, then finishes "
                 "its game); the pool wall-time rate is beside it",
        "wall_s": round(wall, 2), "busy_s_mean": round(float(np.mean(busy)), 2),
        "busy_s_max": round(float(np.max(busy)), 2), "value_wall": round(games / wall, 4),
        "cores_reason": why,
        "sample": (f"oracle/refport.py self-play, C4 {args.sims} sims/move, {workers} worker processes "
                   f"x 1 torch-CPU thread, batch-1 forward, one plays_inferences Manager dict shared by "
                   f"all workers ({entries} entries at the end); {games} games, worker busy time mean "
                   f"{np.mean(busy):.1f}s (pool wall {wall:.1f}s) ({_cpu_model()})"),
    }


def cpu_baseline_native(args, weights):
    """SURVEY.md 8(d)'s stronger CPU line: oracle/az_cpu.c -- the oracle's C
    MCTS (bit-exact on the reference's fixtures) + a batch-1 fp32 C forward,
    one thread per game, the reference's fan-out of worker count, one shared
    insert-only plays_inferences table; same bounded sample length."""
    import cpu_native
    workers, why = cpu_workers(args)
    A = args.width
    flat = cpu_native.fold_for_cpu(weights, args.height, args.width, A, args.depth)
    r = cpu_native.selfplay(flat, args.height, args.width, args.n, True, args.sims, args.depth, workers,
                            args.cpu_baseline_seconds)
    wall = r["seconds"]
    return {
        "value": round(r["games"] / wall, 4), "unit": "games/s", "cores": workers, "kind": "port",
        "expansions_per_s": round(r["expansions"] / wall, 1), "cores_reason": why,
        "cache_hit_rate": round(r["cache_hits"] / max(r["expansions"], 1), 4),
        "sample": (f"oracle/az_cpu.c: C MCTS (oracle/az_oracle.c) + batch-1 fp32 C forward (BN folded, 4 pixels x "
                   f"32 channels per register block), {workers} threads x 1 game, one shared insert-only cache "
                   f"(2^22 entries); C4 {args.sims} sims/move, {r['games']} games / {r['expansions']} expansions in "
                   f"{wall:.1f}s ({_cpu_model()})"),
    }


def cpu_configs0(args, weights):
    """BASELINE configs[0]: C4 via self_play.py, 25 sims/move, 1 CPU worker
    (mono-process: plays_inferences is a plain dict)."""
    import multiprocessing as mp

    import refport
    ctx = mp.get_context("fork")
    job = (args.height, args.width, args.n, True, 25, weights, args.depth, args.cpu_configs0_seconds,
           30_000_000, None)
    t0 = time.perf_counter()
    with ctx.Pool(1) as pool:
        games, exps, busy = pool.map(refport.baseline_worker, [job])[0]
    wall = time.perf_counter() - t0
    return {"config": "BASELINE.json configs[0]: Connect-4 6x7, 25 sims/move, 1 CPU worker",
            "value": round(games / busy, 4), "unit": "games/s", "expansions_per_s": round(exps / busy, 1),
            "cores": 1, "kind": "port", "basis": "games / the worker's own elapsed time",
            "busy_s": round(busy, 2), "wall_s": round(wall, 2),
            "sample": f"oracle/refport.py, {games} games in {busy:.1f}s ({_cpu_model()})"}


def _device_weights(spec, host_w, rank, world, args, dev):
    """Rank 0's init reaches every rank by one flat RCCL broadcast over xGMI."""
    import torch
    import torch.distributed as dist
    flat = torch.cat([torch.from_numpy(host_w[n].reshape(-1)) for n, _ in spec]).to(dev)
    if world > 1:
        if rank != 0:
            flat.zero_()
        if args.dist_backend == "gloo":
            host = flat.cpu()
            dist.broadcast(host, src=0)
            flat.copy_(host)
        else:
            dist.broadcast(flat, src=0)
    named, off = [], 0
    for name, shape in spec:
        k = int(np.prod(shape))
        named.append((name, flat[off:off + k]))
        off += k
    return named, flat


def _reduce(values, op, world, args, dev):
    """All-reduce a list of numbers (float64) over the ranks."""
    if world == 1:
        return list(values)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64,
                     device="cpu" if args.dist_backend == "gloo" else dev)
    dist.all_reduce(t, op=op)
    return t.tolist()


def conv_kernel_name(conv_algo, chess=False, tower=False):
    if conv_algo == 1:
        return "conv3x3_mfma (fp32 MFMA implicit-GEMM 3x3 conv, fused BN/ReLU/residual), one launch per conv"
    if conv_algo == 0 and chess and tower:
        return ("tower16_kernel, input-row form (one launch per lane-simulation: the 118-plane stem conv and the "
                "residual tower's 8 3x3 convs as implicit GEMMs on the 16x16x32 fp16 MFMA -- fp32-accurate, both "
                "operands as two fp16 terms, 3 products per k-step -- activations double-buffered in LDS, 1x1 "
                "projection residuals, head 1x1 convs; the 1880-logit dense heads follow in their own kernels)")
    if conv_algo == 0 and not chess:
        return ("tower16_kernel / tower16_dual_kernel (Connect-4: 96-row tiles of two boards when the launch "
                "holds few live boards, else 128-row tiles of three) (the whole forward in one launch per "
                "lane-simulation: the stem and the "
                "residual tower's 8 3x3 convs as implicit GEMMs on the 16x16x32 fp16 MFMA -- fp32-accurate, both operands "
                "as two fp16 terms, 3 products per k-step -- with activations double-buffered in LDS, 1x1 projection "
                "residuals, head 1x1 convs, dense heads, softmax, tanh)")
    return ("conv16_kernel (direct 3x3 implicit GEMM on the 16x16x32 fp16 MFMA; fp32-accurate: both operands as "
            "two fp16 terms, 3 products per k-step; fused BN/ReLU, 1x1 projection residual and head 1x1 convs; "
            "one launch per conv)")


def conv_roofline(args, conv_algo, per_forward, boards_per_launch, avg_ms, busy_ms, boards_total, launches,
                  direct_flop_per_board, issued_per_board, pmc_file, pmc_key, chess=False, tower=False):
    """roofline of the dominant kernel (the residual tower's convs: the whole
    forward in one tower16_kernel launch, or one conv per launch).
    achieved = ALGORITHMIC FLOP per launch -- the direct convolution's
    2*MACs (19 F*F MACs per pixel per block) x live boards per
    launch / launches per forward -- / the launch's mean duration (HIP events
    on its lane's stream over the timed window); peak = the dense MFMA peak of
    the pipe the kernel issues on (fp16: the two-term split issues 3 fp16
    products per MAC, reported beside it as `issued`)."""
    f16 = conv_algo != 1
    peak = F16_MFMA_PEAK_TFLOPS if f16 else FP32_MFMA_PEAK_TFLOPS
    dtype = "fp16 MFMA (2 terms per fp32 operand, 3 products per MAC)" if f16 else "fp32 MFMA"
    per_launch = boards_per_launch / per_forward
    achieved = per_launch * direct_flop_per_board / (avg_ms * 1e-3) / 1e12 if avg_ms else 0.0
    issued = per_launch * issued_per_board / (avg_ms * 1e-3) / 1e12 if avg_ms else 0.0
    union = boards_total * direct_flop_per_board / (busy_ms * 1e-3) / 1e12 if busy_ms else 0.0
    # PMC (rocprofv3 FETCH_SIZE / WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES passes, profiles/pmc_fold.py):
    # bytes per board x the live batch, and the MFMA-busy fraction -- only when
    # the profile measured THIS build (its az_build_id), else null with the reason
    from custom_alphazero import engine as az
    build, _flags = az.build_id()
    traffic = mfma_busy = None
    pmc_note = f"no PMC profile {os.path.relpath(pmc_file, REPO)}"
    if os.path.exists(pmc_file):
        with open(pmc_file) as fp:
            tj = json.load(fp)
        if pmc_key not in tj:
            pmc_note = f"{os.path.relpath(pmc_file, REPO)} holds no [{pmc_key}] entry"
        elif tj.get("build_id") != build:
            pmc_note = (f"{os.path.relpath(pmc_file, REPO)} measured build {tj.get('build_id')}, this libaz is "
                        f"{build}: traffic and mfma_busy not reported")
        else:
            e = tj[pmc_key]
            traffic = int(e["mean_hbm_bytes_per_board_per_launch"] * boards_per_launch)
            mfma_busy = round(e["mfma_busy"], 4) if e.get("mfma_busy") is not None else None
            pmc_note = (f"{os.path.relpath(pmc_file, REPO)} [{pmc_key}], build {build}: "
                        f"{e['mean_hbm_bytes_per_board_per_launch']:.0f} HBM bytes per board at "
                        f"{e['boards_per_launch']} boards per launch (x live boards/launch here); mfma_busy = "
                        f"SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) of that launch")
    return {
        "kernel": conv_kernel_name(conv_algo, chess, tower),
        "bound": "mfma",
        "achieved": round(achieved, 2),
        "peak": peak,
        "unit": "TFLOP/s",
        "frac": round(achieved / peak, 4),
        "traffic": traffic,
        "traffic_unit": "HBM bytes per launch",
        "mfma_busy": mfma_busy,
        "pmc": pmc_note,
        "build_id": build,
        "dtype": dtype,
        "achieved_basis": (f"direct-convolution FLOP per launch ({int(direct_flop_per_board)} per board x "
                           f"boards_per_launch / {per_forward} launch(es) per forward) / avg_launch_ms (HIP events "
                           f"on each lane's stream, timed region)"),
        "flop_per_board": int(direct_flop_per_board),
        "issued": {"achieved": round(issued, 2), "frac": round(issued / peak, 4),
                   "flop_per_board": int(issued_per_board),
                   "basis": ("MFMA FLOP the kernel issues per board (3 fp16 products per MAC; the tower's own count: "
                             "tile pad rows and stem in, the slot plan's skipped border taps out) x boards per launch "
                             "/ avg_launch_ms")},
        "busy_union": {"achieved": round(union, 2), "frac": round(union / peak, 4),
                       "basis": "all timed boards' direct FLOP / union of the kernel intervals of all lanes"},
        "launches_per_forward": per_forward,
        "boards_per_launch": round(boards_per_launch, 1),
        "avg_launch_ms": round(avg_ms, 4),
        "conv_busy_ms": round(busy_ms, 2),
        "launches_timed": launches,
    }


def chess_cpu_baseline(args, weights):
    import multiprocessing as mp

    import refport
    workers, why = cpu_workers(args)
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(refport.chess_baseline_worker,
                       [(args.sims, weights, args.depth, args.cpu_baseline_seconds, 20_000_000 + i)
                        for i in range(workers)])
    wall = time.perf_counter() - t0
    exps = sum(r[0] for r in res)
    rate = sum(r[0] / r[2] for r in res if r[2] > 0)
    return {"value": round(rate, 2), "unit": "expansions/s", "cores": workers, "kind": "port",
            "basis": "sum over workers of expansions_i / elapsed_i", "wall_s": round(wall, 2),
            "value_wall": round(exps / wall, 2), "cores_reason": why,
            "plies_per_s_est": round(sum(r[1] / r[2] for r in res if r[2] > 0), 4),
            "sample": (f"oracle chess MCTS (C tree, reference arithmetic) + torch-CPU network at batch 1 "
                       f"on Board.full_state, {workers} worker processes x 1 thread, {args.sims} sims/move, "
                       f"{exps} expansions in {wall:.1f}s; the reference's own chess path cannot run "
                       f"under MCTS (chess/board.py:178 vs mcts.py:179)")}


def check_devices(args, world):
    """One rank per GPU: refuse (before any GPU call) a world larger than the
    visible devices, which would stack ranks on one GPU and still print
    n_gpus = world -- unless --share-devices asks for that rehearsal (then
    the line says so).  torch.cuda.device_count() does not initialise the
    GPU on this image."""
    import torch
    n = torch.cuda.device_count()
    if world > n and not args.share_devices:
        print(f"bench.py: {world} ranks but {n} visible GPU(s); refusing to stack ranks on one device "
              f"(--share-devices for a rehearsal)", file=sys.stderr)
        sys.exit(2)
    return n


def _init_dist(args, world, local_rank):
    import torch
    import torch.distributed as dist
    n = check_devices(args, world)
    dev_index = local_rank % max(n, 1)
    if world > 1:
        torch.cuda.set_device(dev_index)
        dist.init_process_group(args.dist_backend)
    return dev_index, torch.device("cuda", dev_index)


def chess_main(args):
    """BASELINE configs[4]: chess, 800 sims/move, 2048 games over 8 GPUs =
    256 concurrent games per GPU (weak scaling).  A game outlasts any short
    window (hundreds of plies x 800 simulations), so value is the MCTS
    node-expansion rate, the metric's second half; plies/s and completed
    games are reported next to it."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from custom_alphazero.model.weights import init_weights, weight_spec
    spec = weight_spec(8, 8, 1880, depth=args.depth, in_channels=118)
    host_w = init_weights(spec, seed=0)
    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = chess_cpu_baseline(args, host_w)
    import torch
    import torch.distributed as dist
    from custom_alphazero import engine as az
    dev_index, dev = _init_dist(args, world, local_rank)
    named, _flat = _device_weights(spec, host_w, rank, world, args, dev)
    eng = az.ChessEngine(mcts_iterations=args.sims, slots=args.slots, evaluator=az.EVAL_NETWORK,
                         max_plies=args.max_plies, depth=args.depth, device=dev_index, conv_algo=args.conv_algo,
                         lanes=args.lanes, cache_log2=args.cache_log2)
    eng.set_weights(named)
    budget = args.slots * 2
    eng.selfplay_begin(first_game=rank * budget, n_games=budget, base_seed=0)
    eng.selfplay_step(args.warmup)
    eng.selfplay_drain()  # (games the untimed moves finished: not the window's)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.timer(True)
    st0 = eng.stats()
    t0 = time.perf_counter()
    # the K moves in one synchronous call, then the drain of the games they
    # finished (inside the timed region).  The Connect-N window's form --
    # enqueue move m, drain move m - 1 -- measured 6% slower here: 1.569 vs
    # 1.674 M expansions/s on one box (profiles/r6/ab_chess_win.txt; kept as
    # AZ_CHESS_ASYNC_WINDOW=1, the drain API is the same)
    parts = []
    if os.environ.get("AZ_CHESS_ASYNC_WINDOW") == "1":
        for _ in range(args.steps):
            eng.selfplay_step(1, sync=False)
            parts.append(eng.selfplay_drain())
    else:
        eng.selfplay_step(args.steps)
    torch.cuda.synchronize()
    parts.append(eng.selfplay_drain())
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st1 = check_device(eng, "the timed window")
    eng.timer(False)
    window = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    drained = len(window["lengths"])
    # ---- N>1: the window's chess games to rank 0 (replay-buffer gather; a
    # chess game outlasts a short window, so often none -- the path runs anyway)
    gather = None
    if world > 1:
        from custom_alphazero import distributed as D
        t_g = time.perf_counter()
        gstats = {}
        gg = D.gather_games(window, device=None if args.dist_backend == "gloo" else dev, stats=gstats)
        gt = time.perf_counter() - t_g
        if rank == 0:
            gather = {"games": int(len(gg["lengths"])), "samples": int(len(gg["moves"])),
                      "policy_entries": int(len(gg["policy_actions"])), "bytes": gstats["wire_bytes"],
                      "bytes_note": "what rank 0 received from the other ranks (its own games stay put)",
                      "seconds": round(gt, 4),
                      "how": f"compact chess records (80-byte positions, u16 moves, sparse root policies: "
                             f"distributed.pack_chess) + per-game counts; a gather of the sizes, then each rank "
                             f"sends its blob to rank 0 only (point-to-point over {args.dist_backend}) after "
                             f"the timed window"}
    d = {k: st1[k] - st0[k] for k in ("games_done", "expansions", "simulations", "plies",
                                      "terminal_visits", "evaluations", "cache_hits")}
    local_evals = d["evaluations"]
    g, e, s, p, ev, dr, hits = _reduce([d["games_done"], d["expansions"], d["simulations"], d["plies"],
                                        d["evaluations"], drained, d["cache_hits"]],
                                       dist.ReduceOp.SUM if world > 1 else None, world, args, dev)
    (elapsed,) = _reduce([elapsed], dist.ReduceOp.MAX if world > 1 else None, world, args, dev)
    F, HW = 128, 64
    direct_flop = HW * 2 * F * F * 19 * args.depth     # direct 3x3 + 1x1 residual, tower only
    issued = 3 * direct_flop if args.conv_algo != 1 else direct_flop  # fp16x2: 3 products per MAC
    launches = st1["conv_launches"]
    tower = st1.get("issued_flop_per_board", 0) > 0  # the one-launch tower (input-row form)
    per_forward = 1 if tower else 2 * args.depth
    if tower:  # the launch also runs the stem conv (118 planes -> F, 3x3): its direct FLOP count too;
        # issued: the tower's own count (stem over the padded planes in, the slot plan's skipped taps out)
        direct_flop += HW * 2 * 118 * 9 * F
        issued = st1["issued_flop_per_board"]
    boards_per_launch = local_evals / max(launches / per_forward, 1)
    avg_ms = st1["conv_ms"] / max(launches, 1)
    roof = conv_roofline(args, args.conv_algo, per_forward, boards_per_launch, avg_ms, st1["conv_busy_ms"],
                         local_evals, launches, direct_flop, issued,
                         os.path.join(REPO, "profiles", "r6", "pmc_chess.json"),
                         ("tower16_rows" if tower else "f16x2") if args.conv_algo != 1 else "direct", chess=True,
                         tower=tower)
    if rank == 0:
        line = {
            "metric": f"MCTS node-expansions/s (Chess, {args.sims} sims/move)",
            "value": round(e / elapsed, 1),
            "unit": "expansions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32-accurate network (fp16 MFMA, two-term split operands, 3 products) / f64 PUCT",
            "data": "synthetic (self-generated games, random-init Keras-default weights, torch seed 0)",
            "config": {
                "workload": (f"Chess (custom_alphazero/chess), {args.sims} sims/move, {args.slots} concurrent "
                             f"games per GPU, (8,8,118) planes, 1880 actions, 128f x {args.depth}-block net "
                             f"(BASELINE.json configs[4], per-GPU shard of 2048 games over 8 GPUs)"),
                "global_batch": args.slots * world,
                "parallelism": f"games sharded over {world} GPU(s)",
            },
            "plies_per_s": round(p / elapsed, 2),
            "simulations_per_s": round(s / elapsed, 1),
            "network_evaluations_per_s": round(ev / elapsed, 1),
            "games_timed": int(g),
            "games_drained": int(dr),
            "transposition_cache": ({
                "capacity": st1["cache_capacity"], "hit_rate": round(hits / max(e, 1), 4),
                "entries": st1["cache_entries"], "inserts": st1["cache_inserts"],
                "dedup_share": round(1 - (ev + hits) / max(e, 1), 4),
                "semantics": "reference plays_inferences (mcts.py:122-143) on chess boards: key = leaf position + "
                             "history form, payload = masked priors + value; identical leaves of one simulation "
                             "share a network row; bit-identical results (LRU eviction, az_tree.h scheme)",
            } if args.cache_log2 else None),
            "games_drained_basis": "games whose records reached the host in the window (az_chess_selfplay_drain "
                                   "after every asynchronous step, and once more after the final synchronize)",
            "replay_buffer_gather": gather,
            "lanes": args.lanes or "auto",
            "roofline": roof,
            "cpu_baseline": base,
        }
        if base:
            line["gpu_over_cpu"] = round(line["value"] / base["value"], 1) if base["value"] else None
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


class WindowGames:
    """The games drained in the timed window (this rank), kept compact for
    the N>1 replay-buffer gather."""

    def __init__(self):
        self.parts = []

    def add(self, d):
        if len(d["lengths"]):
            self.parts.append(d)

    def results(self):
        if not self.parts:
            return None
        return {k: np.concatenate([p[k] for p in self.parts]) for k in
                ("lengths", "results", "expansions", "boards", "policies", "moves")}


def step_and_drain(eng, sink=None):
    """One move for every slot, then the D2H copy of the games it finished."""
    st = eng.selfplay_step(1)
    d = eng.selfplay_drain()
    if sink is not None:
        sink.add(d)
    return st, len(d["lengths"])


def launch_ranks(args):
    """--gpus N is authoritative.  Under a launcher (WORLD_SIZE set) it must
    equal the world size; without one and N > 1, this process starts the N
    ranks itself -- a torch.distributed.run child, before anything here has
    touched the GPU -- and exits with its status (the reference's fan-out is
    likewise one call, self_play.py:98-110).  Returns None when this process
    is a rank and should run the benchmark."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}; refusing to report a mislabelled run",
                  file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def arena_edges_arg(args):
    """az_config.arena_edges for --arena-edges: 0 lets the engine choose the
    overflow-proof size ('proof'); 'bounded' sizes the pools from the measured
    high-water mark (round 4: a lane half held at most 2.09 M of 60.2 M edges
    at configs[1], 1,020 per slot; 38.9 M of 963 M at configs[3]'s 16384-game
    shard, 4,750 per slot): 8*S*A + H*W*A per slot, 5.8x / 4.8x those."""
    if not args.compact or args.arena_edges == "proof":
        return 0
    A, HW = args.width, args.height * args.width
    if args.arena_edges == "bounded":
        return 8 * args.sims * A + HW * A
    return int(args.arena_edges)


def tree_arena(args, st, lanes):
    """The tree memory the engine chose and what the window used of it."""
    A, HW = args.width, args.height * args.width
    safe = args.sims * HW * A + A
    if not args.compact:
        return {"compact": False, "edges_per_slot": st["arena_edges"],
                "bytes_total": 32 * args.slots * st["arena_edges"],
                "rule": f"a static run of {st['arena_edges']} edges per slot (S*H*W*A + A = {safe}: the whole game)"}
    pool, high = st["arena_pool_edges"], st["arena_pool_high"]
    # the per-slot average the pools actually hold (a lane's half is also
    # capped at 2^31 - 1 edges, its indices' range, below arena_edges x slots)
    per_slot = pool // (2 * args.slots)
    proof = per_slot >= safe
    half = pool // (2 * lanes)
    return {
        "compact": True, "sizing": args.arena_edges, "pool_edges_total": pool, "bytes_total": 32 * pool,
        "pool_edges_per_half_per_slot": per_slot, "arena_edges_requested": st["arena_edges"],
        "overflow_proof": proof,
        "high_water_edges_per_lane_half": high, "lane_half_edges": half,
        "high_water_fraction": round(high / max(1, half), 4), "max_retained_edges": st["max_retained"],
        "rule": (f"pooled arenas: each lane owns two halves of {per_slot} edges x its slots; a slot takes "
                 f"{16 * A}-edge chunks of the current half as it expands, and after every move compaction copies "
                 f"each slot's kept subtree (Cheney scan) into the other half, which becomes the current one. "
                 + (f"{per_slot} >= S*H*W*A + A = {safe} per slot: no game can overflow it"
                    if proof else
                    f"{per_slot} < S*H*W*A + A = {safe} per slot ({args.arena_edges}: "
                    + ("8*S*A + H*W*A, ~5x the measured high-water mark" if args.arena_edges == "bounded"
                       else "a request, the 40%-of-free-HBM cap or a lane half's 2^31-edge index range")
                    + "): the slots share the pool, overflow raises a device error (none in this run)")),
    }


def check_device(eng, where):
    """The engine's device error word after a window of asynchronous steps
    (az_selfplay_step without stats returns before the kernels finish): a
    flagged window is not reported."""
    st = eng.stats()
    if st["errors"]:
        print(f"bench.py: device error flags {st['errors']:#x} after {where}; no result reported", file=sys.stderr)
        sys.exit(3)
    return st


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    if args.game == "chess":
        return chess_main(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from custom_alphazero.model.weights import init_weights, weight_spec

    A = args.width
    spec = weight_spec(args.height, args.width, A, depth=args.depth)
    host_w = init_weights(spec, seed=0)

    base = base0 = native = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(args, host_w)
        native = cpu_baseline_native(args, host_w)
        if (args.height, args.width, args.n) == (6, 7, 4) and args.cpu_configs0_seconds > 0:
            base0 = cpu_configs0(args, host_w)

    import torch
    import torch.distributed as dist
    from custom_alphazero import distributed as D
    from custom_alphazero import engine as az

    SUM = dist.ReduceOp.SUM if world > 1 else None
    MAX = dist.ReduceOp.MAX if world > 1 else None
    dev_index, dev = _init_dist(args, world, local_rank)
    devices = [dev_index]
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, dev_index)
    # weights: rank 0's init, one flat RCCL broadcast (~5 MB) to every rank
    named, _flat = _device_weights(spec, host_w, rank, world, args, dev)

    eng = az.Engine(args.height, args.width, args.n, True, args.sims, slots=args.slots,
                    evaluator=az.EVAL_NETWORK, depth=args.depth, device=dev_index,
                    cache_log2=args.cache_log2, lanes=args.lanes, conv_algo=args.conv_algo,
                    compact=bool(args.compact), arena_edges=arena_edges_arg(args), rng_skip=args.rng_skip)
    eng.set_weights(named)
    tree_steps = 3
    total_moves = MAX_PREROLL + 2 * args.steps + tree_steps + args.warmup
    budget = args.slots * (2 + total_moves // 7)   # a C4 game lasts >= 7 plies
    eng.selfplay_begin(first_game=rank * budget, n_games=budget, base_seed=0)

    # ---- untimed: at least --warmup moves, until the cache is stationary
    pre = 0
    while True:
        st, _ = step_and_drain(eng)
        pre += 1
        gen_ok = (not args.cache_log2 or not st["cache_gen_size"]
                  or (st["cache_inserts"] >= CACHE_TURNOVER * st["cache_capacity"]
                      and st["cache_entries"] >= CACHE_FULL * st["cache_capacity"]))
        done = pre >= max(args.warmup, MIN_PREROLL) and gen_ok
        if world > 1:  # every rank runs the same number of untimed moves
            (done,) = _reduce([0.0 if done else 1.0], SUM, world, args, dev)
            done = done == 0.0
        if done or pre >= MAX_PREROLL:
            break

    check_device(eng, "the untimed moves")
    # ---- timed window: K steps, each drained to the host
    window = WindowGames()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the tower timed by HIP events on every launch of each lane
    # (AZ_BENCH_WINDOW_EVENTS=k >= 3: every k-th; 0: none -- on one box every
    # 4th ran 5% SLOWER than every launch, profiles/r6/final/ab_events.txt)
    ev_env = os.environ.get("AZ_BENCH_WINDOW_EVENTS", str(WINDOW_EVENT_STRIDE))
    ev_stride = 1 if ev_env == "tree" else int(ev_env)  # "tree": the select and expand launches too
    eng.timer(ev_stride != 0, tree=ev_env == "tree", every=ev_stride if ev_stride != 0 else 1)
    st0 = eng.stats()
    t0 = time.perf_counter()
    drained = 0
    for _ in range(args.steps):
        # enqueue move m, then copy to the host the games finished by move m-1
        # (az_selfplay_drain waits for move m-1's count snapshot, never for
        # the running move: the GPU stays busy across move boundaries)
        eng.selfplay_step(1, sync=False)
        d = eng.selfplay_drain()
        window.add(d)
        drained += len(d["lengths"])
    torch.cuda.synchronize()
    d = eng.selfplay_drain()  # the window's last moves' games, still inside the timed region
    window.add(d)
    drained += len(d["lengths"])
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st1 = check_device(eng, "the timed window")
    eng.timer(False)
    d = {k: st1[k] - st0[k] for k in ("games_done", "expansions", "simulations", "plies",
                                      "terminal_visits", "cache_hits", "evaluations", "cache_inserts")}
    local_evals = d["evaluations"]
    conv_ms, conv_launches, busy_ms = st1["conv_ms"], st1["conv_launches"], st1["conv_busy_ms"]

    # ---- N>1: the window's games to rank 0 (replay-buffer gather, RCCL)
    gather = None
    if world > 1:
        t_g = time.perf_counter()
        res = window.results()
        if res is None:
            res = {"lengths": np.zeros(0, np.int32), "results": np.zeros(0, np.int32),
                   "expansions": np.zeros(0, np.int32),
                   "boards": np.zeros((0, args.height * args.width, args.height, args.width), np.int8),
                   "policies": np.zeros((0, args.height * args.width, A)),
                   "moves": np.zeros((0, args.height * args.width), np.int32)}
        gstats = {}
        g = D.gather_games(res, device=None if args.dist_backend == "gloo" else dev, stats=gstats)
        gt = time.perf_counter() - t_g
        if rank == 0:
            gather = {"games": int(len(g["lengths"])), "samples": int(len(g["moves"])),
                      "bytes": gstats["wire_bytes"],
                      "bytes_note": "what rank 0 received from the other ranks (its own games stay put)",
                      "seconds": round(gt, 4),
                      "how": f"compact int8 boards + f64 policies + int16 moves + per-game counts; a gather "
                             f"of the sizes, then each rank sends its blob to rank 0 only (point-to-point "
                             f"over {args.dist_backend}) after the timed window (distributed.gather_games)"}

    # ---- tree kernels (select + expand: latency/HBM-bound) timed with HIP
    # events in a short window of their own (4 more events per simulation),
    # priced with SURVEY.md 8d's algorithmic bytes per simulation
    eng.timer(True, tree=True)
    sa = eng.stats()
    for _ in range(tree_steps):
        step_and_drain(eng)
    sb = eng.stats()
    eng.timer(False)
    sims_t = max(sb["simulations"] - sa["simulations"], 1)
    depth = (sb["path_edges"] - sa["path_edges"]) / sims_t
    f_exp = (sb["expansions"] - sa["expansions"]) / sims_t
    bytes_per_sim = 16 * A * depth + 24 * depth + f_exp * (16 * A + 672 + 672 + 64)
    tree_gbs = bytes_per_sim * sims_t / (sb["tree_ms"] * 1e-3) / 1e9 if sb["tree_ms"] else 0.0
    roofline_tree = {
        "kernels": "select_group_kernel + expand_kernel (PUCT descent, backup, prior normalisation; the expand launch also carries the cache inserts)",
        "bound": "hbm", "achieved": round(tree_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(tree_gbs / HBM_PEAK_GBS, 5), "traffic": None,
        "bytes_per_simulation": round(bytes_per_sim, 1), "mean_depth": round(depth, 3),
        "expand_fraction": round(f_exp, 4),
        "avg_launch_ms": round(sb["tree_ms"] / max(sb["tree_launches"], 1), 4),
        "simulations_per_launch": round(sims_t / max(sb["tree_launches"] / 2, 1), 1),
        "basis": "16*A*d + 24*d + f_exp*(16*A + 672 + 672 + 64) bytes per simulation (SURVEY.md 8d) x "
                 "simulations / summed select+expand event time; latency-bound (dependent loads down "
                 "each path), not bandwidth-bound",
    }

    # ---- second window, same slots continuing, cache bypassed: the rate
    # without the reference's plays_inferences semantics (every leaf evaluated)
    off = None
    if args.cache_log2 and not args.no_cache_window:
        eng.cache_enable(False)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        s0 = eng.stats()
        t2 = time.perf_counter()
        g2 = 0
        for _ in range(args.steps):
            g2 += step_and_drain(eng)[1]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el2 = time.perf_counter() - t2
        s1 = eng.stats()
        g2, e2 = _reduce([g2, s1["expansions"] - s0["expansions"]], SUM, world, args, dev)
        (el2,) = _reduce([el2], MAX, world, args, dev)
        off = {"value": round(g2 / el2, 3), "unit": "games/s", "ms_per_step": round(1e3 * el2 / args.steps, 3),
               "expansions_per_s": round(e2 / el2, 1)}

    tot = _reduce([drained, d["games_done"], d["expansions"], d["simulations"], d["plies"], d["cache_hits"],
                   d["evaluations"]], SUM, world, args, dev)
    drained_all, games_all, exp_all, sims_all, plies_all, hits_all, evals_all = tot
    (elapsed,) = _reduce([elapsed], MAX, world, args, dev)
    if st1["active_slots"] < args.slots:
        print(f"warning: rank {rank} ran out of game budget", file=sys.stderr)

    # dominant kernel: the forward's residual-tower convs -- one tower16_kernel
    # launch per forward (AZ_CONV_F16X2), else one launch per conv.  Direct
    # FLOP = SURVEY.md 8d's count (19 F*F MACs per pixel per block: 9F + 9F +
    # the 1x1 F); the fp16x2 kernels issue each MAC as three fp16 products.
    HW, F = args.height * args.width, 128
    direct_flop = HW * 2 * F * F * 19 * args.depth
    issued = 3 * direct_flop if args.conv_algo != 1 else direct_flop
    per_forward = 1 if args.conv_algo == 0 else 2 * args.depth
    conv_avg_ms = conv_ms / max(conv_launches, 1)
    # every lane launches one forward per simulation (timed or not)
    all_launches = args.steps * args.sims * eng.lanes * per_forward
    boards_per_launch = local_evals / max(all_launches / per_forward, 1)
    if ev_stride >= 3:  # the union of the sampled intervals, scaled to every launch
        busy_ms *= ev_stride
    if args.conv_algo == 0 and st1.get("issued_flop_per_board", 0) > 0:
        # the tower reports what it issues: its tiles' pad rows and stem in,
        # the slot plan's skipped border taps (exact zeros) out; the dual
        # launch runs its smaller tiles at <= tower_small_max_boards live
        # boards (judged here by the mean launch)
        issued = st1["issued_flop_per_board"]
        if 0 < boards_per_launch <= st1.get("tower_small_max_boards", -1):
            issued = st1["issued_flop_per_board_small"]
    pmc = os.path.join(REPO, "profiles", "r6", "pmc_tower.json")
    # the PMC entry of this board shape (profiles/r6/collect_pmc.sh: 6x7 "tower16", 9x9 "tower16_9x9")
    pmc_key = {0: "tower16", 1: "direct", 2: "f16x2"}[args.conv_algo]
    if (args.height, args.width) != (6, 7):
        pmc_key += f"_{args.height}x{args.width}"
    roof = conv_roofline(args, args.conv_algo, per_forward, boards_per_launch, conv_avg_ms, busy_ms, local_evals,
                         conv_launches, direct_flop, issued, pmc, pmc_key)
    if ev_stride >= 3:
        roof["event_sampling"] = {
            "every": ev_stride, "launches_all": all_launches,
            "basis": (f"HIP events bracket every {ev_stride}th tower launch of each lane in the timed region "
                      f"(avg_launch_ms over those {conv_launches}); boards_per_launch over all {all_launches} "
                      f"launches (one per lane per simulation); busy_union from the timed launches' union x "
                      f"{ev_stride}")}

    # the same kernels alone on one stream at the live per-lane batch (what a
    # launch costs without the other lane's kernels sharing the CUs)
    if rank == 0:
        nb = max(1, int(round(boards_per_launch)))
        rng = np.random.RandomState(1)
        bx = rng.randint(-1, 2, (nb, args.height, args.width))
        xin = np.stack([bx == 0, bx == 1, bx == -1, np.ones_like(bx, bool)], -1).astype(np.float32)
        eng.forward(xin)
        eng.timer(True)
        for _ in range(10):
            eng.forward(xin)
        si = eng.stats()
        eng.timer(False)
        iso_ms = si["conv_ms"] / max(si["conv_launches"], 1)
        iso = nb * direct_flop / per_forward / (iso_ms * 1e-3) / 1e12
        roof["isolated"] = {"boards": nb, "avg_launch_ms": round(iso_ms, 4), "achieved": round(iso, 2),
                            "frac": round(iso / roof["peak"], 4)}

    cap = st1["cache_capacity"]
    gen_size = st1["cache_gen_size"]
    gen = st1["cache_generation"]
    game_name = "Connect-4 6x7" if (args.height, args.width, args.n) == (6, 7, 4) else \
        f"Connect-{args.n} {args.height}x{args.width}"
    cfg_ref = {(6, 7, 4, 100): "BASELINE.json configs[1]", (9, 9, 5, 200): "BASELINE.json configs[2]",
               (6, 7, 4, 400): "BASELINE.json configs[3], per-GPU shard"}.get(
        (args.height, args.width, args.n, args.sims), "custom")
    if rank == 0:
        line = {
            "metric": f"self-play games/s ({game_name}, {args.sims} sims/move)",
            "value": round(drained_all / elapsed, 3),
            "unit": "games/s",
            "n_gpus": world,
            "rank_devices": devices,
            "shared_devices": len(set(devices)) < len(devices),
            "dist_backend": args.dist_backend if world > 1 else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32-accurate network (fp16 MFMA, two-term split operands, 3 products) / f64 PUCT",
            "data": "synthetic (self-generated games, random-init Keras-default weights, torch seed 0)",
            "config": {
                "workload": (f"{game_name} n={args.n} gravity, {args.sims} sims/move, "
                             f"{args.slots} concurrent games per GPU, 128f x {args.depth}-block net "
                             f"({cfg_ref})"),
                "global_batch": args.slots * world,
                "parallelism": f"games sharded over {world} GPU(s)",
            },
            "lanes": eng.lanes,
            "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
            "untimed_moves": pre,
            "untimed_rule": (f"max(--warmup, {MIN_PREROLL}) moves and until the transposition cache is "
                             f"{CACHE_FULL:.0%} full and has taken {CACHE_TURNOVER}x its capacity in inserts "
                             f"(LRU content turned over: stationary hit rate, profiles/r6/cache_curve*)"),
            "games_timed": int(drained_all),
            "games_timed_basis": "games whose samples reached the host in the window (az_selfplay_drain "
                                 "after every step -- the previous move's games while the next move runs "
                                 "-- and once more after the final synchronize; D2H inside the timed region)",
            "games_finished_on_device": int(games_all),
            "expansions_per_s": round(exp_all / elapsed, 1),
            "simulations_per_s": round(sims_all / elapsed, 1),
            "plies_per_s": round(plies_all / elapsed, 1),
            "network_evaluations_per_s": round(evals_all / elapsed, 1),
            "transposition_cache": ({
                "capacity": cap,
                "hit_rate": round(hits_all / max(exp_all, 1), 4),
                "eviction": ({"inserts_per_generation": gen_size,
                              "rule": "least recently used: every entry is looked up, a hit moves it into the "
                                      "current generation, an insert into a full 16-slot bucket evicts its "
                                      "oldest entry 2+ generations old (az_tree.h)"} if gen_size else None),
                "generation_at_window_end": gen,
                "entries": st1["cache_entries"],
                "fill": round(st1["cache_entries"] / cap, 4) if cap else None,
                "inserts_over_capacity_at_window_end": round(st1["cache_inserts"] / cap, 3) if cap else None,
                "bytes": cap * (32 + 4 + 4 * (A + 1)) if cap else None,
                "age_moves_at_window_start": pre,
                "inserts_in_window": d["cache_inserts"],
                "semantics": "reference plays_inferences (mcts.py:122-143): board -> network output, shared "
                             "by all games on the GPU, emptied when weights change; bit-identical results",
            } if args.cache_log2 else None),
            "tree_arena": tree_arena(args, st1, eng.lanes),
            "cache_off": off,
            "roofline_tree": roofline_tree,
            "roofline": roof,
            "replay_buffer_gather": gather,
            "cpu_baseline": base,
            "cpu_baseline_native": native,
            "cpu_baseline_configs0": base0,
        }
        if base:
            line["gpu_over_cpu"] = round(line["value"] / base["value"], 1) if base["value"] else None
        if native:
            line["gpu_over_cpu_native"] = round(line["value"] / native["value"], 1) if native["value"] else None
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
