#!/usr/bin/env python3
"""Self-play throughput on MI355X: games/s + MCTS node-expansions/s.

Workload (BASELINE.json configs[1]): Connect-4 6x7, n=4, gravity, 100
simulations per move, 4096 concurrent games per GPU, random-init
128-filter x 4-block policy/value network (Keras defaults, torch seed 0).
A "step" is one move for every game slot: `sims` lockstep simulations
(select -> batched network forward -> expand/backup) then a move commit;
finished games are replaced by new ones (game g seeded MT19937(g)), so the
timed window is steady-state.  value = games completed in the K timed steps,
summed over ranks, / max-over-ranks wall time.

Multi-GPU (torchrun, one rank per GPU): games are sharded by global game id
(independent, no data-path collective: scaling "weak"); rank 0's weights
reach the other ranks by one RCCL broadcast over xGMI before timing.

The CPU baseline (rank 0, N=1 only) is oracle/refport.py -- the reference's
self-play structure, pinned to the reference by tests/test_refport.py -- run
as one game per worker process with a 1-thread torch-CPU network, like the
reference's joblib fan-out; it runs before the GPU is touched.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E ~8 TB/s
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no 2:1 sparsity)


def wino_x3():
    """The engines' Winograd kernel: 1 (default) = fp32 products from three bf16
    terms per operand (csrc/az_wino16x.hip), 0 = fp32 MFMA (az_wino16.hip)."""
    v = os.environ.get("AZ_WINO_X3")
    return int(v) if v is not None else 1


def issued_mfma(achieved, conv_flop_per_board, mfma_flop_per_board, conv_algo):
    """The MFMA work the conv kernel issues for `achieved` algorithmic TFLOP/s:
    the Winograd FLOP (2.25x below the direct count at 2x2 tiles) as fp32
    16x16x4 MFMAs, or as six bf16 16x16x32 products per fp32 product."""
    wino = achieved * mfma_flop_per_board / conv_flop_per_board
    if conv_algo == 0 and wino_x3():
        a = 6 * wino
        return {"dtype": "bf16 (3 terms per fp32 operand, 6 products)", "flop_per_board": 6 * mfma_flop_per_board,
                "achieved": round(a, 2), "peak": BF16_MFMA_PEAK_TFLOPS, "frac": round(a / BF16_MFMA_PEAK_TFLOPS, 4)}
    return {"dtype": "fp32", "flop_per_board": mfma_flop_per_board, "achieved": round(wino, 2),
            "peak": FP32_MFMA_PEAK_TFLOPS, "frac": round(wino / FP32_MFMA_PEAK_TFLOPS, 4)}


def conv_kernel_name(conv_algo, chess=False):
    if conv_algo != 0:
        return "conv3x3_mfma (fp32 MFMA implicit-GEMM 3x3 conv, fused BN/ReLU/residual)"
    k = ("wino16x_conv_kernel (Winograd F(2x2,3x3), fp32 products from three bf16 terms per operand on "
         "the 16x16x32 bf16 MFMA" if wino_x3() else
         "wino16_conv_kernel (Winograd F(2x2,3x3) on the fp32 16x16x4 MFMA")
    return k + (", residual tower, 8 launches per forward)" if chess else
                ", 16 tiles per workgroup, fused BN/ReLU and 1x1 projection residual)")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--game", choices=("connect_n", "chess"), default="connect_n",
                    help="chess: BASELINE configs[4] per-GPU shard (256 games, 800 sims/move)")
    ap.add_argument("--steps", type=int, default=None, help="timed moves (30; chess 3)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed moves first (60; chess 2)")
    ap.add_argument("--slots", type=int, default=None, help="concurrent games per GPU (4096; chess 256)")
    ap.add_argument("--sims", type=int, default=None, help="sims per move (100; chess 800)")
    ap.add_argument("--height", type=int, default=6)
    ap.add_argument("--width", type=int, default=7)
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = min(15, cores-1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lanes", type=int, default=0, help="slot groups on separate HIP streams (0 = auto)")
    ap.add_argument("--conv-algo", type=int, default=0, help="0 Winograd, 1 direct")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on MI355X; gloo for rehearsals")
    ap.add_argument("--cache-log2", type=int, default=25,
                    help="transposition cache (the reference's plays_inferences) entries = 2^N; 0 = off")
    ap.add_argument("--no-cache-window", action="store_true",
                    help="skip the second timed window with the cache bypassed")
    args = ap.parse_args()
    chess = args.game == "chess"
    for k, c4, ch in (("steps", 30, 3), ("warmup", 60, 2), ("slots", 4096, 256), ("sims", 100, 800)):
        if getattr(args, k) is None:
            setattr(args, k, ch if chess else c4)
    return args


def cpu_baseline(args, weights):
    """Reference-structured CPU self-play, bounded sample (about budget seconds)."""
    import multiprocessing as mp
    import platform

    import refport
    cores = len(os.sched_getaffinity(0))
    workers = args.cpu_workers or max(1, min(15, cores - 1))
    job = (args.height, args.width, args.n, True, args.sims, weights, args.depth,
           args.cpu_baseline_seconds)
    ctx = mp.get_context("fork")  # no GPU initialised yet in this process
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(refport.baseline_worker, [job + (10_000_000 + 1000 * i,) for i in range(workers)])
    wall = time.perf_counter() - t0
    games = sum(r[0] for r in res)
    exps = sum(r[1] for r in res)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        cpu_model = platform.processor()
    return {
        "value": round(games / wall, 4), "unit": "games/s", "cores": workers,
        "kind": "port", "expansions_per_s": round(exps / wall, 1),
        "sample": (f"oracle/refport.py self-play, C4 {args.sims} sims/move, {workers} worker processes "
                   f"x 1 torch-CPU thread, batch-1 forward, plays_inferences dict kept across each "
                   f"worker's games; {games} games in "
                   f"{wall:.1f}s ({cpu_model})"),
    }


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


def chess_cpu_baseline(args, weights):
    import multiprocessing as mp

    import refport
    cores = len(os.sched_getaffinity(0))
    workers = args.cpu_workers or max(1, min(15, cores - 1))
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(refport.chess_baseline_worker,
                       [(args.sims, weights, args.depth, args.cpu_baseline_seconds, 20_000_000 + i)
                        for i in range(workers)])
    wall = time.perf_counter() - t0
    exps = sum(r[0] for r in res)
    return {"value": round(exps / wall, 2), "unit": "expansions/s", "cores": workers, "kind": "port",
            "plies_per_s_est": round(sum(r[1] for r in res) / wall, 4),
            "sample": (f"oracle chess MCTS (C tree, reference arithmetic) + torch-CPU network at batch 1 "
                       f"on Board.full_state, {workers} worker processes x 1 thread, {args.sims} sims/move, "
                       f"{exps} expansions in {wall:.1f}s; the reference's own chess path cannot run "
                       f"under MCTS (chess/board.py:178 vs mcts.py:179)")}


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
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(dev_index)
        dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", dev_index)
    named, _flat = _device_weights(spec, host_w, rank, world, args, dev)
    eng = az.ChessEngine(mcts_iterations=args.sims, slots=args.slots, evaluator=az.EVAL_NETWORK,
                         max_plies=512, depth=args.depth, device=dev_index, conv_algo=args.conv_algo,
                         lanes=args.lanes)
    eng.set_weights(named)
    budget = args.slots * 2
    eng.selfplay_begin(first_game=rank * budget, n_games=budget, base_seed=0)
    eng.selfplay_step(args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.timer(True)
    st0 = eng.stats()
    t0 = time.perf_counter()
    eng.selfplay_step(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st1 = eng.stats()
    eng.timer(False)
    d = {k: st1[k] - st0[k] for k in ("games_done", "expansions", "simulations", "plies",
                                      "terminal_visits", "evaluations")}
    local_evals = d["evaluations"]
    if world > 1:
        red_dev = "cpu" if args.dist_backend == "gloo" else dev
        t = torch.tensor([d["games_done"], d["expansions"], d["simulations"], d["plies"]],
                         dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        tmax = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        d["games_done"], d["expansions"], d["simulations"], d["plies"] = (int(v) for v in t.tolist())
        elapsed = float(tmax.item())
    F, HW, TB = 128, 64, 16
    conv_flop_per_board = HW * 2 * F * F * 19 * args.depth     # direct 3x3 + 1x1 residual, tower only
    mfma_flop_per_board = (TB * 36 * 2 * F * F * args.depth if args.conv_algo == 0
                           else conv_flop_per_board)
    busy = st1["conv_busy_ms"]
    launches = st1["conv_launches"]
    boards_per_launch = local_evals / max(launches / (2 * args.depth), 1)
    avg_ms = st1["conv_ms"] / max(launches, 1)
    # per launch: algorithmic FLOP of one tower conv / its mean duration (HIP events)
    achieved = boards_per_launch * conv_flop_per_board / (2 * args.depth) / (avg_ms * 1e-3) / 1e12 if avg_ms else 0.0
    union = local_evals * conv_flop_per_board / (busy * 1e-3) / 1e12 if busy else 0.0
    traffic = None
    pmc = os.path.join(REPO, "profiles", "r1", "pmc_chess_traffic.json")
    if os.path.exists(pmc):  # PMC bytes/board (FETCH_SIZE/WRITE_SIZE passes) x live batch
        with open(pmc) as fp:
            traffic = int(json.load(fp)["winograd"]["mean_hbm_bytes_per_board_per_launch"] * boards_per_launch)
    if rank == 0:
        line = {
            "metric": f"MCTS node-expansions/s (Chess, {args.sims} sims/move)",
            "value": round(d["expansions"] / elapsed, 1),
            "unit": "expansions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32 network / f64 PUCT",
            "data": "synthetic (self-generated games, random-init Keras-default weights, torch seed 0)",
            "config": {
                "workload": (f"Chess (custom_alphazero/chess), {args.sims} sims/move, {args.slots} concurrent "
                             f"games per GPU, (8,8,118) planes, 1880 actions, 128f x {args.depth}-block net "
                             f"(BASELINE.json configs[4], per-GPU shard of 2048 games over 8 GPUs)"),
                "global_batch": args.slots * world,
                "parallelism": f"games sharded over {world} GPU(s)",
            },
            "plies_per_s": round(d["plies"] / elapsed, 2),
            "simulations_per_s": round(d["simulations"] / elapsed, 1),
            "games_timed": d["games_done"],
            "terminal_visits": d["terminal_visits"],
            "lanes": args.lanes or "auto",
            "roofline": {
                "kernel": conv_kernel_name(args.conv_algo, chess=True),
                "bound": "mfma",
                "achieved": round(achieved, 2),
                "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (PMC bytes/board, profiles/r1/pmc_chess_traffic.json, "
                                "x live boards/launch)",
                "achieved_basis": "algorithmic (direct-convolution) FLOP per launch (boards_per_launch x "
                                  "algorithmic_flop_per_board / 8 tower launches) / avg_launch_ms (HIP events)",
                "busy_union": {"achieved": round(union, 2), "frac": round(union / FP32_MFMA_PEAK_TFLOPS, 4)},
                "algorithmic_flop_per_board": conv_flop_per_board,
                "mfma_flop_per_board": mfma_flop_per_board,
                "issued": issued_mfma(achieved, conv_flop_per_board, mfma_flop_per_board, args.conv_algo),
                "boards_per_launch": round(boards_per_launch, 1),
                "avg_launch_ms": round(avg_ms, 4),
                "conv_busy_ms": round(busy, 2),
            },
            "cpu_baseline": base,
        }
        if base:
            line["gpu_over_cpu"] = round(line["value"] / base["value"], 1) if base["value"] else None
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.game == "chess":
        return chess_main(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    from custom_alphazero.model.weights import init_weights, weight_spec

    A = args.width
    spec = weight_spec(args.height, args.width, A, depth=args.depth)
    host_w = init_weights(spec, seed=0)

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(args, host_w)

    import torch
    import torch.distributed as dist
    from custom_alphazero import engine as az

    # one rank per GPU; the modulo only matters when rehearsing several ranks
    # on a one-GPU box
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(dev_index)
        dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", dev_index)
    # weights: rank 0's init, one flat RCCL broadcast (~5 MB) to every rank
    named, _flat = _device_weights(spec, host_w, rank, world, args, dev)

    eng = az.Engine(args.height, args.width, args.n, True, args.sims, slots=args.slots,
                    evaluator=az.EVAL_NETWORK, depth=args.depth, device=dev_index,
                    cache_log2=args.cache_log2, lanes=args.lanes, conv_algo=args.conv_algo)
    eng.set_weights(named)
    tree_steps = 3
    budget = args.slots * (2 + (args.warmup + 2 * args.steps + tree_steps) // 5)
    eng.selfplay_begin(first_game=rank * budget, n_games=budget, base_seed=0)

    eng.selfplay_step(args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.timer(True)
    st0 = eng.stats()
    t0 = time.perf_counter()
    eng.selfplay_step(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st1 = eng.stats()
    eng.timer(False)

    # tree kernels (select + expand: latency/HBM-bound) timed with HIP events
    # in a short window of their own (4 more events per simulation), priced
    # with SURVEY.md 8d's algorithmic bytes per simulation
    eng.timer(True, tree=True)
    sa = eng.stats()
    eng.selfplay_step(tree_steps)
    sb = eng.stats()
    eng.timer(False)
    sims_t = max(sb["simulations"] - sa["simulations"], 1)
    depth = (sb["path_edges"] - sa["path_edges"]) / sims_t
    f_exp = (sb["expansions"] - sa["expansions"]) / sims_t
    A = args.width
    bytes_per_sim = 16 * A * depth + 24 * depth + f_exp * (16 * A + 672 + 672 + 64)
    tree_gbs = bytes_per_sim * sims_t / (sb["tree_ms"] * 1e-3) / 1e9 if sb["tree_ms"] else 0.0
    roofline_tree = {
        "kernels": "select_group_kernel + expand_kernel (PUCT descent, backup, prior normalisation)",
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

    # second window, same slots continuing, cache bypassed: the rate without
    # the reference's plays_inferences semantics (every leaf evaluated)
    off = None
    if args.cache_log2 and not args.no_cache_window:
        eng.cache_enable(False)
        if world > 1:
            dist.barrier()
        s0 = eng.stats()
        t0 = time.perf_counter()
        eng.selfplay_step(args.steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el2 = time.perf_counter() - t0
        s1 = eng.stats()
        g2 = s1["games_done"] - s0["games_done"]
        if world > 1:
            t2 = torch.tensor([g2, el2], dtype=torch.float64,
                              device="cpu" if args.dist_backend == "gloo" else dev)
            dist.all_reduce(t2[:1], op=dist.ReduceOp.SUM)
            tm = t2[1:].clone()
            dist.all_reduce(tm, op=dist.ReduceOp.MAX)
            g2, el2 = int(t2[0].item()), float(tm.item())
        off = {"value": round(g2 / el2, 3), "unit": "games/s", "ms_per_step": round(1e3 * el2 / args.steps, 3),
               "expansions_per_s": round((s1["expansions"] - s0["expansions"]) / el2 * world, 1)}

    d = {k: st1[k] - st0[k] for k in ("games_done", "expansions", "simulations", "plies",
                                      "terminal_visits", "cache_hits", "evaluations")}
    conv_ms, conv_launches = st1["conv_ms"], st1["conv_launches"]
    if world > 1:
        red_dev = "cpu" if args.dist_backend == "gloo" else dev
        t = torch.tensor([d["games_done"], d["expansions"], d["simulations"], d["plies"]],
                         dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        tmax = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        d["games_done"], d["expansions"], d["simulations"], d["plies"] = (int(v) for v in t.tolist())
        elapsed = float(tmax.item())
    if st1["active_slots"] < args.slots:
        print(f"warning: rank {rank} ran out of game budget", file=sys.stderr)

    # dominant kernel: the residual tower's 3x3 convs (8 launches per forward at
    # depth 4).  Algorithmic FLOP = the direct convolution (SURVEY.md 8d, 19 F*F
    # MACs per pixel per block: 9F + 9F + the 1x1 F); the Winograd kernel issues
    # fewer MFMA FLOP (16 points per 2x2 tile + 4 residual rows per conv2).
    HW, F = args.height * args.width, 128
    TB = ((args.height + 1) // 2) * ((args.width + 1) // 2)
    conv_flop_per_board = HW * 2 * F * F * 19 * args.depth
    mfma_flop_per_board = (TB * 36 * 2 * F * F * args.depth if args.conv_algo == 0
                           else conv_flop_per_board)
    local_exp = st1["evaluations"] - st0["evaluations"]  # boards the network computed
    conv_avg_ms = conv_ms / max(conv_launches, 1)
    busy_ms = st1["conv_busy_ms"]
    boards_per_launch = local_exp / max(conv_launches / (2 * args.depth), 1)
    # roofline.achieved: algorithmic FLOP of one launch (a conv of the tower,
    # the mean of conv1 and conv2) / the launch's mean duration (HIP events
    # on its lane's stream); with two lanes a launch shares the CUs with the
    # other lane's kernels, so the union-of-busy-time rate is given beside it
    per_launch_flop = boards_per_launch * conv_flop_per_board / (2 * args.depth)
    achieved = per_launch_flop / (conv_avg_ms * 1e-3) / 1e12 if conv_avg_ms else 0.0
    union = (local_exp * conv_flop_per_board) / (busy_ms * 1e-3) / 1e12 if busy_ms else 0.0
    traffic = None
    pmc = os.path.join(REPO, "profiles", "r1", "pmc_conv_traffic.json")
    if os.path.exists(pmc):  # PMC bytes/board (rocprofv3 FETCH_SIZE/WRITE_SIZE) x live batch
        with open(pmc) as fp:
            tj = json.load(fp)
        key = "winograd" if args.conv_algo == 0 else "direct"
        if key in tj:
            traffic = int(tj[key]["mean_hbm_bytes_per_board_per_launch"] * boards_per_launch)

    # the same kernels alone on one stream at the live per-lane batch (what a
    # launch costs without the other lane's kernels sharing the CUs)
    isolated = None
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
        iso = nb * conv_flop_per_board / (2 * args.depth) / (iso_ms * 1e-3) / 1e12
        isolated = {"boards": nb, "avg_launch_ms": round(iso_ms, 4),
                    "achieved": round(iso, 2), "frac": round(iso / FP32_MFMA_PEAK_TFLOPS, 4),
                    "issued": issued_mfma(iso, conv_flop_per_board, mfma_flop_per_board, args.conv_algo)}

    game_name = "Connect-4 6x7" if (args.height, args.width, args.n) == (6, 7, 4) else \
        f"Connect-{args.n} {args.height}x{args.width}"
    cfg_ref = {(6, 7, 4, 100): "BASELINE.json configs[1]", (9, 9, 5, 200): "BASELINE.json configs[2]",
               (6, 7, 4, 400): "BASELINE.json configs[3], per-GPU shard"}.get(
        (args.height, args.width, args.n, args.sims), "custom")
    if rank == 0:
        line = {
            "metric": f"self-play games/s ({game_name}, {args.sims} sims/move)",
            "value": round(d["games_done"] / elapsed, 3),
            "unit": "games/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32 network / f64 PUCT",
            "data": "synthetic (self-generated games, random-init Keras-default weights, torch seed 0)",
            "config": {
                "workload": (f"{game_name} n={args.n} gravity, {args.sims} sims/move, "
                             f"{args.slots} concurrent games per GPU, 128f x {args.depth}-block net "
                             f"({cfg_ref})"),
                "global_batch": args.slots * world,
                "parallelism": f"games sharded over {world} GPU(s)",
            },
            "expansions_per_s": round(d["expansions"] / elapsed, 1),
            "simulations_per_s": round(d["simulations"] / elapsed, 1),
            "plies_per_s": round(d["plies"] / elapsed, 1),
            "games_timed": d["games_done"],
            "network_evaluations_per_s": round(d["evaluations"] / elapsed, 1),
            "transposition_cache": ({"entries": 2 ** args.cache_log2,
                                     "hit_rate": round(d["cache_hits"] / max(d["expansions"], 1), 4),
                                     "semantics": "reference plays_inferences (mcts.py:122-143): board -> "
                                                  "network output, shared by all games, emptied when "
                                                  "weights change; bit-identical results"}
                                    if args.cache_log2 else None),
            "cache_off": off,
            "roofline_tree": roofline_tree,
            "roofline": {
                "kernel": conv_kernel_name(args.conv_algo),
                "bound": "mfma",
                "achieved": round(achieved, 2),
                "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (PMC bytes/board, profiles/r1/pmc_conv_traffic.json, "
                                "x live boards/launch)",
                "achieved_basis": "algorithmic (direct-convolution) FLOP per launch (boards_per_launch x "
                                  "algorithmic_flop_per_board / 8 launches) / avg_launch_ms (HIP events on "
                                  "each lane's stream, timed region)",
                "busy_union": {"achieved": round(union, 2), "frac": round(union / FP32_MFMA_PEAK_TFLOPS, 4),
                               "basis": "all timed boards' algorithmic FLOP / union of the conv intervals of "
                                        "both lanes (launches of the two lanes overlap)"},
                "algorithmic_flop_per_board": conv_flop_per_board,
                "mfma_flop_per_board": mfma_flop_per_board,
                "issued": issued_mfma(achieved, conv_flop_per_board, mfma_flop_per_board, args.conv_algo),
                "boards_per_launch": round(boards_per_launch, 1),
                "avg_launch_ms": round(conv_avg_ms, 4),
                "conv_busy_ms": round(busy_ms, 2),
                "launches_timed": conv_launches,
                "isolated": isolated,
            },
            "cpu_baseline": base,
        }
        if base:
            line["gpu_over_cpu"] = round(line["value"] / base["value"], 1) if base["value"] else None
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
