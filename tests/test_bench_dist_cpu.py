"""bench.py's N>1 glue at world size 2 over gloo on the CPU: the weight
broadcast (_device_weights), the max/sum reductions of the timing and the
counters (_reduce), and the window games' gather to rank 0 (WindowGames +
distributed.gather_games) -- the same functions bench.main runs per rank,
fed with drained-game records of the engine's layout (selfplay_drain).
The GPU side of the same path is tests/test_distributed_gpu.py."""
import argparse
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H, W = 6, 7


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _drained(rank, step, n):
    """n finished games as selfplay_drain returns them (leading game axis,
    padded to H*W plies); contents tagged by (rank, step, game)."""
    P = H * W
    rng = np.random.RandomState(1000 * rank + step)
    lengths = rng.randint(7, P + 1, n).astype(np.int32)
    out = dict(game_ids=np.arange(n, dtype=np.int64) + 100 * rank + 10 * step,
               lengths=lengths, results=rng.randint(-1, 2, n).astype(np.int32),
               expansions=rng.randint(1, 5000, n).astype(np.int32),
               boards=np.zeros((n, P, H, W), np.int8), policies=np.zeros((n, P, W)),
               moves=np.zeros((n, P), np.int32))
    for g in range(n):
        T = lengths[g]
        out["boards"][g, :T] = rng.randint(-1, 2, (T, H, W))
        out["policies"][g, :T] = rng.dirichlet(np.ones(W), T)
        out["moves"][g, :T] = rng.randint(0, W, T)
    return out


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    bench = _bench()
    from custom_alphazero import distributed as D
    from custom_alphazero.model.weights import init_weights, weight_spec
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = argparse.Namespace(dist_backend="gloo")
    dev = torch.device("cpu")

    spec = weight_spec(H, W, W, depth=1)
    host_w = init_weights(spec, seed=0) if rank == 0 else init_weights(spec, seed=123)
    named, flat = bench._device_weights(spec, host_w, rank, world, args, dev)
    ref = init_weights(spec, seed=0)
    for (name, t), (n2, shape) in zip(named, spec):
        assert name == n2
        np.testing.assert_array_equal(t.numpy(), ref[name].reshape(-1))

    (el,) = bench._reduce([1.5 + rank], dist.ReduceOp.MAX, world, args, dev)
    assert el == 1.5 + world - 1
    tot = bench._reduce([rank + 1, 10], dist.ReduceOp.SUM, world, args, dev)
    assert tot == [world * (world + 1) / 2, 10 * world]

    window = bench.WindowGames()
    for step, n in enumerate((2, 0, 3 + rank)):  # a step that drained nothing is skipped
        window.add(_drained(rank, step, n))
    g = D.gather_games(window.results(), device=None)
    if rank == 0:
        np.savez(os.path.join(outdir, "gathered.npz"), **g)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_glue_world2(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    got = dict(np.load(tmp_path / "gathered.npz"))
    bench = _bench()
    from custom_alphazero import distributed as D
    expect = []
    for r in range(world):
        w = bench.WindowGames()
        for step, n in enumerate((2, 0, 3 + r)):
            w.add(_drained(r, step, n))
        expect.append(D._pack(w.results()))
    for k in ("lengths", "results", "expansions", "boards", "policies", "moves"):
        np.testing.assert_array_equal(got[k], np.concatenate([e[k] for e in expect]), err_msg=k)
    assert len(got["lengths"]) == 2 + 3 + 2 + 4
    # and the gathered games expand to the reference's sample layout
    states, pol, rew = D.to_samples(got)
    assert states.shape == (int(got["lengths"].sum()), H, W, 4) and len(rew) == len(pol) == len(states)


def test_bench_refuses_a_mislabelled_world():
    """--gpus N is authoritative: under a launcher whose WORLD_SIZE differs,
    bench.py exits non-zero before touching the GPU or printing a line."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=120, cwd=REPO, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_launch_command_for_n_ranks(monkeypatch):
    """Without a launcher and N > 1, bench.py starts N ranks itself: one
    torch.distributed.run child on 127.0.0.1 with the same arguments."""
    import subprocess
    bench = _bench()
    seen = {}

    class Done:
        returncode = 0

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(bench.sys, "argv", ["bench.py", "--gpus", "4", "--steps", "7"])
    args = argparse.Namespace(gpus=4)
    assert bench.launch_ranks(args) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # one rank, or already under a launcher with the same world: run in-process
    assert bench.launch_ranks(argparse.Namespace(gpus=1)) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.launch_ranks(args) is None


def test_bench_refuses_more_ranks_than_gpus(monkeypatch):
    """One rank per GPU: a world larger than the visible devices exits with
    status 2 before any GPU call (unless --share-devices asks for a
    rehearsal that shares them)."""
    import torch
    bench = _bench()
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    with pytest.raises(SystemExit) as ex:
        bench.check_devices(argparse.Namespace(share_devices=False), 4)
    assert ex.value.code == 2
    assert bench.check_devices(argparse.Namespace(share_devices=True), 4) == 2
    assert bench.check_devices(argparse.Namespace(share_devices=False), 2) == 2


def test_roofline_traffic_only_from_the_same_build(tmp_path):
    """the line's PMC traffic and MFMA-busy fraction come
    from a profile that recorded the libaz build it measured; a profile of
    another build yields null with the reason."""
    import json
    from custom_alphazero import engine as az
    bench = _bench()
    build, _ = az.build_id()
    entry = {"boards_per_launch": 672, "mean_hbm_bytes_per_board_per_launch": 1000.0, "mfma_busy": 0.5}
    f = tmp_path / "pmc.json"
    args = argparse.Namespace()
    for bid, want in ((build, 672 * 1000), ("0123456789abcdef", None)):
        f.write_text(json.dumps({"build_id": bid, "tower16": entry}))
        r = bench.conv_roofline(args, 0, 1, 672.0, 0.2, 10.0, 6720, 10, 104.6e6, 270.5e6, str(f), "tower16")
        assert r["traffic"] == want, r["pmc"]
        assert r["mfma_busy"] == (0.5 if want else None)
        assert r["build_id"] == build
    r = bench.conv_roofline(args, 0, 1, 672.0, 0.2, 10.0, 6720, 10, 104.6e6, 270.5e6, str(tmp_path / "no"), "tower16")
    assert r["traffic"] is None and "no PMC profile" in r["pmc"]


def test_tree_arena_rule_states_the_pool_it_holds():
    """the line's arena rule is the size the pools hold --
    per slot, the pools' edges over both halves and all slots, not the
    requested average (a lane half is also capped at 2^31 - 1 edges)."""
    bench = _bench()
    args = argparse.Namespace(width=7, height=6, sims=100, slots=4096, compact=True, lanes=0,
                              arena_edges="proof")
    safe = 100 * 42 * 7 + 7
    st = dict(arena_edges=safe, arena_pool_edges=2 * 4096 * safe, arena_pool_high=10, max_retained=5)
    r = bench.tree_arena(args, st, 2)
    assert r["overflow_proof"] and r["pool_edges_per_half_per_slot"] == safe and "no game can overflow" in r["rule"]
    capped = dict(st, arena_pool_edges=2 * 2 * ((1 << 31) - 1))  # two lanes, each half at the index cap
    args.slots, args.sims = 65536, 400
    r = bench.tree_arena(args, capped, 2)
    assert not r["overflow_proof"] and r["pool_edges_per_half_per_slot"] == 2 * ((1 << 31) - 1) // 65536
    assert "share the pool" in r["rule"]


def test_bounded_arena_is_sized_from_the_measured_high_water_mark():
    """--arena-edges bounded (the default) asks for
    8*S*A + H*W*A edges per slot -- 5,894 at configs[1], ~5.8x the 1,020 per
    slot a lane half held at its high-water mark in round 4 -- instead of
    the overflow-proof 29,407; the line states the pool and the fraction the
    window's high-water mark used."""
    bench = _bench()
    args = argparse.Namespace(width=7, height=6, sims=100, slots=4096, compact=True, lanes=0,
                              arena_edges="bounded")
    assert bench.arena_edges_arg(args) == 8 * 100 * 7 + 42 * 7 == 5894
    assert bench.arena_edges_arg(argparse.Namespace(**dict(vars(args), arena_edges="proof"))) == 0
    assert bench.arena_edges_arg(argparse.Namespace(**dict(vars(args), arena_edges="1234"))) == 1234
    st = dict(arena_edges=5894, arena_pool_edges=2 * 4096 * 5894, arena_pool_high=2_090_000, max_retained=2485)
    r = bench.tree_arena(args, st, 2)
    assert not r["overflow_proof"] and r["sizing"] == "bounded"
    assert r["lane_half_edges"] == 2048 * 5894 and r["high_water_fraction"] == round(2_090_000 / (2048 * 5894), 4)
    assert "measured high-water mark" in r["rule"]
