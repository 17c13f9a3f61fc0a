"""RCCL on the box's one GPU: the nccl-only code of the N>1 path.

RCCL does not put two ranks on one device, so the two-rank rehearsals
(tests/test_distributed_gpu.py) run over gloo, and the device-memory
collectives -- the weight broadcast and the replay-buffer gather on the
rank's GPU (custom_alphazero.distributed, self_play.py:96-118 in the
reference) -- would otherwise run only on the driver's multi-GPU node.  Here
a one-rank nccl group drives them through RCCL on cuda:0: the broadcast
weights are the host weights bit for bit, bench.py's broadcast and
all-reduces (their multi-rank branches) run on the device, and the games
gathered through RCCL are one engine's games bit for bit.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H, W, N, S = 6, 7, 4, 16
N_GAMES = 12
BASE_SEED = 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _paths():
    for p in (os.path.join(REPO, "custom-alphazero_amd"), REPO):
        if p not in sys.path:
            sys.path.insert(0, p)


def _spec_and_host():
    from custom_alphazero.model.weights import init_weights, weight_spec
    spec = weight_spec(H, W, W)
    return spec, init_weights(spec, seed=9, randomize_bn=True)


def _worker(rank, port, outdir):
    _paths()
    import torch
    import torch.distributed as dist
    from custom_alphazero import distributed as D
    from custom_alphazero import engine as az
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    spec, host = _spec_and_host()
    named = D.broadcast_weights([(n, torch.from_numpy(host[n])) for n, _ in spec])
    for (n, t) in named:  # on the rank's GPU (collective_device under nccl), unchanged
        assert t.device == dev, n
        np.testing.assert_array_equal(t.cpu().numpy(), host[n].astype(np.float32), err_msg=n)
    # bench.py's own multi-rank branches (taken when world > 1) on the same group
    import argparse
    import bench
    a = argparse.Namespace(dist_backend="nccl")
    bnamed, flat = bench._device_weights(spec, host, 0, 2, a, dev)
    assert flat.device == dev
    for (n, t) in bnamed:
        np.testing.assert_array_equal(t.cpu().numpy().reshape(host[n].shape), host[n], err_msg=n)
    assert bench._reduce([1.5, 2.0], dist.ReduceOp.SUM, 2, a, dev) == [1.5, 2.0]
    assert bench._reduce([3.0], dist.ReduceOp.MAX, 2, a, dev) == [3.0]
    devices = [None]
    dist.all_gather_object(devices, 0)
    assert devices == [0]
    eng = az.Engine(H, W, N, True, S, slots=8, evaluator=az.EVAL_NETWORK, compact=True)
    eng.set_weights(named)
    g = D.selfplay_sharded(D.engine_runner(eng), N_GAMES, BASE_SEED)  # gather: RCCL gather (+ point-to-point for other ranks) on cuda:0
    eng.close()
    np.savez(os.path.join(outdir, "rccl.npz"), **g)
    # the chess record (configs[4]) through the same RCCL gather from device memory
    ceng = az.ChessEngine(mcts_iterations=8, slots=4, evaluator=az.EVAL_SYNTHETIC, max_plies=8)
    cg = D.selfplay_sharded(D.engine_runner(ceng), 6, 5)
    ceng.close()
    np.savez(os.path.join(outdir, "rccl_chess.npz"), **cg)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_rccl_weight_broadcast_and_game_gather_on_device(tmp_path):
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path)), nprocs=1, start_method="spawn")
    got = dict(np.load(tmp_path / "rccl.npz"))
    _paths()
    from custom_alphazero import distributed as D
    from custom_alphazero import engine as az
    spec, host = _spec_and_host()
    eng = az.Engine(H, W, N, True, S, slots=8, evaluator=az.EVAL_NETWORK, compact=True)
    eng.set_weights([(n, host[n]) for n, _ in spec])
    eng.selfplay_run(0, N_GAMES, BASE_SEED)
    ref = D._pack(eng.selfplay_results())
    eng.close()
    assert len(got["lengths"]) == N_GAMES
    for k in ("lengths", "results", "expansions", "boards", "moves"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(got["policies"].view(np.uint64), ref["policies"].view(np.uint64))
    cgot = dict(np.load(tmp_path / "rccl_chess.npz"))
    ceng = az.ChessEngine(mcts_iterations=8, slots=4, evaluator=az.EVAL_SYNTHETIC, max_plies=8)
    cref = D.pack_chess(D.engine_runner(ceng)(0, 6, 5))
    ceng.close()
    assert len(cgot["lengths"]) == 6
    for k, v in cref.items():
        np.testing.assert_array_equal(cgot[k].view(np.uint8), v.view(np.uint8), err_msg=k)
