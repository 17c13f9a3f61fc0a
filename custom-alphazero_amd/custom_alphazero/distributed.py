"""Multi-GPU self-play: one process per GPU, games sharded by global game id.

The reference's only parallelism is one game per OS process
(self_play.py:98-110), with the model shipped by disk and results by
pickling; here each rank owns a contiguous block of global game ids and runs
them on its own device with no exchange during search.  Two collectives
remain, both over torch.distributed ("nccl" = RCCL over xGMI on MI355X,
"gloo" on CPU for tests):
  * broadcast_weights: rank 0's weights, flattened into ONE buffer (~5 MB for
    the 128x4 net), one broadcast -- the analogue of every worker loading the
    best model from disk (utils.py:64-78);
  * gather_games: each rank's finished games to rank 0 only, in global game
    order (a gather of the sizes, then point-to-point sends to rank 0),
    shipped compact (canonical int8 boards, float64 policies, int16 moves, one
    result per game) and expanded to full_state only on rank 0 -- the
    analogue of joblib's result return (self_play.py:112-118).
Because a game's trajectory depends only on its seed (base_seed + game id)
and the per-board evaluator, the gathered samples are identical for any
number of ranks (tests/test_distributed_cpu.py).
"""
from typing import Callable, Dict, List, Sequence, Tuple

import numpy as np


def collective_device(device=None):
    """Where collective buffers must live: the caller's device, else this
    rank's current GPU under nccl (RCCL moves device memory only), else the
    CPU (gloo)."""
    import torch
    import torch.distributed as dist
    if device is not None:
        return torch.device(device)
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def shard(n_games: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of global game ids owned by `rank`: (first, count)."""
    base, extra = divmod(int(n_games), int(world))
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def broadcast_weights(named: Sequence[Tuple[str, "object"]], device=None, src: int = 0):
    """Broadcast a list of (name, tensor) from `src` with a single collective.
    Returns the list of (name, tensor-view) on every rank (views into one
    flat buffer on `device`)."""
    import torch
    import torch.distributed as dist

    shapes = [(name, tuple(t.shape)) for name, t in named]
    if dist.get_rank() == src:
        flat = torch.cat([torch.as_tensor(t).reshape(-1).float() for _, t in named])
    else:
        total = sum(int(np.prod(s)) for _, s in shapes)
        flat = torch.zeros(total, dtype=torch.float32)
    flat = flat.to(collective_device(device))
    dist.broadcast(flat, src=src)
    out, off = [], 0
    for name, shape in shapes:
        k = int(np.prod(shape))
        out.append((name, flat[off:off + k].view(shape)))
        off += k
    return out


def _pack(results: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Per-rank engine results -> compact flat arrays."""
    lengths = results["lengths"].astype(np.int64)
    n = len(lengths)
    boards = np.concatenate([results["boards"][g, :lengths[g]] for g in range(n)]) \
        if n else np.zeros((0,) + results["boards"].shape[2:], np.int8)
    policies = np.concatenate([results["policies"][g, :lengths[g]] for g in range(n)]) \
        if n else np.zeros((0, results["policies"].shape[2]), np.float64)
    moves = np.concatenate([results["moves"][g, :lengths[g]] for g in range(n)]).astype(np.int16) \
        if n else np.zeros(0, np.int16)
    return dict(lengths=lengths, results=results["results"].astype(np.int8), boards=boards,
                policies=policies, moves=moves,
                expansions=results["expansions"].astype(np.int64))


def gather_games(results: Dict[str, np.ndarray], device=None, dst: int = 0, stats=None):
    """Gather every rank's compact games to `dst` only: the per-rank sizes by
    one `gather` of three int64s, then each other rank `send`s its byte blob
    (exact length, no padding) and `dst` `recv`s them in rank order -- under
    nccl both are RCCL point-to-point transfers between the ranks' GPUs over
    xGMI; no rank but `dst` receives or holds another rank's games.  Returns
    the concatenated dict on `dst`, None elsewhere; `stats` (a dict) gets
    `wire_bytes`, the bytes `dst` received from the other ranks."""
    import torch
    import torch.distributed as dist

    packed = _pack(results)
    order = ("lengths", "results", "expansions", "boards", "policies", "moves")
    blob = b"".join(np.ascontiguousarray(packed[k]).tobytes() for k in order)
    world, rank = dist.get_world_size(), dist.get_rank()
    device = collective_device(device)
    sizes = torch.tensor([len(blob), len(packed["lengths"]), len(packed["moves"])], dtype=torch.int64,
                         device=device)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)] if rank == dst else None
    dist.gather(sizes, gather_list=all_sizes, dst=dst)
    if rank != dst:
        if blob:
            dist.send(torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device), dst=dst)
        return None
    all_sizes = [[int(v) for v in t.cpu().tolist()] for t in all_sizes]
    bufs, reqs = [], []
    for r in range(world):
        if r == dst or all_sizes[r][0] == 0:
            bufs.append(None)
            continue
        bufs.append(torch.empty(all_sizes[r][0], dtype=torch.uint8, device=device))
        reqs.append(dist.irecv(bufs[r], src=r))
    for q in reqs:
        q.wait()
    if stats is not None:
        stats["wire_bytes"] = int(sum(all_sizes[r][0] for r in range(world) if r != dst))
    board_shape = packed["boards"].shape[1:]
    A = packed["policies"].shape[1]
    parts: List[Dict[str, np.ndarray]] = []
    for r in range(world):
        raw = blob if r == dst else (bufs[r].cpu().numpy().tobytes() if bufs[r] is not None else b"")
        n_games, n_samples = all_sizes[r][1], all_sizes[r][2]
        spec = [("lengths", np.int64, (n_games,)), ("results", np.int8, (n_games,)),
                ("expansions", np.int64, (n_games,)),
                ("boards", np.int8, (n_samples,) + tuple(board_shape)),
                ("policies", np.float64, (n_samples, A)), ("moves", np.int16, (n_samples,))]
        off, part = 0, {}
        for k, dt, shape in spec:
            nbytes = int(np.prod(shape)) * np.dtype(dt).itemsize
            part[k] = np.frombuffer(raw[off:off + nbytes], dtype=dt).reshape(shape)
            off += nbytes
        parts.append(part)
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def to_samples(g: Dict[str, np.ndarray]):
    """Compact games -> (states f32 [M,H,W,4], policies f64, rewards int64),
    the reference's sample layout (self_play.py:112-118)."""
    b = g["boards"]
    states = np.zeros(b.shape + (4,), np.float32)
    states[..., 0] = b == 0
    states[..., 1] = b == 1
    states[..., 2] = b == -1
    states[..., 3] = 1.0
    rewards = []
    for T, res in zip(g["lengths"], g["results"]):
        r = np.repeat(np.int64(res), int(T))
        r[-2::-2] = -r[-2::-2]
        rewards.append(r)
    rewards = np.concatenate(rewards) if rewards else np.zeros(0, np.int64)
    return states, g["policies"], rewards


def selfplay_sharded(runner: Callable[[int, int, int], Dict[str, np.ndarray]], n_games: int,
                     base_seed: int, device=None):
    """Run this rank's shard with `runner(first_game, count, base_seed)` (an
    engine's selfplay_run + selfplay_results) and gather to rank 0."""
    import torch.distributed as dist

    first, count = shard(n_games, dist.get_world_size(), dist.get_rank())  # device: collective_device
    results = runner(first, count, base_seed)
    return gather_games(results, device=device)


def engine_runner(engine):
    """Adapter: a custom_alphazero.engine.Engine as a selfplay_sharded runner."""
    def run(first, count, base_seed):
        engine.selfplay_run(first, count, base_seed)
        return engine.selfplay_results()
    return run
