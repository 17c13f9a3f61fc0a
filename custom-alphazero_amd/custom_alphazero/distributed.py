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
    shipped compact -- Connect-N: canonical int8 boards, float64 policies,
    int16 moves, one result per game; chess (BASELINE configs[4]): the 80-byte
    positions, u16 moves and the sparse root policies (pack_chess) -- and
    expanded to full_state only on rank 0: the analogue of joblib's result
    return (self_play.py:112-118).
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
    """Per-rank Connect-N engine results -> compact flat arrays."""
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


POS_BYTES = 80  # sizeof(az_chess_pos), include/az_chess.h


def pack_chess(results: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Per-rank chess engine results (ChessEngine.selfplay_results or
    selfplay_drain: dense [game][max_plies] rows) -> the compact chess record:
    per game its id, length, result, termination and expansions; per sample
    (ply) the canonical root position's 80 bytes (az_chess_pos), the move
    played and the root's edge count; per root edge its action index and
    visit probability (the sparse MCTS.play policy, mcts.py:182-222) -- only
    the plies each game played and the edges each root had."""
    lengths = np.asarray(results["lengths"], np.int64)
    n = len(lengths)
    ids = np.asarray(results["game_ids"], np.int64) if "game_ids" in results else np.full(n, -1, np.int64)
    pos = np.ascontiguousarray(results["positions"])
    rows = [(g, int(lengths[g])) for g in range(n)]
    positions = np.concatenate([pos[g, :T].view(np.uint8).reshape(T, POS_BYTES) for g, T in rows]) \
        if n else np.zeros((0, POS_BYTES), np.uint8)
    moves = np.concatenate([results["moves"][g, :T] for g, T in rows]).astype(np.uint16) \
        if n else np.zeros(0, np.uint16)
    pn = np.concatenate([results["policy_n"][g, :T] for g, T in rows]).astype(np.int64) \
        if n else np.zeros(0, np.int64)
    M = results["policy_actions"].shape[-1] if n else 1
    if n:
        pa = np.concatenate([results["policy_actions"][g, :T] for g, T in rows])
        pp = np.concatenate([results["policy_probs"][g, :T] for g, T in rows])
        keep = np.arange(M)[None, :] < pn[:, None]
        actions, probs = pa[keep].astype(np.int16), pp[keep].astype(np.float64)
    else:
        actions, probs = np.zeros(0, np.int16), np.zeros(0, np.float64)
    return dict(game_ids=ids, lengths=lengths, results=np.asarray(results["results"]).astype(np.int8),
                terminations=np.asarray(results["terminations"]).astype(np.int8),
                expansions=np.asarray(results["expansions"]).astype(np.int64), positions=positions,
                moves=moves, policy_n=pn.astype(np.int16), policy_actions=actions, policy_probs=probs)


# wire layouts: (field, dtype, leading axis: "games" | "samples" | "entries", trailing shape)
_WIRE = {
    "connect_n": [("lengths", np.int64, "games", ()), ("results", np.int8, "games", ()),
                  ("expansions", np.int64, "games", ()), ("boards", np.int8, "samples", None),
                  ("policies", np.float64, "samples", None), ("moves", np.int16, "samples", ())],
    "chess": [("game_ids", np.int64, "games", ()), ("lengths", np.int64, "games", ()),
              ("results", np.int8, "games", ()), ("terminations", np.int8, "games", ()),
              ("expansions", np.int64, "games", ()), ("positions", np.uint8, "samples", (POS_BYTES,)),
              ("moves", np.uint16, "samples", ()), ("policy_n", np.int16, "samples", ()),
              ("policy_actions", np.int16, "entries", ()), ("policy_probs", np.float64, "entries", ())],
}


def gather_games(results: Dict[str, np.ndarray], device=None, dst: int = 0, stats=None):
    """Gather every rank's compact games to `dst` only: the per-rank sizes by
    one `gather` of four int64s (bytes, games, samples, policy entries), then
    each other rank `send`s its byte blob (exact length, no padding) and `dst`
    `recv`s them in rank order -- under nccl both are RCCL point-to-point
    transfers between the ranks' GPUs over xGMI; no rank but `dst` receives or
    holds another rank's games.  Connect-N records (engine results: boards,
    policies, moves) or chess records (ChessEngine results: positions,
    sparse policies; pack_chess) -- every rank passes the same kind.  Returns
    the concatenated dict on `dst`, None elsewhere; `stats` (a dict) gets
    `wire_bytes`, the bytes `dst` received from the other ranks."""
    import torch
    import torch.distributed as dist

    kind = "chess" if "positions" in results else "connect_n"
    packed = pack_chess(results) if kind == "chess" else _pack(results)
    spec = _WIRE[kind]
    blob = b"".join(np.ascontiguousarray(packed[k]).tobytes() for k, _, _, _ in spec)
    n_entries = len(packed["policy_actions"]) if kind == "chess" else 0
    world, rank = dist.get_world_size(), dist.get_rank()
    device = collective_device(device)
    sizes = torch.tensor([len(blob), len(packed["lengths"]), len(packed["moves"]), n_entries], dtype=torch.int64,
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
    trailing = {"boards": packed["boards"].shape[1:], "policies": packed["policies"].shape[1:]} \
        if kind == "connect_n" else {}
    parts: List[Dict[str, np.ndarray]] = []
    for r in range(world):
        raw = blob if r == dst else (bufs[r].cpu().numpy().tobytes() if bufs[r] is not None else b"")
        count = {"games": all_sizes[r][1], "samples": all_sizes[r][2], "entries": all_sizes[r][3]}
        off, part = 0, {}
        for k, dt, axis, tail in spec:
            shape = (count[axis],) + tuple(trailing[k] if tail is None else tail)
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
    """Adapter: a custom_alphazero.engine.Engine (or ChessEngine) as a
    selfplay_sharded runner (chess results carry their game ids)."""
    def run(first, count, base_seed):
        engine.selfplay_run(first, count, base_seed)
        res = engine.selfplay_results()
        if "positions" in res:
            res["game_ids"] = first + np.arange(count, dtype=np.int64)
        return res
    return run
