"""The drop-in Python API on the GPU: MCTS / play_game / play / PolicyValueModel
against the reference's golden vectors (synthetic evaluator) and the float64
Keras restatement (network)."""
import numpy as np
import pytest

import keras_ref
import oracle
from custom_alphazero import self_play
from custom_alphazero.config import ConfigConnectN, ConfigSelfPlay
from custom_alphazero.connect_n.board import Board
from custom_alphazero.mcts.mcts import MCTS, SyntheticEvaluator
from custom_alphazero.model.tensorflow.model import PolicyValueModel

pytestmark = pytest.mark.gpu


@pytest.fixture
def game_cfg():
    saved = (ConfigConnectN.board_height, ConfigConnectN.board_width, ConfigConnectN.n,
             ConfigConnectN.gravity, ConfigSelfPlay.mcts_iterations)

    def set_(z):
        ConfigConnectN.board_height, ConfigConnectN.board_width = int(z["height"]), int(z["width"])
        ConfigConnectN.n, ConfigConnectN.gravity = int(z["n"]), bool(z["gravity"])
        ConfigSelfPlay.mcts_iterations = int(z["sims"])

    yield set_
    (ConfigConnectN.board_height, ConfigConnectN.board_width, ConfigConnectN.n,
     ConfigConnectN.gravity, ConfigSelfPlay.mcts_iterations) = saved


@pytest.mark.parametrize("name", ["c4_s25", "c5_9x9_s50", "nograv_5x5_s25"])
def test_play_game_api_matches_reference(golden, game_cfg, monkeypatch, name):
    """self_play.play_game with the reference's own seeding (time patched)."""
    z = golden("mcts_" + name)
    game_cfg(z)
    all_moves = Board.get_all_possible_moves()
    off = 0
    for g, seed in enumerate(z["seed"][:2]):
        monkeypatch.setattr(self_play.time, "time", lambda s=seed: float(s))
        states, policies, rewards, mcts = self_play.play_game(
            0, all_moves, int(z["sims"]), "test-run", {}, model=SyntheticEvaluator())
        T = int(z["game_len"][g])
        sl = slice(off, off + T)
        np.testing.assert_array_equal(states, z["state"][sl])
        np.testing.assert_array_equal(policies.view(np.uint64), z["policy"][sl].view(np.uint64))
        np.testing.assert_array_equal(rewards, z["reward"][sl])
        # tree views: the played path carries the reference's edge statistics
        node = mcts.root
        for ply in range(T):
            played = [e for e in node.edges if e.played]
            assert len(played) == 1
            gi = off + ply
            k = int(z["n_edges"][gi])
            assert [e.visit_count for e in node.edges] == z["edge_n"][gi, :k].tolist()
            np.testing.assert_array_equal(np.array([e.total_action_value for e in node.edges]),
                                          z["edge_w"][gi, :k])
            assert played[0].greedily_played == bool(z["greedy"][gi])
            node = played[0].child
        off += T
        monkeypatch.undo()


@pytest.fixture
def noise_on():
    from custom_alphazero.config import ConfigMCTS
    ConfigMCTS.enable_dirichlet_noise = True
    yield
    ConfigMCTS.enable_dirichlet_noise = False


@pytest.mark.parametrize("name", ["c4_s25_noise", "nograv_5x5_s25_noise"])
def test_play_game_with_root_noise_matches_reference(golden, game_cfg, monkeypatch, noise_on, name):
    """self_play.play_game with ConfigMCTS.enable_dirichlet_noise: the game
    runs on the device with its np.random stream (MT19937(seed) past the
    model construction's draws) -- the reference's noisy play_game, bitwise."""
    z = golden("mcts_" + name)
    game_cfg(z)
    off = 0
    for g, seed in enumerate(z["seed"][:2]):
        monkeypatch.setattr(self_play.time, "time", lambda s=seed: float(s))
        states, policies, rewards, _ = self_play.play_game(0, Board.get_all_possible_moves(), int(z["sims"]),
                                                           "test-run", {}, model=SyntheticEvaluator())
        T = int(z["game_len"][g])
        np.testing.assert_array_equal(states, z["state"][off:off + T])
        np.testing.assert_array_equal(policies.view(np.uint64), z["policy"][off:off + T].view(np.uint64))
        np.testing.assert_array_equal(rewards, z["reward"][off:off + T])
        off += T
        monkeypatch.undo()


@pytest.mark.parametrize("name", ["c4_s25_noise", "c5_9x9_s50_noise", "nograv_5x5_s25_noise"])
def test_mcts_with_root_noise_matches_reference(golden, game_cfg, noise_on, name):
    """The single-tree MCTS API with ConfigMCTS.enable_dirichlet_noise: each
    search draws its root-noise vectors from numpy's global stream
    (mcts.root_noise_rows, az_tree_search_noise), then play() its one
    random_sample -- the reference's stream order, so a seeded game is the
    reference's noisy game bit for bit (root edge statistics every ply)."""
    z = golden("mcts_" + name)
    game_cfg(z)
    S = int(z["sims"])
    all_moves = Board.get_all_possible_moves()
    off = 0
    for g, seed in enumerate(z["seed"][:2]):
        np.random.seed(int(seed))
        np.random.rand(1, int(z["height"]), int(z["width"]), 4)  # play_game's model construction
        m = MCTS(Board(), all_moves, False, {}, model=SyntheticEvaluator())
        T = int(z["game_len"][g])
        for ply in range(T):
            m.search(S)
            gi = off + ply
            k = int(z["n_edges"][gi])
            edges = m.current_root.edges
            assert [e.visit_count for e in edges] == z["edge_n"][gi, :k].tolist(), (g, ply)
            np.testing.assert_array_equal(np.array([e.total_action_value for e in edges]), z["edge_w"][gi, :k])
            _, _, policy, move = m.play(m.board.fullmove_number >= 8, return_details=True)
            np.testing.assert_array_equal(policy.view(np.uint64), z["policy"][gi].view(np.uint64))
            assert all_moves.index(move) == z["moves"][gi]
        assert m.board.is_game_over()
        off += T


def test_batched_play_matches_reference(golden, game_cfg):
    z = golden("mcts_c4_s25")
    game_cfg(z)
    states, policies, rewards, records = self_play.play(
        "test-run", {}, model=SyntheticEvaluator(), n_games=16, base_seed=0)
    np.testing.assert_array_equal(states, z["state"])
    np.testing.assert_array_equal(policies.view(np.uint64), z["policy"].view(np.uint64))
    np.testing.assert_array_equal(rewards, z["reward"])
    assert [r.length for r in records] == z["game_len"].tolist()
    assert [r.expansions for r in records] == z["expansions"].tolist()


def test_batched_play_cache_follows_plays_inferences(golden, game_cfg):
    """The device cache is the caller's plays_inferences: kept across calls
    with the same dict (hits on the second call), emptied for a new dict;
    results identical either way (self_play.py:145-146, mcts.py:122-143)."""
    z = golden("mcts_c4_s25")
    game_cfg(z)
    shared = {}
    hits = []  # per call (az_selfplay_begin resets the counters)
    outs = []
    for d in (shared, shared, {}):
        outs.append(self_play.play("test-run", d, model=SyntheticEvaluator(), n_games=16, base_seed=0))
        hits.append(next(iter(self_play._ENGINES.values())).stats()["cache_hits"])
    for out in outs[1:]:
        np.testing.assert_array_equal(out[0], outs[0][0])
        np.testing.assert_array_equal(out[1].view(np.uint64), outs[0][1].view(np.uint64))
    # same dict: the replayed games find their boards already cached; a fresh
    # dict starts empty again
    assert hits[1] > hits[0] and hits[2] == hits[0]


def test_mcts_deterministic_play_is_argmax(game_cfg, golden):
    game_cfg(golden("mcts_c4_s25"))
    m = MCTS(Board(), Board.get_all_possible_moves(), False, {}, model=SyntheticEvaluator())
    m.search(30)
    visits = [e.visit_count for e in m.current_root.edges]
    state = np.random.get_state()
    b = m.play(deterministic=True)
    assert b.played_moves[-1].x == int(np.argmax(visits))
    assert np.random.get_state()[2] == state[2]  # no RNG draw when deterministic


def test_policy_value_model_matches_keras(game_cfg, golden):
    game_cfg(golden("mcts_c4_s25"))
    model = PolicyValueModel(input_dim=(6, 7, 4), action_space=7, seed=3)
    rng = np.random.RandomState(0)
    x = oracle.full_state(rng.randint(-1, 2, (9, 6, 7)).astype(np.int8))
    probs, value = model(x)
    p, v = probs.numpy(), value.numpy()
    assert p.shape == (9, 7) and v.shape == (9, 1)
    w = dict(zip(model.weight_names, model.get_weights()))
    rp, rv = keras_ref.forward(w, x, depth=4)
    assert np.abs(p - rp).max() < 1e-5 and np.abs(v[:, 0] - rv).max() < 1e-5
    # the reference's batch-1 idiom (mcts.py:131-137)
    pp, vv = model(np.expand_dims(x[0], 0))
    assert pp.numpy().ravel().shape == (7,) and isinstance(vv.numpy().item(), float)


def test_model_save_load_roundtrip(tmp_path, game_cfg, golden):
    game_cfg(golden("mcts_c4_s25"))
    a = PolicyValueModel((6, 7, 4), 7, seed=1)
    a.steps = 12
    a.save_with_meta(str(tmp_path))
    # the reference's files: Model.save_weights(path/model) -> a TF checkpoint
    # (model.py:203-204), read back here without TensorFlow
    for f in ("model.index", "model.data-00000-of-00001", "checkpoint", "meta.json",
              "MODEL_SAVED_SUCCESSFULLY"):
        assert (tmp_path / f).exists(), f
    b = PolicyValueModel((6, 7, 4), 7, seed=2)
    assert not a.is_equal(b)
    b.load_with_meta(str(tmp_path))
    assert a.is_equal(b) and b.steps == 12
    x = np.zeros((1, 6, 7, 4), np.float32)
    x[..., 0] = 1
    x[..., 3] = 1
    np.testing.assert_array_equal(a(x)[0].numpy(), b(x)[0].numpy())


def test_mcts_with_network_model_plays_legal_game(game_cfg, golden):
    game_cfg(golden("mcts_c4_s25"))
    model = PolicyValueModel((6, 7, 4), 7, seed=0)
    np.random.seed(4)
    states, policies, rewards, mcts = self_play.play_game(0, Board.get_all_possible_moves(), 20,
                                                          "test-run", {}, model=model)
    assert len(states) == len(policies) == len(rewards) >= 7
    np.testing.assert_allclose(policies.sum(axis=1), 1.0)
    assert abs(int(rewards[-1])) in (0, 1)


def test_self_play_run_loop(tmp_path, golden, game_cfg, monkeypatch):
    """self_play.run = the reference __main__ loop: samples.npz checkpoints,
    draws dropped, the queue payload handed to the sink, plays_inferences kept
    while the best model's hash is unchanged."""
    from custom_alphazero.config import ConfigPath
    z = golden("mcts_c4_s25")
    game_cfg(z)
    monkeypatch.setattr(ConfigPath, "results_dir", str(tmp_path))
    monkeypatch.setattr(ConfigSelfPlay, "games_per_call", 16)
    monkeypatch.setattr(ConfigSelfPlay, "base_seed", 0)
    sink = []
    counts = self_play.run("run-x", iterations=2, queue_sink=sink.append,
                           model_loader=lambda run_id: SyntheticEvaluator())
    keep = z["reward"] != 0
    assert counts == [int(keep.sum())] * 2
    assert len(sink) == 2
    np.testing.assert_array_equal(np.asarray(sink[0]["states"], np.float32), z["state"][keep])
    saved = np.load(tmp_path / "connect_n" / "run-x" / ConfigPath.self_play_dir / "iteration_1" /
                    ConfigPath.samples_file)
    np.testing.assert_array_equal(saved["values"], z["reward"][keep])


def test_tree_views_serve_the_reference_visualizer(game_cfg, golden):
    """The device tree's UCTNode/UCTEdge views carry every attribute the
    reference's MctsVisualizer reads or writes (visualize_mcts.py:40-125:
    node.edges/board.repr_graphviz()/evaluated_value, edge.parent/child/
    prior/visit_count/action/played/greedily_played, edge.proportion_n set
    per parent), and the played root edge is the one play() chose."""
    game_cfg(golden("mcts_c4_s25"))
    m = MCTS(Board(), Board.get_all_possible_moves(), False, {}, model=SyntheticEvaluator())
    m.search(25)
    m.play(greedy=True)
    frontier, seen = [m.root], 0
    while frontier:
        node = frontier.pop()
        assert isinstance(node.board.repr_graphviz(), str)
        assert node.evaluated_value is None or isinstance(node.evaluated_value, float)
        visits = sum(e.visit_count for e in node.edges)
        for e in node.edges:
            assert e.parent is node and isinstance(e.prior, float) and e.action is not None
            assert isinstance(e.played, bool) and isinstance(e.greedily_played, bool)
            e.proportion_n = e.visit_count / visits if visits else 0.0
            seen += 1
            if e.visit_count > 0 and e.child is not None:
                frontier.append(e.child)
    assert seen > len(m.root.edges) and sum(e.visit_count for e in m.root.edges) == 24
    played = [e for e in m.root.edges if e.played]
    assert len(played) == 1 and played[0].greedily_played
    assert played[0].visit_count == max(e.visit_count for e in m.root.edges)


def test_load_with_meta_accepts_reference_hash(tmp_path, game_cfg, golden):
    """A meta.json whose hash the reference computed (sum of md5(str(w)),
    model.py:172-177, digests taken under legacy numpy) validates; a wrong
    hash is refused like the reference's assertion (model.py:199-201)."""
    import json
    import os

    from custom_alphazero.config import ConfigPath
    from custom_alphazero.model.weights import init_weights, weight_spec
    game_cfg(golden("mcts_c4_s25"))
    case = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "weight_hash.json")))["c4_seed0"]
    w = init_weights(weight_spec(6, 7, 7), seed=0)
    np.savez(tmp_path / (ConfigPath.model_prefix + ".npz"), **w)
    (tmp_path / ConfigPath.model_meta).write_text(json.dumps({"steps": 3, "learning_rate": 0.01,
                                                             "hash": int(case["hash"])}))
    (tmp_path / ConfigPath.model_success).write_bytes(b"")
    m = PolicyValueModel((6, 7, 4), 7, seed=5)
    m.load_with_meta(str(tmp_path))
    assert m.hash == int(case["hash"]) and m.steps == 3
    (tmp_path / ConfigPath.model_meta).write_text(json.dumps({"steps": 3, "hash": int(case["hash"]) + 1}))
    with pytest.raises(AssertionError):
        m.load_with_meta(str(tmp_path))
    # a checkpoint an earlier build of this package wrote (raw-bytes md5 as
    # `hash`), and this build's own meta.json (both hashes) also load
    (tmp_path / ConfigPath.model_meta).write_text(json.dumps({"steps": 4, "hash": m.content_hash}))
    m.load_with_meta(str(tmp_path))
    assert m.steps == 4
    m.save_with_meta(str(tmp_path))
    meta = json.loads((tmp_path / ConfigPath.model_meta).read_text())
    assert meta["hash"] == int(case["hash"]) and meta["content_hash"] == m.content_hash
    m.load_with_meta(str(tmp_path))


def test_play_engine_runs_the_benched_lanes():
    """The drop-in play()'s engine at configs[1]'s 4096 slots runs the lane
    count bench.py reports: the package import gave the process the 8 HIP
    hardware queues bench.py asks for, so the auto rule picks 3 lanes
    (VERDICT r5 item 6)."""
    import os
    assert int(os.environ["GPU_MAX_HW_QUEUES"]) >= 8
    eng = self_play._batched_engine(SyntheticEvaluator(), 4096, sims=4)
    assert eng.lanes == 3
