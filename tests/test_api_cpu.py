"""Host-side drop-in API (connect_n Board/Move, normalize_probabilities)
against the reference's own outputs (golden vectors)."""
import os
import sys

import numpy as np
import pytest

from custom_alphazero.config import ConfigConnectN
from custom_alphazero.connect_n.board import Board
from custom_alphazero.connect_n.move import Move
from custom_alphazero.mcts.utils import normalize_probabilities

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "custom-alphazero_amd")


@pytest.fixture
def game_cfg():
    saved = (ConfigConnectN.board_height, ConfigConnectN.board_width, ConfigConnectN.n,
             ConfigConnectN.gravity)

    def set_(h, w, n, g):
        ConfigConnectN.board_height, ConfigConnectN.board_width = h, w
        ConfigConnectN.n, ConfigConnectN.gravity = n, g

    yield set_
    set_(*saved)


@pytest.mark.parametrize("name", ["c4", "c5_9x9", "nograv_5x5"])
def test_board_api_matches_reference(golden, game_cfg, name):
    z = golden("board_" + name)
    H, W, n, grav = int(z["height"]), int(z["width"]), int(z["n"]), bool(z["gravity"])
    game_cfg(H, W, n, grav)
    all_moves = Board.get_all_possible_moves()
    assert len(all_moves) == (W if grav else W * H)
    games = z["game"]
    idx = 0
    for g in np.unique(games)[:40]:
        sel = np.flatnonzero(games == g)
        board = Board()
        for i in sel:
            board.play(all_moves[int(z["move"][i])], keep_same_player=True)
            np.testing.assert_array_equal(board.array, z["array"][i])
            assert board.is_game_over() == bool(z["game_over"][i])
            res = board.get_result(keep_same_player=True)
            assert (-9 if res is None else res) == z["result"][i]
            np.testing.assert_array_equal(board.legal_moves_mask(all_moves), z["mask"][i])
            order = [all_moves.index(m) for m in board.moves]
            k = int(z["n_moves"][i])
            assert order == z["moves_order"][i][:k].tolist()
            assert board.fullmove_number == z["fullmove"][i]
            fs = board.full_state
            assert fs.dtype == np.float32 and fs.shape == (H, W, 4)
            idx += 1
    assert idx > 100


def test_board_play_on_copy_and_repr(game_cfg):
    game_cfg(6, 7, 4, True)
    b = Board()
    c = b.play(Move(True, 3), on_copy=True, keep_same_player=True)
    assert b.fullmove_number == 0 and c.fullmove_number == 1
    assert repr(c).splitlines()[-1] == "...O..." and b != c
    assert c.turn == 1 and c.played_moves == [Move(True, 3)]
    assert Board.from_one_hot(c.array_one_hot)[5, 3] == -1


def test_normalize_matches_reference(golden):
    z = golden("numerics")
    for vin, vout, n, is64 in zip(z["norm_in"], z["norm_out"], z["norm_len"], z["norm_out_is64"]):
        r = normalize_probabilities(vin[:n])
        assert (r.dtype == np.float64) == bool(is64)
        np.testing.assert_array_equal(np.asarray(r, np.float64).view(np.uint64),
                                      vout[:n].view(np.uint64))


def test_queue_payload_matches_append_queue_schema(tmp_path):
    """append_queue's JSON body (serving/factory.py:69-80): nested lists with
    ModelAppendQueueInputs' shapes; round-trips to the same arrays."""
    import json

    from custom_alphazero import self_play
    rng = np.random.RandomState(0)
    states = rng.rand(3, 6, 7, 4).astype(np.float32)
    policies = rng.rand(3, 7)
    values = np.array([1, -1, 1])
    body = self_play.queue_payload(states, policies, values)
    assert set(body) == {"states", "policies", "values"}
    assert len(body["states"]) == 3 and len(body["states"][0]) == 6 and len(body["states"][0][0][0]) == 4
    path = self_play.write_queue_payload(str(tmp_path / "q.json"), states, policies, values)
    back = json.load(open(path))
    np.testing.assert_array_equal(np.asarray(back["states"], np.float32), states)
    np.testing.assert_array_equal(np.asarray(back["policies"]), policies)
    np.testing.assert_array_equal(np.asarray(back["values"]), values)


def test_reference_weight_hash_matches_legacy_numpy(golden_dir):
    """PolicyValueModel.hash is the reference's sum of md5(str(weight)) over
    Keras get_weights() (model/tensorflow/model.py:172-177); the digests were
    taken under numpy 1.26 (tests/golden/make_weight_hash.py)."""
    import json
    import os

    from custom_alphazero.model.weights import (content_hash, init_weights, keras_order, reference_hash,
                                                weight_spec)
    cases = json.load(open(os.path.join(golden_dir, "weight_hash.json")))
    for case in cases.values():
        H, W, A, C = case["shape"]
        spec = weight_spec(H, W, A, in_channels=C)
        w = init_weights(spec, seed=case["seed"], randomize_bn=case["randomize_bn"])
        names = keras_order(spec)
        assert names == case["names"]
        assert str(reference_hash([w[n] for n in names])) == case["hash"]
    # the reference hash sees only the corners of arrays over 1000 elements
    k = w["block0.conv1.kernel"].copy()
    k[1, 1, 64, 64] += 1.0
    w2 = dict(w, **{"block0.conv1.kernel": k})
    assert reference_hash([w2[n] for n in names]) == reference_hash([w[n] for n in names])
    assert content_hash([w2[n] for n in names]) != content_hash([w[n] for n in names])


def test_dirichlet_noise_paths():
    """Root Dirichlet noise (mcts.py:70-85) runs in Connect-N self-play, the
    MCTS tree API and the arena; chess refuses it rather than ignore it."""
    from custom_alphazero.config import ConfigMCTS, check_mcts_config
    check_mcts_config()
    ConfigMCTS.enable_dirichlet_noise = True
    try:
        for path in ("selfplay", "tree"):
            check_mcts_config(path)
        with pytest.raises(NotImplementedError):
            check_mcts_config("chess")
    finally:
        ConfigMCTS.enable_dirichlet_noise = False


def test_root_noise_rows_are_numpys_dirichlet_draws():
    """The tree API's host-drawn root noise: rng.dirichlet(0.03 * ones(k)) per
    row, in order, padded to the action space (mcts.py:74-78)."""
    from custom_alphazero.mcts.mcts import root_noise_rows
    rows = root_noise_rows(np.random.RandomState(3), 5, 4, 7)
    rs = np.random.RandomState(3)
    for r in range(4):
        np.testing.assert_array_equal(rows[r, :5], rs.dirichlet(np.ones(5) * 0.03))
    assert not rows[:, 5:].any()
    assert root_noise_rows(np.random.RandomState(3), 5, 0, 7).shape == (1, 7)


@pytest.mark.parametrize("env,want", [({}, "8"), ({"GPU_MAX_HW_QUEUES": "4"}, "8"),
                                      ({"GPU_MAX_HW_QUEUES": "12"}, "12"),
                                      ({"GPU_MAX_HW_QUEUES": "4", "AZ_KEEP_HW_QUEUES": "1"}, "4")])
def test_package_import_sets_the_benched_hw_queues(env, want):
    """Importing the package before HIP initialises gives the process the 8
    hardware queues bench.py runs with (the engine's auto rule then picks 3
    lanes at 1536-4096 slots, as in the bench line), unless the caller set
    more or asked to keep its value."""
    import subprocess
    e = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "AZ_KEEP_HW_QUEUES")}
    e.update(env)
    code = ("import os, sys; sys.path.insert(0, %r); import custom_alphazero; "
            "print(os.environ['GPU_MAX_HW_QUEUES'])" % PKG)
    out = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == want
