"""Configuration, same class-constant layout as the reference
(custom_alphazero/config.py:7-125); only the fields the self-play path reads
are honoured, plus engine sizing knobs marked as additions."""


class ConfigGeneral:
    game = "connect_n"
    self_play_gpu_index = "0"   # the reference runs self-play on CPU ("-1")
    serving_gpu_index = "-1"
    training_gpu_index = "0"
    concurrency = False
    mono_process = False
    http_inference = False


class ConfigSelfPlay:
    discounting_factor = 1
    samples_checkpoint_frequency = 1
    mcts_iterations = 250
    exclude_null_games = True
    # additions: the batched engine replaces joblib's one-game-per-process fan-out
    games_per_call = 4096        # games per play() call (reference: cpu_count()-1)
    concurrent_games = 4096      # device slots (trees in flight)
    base_seed = None             # None -> time-based like self_play.py:45
    cache_log2 = 26              # device plays_inferences entries (2^k, LRU; 2^26 = 4.6 GB for C4); 0 = no cache
    lanes = 0                    # slot groups on separate HIP streams (0 = auto)
    chess_concurrent_games = 256 # chess device slots (BASELINE configs[4]: 2048 games / 8 GPUs)
    chess_max_plies = 512        # chess games stop (as draws) here; the reference has no cap
    chess_cache_log2 = 0         # chess plays_inferences entries (2^k, ~1.1 KB each; 0 = off: slower in
                                 # the opening at 0.18 hits, profiles/r6/ab_chess_r5.txt)


class ConfigChess:
    piece_symbols = [None, "p", "n", "b", "r", "q", "k"]
    initial_board_fen = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR"
    initial_turn = "w"
    initial_castling_rights = "KQkq"
    initial_ep_quare = "-"
    initial_halfmove_clock = "0"
    initial_fullmove_number = "1"
    board_size = 8
    number_unique_pieces = 12
    # addition: HIP device the chess board kernels run on (include/az_chess.h)
    device = 0


class ConfigConnectN:
    board_width = 7
    board_height = 6
    n = 4
    gravity = True
    black = -1
    empty = 0
    white = 1
    pieces = {-1: "O", 0: ".", 1: "X"}
    directions = [(0, 1), (1, 1), (1, 0), (1, -1)]


class ConfigMCTS:
    exploration_constant = 1.5
    enable_dirichlet_noise = False  # the reference disables it too (config.py:52)
    dirichlet_noise_value = 0.03
    dirichlet_noise_ratio = 0.25
    index_move_greedy = 8
    use_solver = False


class ConfigModel:
    training_epochs = 1
    batch_size = 256
    l2_penalization_term = 1e-4
    depth = 4
    maximum_learning_rate = 1e-2
    minimum_learning_rate = 1e-4
    momentum = 0.9
    filters = 128
    # additions: Keras defaults the reference relies on implicitly
    value_hidden = 256            # ValueHead hidden_dim (model/tensorflow/model.py:110)
    bn_epsilon = 1e-3             # tf.keras BatchNormalization default
    forward_batch = 1024          # az_forward chunk (device buffer rows)


class ConfigServing:
    evaluation_games_number = 150   # config.py:89
    replace_min_score = 0.55        # config.py:90
    evaluate_with_mcts = False      # config.py:92


class ConfigPath:
    results_dir = "results"
    self_play_dir = "self_play"
    training_dir = "training"
    evaluation_dir = "evaluation"
    samples_file = "samples.npz"
    model_prefix = "model"
    model_meta = "meta.json"
    model_success = "MODEL_SAVED_SUCCESSFULLY"


def check_mcts_config(path: str = "tree"):
    """Refuse MCTS settings an engine path does not implement instead of
    silently ignoring them.  Dirichlet root noise (mcts.py:70-85, used by
    select at :113-116; disabled in the reference, config.py:52) runs in
    Connect-N self-play (path "selfplay": self_play.play / play_game, whose
    games own their np.random streams on the device, MT19937 seeded like
    self_play.py:45) and in the Connect-N tree API and arena (path "tree":
    the caller's np.random.dirichlet draws, az_tree_search_noise).  Chess
    (path "chess") has no root noise: the reference's chess MCTS cannot run
    (chess/board.py:178 vs mcts.py:179), so there is no behaviour to match."""
    if ConfigMCTS.enable_dirichlet_noise and path == "chess":
        raise NotImplementedError(
            "ConfigMCTS.enable_dirichlet_noise=True is not implemented for chess on the MI355X engine "
            "(Connect-N self-play, MCTS and the arena draw it)")
