"""MI355X-native drop-in for custom_alphazero's self-play path.

Same import paths as the reference (custom_alphazero.mcts.mcts.MCTS,
custom_alphazero.self_play.play_game, custom_alphazero.model.tensorflow.model.
PolicyValueModel, custom_alphazero.connect_n.board.Board, custom_alphazero.config);
the search and the network run in libaz (HIP, gfx950) through ctypes.
"""
__all__ = ["config", "engine"]
