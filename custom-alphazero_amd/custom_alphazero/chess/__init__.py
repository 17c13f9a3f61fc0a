"""Chess board seam (reference custom_alphazero/chess/): Board, Move and
get_all_possible_moves over libaz's chess kernels (include/az_chess.h)."""
