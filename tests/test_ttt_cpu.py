"""CPU checks of the TicTacToe host entry points: the parameter count and the
tch-default init match the oracle's (model/tictactoe.rs construction order)."""
import numpy as np


def test_ttt_params_match_oracle(oracle):
    import spai_ttt
    for blocks in (0, 2, 4):
        assert spai_ttt.num_params(blocks) == oracle.num_params(oracle.GAME_TICTACTOE, blocks, 64)
        assert np.array_equal(spai_ttt.init_params(blocks, 5), oracle.init_params(oracle.GAME_TICTACTOE, blocks, 64, 5))
