"""CPU-only checks of the C ABI library: it loads, exports every symbol that
include/spai.h declares, host-only entry points agree with the oracle, and the
device path fails loudly (no CPU fallback) when no GPU is present."""
import os
import re

import numpy as np
import pytest

from conftest import REPO


@pytest.fixture(scope="module")
def spai():
    import spai as s
    s.lib()
    return s


def test_header_symbols_exported(spai):
    with open(os.path.join(REPO, "include", "spai.h")) as f:
        hdr = f.read()
    declared = set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(spai_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    assert declared == set(spai.SYMBOLS), declared ^ set(spai.SYMBOLS)
    lib = spai.lib()
    for s in declared:
        assert hasattr(lib, s), s


def test_version_and_config(spai):
    import ctypes as C
    assert spai.lib().spai_version().startswith(b"spai")
    cfg = spai.Config()
    assert spai.lib().spai_config_default(spai.GAME_CONNECT4, C.byref(cfg)) == 0
    assert (cfg.c, cfg.num_searches, cfg.temperature, cfg.max_trees) == (2.0, 600, 1.25, 100)  # mcts.rs:46-59
    assert spai.lib().spai_config_default(spai.GAME_CHESS, C.byref(cfg)) == -7


@pytest.mark.parametrize("blocks", [0, 2, 6])
def test_param_count_and_init_match_oracle(spai, oracle, blocks):
    assert spai.num_params(blocks) == oracle.num_params(oracle.GAME_CONNECT4, blocks, 64)
    np.testing.assert_array_equal(spai.init_params(blocks, seed=3), oracle.init_params(oracle.GAME_CONNECT4, blocks, 64, 3))


def test_survey_param_and_flop_counts(spai):
    # 476,399 trainable params for 6x64 (+ 1,734 BN running stats)
    assert spai.num_params(6) == 476399 + 2 * (13 * 64 + 32 + 3)
    import bench
    assert bench.flops_per_eval(6) == 39_016_572
    assert bench.flops_per_eval(4) == 26_630_268


def test_no_gpu_fails_loudly(spai):
    if spai.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(spai.SpaiError) as ei:
        spai.Engine(num_searches=4, max_trees=4)
    assert ei.value.code == -4


def test_null_arguments_rejected(spai):
    import ctypes as C
    assert spai.lib().spai_engine_create(1, None, 0, None) == -1
    assert b"NULL" in spai.lib().spai_last_error()
    assert spai.lib().spai_search(None, 0, None, 0, None, None, None, None) == -1
