"""The oracle's self-play sampler (or_self_play: Philox uniform, WeightedIndex
over visits^T) in distribution: >= 10^5 draws (6400 games, hash evaluator) fit
P(child) = N^T / sum N^T at T = 1.25 and reject T = 1 and T = 1.5
(tests/sampling_stats.py; the device move step is held to the same test in
test_gpu_parity.py::test_self_play_sampling_frequencies and to the oracle bit
for bit in test_self_play_device_sampling_matches_oracle)."""
import numpy as np

from sampling_stats import rank_chi2


def test_oracle_sampler_distribution(oracle):
    r = oracle.self_play(oracle.GAME_CONNECT4, 6400, 32, 17, eval_kind=oracle.EVAL_HASH, max_plies=42,
                         temperature=1.25)
    mv = r["moves"][r["game"], r["ply"]]
    assert len(mv) >= 100_000, len(mv)
    c, p, obs, exp = rank_chi2(r["policy"], mv, 1.25)
    assert p > 1e-4, (c, p, obs, exp)
    for t_alt in (1.0, 1.5):
        assert rank_chi2(r["policy"], mv, t_alt)[1] < 1e-12
