"""Policy trait methods (game/mod.rs:35-44) through the C ABI (host functions of
libspai.so, no GPU needed), checked against the oracle restatement
(oracle/spai_oracle.c or_policy_best_action / or_policy_sample, or_nd_sum).

Pinning: the Rust toolchain is absent, so the reference and rand 0.8.5 cannot
run here.  get_best_action is pinned by hand-derived known answers for
f32::total_cmp (ties -> last index, -0 < +0, NaN above +inf); sample by
hand-derived boundaries of rand's WeightedIndex (first running total strictly
greater than the draw).  Everything else: library == oracle, bit for bit."""
import ctypes as C

import numpy as np
import pytest

import spai


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def test_best_action_known_answers():
    assert spai.policy_best_action([0.1, 0.5, 0.5, 0.2]) == 2          # last of equal maxima
    assert spai.policy_best_action([0.0, -0.0]) == 0                   # -0 < +0 under total_cmp
    assert spai.policy_best_action([-0.0, 0.0]) == 1
    assert spai.policy_best_action([np.nan, 1.0, np.inf]) == 0         # +NaN is the largest
    assert spai.policy_best_action([-np.nan, -np.inf, -1.0]) == 2      # -NaN is the smallest
    assert spai.policy_best_action([3.0]) == 0
    with pytest.raises(spai.SpaiError):
        spai.policy_best_action([])


def test_sample_known_answers():
    p = [0.2, 0.3, 0.5]   # running totals before each later weight: 0.2, 0.5; total 1.0
    got = [spai.policy_sample(p, 1.0, u) for u in (0.0, 0.19, 0.2, 0.21, 0.49, 0.5, 0.51, 1.0 - 2 ** -23)]
    assert got == [0, 0, 1, 1, 1, 2, 2, 2]
    assert spai.policy_sample([0.0, 0.0, 1.0], 1.25, 0.0) == 2          # zero weights are never drawn
    assert spai.policy_sample([1.0, 0.0, 0.0], 1.25, 0.999) == 0
    for bad in ([], [0.0, 0.0], [0.5, -0.1], [np.nan, 1.0]):
        with pytest.raises(spai.SpaiError):
            spai.policy_sample(bad, 1.0, 0.5)
    with pytest.raises(spai.SpaiError):
        spai.policy_sample([1.0], 1.0, 1.0)                              # u01 must be < 1


def test_normalize_matches_ndarray_sum(oracle):
    rng = np.random.default_rng(1)
    for n in (7, 9, 4672, 13):
        p = rng.random(n).astype(np.float32) * rng.integers(0, 2, n).astype(np.float32)
        p[0] = 0.25
        ref = p / np.float32(oracle.lib().or_nd_sum(_f(p), n))
        assert np.array_equal(spai.policy_normalize(p), ref)


@pytest.mark.parametrize("n", [7, 9, 4672])
def test_best_action_and_sample_match_oracle(oracle, n):
    L = oracle.lib()
    rng = np.random.default_rng(n)
    for trial in range(300):
        kind = trial % 4
        if kind == 0:    # visit-count-like policies with ties
            p = rng.integers(0, 6, n).astype(np.float32)
        elif kind == 1:  # sparse softmax-like
            p = (rng.random(n) * (rng.random(n) < 0.05)).astype(np.float32)
        elif kind == 2:  # normalized
            p = rng.random(n).astype(np.float32)
            p /= p.sum()
        else:            # signed values, zeros of both signs
            p = rng.normal(size=n).astype(np.float32)
            p[rng.integers(0, n, 3)] = 0.0
            p[rng.integers(0, n, 3)] = -0.0
        assert spai.policy_best_action(p) == L.or_policy_best_action(_f(p), n)
        if kind == 3 or not p.any():
            continue
        for t in (1.0, 1.25, 0.5):
            # rand's f32 draws: (u32 >> 9) * 2^-23, incl. the extremes
            for u in [0.0, 1.0 - 2 ** -23] + list((rng.integers(0, 1 << 23, 6) * 2.0 ** -23)):
                u = float(np.float32(u))
                assert spai.policy_sample(p, t, u) == L.or_policy_sample(_f(p), n, t, u), (trial, t, u)


def test_sample_frequencies_follow_weights():
    p = np.array([1, 0, 3, 4, 0, 2, 0], np.float32)
    w = p ** 1.25
    counts = np.zeros(7)
    for k in range(1 << 14):
        counts[spai.policy_sample(p, 1.25, k * 2.0 ** -14)] += 1
    assert np.allclose(counts / counts.sum(), w / w.sum(), atol=2e-4)
