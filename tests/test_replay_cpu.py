"""Replay ring (learner_concurrent.rs:244-290, main.rs:142) and the 30 % subsample
(choose_multiple), host-only: checked against a plain Python model of HeapRb's
push_iter_overwrite / pop_iter().take(n)."""
import collections

import numpy as np
import pytest

spai = pytest.importorskip("spai")


def _samples(rng, n, tag):
    s = rng.random((n, 126)).astype(np.float32)
    s[:, 0] = tag + np.arange(n)          # unique id per sample
    p = rng.random((n, 7)).astype(np.float32)
    v = rng.choice(np.array([-1, 0, 1], np.float32), n)
    return s, p, v


def test_replay_ring_matches_model():
    rng = np.random.default_rng(0)
    cap = 50
    r = spai.Replay(cap)
    model = collections.deque(maxlen=cap)   # append drops the oldest when full
    tag = 0
    for step in range(40):
        n = int(rng.integers(0, 23))
        s, p, v = _samples(rng, n, tag)
        tag += 1000
        r.push(s, p, v)
        for i in range(n):
            model.append((s[i].copy(), p[i].copy(), v[i]))
        assert len(r) == len(model)
        if step % 3 == 2 and len(model) >= 8:
            k = int(rng.integers(1, 9))
            gs, gp, gv = r.pop(k)
            for i in range(k):
                ms, mp, mv = model.popleft()
                np.testing.assert_array_equal(gs[i], ms)
                np.testing.assert_array_equal(gp[i], mp)
                assert gv[i] == mv
    with pytest.raises(spai.SpaiError):    # fewer buffered than requested
        r.pop(len(r) + 1)
    r.close()


def test_choose_multiple():
    a = spai.choose_multiple(100, 30, seed=5, stream=7)
    assert len(a) == 30 and len(set(a.tolist())) == 30 and a.max() < 100
    np.testing.assert_array_equal(a, spai.choose_multiple(100, 30, seed=5, stream=7))   # deterministic
    assert not np.array_equal(a, spai.choose_multiple(100, 30, seed=5, stream=8))
    assert sorted(spai.choose_multiple(10, 10, seed=1).tolist()) == list(range(10))
    assert len(spai.choose_multiple(5, 9)) == 5
    # uniform: every index about equally likely over many streams
    counts = np.zeros(20)
    for st in range(2000):
        counts[spai.choose_multiple(20, 6, seed=3, stream=st)] += 1
    assert counts.min() > 0.8 * counts.mean() and counts.max() < 1.2 * counts.mean()
