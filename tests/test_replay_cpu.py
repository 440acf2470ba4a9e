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


def _c4_samples(rng, n):
    s = np.zeros((n, 3, 42), np.float32)
    cell = rng.integers(0, 3, (n, 42))
    for c in range(3):
        s[:, c] = cell == c
    p = rng.random((n, 7)).astype(np.float32)
    p /= p.sum(1, keepdims=True)
    return s.reshape(n, 126), p, rng.choice(np.array([-1, 0, 1], np.float32), n)


def test_pipeline_event_model_catches_faults():
    """tests/pipeline_model.py (the checker of the GPU pipeline tests) accepts a
    correct HeapRb event stream and rejects a reordered batch, a wrong subsample
    size and a sample trained before its weights were published"""
    import copy

    from pipeline_model import POP, PUSH, check_events, subsample_size
    rng = np.random.default_rng(1)
    cap, B = 40, 8
    ring = collections.deque()
    events, pushed, over, pops = [], 0, 0, 0
    for b in range(6):
        pos = int(rng.integers(20, 60))
        k = subsample_size(pos, 0.3)
        s, p, v = _c4_samples(rng, k)
        for i in range(k):
            if len(ring) == cap:
                ring.popleft()
                over += 1
            ring.append((s[i], p[i], v[i]))
        pushed += k
        events.append(dict(kind=PUSH, worker=0, batch=b, version=b // 2, n=k, positions=pos, ring_size=len(ring),
                           states=s, policies=p, values=v))
        while len(ring) >= B:
            got = [ring.popleft() for _ in range(B)]
            events.append(dict(kind=POP, worker=0, batch=pops, version=b // 2 + 1, n=B, positions=0,
                               ring_size=len(ring), states=np.stack([g[0] for g in got]),
                               policies=np.stack([g[1] for g in got]), values=np.array([g[2] for g in got])))
            pops += 1
    stats = dict(samples_pushed=pushed, samples_overwritten=over, batches_trained=pops,
                 positions=sum(e["positions"] for e in events if e["kind"] == PUSH))
    check_events(events, stats, cap, B, 0.3, batches_expected=pops, workers=1)
    first_pop = next(i for i, e in enumerate(events) if e["kind"] == POP)
    bad = copy.deepcopy(events)                       # two samples of a batch swapped
    bad[first_pop]["states"][[0, 1]] = bad[first_pop]["states"][[1, 0]]
    with pytest.raises(AssertionError):
        check_events(bad, stats, cap, B, 0.3)
    bad = copy.deepcopy(events)                       # (positions * 0.3) as usize violated
    bad[0]["positions"] += 10
    with pytest.raises(AssertionError):
        check_events(bad, stats, cap, B, 0.3)
    bad = copy.deepcopy(events)                       # played with weights not yet published
    bad[0]["version"] = 99
    with pytest.raises(AssertionError):
        check_events(bad, stats, cap, B, 0.3)
