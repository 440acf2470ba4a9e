"""A model of the reference's replay hand-off for checking spai_pipeline_run's
event stream (test infrastructure).

train_concurrent (main.rs:137-235) shares one HeapRb of capacity batch*100
(main.rs:142) between the self-play workers and the trainer:
  * a worker pushes `(len as f32 * 0.3) as usize` randomly chosen positions of
    each finished self-play batch with push_iter_overwrite
    (learner_concurrent.rs:278-283): when full, the oldest sample is dropped;
  * the trainer waits for >= batch_size samples and takes the oldest
    batch_size with pop_iter().take(batch_size) (learner_concurrent.rs:94-101);
  * after each iteration of batches it publishes its weights (:153-159), which
    the workers load before their next self-play batch (:260-264).

`check_events` replays the observer's events (spai.pipeline_run(events=[...]),
delivered under the ring lock, in ring order) through a deque model and checks:
every popped batch equals the model's oldest samples bit for bit, the ring size
after each event, the subsample size of every push, that no sample is trained
on before the weights it was played with were published, that each worker's
weight versions never go backwards, and the totals in the returned stats.
"""
import collections

import numpy as np

PUSH, POP = 0, 1


def subsample_size(positions, fraction):
    """(len as f32 * fraction) as usize: f32 product, truncated"""
    return int(np.float32(positions) * np.float32(fraction))


def check_sample_shapes(states, policies, values):
    """every sample is a C4 position (planes mine/theirs/empty partition each cell),
    a normalised visit policy and a game outcome in {-1, 0, 1}"""
    enc = states.reshape(-1, 3, 42)
    assert np.all(np.isin(enc, (0.0, 1.0)))
    assert np.all(enc.sum(1) == 1.0)
    assert np.all(np.abs(policies.sum(1) - 1.0) < 1e-5) and np.all(policies >= 0)
    assert np.all(np.isin(values, (-1.0, 0.0, 1.0)))


def check_events(events, stats, capacity, batch_size, fraction, batches_expected=None, workers=None):
    model = collections.deque()     # (state, policy, value, version)
    pushed = overwritten = popped = positions = 0
    last_version = {}               # worker -> weight version of its previous batch
    next_batch = {}                 # worker -> expected next batch number
    pops = 0
    published = 0                   # versions published, as seen by the trainer's pops
    pending_push_versions = []      # push versions not yet bounded by a later pop
    for ev in events:
        n = ev["n"]
        if ev["kind"] == PUSH:
            w = ev["worker"]
            if workers is not None:
                assert w < workers, ev["worker"]
            assert ev["batch"] == next_batch.get(w, 0), (w, ev["batch"])
            next_batch[w] = ev["batch"] + 1
            assert n == subsample_size(ev["positions"], fraction), (ev["positions"], n)
            assert ev["version"] >= last_version.get(w, 0), (w, ev["version"])
            last_version[w] = ev["version"]
            check_sample_shapes(ev["states"], ev["policies"], ev["values"])
            for i in range(n):
                if len(model) == capacity:
                    model.popleft()
                    overwritten += 1
                model.append((ev["states"][i], ev["policies"][i], ev["values"][i], ev["version"]))
            pushed += n
            positions += ev["positions"]
            pending_push_versions.append(ev["version"])
        else:
            assert ev["kind"] == POP, ev["kind"]
            assert n == batch_size
            assert ev["batch"] == pops, (ev["batch"], pops)
            assert ev["version"] >= published   # publishing is monotone
            published = ev["version"]
            # a push's weights were published no later than this pop saw
            assert all(v <= published for v in pending_push_versions), (pending_push_versions, published)
            pending_push_versions = []
            assert len(model) >= n
            for i in range(n):
                s, p, v, ver = model.popleft()
                np.testing.assert_array_equal(ev["states"][i], s)
                np.testing.assert_array_equal(ev["policies"][i], p)
                assert ev["values"][i] == v
                assert ver <= published
            popped += n
            pops += 1
        assert ev["ring_size"] == len(model), (ev["ring_size"], len(model))
    assert stats["samples_pushed"] == pushed
    assert stats["samples_overwritten"] == overwritten
    assert stats["positions"] == positions
    assert stats["batches_trained"] == pops
    if batches_expected is not None:
        assert pops == batches_expected
    return dict(pushed=pushed, popped=popped, overwritten=overwritten, pops=pops, pushes=sum(next_batch.values()),
                workers_seen=len(next_batch), max_push_version=max(last_version.values(), default=0))
