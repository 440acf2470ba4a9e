"""Fault behaviour on the GPU: a NaN anywhere in the PUCT scores stops the
search with SPAI_ERR_NAN, where the reference panics in
`partial_cmp().unwrap()` (mcts.rs:106-109, quirk Q11).

A net whose value bias is NaN makes every backed-up W NaN.  After the first
visit of a root child, that child's q = ((-W/N)+1)/2 is NaN while its unvisited
siblings still score finite UCBs, so the NaN sits on a child other than the
first (the first selection from a uniform root goes to the LAST child, Q2).
Only an OR over all of a tree's lanes catches it (a lane-0-only
report missed it and let the lanes' argmax split).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spai():
    import spai as s
    assert s.device_count() > 0, "no GPU visible"
    return s


def test_c4_nan_value_reports_nan(spai):
    e = spai.Engine(num_searches=8, max_trees=64, eval_kind=spai.EVAL_NET, seed=1)
    p = spai.init_params(2, 64, seed=3)
    p[-1] = np.nan   # value-head linear bias (model/connect_four.rs:69-70)
    net = spai.Net(e, 2, p)
    e.set_net(net)
    e.trees_create(64)
    with pytest.raises(spai.SpaiError) as ex:
        e.search(np.arange(64))
    assert ex.value.code == -5
    # a clean net on a fresh set of trees still searches normally afterwards
    net.close()
    net = spai.Net(e, 2, spai.init_params(2, 64, seed=3))
    e.set_net(net)
    e.trees_create(64)
    pol, ids, vis, nc = e.search(np.arange(64))
    assert np.all(vis.sum(1) == 7)   # the first iteration expands the root itself
    net.close()
    e.close()


def test_ttt_nan_value_reports_nan(spai):
    import spai_ttt
    e = spai_ttt.TTTEngine(num_searches=8, max_trees=8, eval_kind=spai_ttt.EVAL_NET)
    p = spai_ttt.init_params(2, seed=3)
    p[-1] = np.nan
    net = spai_ttt.TTTNet(e, 2, p)
    e.set_net(net)
    e.trees_create(8)
    with pytest.raises(spai.SpaiError) as ex:
        e.search(np.arange(8))
    assert ex.value.code == -5
    net.close()
    e.close()


def test_chess_nan_value_reports_nan(spai):
    import spai_chess
    e = spai_chess.ChessEngine(num_searches=6, max_trees=2, eval_kind=spai_chess.EVAL_NET)
    p = spai_chess.init_params(1, seed=3)
    p[-1] = np.nan   # value linear 256 -> 1 bias (model/chess.rs)
    net = spai_chess.ChessNet(e, 1, p)
    e.set_net(net)
    e.trees_create(2)
    with pytest.raises(spai.SpaiError) as ex:
        e.search(np.arange(2))
    assert ex.value.code == -5
    net.close()
    e.close()


def test_c4_zero_searches_on_a_fresh_engine(spai):
    """num_searches = 0 on a fresh engine (the per-iteration counters
    were not allocated, and the memset of a null buffer failed): the search returns
    with no children, and the root policy is Policy::normalize of all-zero visits,
    0/0 = NaN as in the reference (mcts.rs:310-331 with an unexpanded root)"""
    e = spai.Engine(num_searches=4, max_trees=8, eval_kind=spai.EVAL_HASH, seed=2)
    e.trees_create(8)
    pol, ids, vis, nc = e.search(np.arange(8), 0)
    assert np.all(nc == 0) and np.all(vis == 0)
    assert np.all(np.isnan(pol))
    pol, ids, vis, nc = e.search(np.arange(8), 4)   # the engine still searches afterwards
    assert np.all(nc == 7) and np.all(vis.sum(1) == 3)
    e.close()
