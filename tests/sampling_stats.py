"""Goodness of fit of self-play move draws to the reference's rule
(learner_concurrent.rs:189-193: WeightedIndex over visit_count.powf(T), drawn
with the unseeded thread_rng, so only the distribution can be compared).

Each recorded position holds its root visit policy (normalised visits, mcts.rs:
310-331) and the played column.  Children are ranked by visits (descending, ties
by column); the observed counts of the played child's rank are compared with
the expected counts sum_pos N_child^T / sum N^T by a chi-square test (categories
with fewer than 5 expected draws pooled)."""
import numpy as np
from scipy.stats import chi2


def rank_observed(policy, moves):
    pol = np.asarray(policy, np.float64)
    mv = np.asarray(moves, np.int64)
    rows = np.arange(len(mv))
    order = np.lexsort((np.broadcast_to(np.arange(pol.shape[1]), pol.shape), -pol), axis=1)
    rank_of = np.empty_like(order)
    rank_of[rows[:, None], order] = np.arange(pol.shape[1])[None, :]
    observed = np.bincount(rank_of[rows, mv], minlength=pol.shape[1]).astype(np.float64)
    return pol, rank_of, observed


def rank_chi2(policy, moves, temperature):
    """(chi-square statistic, p-value, observed, expected) of the draws under P = N^T / sum N^T"""
    pol, rank_of, observed = rank_observed(policy, moves)
    legal = pol > 0
    w = np.where(legal, pol, 0.0) ** temperature
    q = w / w.sum(1, keepdims=True)
    expected = np.zeros(pol.shape[1])
    np.add.at(expected, rank_of.ravel(), q.ravel())
    keep = expected >= 5
    o = np.append(observed[keep], observed[~keep].sum())
    x = np.append(expected[keep], expected[~keep].sum())
    if x[-1] < 5:
        o, x = o[:-1], x[:-1]
    c = float(((o - x) ** 2 / x).sum())
    return c, float(chi2.sf(c, len(x) - 1)), observed, expected
