"""Serving coalescer (fenix_amd/coalesce.py) on the CPU with a stand-in search:
concurrent single-query requests are batched, every request gets exactly its
own top-k, failures reach every request of the failing batch."""

from __future__ import annotations

import threading
import time

import numpy as np
import pytest

from fenix_amd.coalesce import Coalescer


def brute(x: np.ndarray):
    """(queries, K) -> ((dist asc, row asc) top-K) over x, like the engine."""
    def run(qs: np.ndarray, k: int):
        d = np.sqrt(((qs[:, None, :].astype(np.float64) - x[None]) ** 2).sum(-1))
        order = np.lexsort((np.broadcast_to(np.arange(x.shape[0]), d.shape), d), axis=-1)[:, :k]
        return np.take_along_axis(d, order, 1).astype(np.float32), order.astype(np.int64)
    return run


def test_concurrent_requests_are_batched_and_exact():
    rs = np.random.RandomState(0)
    x = rs.randn(500, 16).astype(np.float32)
    qs = rs.randn(40, 16).astype(np.float32)
    ks = [1 + (i * 7) % 23 for i in range(len(qs))]
    inner = brute(x)
    calls = []

    def run(q, k):
        calls.append(q.shape[0])
        time.sleep(0.02)  # the "device" is busy: later requests queue up
        return inner(q, k)

    c = Coalescer()
    out = [None] * len(qs)
    barrier = threading.Barrier(len(qs))

    def client(i):
        barrier.wait()
        out[i] = c.search("col", run, qs[i], ks[i])

    ts = [threading.Thread(target=client, args=(i,)) for i in range(len(qs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert sum(calls) == len(qs) and len(calls) < len(qs)
    assert c.requests == len(qs) and c.batches == len(calls)
    for i, (d, r) in enumerate(out):
        ed, er = inner(qs[i : i + 1], ks[i])
        assert d.shape == (1, ks[i]) and r.shape == (1, ks[i])
        np.testing.assert_array_equal(r, er)
        np.testing.assert_array_equal(d, ed)


def test_single_request_runs_at_once_and_keys_do_not_mix():
    rs = np.random.RandomState(1)
    xa, xb = rs.randn(50, 4).astype(np.float32), rs.randn(60, 4).astype(np.float32)
    c = Coalescer()
    q = rs.randn(4).astype(np.float32)
    da, ra = c.search("a", brute(xa), q, 5)
    db, rb = c.search("b", brute(xb), q, 5)
    np.testing.assert_array_equal(ra, brute(xa)(q[None], 5)[1])
    np.testing.assert_array_equal(rb, brute(xb)(q[None], 5)[1])
    assert c.batches == 2


def test_failure_reaches_every_request_of_the_batch_and_recovers():
    c = Coalescer()
    gate = threading.Event()
    n = 6
    errors = []

    def run(q, k):
        gate.wait(5)
        raise RuntimeError("device lost")

    def client():
        try:
            c.search("k", run, np.zeros(3, np.float32), 2)
        except RuntimeError as e:
            errors.append(str(e))

    ts = [threading.Thread(target=client) for _ in range(n)]
    for t in ts:
        t.start()
    time.sleep(0.1)
    gate.set()
    for t in ts:
        t.join(10)
    assert errors == ["device lost"] * n
    # the key is free again afterwards
    d, r = c.search("k", lambda q, k: (np.zeros((1, k), np.float32), np.zeros((1, k), np.int64)),
                    np.zeros(3, np.float32), 2)
    assert r.shape == (1, 2)


@pytest.mark.parametrize("max_batch", [1, 3])
def test_max_batch_bounds_each_batch(max_batch):
    rs = np.random.RandomState(2)
    x = rs.randn(100, 8).astype(np.float32)
    inner = brute(x)
    sizes = []

    def run(q, k):
        sizes.append(q.shape[0])
        time.sleep(0.01)
        return inner(q, k)

    c = Coalescer(max_batch=max_batch)
    qs = rs.randn(10, 8).astype(np.float32)
    res = [None] * 10
    ts = [threading.Thread(target=lambda i=i: res.__setitem__(i, c.search(0, run, qs[i], 3)))
          for i in range(10)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    assert max(sizes) <= max_batch and sum(sizes) == 10
    for i in range(10):
        np.testing.assert_array_equal(res[i][1], inner(qs[i : i + 1], 3)[1])
