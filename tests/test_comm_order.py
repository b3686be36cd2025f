"""The single-process RCCL exchange under concurrent searches (CPU, library
stubbed).

A Flight server answers requests on concurrent gRPC threads (reference:
src/fenix/flight.py:62-77), and ``engine._search_all`` over shards on distinct
devices ends in one grouped all-gather per search (``DeviceComm.allgather`` ->
``fx_allgather_topk``).  Two enqueues that overlap can order the collectives
differently on two devices, and RCCL then hangs.  Here the
library is a stand-in whose ``fx_allgather_topk`` really all-gathers host
buffers, records which thread is inside it, and sleeps so that an unlocked
overlap is near certain; the devices are ``cpu:0 … cpu:3`` stand-ins and each
device's engine is a brute-force numpy search.

* 8 threads × mixed metrics and masks: never two threads inside the call, every
  result equals brute force over the whole table;
* the same run with ``COLLECTIVE_LOCK`` replaced by a no-op does overlap
  (the test can see the hazard);
* a communicator that cannot be created falls back to peer copies, once
  warned, with the same results.
"""

from __future__ import annotations

import contextlib
import ctypes
import threading
import time
import types

import numpy as np
import pytest
import torch

from fenix_amd import _lib, engine


def _brute(x: np.ndarray, rows: np.ndarray, q: np.ndarray, metric: int, k: int,
           keep: np.ndarray | None):
    """(dist asc, row asc) top-k of q over x; rows = global row ids."""
    x64, q64 = x.astype(np.float64), q.astype(np.float64)
    if metric == _lib.METRIC_L2:
        d = np.sqrt(((q64[:, None, :] - x64[None]) ** 2).sum(-1))
    else:
        d = -(q64 @ x64.T)
    d = d.astype(np.float32)
    if keep is not None:
        d[:, ~keep] = np.inf
    out_d = np.full((q.shape[0], k), np.inf, np.float32)
    out_r = np.full((q.shape[0], k), -1, np.int64)
    for i in range(q.shape[0]):
        ok = np.isfinite(d[i])
        di, ri = d[i][ok], rows[ok]
        o = np.lexsort((ri, di))[:k]
        out_d[i, :o.size], out_r[i, :o.size] = di[o], ri[o]
    return out_d, out_r


class _FakeEngine:
    """Stands in for ``engine.Engine`` on one fake device."""

    def __init__(self) -> None:
        self.lock = threading.Lock()

    def search(self, shards, queries, metric, k, masks=None, counts=None):
        xs = np.concatenate([s.x for s in shards])
        rows = np.concatenate([s.row_base + np.arange(s.n) for s in shards])
        keep = None
        if masks is not None:
            keep = np.concatenate([m if m is not None else np.ones(s.n, bool)
                                   for m, s in zip(masks, shards)])
        d, r = _brute(xs, rows, queries.numpy(), metric, k, keep)
        return torch.from_numpy(d), torch.from_numpy(r)

    def merge(self, dist, row, k):
        nq = dist.shape[0]
        d, r = dist.reshape(nq, -1).numpy(), row.reshape(nq, -1).numpy()
        out_d = np.empty((nq, k), np.float32)
        out_r = np.empty((nq, k), np.int64)
        for i in range(nq):
            o = np.lexsort((r[i], d[i]))[:k]
            out_d[i], out_r[i] = d[i][o], r[i][o]
        return torch.from_numpy(out_d), torch.from_numpy(out_r)


class _FakeLib:
    """fx_comm_init_all / fx_allgather_topk over host memory, with a probe of
    how many threads are inside the all-gather at once."""

    def __init__(self, init_rc: int = 0) -> None:
        self.init_rc = init_rc
        self.inside = 0
        self.max_inside = 0
        self.calls = 0
        self._m = threading.Lock()

    def fx_last_error(self):
        return b"stub: no RCCL"

    def fx_max_k(self):
        return 1024

    def fx_comm_init_all(self, n, ids, href):
        if self.init_rc:
            return self.init_rc
        href._obj.value = 0x1000 + n
        return 0

    def fx_comm_destroy(self, h):
        return 0

    def fx_allgather_topk(self, handle, src_d, src_r, nq, k, dst_d, dst_r, streams):
        with self._m:
            self.inside += 1
            self.calls += 1
            self.max_inside = max(self.max_inside, self.inside)
        try:
            n = len(src_d)
            count = nq * k
            for j in range(n):          # one "device" at a time, like the group enqueue
                time.sleep(0.002)
                for i in range(n):
                    ctypes.memmove(dst_d[j] + i * count * 4, src_d[i], count * 4)
                    ctypes.memmove(dst_r[j] + i * count * 8, src_r[i], count * 8)
        finally:
            with self._m:
                self.inside -= 1
        return 0


@pytest.fixture
def stubbed(monkeypatch):
    ndev = 4
    fakes = {g: _FakeEngine() for g in range(ndev)}
    lib = _FakeLib()
    monkeypatch.setattr(_lib, "load", lambda: lib)
    monkeypatch.setattr(engine.Engine, "get", classmethod(lambda cls, dev=None: fakes[dev.index]))
    monkeypatch.setattr(torch.cuda, "device", lambda dev: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "current_stream",
                        lambda dev=None: types.SimpleNamespace(cuda_stream=dev.index))
    monkeypatch.setattr(engine.DeviceComm, "_cache", {})
    monkeypatch.setattr(engine.DeviceComm, "_failed", {})
    monkeypatch.delenv("FENIX_AMD_GATHER", raising=False)

    rs = np.random.RandomState(7)
    d = 24
    x = rs.randn(4 * 300 + 37, d).astype(np.float32)
    cuts = [0, 300, 610, 900, x.shape[0]]     # ragged shards, one per fake device
    shards = []
    for g in range(ndev):
        lo, hi = cuts[g], cuts[g + 1]
        s = types.SimpleNamespace(x=x[lo:hi], n=hi - lo, row_base=lo,
                                  data=types.SimpleNamespace(device=torch.device("cpu", g)))
        shards.append(s)
    return lib, x, shards


def _drive(x, shards, threads=8, reps=6):
    """Run ``engine._search_all`` from ``threads`` threads with mixed metrics,
    k and masks; return the mismatches against brute force."""
    rs = np.random.RandomState(11)
    jobs = []
    for t in range(threads):
        for r in range(reps):
            metric = (_lib.METRIC_L2, _lib.METRIC_IP)[(t + r) % 2]
            k = (5, 17, 40)[(t * reps + r) % 3]
            q = rs.randn(1 + (t % 3), x.shape[1]).astype(np.float32)
            keep = rs.rand(x.shape[0]) < 0.6 if r % 3 == 2 else None
            jobs.append((t, metric, k, q, keep))
    bad = []
    barrier = threading.Barrier(threads)

    def worker(t):
        barrier.wait()
        for (tt, metric, k, q, keep) in jobs:
            if tt != t:
                continue
            masks = None
            if keep is not None:
                masks = [keep[s.row_base:s.row_base + s.n] for s in shards]
            d, r = engine._search_all(shards, torch.from_numpy(q), metric, k, masks)
            ed, er = _brute(x, np.arange(x.shape[0]), q, metric, k, keep)
            if not (np.array_equal(r.numpy(), er) and np.array_equal(d.numpy(), ed)):
                bad.append((t, metric, k))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    return bad, len(jobs)


def test_concurrent_exchanges_never_overlap(stubbed):
    lib, x, shards = stubbed
    before = engine.GATHERS["rccl"]
    bad, njobs = _drive(x, shards)
    assert bad == []
    assert lib.calls == njobs
    assert engine.GATHERS["rccl"] - before == njobs
    assert lib.max_inside == 1


def test_unlocked_exchanges_do_overlap(stubbed, monkeypatch):
    """Negative control: without the lock the stub sees overlapping enqueues,
    so the test above can fail."""
    lib, x, shards = stubbed
    monkeypatch.setattr(engine, "COLLECTIVE_LOCK", contextlib.nullcontext())
    _drive(x, shards)
    assert lib.max_inside > 1


def test_comm_init_failure_falls_back_to_peer_copies(stubbed):
    lib, x, shards = stubbed
    lib.init_rc = -2      # FX_EUNSUPPORTED: RCCL missing
    before = dict(engine.GATHERS)
    with pytest.warns(RuntimeWarning, match="peer copies"):
        bad, njobs = _drive(x, shards, threads=4, reps=3)
    assert bad == []
    assert lib.calls == 0
    assert engine.GATHERS["p2p"] - before["p2p"] == njobs
    assert engine.GATHERS["rccl"] == before["rccl"]
