"""N>1 path on CPU: world_size-2 gloo processes exercise the row sharding and
the all-gather of per-shard top-k used by bench.py / sharded_search over RCCL.

Each rank computes its shard's top-k with the CPU oracle (the GPU scan is
covered by the gpu tests), exchanges it with ``allgather_topk`` and checks
that the (distance, row) merge of the gathered lists equals the oracle's
global top-k — the decomposition the multi-GPU path relies on."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fenix_amd.distributed import allgather_topk, shard_rows


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O

        n_total, d, k = 9001, 48, 25
        base, n_local = shard_rows(n_total, world, rank)
        x = O.fill_normal(n_local, d, seed=0, row_base=base)  # this rank's rows only
        q = O.fill_normal(3, d, seed=1)
        results = {}
        for metric in ("l2", "cosine", "inner_product"):
            od, orow = O.knn(x, q, metric, k, row_base=base, threads=1)
            dl = torch.from_numpy(od.astype(np.float32))
            rl = torch.from_numpy(orow)
            gd, gr = allgather_topk(dl, rl)
            results[metric] = (gd.numpy(), gr.numpy())
        # bit-exact transport of special values
        special = torch.tensor([[np.nan, -0.0, np.inf, 1.5]], dtype=torch.float32)
        sd, sr = allgather_topk(special, torch.tensor([[rank, -1, 3, 4]]))
        results["special"] = (sd.numpy(), sr.numpy())
        result_q.put((rank, results))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_shard_rows_partition():
    for n in (0, 1, 7, 10_000_000, 80_000_001):
        for world in (1, 2, 3, 8):
            spans = [shard_rows(n, world, r) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(s[1] for s in spans) == n
            for (b0, n0), (b1, _) in zip(spans, spans[1:]):
                assert b0 + n0 == b1
            assert max(s[1] for s in spans) - min(s[1] for s in spans) <= 1
    with pytest.raises(ValueError):
        shard_rows(10, 2, 2)


def test_gloo_world2_gather_and_merge():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 2
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    from oracle import oracle as O

    x_all = O.fill_normal(9001, 48, seed=0)
    qv = O.fill_normal(3, 48, seed=1)
    for metric in ("l2", "cosine", "inner_product"):
        d0, r0 = got[0][metric]
        d1, r1 = got[1][metric]
        np.testing.assert_array_equal(d0, d1)  # every rank holds the same gather
        np.testing.assert_array_equal(r0, r1)
        assert d0.shape == (3, world, 25)
        od, orow = O.knn(x_all, qv, metric, 25)
        for i in range(3):
            dd = np.asarray(d0[i], dtype=np.float64).ravel()
            rr = r0[i].ravel()
            order = np.lexsort((rr, dd))[:25]
            np.testing.assert_array_equal(rr[order], orow[i])
    sd, sr = got[0]["special"]
    assert np.isnan(sd[0, 0, 0]) and np.signbit(sd[0, 0, 1]) and np.isinf(sd[0, 0, 2])
    assert list(sr[0, :, 0]) == [0, 1]


class _HostEngine:
    """Stand-in for fenix_amd.engine.Engine with the two calls sharded_search
    makes (search, merge), computed by the CPU oracle and a host (distance,
    row) merge: exercises the distributed control flow without a GPU."""

    def __init__(self):
        import threading

        self.lock = threading.Lock()

    def search(self, shards, queries, metric, k):
        from oracle import oracle as O

        (sh,) = shards
        od, orow = O.knn(sh.data, queries.numpy(), sh.metric_name, k, row_base=sh.row_base,
                         threads=1)
        return torch.from_numpy(od.astype(np.float32)), torch.from_numpy(orow)

    def merge(self, d, r, k):
        d, r = d.numpy(), r.numpy()
        outd = np.empty((d.shape[0], k), np.float32)
        outr = np.empty((d.shape[0], k), np.int64)
        for i in range(d.shape[0]):
            dd, rr = d[i].ravel().astype(np.float64), r[i].ravel()
            o = np.lexsort((rr, dd))[:k]
            outd[i], outr[i] = dd[o], rr[o]
        return torch.from_numpy(outd), torch.from_numpy(outr)


def _sharded_worker(rank, world, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from types import SimpleNamespace

        from fenix_amd.distributed import sharded_search
        from oracle import oracle as O

        n_total, d, k = 7003, 40, 30
        base, n_local = shard_rows(n_total, world, rank)
        q = torch.from_numpy(O.fill_normal(4, d, seed=5))
        out = {}
        for metric in ("l2", "cosine", "inner_product"):
            sh = SimpleNamespace(data=O.fill_normal(n_local, d, seed=4, row_base=base),
                                 row_base=base, metric_name=metric)
            md, mr = sharded_search(_HostEngine(), sh, q, 0, k)
            out[metric] = (md.numpy(), mr.numpy())
        result_q.put((rank, out))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_gloo_world3_sharded_search_equals_whole():
    """fenix_amd.distributed.sharded_search over 3 gloo ranks (uneven shards):
    every rank returns the global top-k of the whole corpus, rows numbered
    globally through each shard's row_base."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 3
    port = _port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    from oracle import oracle as O

    x_all = O.fill_normal(7003, 40, seed=4)
    qv = O.fill_normal(4, 40, seed=5)
    for metric in ("l2", "cosine", "inner_product"):
        od, orow = O.knn(x_all, qv, metric, 30)
        for r in range(world):
            np.testing.assert_array_equal(got[r][metric][1], orow)
            np.testing.assert_allclose(got[r][metric][0], od, rtol=1e-6, atol=1e-6)
