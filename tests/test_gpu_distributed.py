"""The multi-rank search path on the GPU: fenix_amd.distributed.sharded_search
run by 2 ranks (gloo process group, both ranks on the one GPU of the box:
RCCL refuses two ranks on one device), each scanning its row shard with the
HIP kernels, all-gathering its top-k and merging with fx_topk_merge.  The
merged rows and distance bits must equal the 1-rank search over the whole
corpus, and the rows must equal the CPU oracle's (row-range
shards, topk(all) == merge(topk(shards)))."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import oracle as O
from tests.parity import check_topk

pytestmark = pytest.mark.gpu

N_PER_RANK, D, NQ, K = 300_000, 256, 3, 100
METRICS = ("l2", "cosine", "inner_product")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, result_q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fenix_amd import _lib
        from fenix_amd.distributed import shard_rows, sharded_search
        from fenix_amd.engine import Engine, Shard

        eng = Engine.get(torch.device("cuda", 0))
        base, n_local = shard_rows(N_PER_RANK * world, world, rank)
        x = torch.empty((n_local, D), dtype=torch.float32, device=eng.device)
        eng.fill(x, seed=81, row_base=base)
        q = torch.from_numpy(O.fill_normal(NQ, D, seed=82))
        out = {}
        for metric in METRICS:
            md, mr = sharded_search(eng, Shard(x, base), q, _lib.METRICS[metric], K)
            out[metric] = (md.cpu().numpy(), mr.cpu().numpy())
        torch.cuda.synchronize()
        result_q.put((rank, out))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_two_rank_sharded_search_equals_one_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=180) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)

    from fenix_amd import _lib
    from fenix_amd.engine import Engine, Shard

    eng = Engine.get(torch.device("cuda", 0))
    n = N_PER_RANK * world
    x = torch.empty((n, D), dtype=torch.float32, device=eng.device)
    eng.fill(x, seed=81)
    qv = O.fill_normal(NQ, D, seed=82)
    xh = O.fill_normal(n, D, seed=81)
    for metric in METRICS:
        wd, wr = eng.search([Shard(x, 0)], torch.from_numpy(qv), _lib.METRICS[metric], K)
        wd, wr = wd.cpu().numpy(), wr.cpu().numpy()
        for r in range(world):
            gd, gr = got[r][metric]
            np.testing.assert_array_equal(gr, wr)
            np.testing.assert_array_equal(gd.view(np.uint32), wd.view(np.uint32))
        od, orow = O.knn(xh, qv, metric, K)
        check_topk(wd, wr, od, orow, xh, qv, metric)
        np.testing.assert_array_equal(wr, orow)
