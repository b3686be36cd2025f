"""The int8 filter image on corpora whose order is not random: the reference
test's clustered distribution (x + 10 x0 per 1 000-row batch,
/root/reference/tests/test_flight.py:21-22) and a corpus sorted by one
component.  The filter's thresholds come from tile-strided samples; the
image stores its rows in a permuted order (fx_filter_image8_perm), so the
samples are equidistributed over the corpus whatever its order.  Every search
must equal the exact f32 scan bit for bit, and, on these corpora, no query may
overflow the candidate buffer (which would send it to the exact scan: correct,
but 1.3x slower than the scan alone).  The shard is >= 4 GiB, so single
queries take the image (capi.hip use_batched)."""

from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from fenix_amd import _lib
from fenix_amd.engine import Engine, Shard
from oracle import oracle as O
from tests.parity import check_topk

pytestmark = pytest.mark.gpu

N, D, K = 1_500_000, 768, 100  # 4.6 GB of f32 rows
METRICS = ("l2", "cosine", "inner_product")
STATS = {}


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = Engine.get(torch.device("cuda", 0))
    yield e
    e.clear_images()
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "clustered_counts.json"), "w") as f:
        json.dump(STATS, f, indent=1)


def _queries(x: torch.Tensor, seed: int) -> dict:
    g = torch.Generator(device="cpu").manual_seed(seed)
    normal = torch.from_numpy(O.fill_normal(1, D, seed=seed))
    rows = [5, 777_777, N - 1]
    near = [x[r : r + 1].cpu() + 0.5 * torch.randn((1, D), generator=g) for r in rows]
    uniform = torch.rand((1, D), generator=g)  # pc.random(D), as the reference test searches
    return {"normal": normal, "near0": near[0], "near1": near[1], "near2": near[2],
            "uniform": uniform}


def _search(eng, shard, q, metric, k):
    q = q.to(eng.device, torch.float32).contiguous()
    od = torch.empty((q.shape[0], k), dtype=torch.float32, device=eng.device)
    orow = torch.empty((q.shape[0], k), dtype=torch.int64, device=eng.device)
    st = eng.scan(shard, q, metric, k)
    counts, cap = eng.filter_counts(shard, q.shape[0], metric, k, st)
    eng.reduce(shard, q, metric, k, st, od, orow)
    return od.cpu().numpy(), orow.cpu().numpy(), counts, cap


def _check_against_scan(eng, shard, name, q, metric, k=K, allow_overflow=False):
    m = _lib.METRICS[metric]
    fd, fr, counts, cap = _search(eng, shard, q, m, k)
    assert counts is not None, "the search did not run the filter"
    with _lib.options(single_query_image=0, batched=0):
        sd, sr, c2, _ = _search(eng, shard, q, m, k)
    assert c2 is None
    np.testing.assert_array_equal(fr, sr)
    np.testing.assert_array_equal(fd.view(np.uint32), sd.view(np.uint32))
    STATS[f"{name}/{metric}/nq{q.shape[0]}/k{k}"] = {"cap": cap, "max_count": int(counts.max()),
                                                    "mean_count": float(counts.mean())}
    STATS[f"{name}/{metric}/nq{q.shape[0]}/k{k}"]["overflowed"] = int((counts > cap).sum())
    if not allow_overflow:
        assert counts.max() <= cap, f"{name} {metric}: a query overflowed ({counts.max()} > {cap})"
    return fd, fr


def test_clustered_single_queries_through_image(eng):
    x = torch.empty((N, D), dtype=torch.float32, device=eng.device)
    eng.fill(x, seed=301, cluster=1000)
    shard = Shard(x, 0)
    for metric in METRICS:
        assert _lib.filter_image_used(N, D, _lib.DTYPE_F32, 1, K, _lib.METRICS[metric])
    qs = _queries(x, 302)
    for metric in METRICS:
        for name, q in qs.items():
            fd, fr = _check_against_scan(eng, shard, f"cluster1000/{name}", q, metric)
            if name == "near1":  # and the float64 oracle over the same rows
                qh = q.numpy()
                od, orow = O.knn_gen(N, D, 301, qh, metric, K, cluster=1000, threads=16)
                check_topk(fd, fr, od, orow, x[:2000].cpu().numpy(), qh, metric)
    # a batch: queries inside clusters and generic ones (the batched filter
    # over the image).  Generic queries against clustered rows are the int8
    # bounds' weak case (a row's quantisation error scales with its cluster
    # centre, not with the spread inside the cluster): some may overflow the
    # buffer and be recomputed by the exact scan, results stay exact
    batch = torch.cat([qs["near0"], qs["near1"], qs["near2"],
                       torch.from_numpy(O.fill_normal(61, D, seed=303))])
    for metric in METRICS:
        _check_against_scan(eng, shard, "cluster1000/batch", batch, metric, allow_overflow=True)
    eng.clear_images()


def test_sorted_corpus_through_image(eng):
    """Rows sorted by their first component: the rows nearest to a query along
    e_0 form one contiguous block at the end of the corpus."""
    x = torch.empty((N, D), dtype=torch.float32, device=eng.device)
    eng.fill(x, seed=311)
    order = torch.argsort(x[:, 0])
    x = x[order].contiguous()
    shard = Shard(x, 0)
    e0 = torch.zeros((1, D))
    e0[0, 0] = 6.0
    for metric in METRICS:
        _check_against_scan(eng, shard, "sorted/e0", e0, metric)
        if _lib.filter_image_used(N, D, _lib.DTYPE_F32, 1, 1000, _lib.METRICS[metric]):
            _check_against_scan(eng, shard, "sorted/e0", e0, metric, k=1000)
    eng.clear_images()
