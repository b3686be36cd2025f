"""Search over a quint8 tensor column on the GPU (FX_DTYPE_QU8: 1-byte codes
dequantised in the scan's registers) against the oracle on the dequantised
values (oracle.dequantize = QUInt8NDArray.dequantize, quint8.py:53-54)."""

from __future__ import annotations

import socket

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pytest
import torch

import fenix_amd
from fenix_amd.ex.arrow import quint8 as Q
from fenix_amd.io import index, table
from oracle import oracle as O
from tests.parity import check_topk

pytestmark = pytest.mark.gpu

METRICS = ["l2", "inner_product", "cosine"]


@pytest.fixture(scope="module")
def qenv(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = str(tmp_path_factory.mktemp("q8"))
    n, d = 60_000, 128
    x = O.fill_normal(n, d, seed=71, cluster=1000)
    a = Q.from_numpy(x)
    src = pa.table({"id": pa.array(np.arange(n, dtype=np.int64)), "vector": a})
    table.make(root, "q/t", src.to_reader(max_chunksize=1000))
    deq = O.dequantize(a.codes(), a.type.scale, a.type.shift)
    return dict(root=root, x=deq, codes=a.codes(), type=a.type, n=n, d=d)


@pytest.mark.parametrize("metric", METRICS)
def test_quint8_search_matches_oracle(qenv, metric):
    t = O.fill_normal(1, qenv["d"], seed=72)[0]
    r = index.call(qenv["root"], None, "q/t", "vector", target=t, metric=metric, maxval=20)
    assert r.schema.field("__DISTANCE__").type == pa.float32()
    assert Q.is_quint8(r.schema.field("vector").type)
    od, orow = O.knn(qenv["x"], t[None], metric, 20)
    check_topk(r.column("__DISTANCE__").to_numpy()[None], r.column("id").to_numpy()[None], od,
               orow, qenv["x"], t[None], metric)
    got = r.column("vector").chunk(0).codes()  # combine_chunks: one chunk
    np.testing.assert_array_equal(got, qenv["codes"][r.column("id").to_numpy()])


def test_quint8_whole_table_distances(qenv):
    t = O.fill_normal(1, qenv["d"], seed=73)[0]
    r = index.call(qenv["root"], None, "q/t", "vector", target=t, metric="l2", select=["id"])
    ref = O.distances(qenv["x"], t[None], "l2")[0]
    assert np.all(np.abs(r.column("__DISTANCE__").to_numpy() - ref) <= 1e-5 * np.abs(ref).max())


@pytest.mark.parametrize("metric", ["l2", "cosine"])
def test_quint8_selective_filter_row_list(qenv, metric):
    """< 50 % kept: compacted row list through fx_knn_search_ex."""
    t = O.fill_normal(1, qenv["d"], seed=74)[0]
    expr = pc.field("id") < 9_000
    r = index.call(qenv["root"], None, "q/t", "vector", target=t, metric=metric,
                   select=["id"], filter=expr, maxval=15)
    mask = np.arange(qenv["n"]) < 9_000
    od, orow = O.knn(qenv["x"], t[None], metric, 15, mask=mask)
    check_topk(r.column("__DISTANCE__").to_numpy()[None], r.column("id").to_numpy()[None], od,
               orow, qenv["x"], t[None], metric)


def test_quint8_over_flight(qenv, tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    server = fenix_amd.Server(str(tmp_path), host="127.0.0.1", port=port)
    try:
        f = fenix_amd.Flight(host="127.0.0.1", port=port)
        f.make_table("q/f", table.load(qenv["root"], "q/t").to_reader())
        t = O.fill_normal(1, qenv["d"], seed=75)[0]
        r = f.search(target=t, source="q/f", column="vector", metric="dot", maxval=10)
        od, orow = O.knn(qenv["x"], t[None], "dot", 10)
        check_topk(r.column("__DISTANCE__").to_numpy()[None], r.column("id").to_numpy()[None],
                   od, orow, qenv["x"], t[None], "dot")
    finally:
        server.shutdown()


@pytest.mark.parametrize("metric", METRICS)
def test_quint8_dma_ring_equals_register_tiles(qenv, metric):
    """The LDS-DMA ring (unmasked scans) and the register tiles (masked scans,
    option "q8_dma" 0) compute the same distances bit for bit, top-k and all
    rows."""
    from fenix_amd import _lib
    from fenix_amd.engine import Engine, Shard

    eng = Engine.get(torch.device("cuda", 0))
    codes = torch.from_numpy(qenv["codes"].reshape(qenv["n"], qenv["d"])).to(eng.device)
    shard = Shard(codes, 0, float(qenv["type"].scale), int(qenv["type"].shift))
    q = torch.from_numpy(O.fill_normal(1, qenv["d"], seed=74))
    m = _lib.METRICS[metric]
    dd, dr = eng.search([shard], q, m, 50)
    da = eng.distances(shard, q, m)
    with _lib.options(q8_dma=0):
        rd, rr = eng.search([shard], q, m, 50)
        ra = eng.distances(shard, q, m)
    assert torch.equal(dr, rr)
    assert torch.equal(dd.view(torch.int32), rd.view(torch.int32))
    assert torch.equal(da.view(torch.int32), ra.view(torch.int32))
