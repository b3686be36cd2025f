"""End-to-end drop-in tests, structured like the reference's
tests/test_flight.py: an in-process Server on loopback, a 100 000 x 256
float32 source written in 1 000-row batches with the reference's clustered
distribution (x + 10 * x[0] per batch, test_flight.py:17-35), and searches for
every metric.  Beyond the reference (which checks only row count and schema,
test_flight.py:111-114) the row ids are checked against the CPU oracle."""

from __future__ import annotations

import socket

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pytest
import torch

import fenix_amd
from fenix_amd.io import index
from oracle import oracle as O
from tests.parity import check_topk

pytestmark = pytest.mark.gpu

VECTOR_SIZE = 256
NUM_VECTORS = 100_000
BATCH_SIZE = 1_000
VECTOR = pa.list_(pa.float32(), list_size=VECTOR_SIZE)
SCHEMA = pa.schema({"id": pa.int64(), "vector": VECTOR})
METRICS = ["cosine", "dot", "inner_product", "l2", "euclidean"]


def batches(x, batch=BATCH_SIZE, value=np.float32):
    out = []
    d = x.shape[1]
    for s in range(0, x.shape[0], batch):
        part = x[s : s + batch].astype(value)
        a = pa.FixedSizeListArray.from_arrays(pa.array(part.ravel()), list_size=d)
        i = pa.array(np.arange(s, s + len(part), dtype=np.int64))
        out.append(pa.record_batch([i, a], names=["id", "vector"]))
    return out


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = str(tmp_path_factory.mktemp("fenix"))
    port = _port()
    server = fenix_amd.Server(root, host="127.0.0.1", port=port)
    x = O.fill_normal(NUM_VECTORS, VECTOR_SIZE, seed=21, cluster=BATCH_SIZE)
    source = pa.Table.from_batches(batches(x), SCHEMA)
    flight = fenix_amd.Flight(host="127.0.0.1", port=port)
    flight.make_table("test/table", source.to_reader())
    yield dict(root=root, server=server, flight=flight, x=x, source=source)
    server.shutdown()


def test_make_table(env):
    table = env["flight"].read_table("test/table").read_all()
    assert env["source"] == table


@pytest.mark.parametrize("metric", METRICS)
def test_search_without_index(env, metric):
    target = O.fill_normal(1, VECTOR_SIZE, seed=22)[0]
    result = env["flight"].search(target=target, source="test/table", column="vector",
                                  metric=metric, maxval=10)
    assert result.num_rows == 10
    assert result.schema == pa.schema([*SCHEMA, pa.field("__DISTANCE__", VECTOR.value_type)])
    od, orow = O.knn(env["x"], target[None], metric, 10)
    check_topk(result.column("__DISTANCE__").to_numpy()[None],
               result.column("id").to_numpy()[None], od, orow, env["x"], target[None], metric)
    # the gathered vectors are the rows' own vectors
    vec = np.stack(result.column("vector").to_numpy(zero_copy_only=False))
    np.testing.assert_array_equal(vec, env["x"][result.column("id").to_numpy()])


def test_search_random_target_like_reference(env):
    """The reference test's exact call: pc.random(256) cast to float32."""
    target = pc.random(VECTOR_SIZE).cast(VECTOR.value_type)
    for metric in METRICS:
        r = env["flight"].search(target=target, source="test/table", column="vector",
                                 metric=metric, maxval=10)
        assert r.num_rows == 10
        d = r.column("__DISTANCE__").to_numpy()
        assert np.all(np.diff(d) >= 0)


def test_search_select_and_filter(env):
    target = O.fill_normal(1, VECTOR_SIZE, seed=23)[0]
    expr = (pc.field("id") >= 30_000) & (pc.field("id") < 70_000)
    r = env["flight"].search(target=target, source="test/table", column="vector", metric="l2",
                             select=["id"], filter=expr, maxval=25)
    assert r.schema == pa.schema([pa.field("id", pa.int64()),
                                  pa.field("__DISTANCE__", pa.float32())])
    mask = (np.arange(NUM_VECTORS) >= 30_000) & (np.arange(NUM_VECTORS) < 70_000)
    od, orow = O.knn(env["x"], target[None], "l2", 25, mask=mask)
    check_topk(r.column("__DISTANCE__").to_numpy()[None], r.column("id").to_numpy()[None], od,
               orow, env["x"], target[None], "l2")


def test_search_maxval_none_returns_whole_table(env):
    target = O.fill_normal(1, VECTOR_SIZE, seed=24)[0]
    r = env["flight"].search(target=target, source="test/table", column="vector", metric="cosine",
                             select=["id"])
    assert r.num_rows == NUM_VECTORS
    np.testing.assert_array_equal(r.column("id").to_numpy(), np.arange(NUM_VECTORS))
    ref = O.distances(env["x"], target[None], "cosine")[0]
    assert np.all(np.abs(r.column("__DISTANCE__").to_numpy() - ref) <= 1e-5)


def test_multi_source_global_rows(env):
    root = env["root"]
    y = O.fill_normal(5_000, VECTOR_SIZE, seed=25)
    env["flight"].make_table("test/other", pa.Table.from_batches(batches(y), SCHEMA).to_reader())
    target = O.fill_normal(1, VECTOR_SIZE, seed=26)[0]
    r = index.call(root, None, ["test/other", "test/table"], "vector", target=target,
                   metric="inner_product", maxval=50)
    both = np.concatenate([y, env["x"]])
    od, orow = O.knn(both, target[None], "inner_product", 50)
    # the id column restarts per source; recover global positions from the vectors
    vec = np.stack(r.column("vector").to_numpy(zero_copy_only=False))
    od_ids = orow[0]
    np.testing.assert_array_equal(vec, both[od_ids])


def test_rewrite_restages(env):
    root = env["root"]
    z = O.fill_normal(3_000, VECTOR_SIZE, seed=27)
    env["flight"].make_table("test/mut", pa.Table.from_batches(batches(z), SCHEMA).to_reader())
    t = O.fill_normal(1, VECTOR_SIZE, seed=28)[0]
    r1 = index.call(root, None, "test/mut", "vector", target=t, metric="l2", maxval=5)
    z2 = O.fill_normal(3_000, VECTOR_SIZE, seed=29)
    env["flight"].make_table("test/mut", pa.Table.from_batches(batches(z2), SCHEMA).to_reader())
    r2 = index.call(root, None, "test/mut", "vector", target=t, metric="l2", maxval=5)
    od, orow = O.knn(z2, t[None], "l2", 5)
    np.testing.assert_array_equal(r2.column("id").to_numpy(), orow[0])
    assert not r1.equals(r2)


def test_float16_column(env):
    root = env["root"]
    h = O.fill_normal(20_000, 128, seed=30)
    vt = pa.list_(pa.float16(), 128)
    sch = pa.schema({"id": pa.int64(), "vector": vt})
    env["flight"].make_table("test/half",
                             pa.Table.from_batches(batches(h, value=np.float16), sch).to_reader())
    t = O.fill_normal(1, 128, seed=31)[0]
    r = index.call(root, None, "test/half", "vector", target=t, metric="inner_product",
                   maxval=100)
    assert r.schema.field("__DISTANCE__").type == pa.float16()
    xh = h.astype(np.float16)
    qh = t.astype(np.float16).astype(np.float32)[None]
    od, orow = O.knn(xh, qh, "inner_product", 100)
    # fp16 output distances: compare ids, and values at fp16 resolution
    np.testing.assert_array_equal(r.column("id").to_numpy(), orow[0])
    got = r.column("__DISTANCE__").to_numpy().astype(np.float64)
    assert np.all(np.abs(got - od[0]) <= 2 ** -10 * np.abs(od[0]))


def test_table_source_and_coder_distance(env):
    src = env["source"].slice(0, 4_000)
    t = O.fill_normal(1, VECTOR_SIZE, seed=32)[0]
    r = index.call("", None, src, "vector", target=t, metric="dot", maxval=7)
    od, orow = O.knn(env["x"][:4_000], t[None], "dot", 7)
    np.testing.assert_array_equal(r.column("id").to_numpy(), orow[0])
    u = torch.from_numpy(O.fill_normal(3, VECTOR_SIZE, seed=33))
    v = torch.from_numpy(env["x"][:1000])
    for metric in ("l2", "cosine", "dot"):
        got = fenix_amd.io.coder.distance(u, v, metric).numpy()
        ref = O.fenix_distance(u.numpy(), v.numpy(), metric)
        scale = 1.0 if metric == "cosine" else float(np.abs(ref).max())
        assert got.shape == (3, 1000)
        assert np.all(np.abs(got - ref) <= 1e-5 * scale)


def test_sharded_over_devices(env, monkeypatch):
    """FENIX_AMD_DEVICES row-shards the staged column (here 3 shards on one GPU;
    on a node, one per GPU); results are identical to the unsharded search."""
    root = env["root"]
    t = O.fill_normal(1, VECTOR_SIZE, seed=34)[0]
    base = index.call(root, None, "test/table", "vector", target=t, metric="l2", maxval=100)
    monkeypatch.setenv("FENIX_AMD_DEVICES", "0,0,0")
    sh = index.call(root, None, "test/table", "vector", target=t, metric="l2", maxval=100)
    assert sh.equals(base)
    expr = pc.field("id") >= 50_000
    sf = index.call(root, None, ["test/table", "test/table"], "vector", target=t,
                    metric="cosine", filter=expr, maxval=30)
    both = np.concatenate([env["x"], env["x"]])
    mask = np.concatenate([np.arange(NUM_VECTORS) >= 50_000] * 2)
    od, orow = O.knn(both, t[None], "cosine", 30, mask=mask)
    vec = np.stack(sf.column("vector").to_numpy(zero_copy_only=False))
    np.testing.assert_array_equal(vec, both[orow[0]])
    full = index.call(root, None, "test/table", "vector", target=t, metric="dot", select=["id"])
    ref = O.distances(env["x"], t[None], "dot")[0]
    assert np.all(np.abs(full.column("__DISTANCE__").to_numpy() - ref) <= 1e-5 * np.abs(ref).max())


def test_registered_distance_udf(env):
    """pc.call_function("distance:{metric}:{T}:{D}", ...) as in index.py:162."""
    t = O.fill_normal(1, VECTOR_SIZE, seed=35)[0]
    for metric in ("l2", "cosine", "dot"):
        func = index.register_distance(metric, VECTOR)
        assert func == f"distance:{metric}:float:{VECTOR_SIZE}"
        assert index.register_distance(metric, VECTOR) == func  # idempotent
        col = env["source"].column("vector").slice(0, 3_500)  # several chunks
        got = pc.call_function(func, [col, pa.scalar(t, type=VECTOR)]).to_numpy()
        ref = O.distances(env["x"][:3_500], t[None], metric)[0]
        scale = 1.0 if metric == "cosine" else float(np.abs(ref).max())
        assert np.all(np.abs(got - ref) <= 1e-5 * scale)


def test_concurrent_searches_match_sequential(env):
    """Flight handlers run on several gRPC threads at once (the reference has no
    locking, flight.py:62-77): 8 client threads searching together get exactly
    the results they get one at a time."""
    from concurrent.futures import ThreadPoolExecutor

    port = env["flight"].port
    targets = O.fill_normal(16, VECTOR_SIZE, seed=36)
    metrics = ["l2", "cosine", "dot", "euclidean"]

    def one(i):
        f = fenix_amd.Flight(host="127.0.0.1", port=port)
        r = f.search(target=targets[i], source="test/table", column="vector",
                     metric=metrics[i % 4], select=["id"], maxval=20 + i)
        return r.column("id").to_numpy(), r.column("__DISTANCE__").to_numpy()

    seq = [one(i) for i in range(16)]
    with ThreadPoolExecutor(8) as pool:
        par = list(pool.map(one, range(16)))
    for (a, da), (b, db) in zip(seq, par):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(da, db)


def test_maxval_above_fused_k(env):
    """maxval = 2 500 (> the fused path's 1 024): same rows as the oracle."""
    target = O.fill_normal(1, VECTOR_SIZE, seed=37)[0]
    r = env["flight"].search(target=target, source="test/table", column="vector", metric="l2",
                             select=["id"], maxval=2500)
    assert r.num_rows == 2500
    od, orow = O.knn(env["x"], target[None], "l2", 2500)
    check_topk(r.column("__DISTANCE__").to_numpy()[None], r.column("id").to_numpy()[None], od,
               orow, env["x"], target[None], "l2")


def test_empty_source(env):
    """A source with no rows: the reference returns an empty table with the
    output schema (index.py:165 not taken); so does the GPU path."""
    empty = pa.Table.from_batches([], SCHEMA)
    env["flight"].make_table("test/empty", empty.to_reader())
    t = O.fill_normal(1, VECTOR_SIZE, seed=38)[0]
    r = env["flight"].search(target=t, source="test/empty", column="vector", metric="l2",
                             maxval=10)
    assert r.num_rows == 0
    assert r.schema == pa.schema([*SCHEMA, pa.field("__DISTANCE__", pa.float32())])
    both = index.call(env["root"], None, ["test/empty", "test/table"], "vector", target=t,
                      metric="l2", select=["id"], maxval=5)
    od, orow = O.knn(env["x"], t[None], "l2", 5)
    np.testing.assert_array_equal(both.column("id").to_numpy(), orow[0])


def test_hbm_budget_evicts_and_restages(env, monkeypatch):
    """With an HBM budget below two staged columns (FENIX_AMD_HBM_BUDGET), the
    second table's staging evicts the first (least recently used); the first
    is restaged on its next search, with identical results."""
    from fenix_amd import engine

    root = env["root"]
    x2 = O.fill_normal(NUM_VECTORS, VECTOR_SIZE, seed=91)
    env["flight"].make_table("test/table2", pa.Table.from_batches(batches(x2), SCHEMA).to_reader())
    t = O.fill_normal(1, VECTOR_SIZE, seed=92)[0]
    engine.CACHE.clear()
    engine.RESIDENT.evict_all(engine.Residency.IMAGE)  # images of earlier tests' corpora
    first = index.call(root, None, "test/table", "vector", target=t, metric="l2", maxval=50)
    col_bytes = NUM_VECTORS * VECTOR_SIZE * 4
    monkeypatch.setenv("FENIX_AMD_HBM_BUDGET", str(int(1.5 * col_bytes)))
    ev0 = engine.RESIDENT.evictions
    other = index.call(root, None, "test/table2", "vector", target=t, metric="l2", maxval=50)
    assert engine.RESIDENT.evictions == ev0 + 1
    assert engine.RESIDENT.used(0) <= 1.5 * col_bytes
    od, orow = O.knn(x2, t[None], "l2", 50)
    np.testing.assert_array_equal(other.column("id").to_numpy(), orow[0])
    again = index.call(root, None, "test/table", "vector", target=t, metric="l2", maxval=50)
    assert engine.RESIDENT.evictions == ev0 + 2  # table2 made room for table's restaging
    assert again.equals(first)
    monkeypatch.delenv("FENIX_AMD_HBM_BUDGET")
    engine.CACHE.clear()


def test_configs0_100k_x128_l2_k10(env):
    """BASELINE configs[0] at its workload: 100 000 x 128 float32 rows (i.i.d.
    N(0,1), written by Flight.make_table in 1 000-row batches), L2, k = 10,
    single queries, through io.index.call (index.py:81-170) and through
    Flight.search (flight.py:242-288): ids bit-exact against the float64
    oracle, distances within 1e-5 relative."""
    root = env["root"]
    x0 = O.fill_normal(100_000, 128, seed=1000)
    sch = pa.schema({"id": pa.int64(), "vector": pa.list_(pa.float32(), 128)})
    env["flight"].make_table("test/cfg0", pa.Table.from_batches(batches(x0), sch).to_reader())
    targets = O.fill_normal(8, 128, seed=1001)
    od, orow = O.knn(x0, targets, "l2", 10)
    for i, t in enumerate(targets):
        direct = index.call(root, None, "test/cfg0", "vector", target=t, metric="l2", maxval=10)
        remote = env["flight"].search(target=t, source="test/cfg0", column="vector",
                                      metric="euclidean" if i % 2 else "l2", maxval=10)
        for r in (direct, remote):
            assert r.num_rows == 10
            assert r.schema == pa.schema([*sch, pa.field("__DISTANCE__", pa.float32())])
            np.testing.assert_array_equal(r.column("id").to_numpy(), orow[i])
            got = r.column("__DISTANCE__").to_numpy().astype(np.float64)
            assert np.all(np.abs(got - od[i]) <= 1e-5 * np.abs(od[i]))
            vec = np.stack(r.column("vector").to_numpy(zero_copy_only=False))
            np.testing.assert_array_equal(vec, x0[orow[i]])


def test_image_budget_never_evicts_its_corpus(env, monkeypatch):
    """A budget between the staged corpus alone and corpus + filter image: the
    optional image is not built (it never evicts a corpus, least of all the
    one it is for), the corpus stays resident and the batched search still
    equals the scan (image reservations evict images only)."""
    from fenix_amd import _lib, engine

    root = env["root"]
    engine.CACHE.clear()
    engine.RESIDENT.evict_all()
    t = O.fill_normal(1, VECTOR_SIZE, seed=93)[0]
    index.call(root, None, "test/table", "vector", target=t, metric="l2", maxval=5)
    (entry,) = engine.CACHE._entries.values()
    piece = entry.pieces[0]
    col_bytes = NUM_VECTORS * VECTOR_SIZE * 4
    monkeypatch.setenv("FENIX_AMD_HBM_BUDGET", str(int(col_bytes * 1.1)))  # image: +0.27x
    eng = engine.Engine.get(piece.device)
    eng.clear_images()
    ev0 = engine.RESIDENT.evictions
    qs = torch.from_numpy(O.fill_normal(16, VECTOR_SIZE, seed=94))
    shard = engine.Shard(piece.data, 0)
    assert _lib.filter_image_used(shard.n, shard.d, shard.dtype_id, 16, 50, _lib.METRIC_L2)
    bd, br = eng.search([shard], qs, _lib.METRIC_L2, 50)
    assert id(piece.data) not in eng._images  # no room: no image
    assert engine.RESIDENT.evictions == ev0
    assert entry.key in engine.CACHE
    with _lib.options(batched=0):
        sd, sr = eng.search([shard], qs, _lib.METRIC_L2, 50)
    np.testing.assert_array_equal(br.cpu().numpy(), sr.cpu().numpy())
    np.testing.assert_array_equal(bd.cpu().numpy().view(np.uint32),
                                  sd.cpu().numpy().view(np.uint32))
    monkeypatch.setenv("FENIX_AMD_HBM_BUDGET", str(int(col_bytes * 1.5)))
    eng.search([shard], qs, _lib.METRIC_L2, 50)
    assert id(piece.data) in eng._images  # room again: built, corpus still resident
    assert entry.key in engine.CACHE and engine.RESIDENT.evictions == ev0
    monkeypatch.delenv("FENIX_AMD_HBM_BUDGET")
    eng.clear_images()
    engine.CACHE.clear()


def test_remove(env):
    flight = env["flight"]
    flight.remove()
    import os

    assert not os.path.exists(env["root"])

