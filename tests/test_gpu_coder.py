"""GPU parity of the coded index (fenix_amd/csrc/knn_code.hip) against the CPU
oracle (oracle/coder.py) and the reference's own outputs
(tests/golden/g5_coder.npz), through the C ABI; then the reference's
index tests (tests/test_flight.py:62-95, 130-164 of nrlugg/fenix) end to end
over Flight, with the probe search checked row by row against the oracle."""

from __future__ import annotations

import json
import os
import socket

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pytest
import torch

import fenix_amd
from fenix_amd import _lib
from fenix_amd.engine import Engine
from fenix_amd.io import coder, index
from oracle import coder as OC
from oracle import oracle as O

pytestmark = pytest.mark.gpu

METRICS = ["l2", "inner_product", "cosine"]


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return Engine.get(torch.device("cuda", 0))


@pytest.fixture(scope="module")
def g5(golden_dir):
    g = np.load(f"{golden_dir}/g5_coder.npz")
    return g, json.loads(str(g["meta"]))


def _assign_ok(x, cw, metric, got_index, got_dist=None):
    """Per-codebook argmin vs float64: equal, or a near-tie (the two
    codewords' float64 distances within 1e-5 relative)."""
    nb, ks, _ = cw.shape
    d = OC.distance(x, cw.reshape(nb * ks, -1), metric).reshape(-1, nb, ks)
    ref = np.argmin(d, axis=2)
    bad = got_index != ref
    if bad.any():
        r, j = np.nonzero(bad)
        dg = d[r, j, got_index[r, j]]
        dr = d[r, j, ref[r, j]]
        scale = np.maximum(np.abs(dr), 1.0 if metric != "cosine" else 1e-3)
        assert np.all(np.abs(dg - dr) <= 1e-5 * scale), (bad.sum(), np.abs(dg - dr).max())
        assert bad.mean() < 1e-3
    if got_dist is not None:
        best = np.take_along_axis(d, got_index[..., None], axis=2)[..., 0]
        scale = 1.0 if metric == "cosine" else np.abs(best).max()
        assert np.all(np.abs(got_dist - best) <= 2e-5 * max(scale, 1.0))
    return ref


# ---------------------------------------------------------------- kernels


@pytest.mark.parametrize("metric", METRICS)
@pytest.mark.parametrize("nb,ks,d", [(2, 8, 64), (3, 5, 48), (2, 37, 128), (1, 64, 96),
                                     (2, 300, 64), (4, 16, 50)])
def test_code_assign_matches_oracle(eng, metric, nb, ks, d):
    n = 3000
    x = O.fill_normal(n, d, seed=41, cluster=100)
    cw = O.fill_normal(nb * ks, d, seed=42).reshape(nb, ks, d)
    xt = torch.from_numpy(x).to(eng.device)
    idx, code, dist = eng.code_assign(xt, torch.from_numpy(cw), _lib.METRICS[metric], index=True,
                                      code=True, dist=True)
    torch.cuda.synchronize()
    idx, code, dist = idx.cpu().numpy(), code.cpu().numpy(), dist.cpu().numpy()
    _assign_ok(x, cw, metric, idx, dist)
    expect = np.zeros(n, np.int64)
    for j in range(nb):
        expect = expect * ks + idx[:, j]
    np.testing.assert_array_equal(code, expect)


@pytest.mark.parametrize("metric", METRICS)
def test_code_assign_float16_and_tail_rows(eng, metric):
    n, d, nb, ks = 1001, 40, 2, 12  # n % 128 != 0, d % 32 != 0
    x = O.fill_normal(n, d, seed=43).astype(np.float16)
    cw = O.fill_normal(nb * ks, d, seed=44).reshape(nb, ks, d)
    xt = torch.from_numpy(x).to(eng.device)
    idx, _, _ = eng.code_assign(xt, torch.from_numpy(cw), _lib.METRICS[metric], index=True,
                                code=False)
    torch.cuda.synchronize()
    _assign_ok(x.astype(np.float32), cw, metric, idx.cpu().numpy())


@pytest.mark.parametrize("metric", METRICS)
def test_code_assign_repeats_bit_exactly(eng, metric):
    """The MFMA code assignment repeated on the same rows returns the same
    indices and the same distance bits every time: an accumulator read before
    its MFMA landed (the hazard DESIGN.md §3.6e audits) would move a near-tie
    index or a distance's low bits between runs.  Many rows (every CU busy,
    two waves per SIMD), wide codebooks, a tail tile."""
    n, d, nb, ks = 200_003, 256, 2, 256
    x = torch.empty((n, d), dtype=torch.float32, device=eng.device)
    eng.fill(x, seed=47, cluster=1000)
    cw = torch.from_numpy(O.fill_normal(nb * ks, d, seed=48).reshape(nb, ks, d))
    ref = None
    for _ in range(6):
        idx, _, dist = eng.code_assign(x, cw, _lib.METRICS[metric], index=True, code=False,
                                       dist=True)
        got = (idx.cpu().numpy(), dist.cpu().numpy().view(np.uint32))
        if ref is None:
            ref = got
            continue
        np.testing.assert_array_equal(got[0], ref[0], err_msg="indices moved")
        np.testing.assert_array_equal(got[1], ref[1], err_msg="distance bits moved")


def test_code_assign_unaligned_rows(eng):
    n, d, nb, ks = 700, 33, 2, 8  # odd d: scalar staging path
    x = O.fill_normal(n, d, seed=45)
    cw = O.fill_normal(nb * ks, d, seed=46).reshape(nb, ks, d)
    xt = torch.from_numpy(x).to(eng.device)
    idx, _, _ = eng.code_assign(xt, torch.from_numpy(cw), _lib.METRIC_L2, index=True, code=False)
    torch.cuda.synchronize()
    _assign_ok(x, cw, "l2", idx.cpu().numpy())


@pytest.mark.parametrize("metric", ["l2", "cosine", "dot"])
def test_kmeans_step_matches_reference(eng, g5, metric):
    g, meta = g5
    u = meta["update"]
    q = O.fill_normal(u["nb"] * u["ks"], u["D"], seed=u["q_seed"]).reshape(u["nb"], u["ks"], u["D"])
    v = O.fill_normal(u["nb"] * u["bs"], u["D"], seed=u["v_seed"], cluster=u["v_cluster"])
    out = coder.update(torch.from_numpy(q), torch.from_numpy(v.reshape(u["nb"], u["bs"], -1)),
                       metric).numpy()
    ref = g[f"update_{metric}"]
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()
    # single-codebook form (what vmap maps over)
    one = coder.update(torch.from_numpy(q[0]), torch.from_numpy(v[: u["bs"]]), metric).numpy()
    np.testing.assert_array_equal(one, out[0])


@pytest.mark.parametrize("metric", ["l2", "cosine", "dot"])
def test_coder_call_matches_reference(eng, g5, metric):
    g, meta = g5
    c = meta["call"]
    cw = O.fill_normal(c["nb"] * c["ks"], c["D"], seed=c["cw_seed"]).reshape(c["nb"], c["ks"], c["D"])
    x = O.fill_normal(c["n"], c["D"], seed=c["x_seed"], cluster=c["x_cluster"])
    t = O.fill_normal(c["nt"], c["D"], seed=c["t_seed"])
    coding = {"tensor": torch.from_numpy(cw), "column": pa.list_(pa.float32(), c["D"]),
              "config": {"metric": metric, "codebook_size": c["ks"], "num_codebooks": c["nb"],
                         "batch_size": 1, "num_epochs": 1}}
    np.testing.assert_array_equal(coder.call(x, coding, 1)[:, 0], g[f"call_codes_{metric}"])
    np.testing.assert_array_equal(coder.call(t, coding, c["probes"]), g[f"call_probe_{metric}"])
    np.testing.assert_array_equal(coder.call(t, coding, None), g[f"call_sort_{metric}"])
    # return types follow the target (coder.py:188-194)
    assert isinstance(coder.call(torch.from_numpy(t), coding, 3), torch.Tensor)
    arr = pa.FixedSizeListArray.from_arrays(pa.array(t.ravel()), list_size=c["D"])
    la = coder.call(arr, coding, 2)
    assert la.type == pa.list_(pa.int64()) and len(la) == c["nt"]
    with pytest.raises(RuntimeError):
        coder.call(t, coding, c["ks"] ** c["nb"] + 1)


def test_code_probe_mask_and_count(eng):
    nb, ks, n = 2, 6, 5000
    rs = np.random.RandomState(3)
    cw_dist = torch.from_numpy(rs.rand(1, nb, ks).astype(np.float32))
    codes, scores, sel = eng.code_probe(cw_dist, 7)
    torch.cuda.synchronize()
    s = OC.composite(cw_dist.numpy().reshape(1, -1).astype(np.float64), nb, ks)[0]
    np.testing.assert_array_equal(codes.cpu().numpy()[0], np.argsort(s, kind="stable")[:7])
    assert np.all(np.diff(scores.cpu().numpy()[0]) >= 0)
    row_code = rs.randint(-1, ks**nb + 2, size=n).astype(np.int64)  # includes out-of-range
    filt = rs.rand(n) < 0.5
    mk, cnt = eng.code_mask(torch.from_numpy(row_code).to(eng.device), sel[0], ks**nb,
                            fenix_amd.engine.device_mask(filt, eng.device))
    torch.cuda.synchronize()
    got = np.unpackbits(mk.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    expect = np.isin(row_code, codes.cpu().numpy()[0]) & filt
    np.testing.assert_array_equal(got, expect)
    assert int(cnt.item()) == int(expect.sum())


# ---------------------------------------------------------------- io.coder.make


@pytest.fixture(scope="module")
def root(tmp_path_factory):
    return str(tmp_path_factory.mktemp("fenix_coder"))


@pytest.mark.parametrize("metric", ["l2", "cosine", "dot"])
def test_coder_make_matches_reference(eng, g5, root, metric):
    g, meta = g5
    mk = meta["make"]
    x = O.fill_normal(mk["n"], mk["D"], seed=mk["x_seed"], cluster=mk["x_cluster"])
    src = "g5/src"
    if not os.path.exists(os.path.join(root, "sources", src + ".arrow")):
        arr = pa.FixedSizeListArray.from_arrays(pa.array(x.ravel()), list_size=mk["D"])
        t = pa.table({"id": pa.array(np.arange(mk["n"], dtype=np.int64)), "vector": arr})
        fenix_amd.io.table.make(root, src, t.to_reader(max_chunksize=1000))
    cfg = {k: mk[k] for k in ("codebook_size", "num_codebooks", "batch_size", "num_epochs")}
    np.random.seed(mk["np_seed"])
    code = coder.make(root, f"g5/{metric}", src, "vector", {"metric": metric, **cfg})
    ref = g[f"make_{metric}"]
    got = code["tensor"].numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()
    assert code["column"] == pa.list_(pa.float32(), mk["D"])
    assert f"g5/{metric}" in list(coder.list(root))
    again = coder.load(root, f"g5/{metric}")
    np.testing.assert_array_equal(again["tensor"].numpy(), got)


# ---------------------------------------------------------------- over Flight

VECTOR_SIZE = 256
NUM_VECTORS = 100_000
VECTOR = pa.list_(pa.float32(), list_size=VECTOR_SIZE)
SCHEMA = pa.schema({"id": pa.int64(), "vector": VECTOR})
REF_METRICS = ["cosine", "dot", "inner_product", "l2", "euclidean"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def fl_env(eng, tmp_path_factory):
    r = str(tmp_path_factory.mktemp("fenix_index"))
    port = _port()
    server = fenix_amd.Server(r, host="127.0.0.1", port=port)
    x = O.fill_normal(NUM_VECTORS, VECTOR_SIZE, seed=51, cluster=1000)
    batches = []
    for s in range(0, NUM_VECTORS, 1000):
        a = pa.FixedSizeListArray.from_arrays(pa.array(x[s : s + 1000].ravel()), VECTOR_SIZE)
        batches.append(pa.record_batch([pa.array(np.arange(s, s + 1000, dtype=np.int64)), a],
                                       names=["id", "vector"]))
    source = pa.Table.from_batches(batches, SCHEMA)
    flight = fenix_amd.Flight(host="127.0.0.1", port=port)
    flight.make_table("test/table", source.to_reader())
    yield dict(root=r, server=server, flight=flight, x=x, source=source)
    server.shutdown()


@pytest.mark.parametrize("metric", REF_METRICS)
def test_make_index_like_reference(fl_env, metric):
    """tests/test_flight.py:62-95 of the reference, plus code parity."""
    flight = fl_env["flight"]
    coding = f"test/{metric}"
    flight.make_index(name=coding, source="test/table", column="vector",
                      config={"metric": metric, "codebook_size": 8, "num_codebooks": 2,
                              "batch_size": 2560, "num_epochs": 5})
    t = flight.read_table("test/table", coding, "vector").read_all()
    assert fl_env["source"] == t.drop(["__CODED_ID__"])
    assert t.schema == pa.schema([*fl_env["source"].schema, pa.field("__CODED_ID__", pa.int64())])
    # every stored code is the composite argmin under the trained codebooks
    code = coder.load(fl_env["root"], coding)
    ref = OC.call(fl_env["x"], code["tensor"].numpy(), metric, 1)[:, 0]
    got = t.column("__CODED_ID__").to_numpy()
    assert (got != ref).mean() < 1e-3


@pytest.mark.parametrize("metric", REF_METRICS)
def test_search_with_index_like_reference(fl_env, metric):
    """tests/test_flight.py:130-164 of the reference, plus row parity: the
    result is the exact top-10 over the rows whose code is among the 16
    probed composites."""
    flight = fl_env["flight"]
    coding = f"test/{metric}"
    target = O.fill_normal(1, VECTOR_SIZE, seed=52)[0]
    result = flight.search(target=target, source="test/table", column="vector", metric=metric,
                           coding=coding, maxval=10, probes=16)
    assert result.num_rows == 10
    assert result.schema == pa.schema([*SCHEMA, pa.field("__CODED_ID__", pa.int64()),
                                       pa.field("__DISTANCE__", VECTOR.value_type)])
    code = coder.load(fl_env["root"], coding)
    probe = OC.call(target[None], code["tensor"].numpy(), code["config"]["metric"], 16)[0]
    rows_code = index.load(fl_env["root"], coding, "test/table", "vector") \
        .column("__CODED_ID__").to_numpy()
    mask = np.isin(rows_code, probe)
    od, orow = O.knn(fl_env["x"], target[None], metric, 10, mask=mask)
    np.testing.assert_array_equal(result.column("id").to_numpy(), orow[0])
    assert np.all(np.isin(result.column("__CODED_ID__").to_numpy(), probe))


def test_probe_search_filter_select_and_whole(fl_env):
    root = fl_env["root"]
    coding = "test/l2"
    target = O.fill_normal(1, VECTOR_SIZE, seed=53)[0]
    code = coder.load(root, coding)
    probe = OC.call(target[None], code["tensor"].numpy(), "l2", 5)[0]
    rows_code = index.load(root, coding, "test/table", "vector").column("__CODED_ID__").to_numpy()
    expr = pc.field("id") >= 40_000
    keep = np.isin(rows_code, probe) & (np.arange(NUM_VECTORS) >= 40_000)
    # metric defaults to the coding's (index.py:119-120)
    r = index.call(root, coding, "test/table", "vector", target=target, select=["id"],
                   filter=expr, maxval=25, probes=5)
    od, orow = O.knn(fl_env["x"], target[None], "l2", 25, mask=keep)
    np.testing.assert_array_equal(r.column("id").to_numpy(), orow[0])
    # maxval None: every probed row, in table order, with its distance
    w = index.call(root, coding, "test/table", "vector", target=target, metric="l2",
                   select=["id", "__CODED_ID__"], filter=expr, probes=5)
    np.testing.assert_array_equal(w.column("id").to_numpy(), np.nonzero(keep)[0])
    ref = O.distances(fl_env["x"][keep], target[None], "l2")[0]
    assert np.all(np.abs(w.column("__DISTANCE__").to_numpy() - ref) <= 1e-5 * np.abs(ref).max())
    # sharded over several (here: repeated) devices: identical
    os.environ["FENIX_AMD_DEVICES"] = "0,0,0"
    try:
        r3 = index.call(root, coding, "test/table", "vector", target=target, select=["id"],
                        filter=expr, maxval=25, probes=5)
    finally:
        del os.environ["FENIX_AMD_DEVICES"]
    assert r3.equals(r)


def test_coding_without_probes_is_brute_force_with_codes(fl_env):
    """coding given, probes None (index.py:93-96, 113 not taken): the joined
    table is searched exhaustively; the code column rides along."""
    root = fl_env["root"]
    target = O.fill_normal(1, VECTOR_SIZE, seed=54)[0]
    r = index.call(root, "test/l2", "test/table", "vector", target=target, metric="cosine",
                   maxval=12)
    assert r.schema.names == ["id", "vector", "__CODED_ID__", "__DISTANCE__"]
    od, orow = O.knn(fl_env["x"], target[None], "cosine", 12)
    np.testing.assert_array_equal(r.column("id").to_numpy(), orow[0])
    codes = index.load(root, "test/l2", "test/table", "vector").column("__CODED_ID__").to_numpy()
    np.testing.assert_array_equal(r.column("__CODED_ID__").to_numpy(), codes[orow[0]])


def test_drop_index(fl_env):
    root = fl_env["root"]
    flight = fl_env["flight"]
    assert "test/table/vector/test/dot" in list(index.list(root))
    flight.drop_index("test/dot")
    assert "test/dot" not in list(coder.list(root))
    assert "test/table/vector/test/dot" not in list(index.list(root))
    assert "test/table/vector/test/l2" in list(index.list(root))
