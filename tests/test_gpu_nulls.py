"""Null embedding slots, pinned to the reference's own outputs (tests/golden
g7_nulls.npz, written by tests/golden/make_golden.py from fenix.io.index.call).

The reference scans a null slot's stored values: ``from_arrow`` hands the
list array's VALUES to DLPack and never looks at the list's validity
(src/fenix/io/torch/torch.py:6-10), the UDF computes a distance for every row
(src/fenix/io/index/index.py:162-163) and ``take`` keeps the slot null in the
result (index.py:166-168).  Here the slot's stored values are staged and
scanned the same way; the k winning vectors are gathered from HBM and the
slot's validity is reapplied (io.index._gather_vectors).  Both branches of
io.index._take_columns are covered: maxval 10 (select path, vectors gathered
from HBM with the null mask) and maxval None / 5000 > rows (the whole table in
row order, the column passed through).  Nulls inside the values (a slot built
from Python ``None``) make the reference's from_dlpack raise ArrowTypeError,
and so does this engine.
"""

from __future__ import annotations

import json
import os
import socket

import numpy as np
import pyarrow as pa
import pytest
import torch

import fenix_amd
from fenix_amd.io import index, table
from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "g7_nulls.npz")


def _corpus(meta):
    x = O.fill_normal(meta["n"], meta["d"], meta["seed"])
    q = O.fill_normal(meta["nq"], meta["d"], meta["qseed"])
    x[17] = q[0]
    x[1777] = q[1] + np.float32(0.01)
    return x, q


def _source(x, nulls, chunk=1000):
    n, d = x.shape
    mask = np.zeros(n, dtype=bool)
    mask[nulls] = True
    schema = pa.schema({"id": pa.int64(), "vector": pa.list_(pa.float32(), d)})
    batches = []
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        arr = pa.FixedSizeListArray.from_arrays(pa.array(x[s:e].ravel()), list_size=d,
                                                mask=pa.array(mask[s:e]))
        batches.append(pa.record_batch([pa.array(np.arange(s, e, dtype=np.int64)), arr],
                                       names=["id", "vector"]))
    return pa.RecordBatchReader.from_batches(schema, batches), mask


@pytest.fixture(scope="module")
def g7(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z = np.load(GOLDEN)
    meta = json.loads(str(z["meta"]))
    x, q = _corpus(meta)
    root = str(tmp_path_factory.mktemp("nulls"))
    reader, mask = _source(x, meta["nulls"])
    table.make(root, "g7", reader)
    return dict(z=z, meta=meta, x=x, q=q, root=root, mask=mask)


def _check(g7, t, metric, tag, i):
    z, x, mask = g7["z"], g7["x"], g7["mask"]
    ids = t.column("id").to_numpy()
    np.testing.assert_array_equal(ids, z[f"{metric}_{tag}_ids"][i], err_msg=f"{metric} {tag}")
    np.testing.assert_array_equal(t.column("vector").is_null().to_numpy(zero_copy_only=False),
                                  z[f"{metric}_{tag}_null"][i])
    # distances: the float64 oracle over the stored values, 1e-5 relative
    # (scaled by |q| where an L2 distance is near zero)
    ref = O.distances(x[ids], g7["q"][i : i + 1], metric)[0]
    got = t.column("__DISTANCE__").to_numpy().astype(np.float64)
    scale = max(float(np.linalg.norm(g7["q"][i])), 1.0)
    assert np.all(np.abs(got - ref) <= 1e-5 * np.maximum(np.abs(ref), scale)), (metric, tag)
    # the non-null vectors are the stored rows; null slots stay null
    vec = t.column("vector")
    keep = ~mask[ids]
    got_vec = np.stack(vec.filter(pa.array(keep)).to_numpy(zero_copy_only=False))
    np.testing.assert_array_equal(got_vec, x[ids[keep]])


@pytest.mark.parametrize("metric", ["l2", "cosine", "inner_product"])
@pytest.mark.parametrize("maxval", [10, None, 5000])
def test_null_slots_match_reference_index_call(g7, metric, maxval):
    tag = "all" if maxval is None else str(maxval)
    for i, qv in enumerate(g7["q"]):
        t = index.call(g7["root"], None, "g7", "vector", target=qv, metric=metric, maxval=maxval)
        assert t.schema.names == ["id", "vector", "__DISTANCE__"]
        _check(g7, t, metric, tag, i)


def test_null_slots_through_flight(g7, tmp_path):
    """The same through Flight.search (do_exchange -> io.index.call), with the
    source written by Flight.make_table, at maxval 10 and None."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    server = fenix_amd.Server(str(tmp_path), host="127.0.0.1", port=port)
    try:
        flight = fenix_amd.Flight(host="127.0.0.1", port=port)
        reader, _ = _source(g7["x"], g7["meta"]["nulls"])
        flight.make_table("g7", reader)
        for metric in ("l2", "inner_product"):
            for maxval, tag in ((10, "10"), (None, "all")):
                for i, qv in enumerate(g7["q"]):
                    t = flight.search(target=qv, source="g7", column="vector", metric=metric,
                                      maxval=maxval)
                    _check(g7, t, metric, tag, i)
    finally:
        server.shutdown()


def test_nulls_inside_values_raise_like_reference(g7, tmp_path):
    """A null slot built from Python None puts nulls into the list's values;
    the reference's from_dlpack raises ArrowTypeError (g7 meta records the
    message) and so does staging here."""
    x = g7["x"][:1000]
    rows = [None if i in (3, 17) else [float(v) for v in r] for i, r in enumerate(x)]
    vt = pa.list_(pa.float32(), x.shape[1])
    b = pa.record_batch([pa.array(np.arange(1000, dtype=np.int64)), pa.array(rows, type=vt)],
                        names=["id", "vector"])
    root = str(tmp_path)
    table.make(root, "child", pa.RecordBatchReader.from_batches(b.schema, [b]))
    want = g7["meta"]["child_nulls_error"].split(": ", 1)
    with pytest.raises(pa.ArrowTypeError, match=want[1].rstrip(".")):
        index.call(root, None, "child", "vector", target=g7["q"][0], metric="l2", maxval=10)
