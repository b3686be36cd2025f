"""Host-side logic of the drop-in surface, on CPU: target normalisation,
filter -> mask, chunk-aware gather, storage format, error behaviour, and that
the product path refuses to run without the GPU (no CPU fallback)."""

from __future__ import annotations

import os
import pickle

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pytest
import torch

import fenix_amd
from fenix_amd import engine
from fenix_amd.io import index, table
from fenix_amd.io import torch as io_torch
from oracle import oracle as O

D = 16


def make_source(root, name, n=2500, chunk=1000, seed=0, value=pa.float32()):
    x = O.fill_normal(n, D, seed)
    vt = pa.list_(value, list_size=D)
    batches = []
    for s in range(0, n, chunk):
        part = x[s : s + chunk]
        vals = pa.array(part.ravel().astype(np.float16 if value == pa.float16() else np.float32))
        arr = pa.FixedSizeListArray.from_arrays(vals, list_size=D)
        ids = pa.array(np.arange(s, s + len(part), dtype=np.int64))
        batches.append(pa.record_batch([ids, arr], names=["id", "vector"]))
    schema = pa.schema({"id": pa.int64(), "vector": vt})
    return table.make(root, name, pa.RecordBatchReader.from_batches(schema, batches)), x


def test_table_roundtrip_and_listing(tmp_path):
    root = str(tmp_path)
    t, x = make_source(root, "a/b")
    assert t.num_rows == 2500 and t.column("vector").num_chunks == 3
    assert table.load(root, "a/b") == t
    both = table.load(root, ["a/b", "a/b"])
    assert both.num_rows == 5000
    assert list(table.list(root)) == ["a/b"]
    table.drop(root, "a/b")
    assert list(table.list(root)) == []


def test_rewrite_keeps_mapped_versions_valid(tmp_path):
    """do_put -> io.table.make rewrites a source while searches may hold its
    mmap (the resident caches keep them across calls): the old mapping must
    stay readable, and the version key must change even when the new file has
    the same size and lands in the same mtime tick."""
    from fenix_amd.io import _resident, arrow

    root = str(tmp_path)
    t1, x1 = make_source(root, "s", seed=0)
    p = table.path(root, "s")
    key1, mapped = _resident.load_table(p)
    old_ns = os.stat(p).st_mtime_ns
    t2, x2 = make_source(root, "s", seed=1)  # same shape -> same size
    os.utime(p, ns=(old_ns, old_ns))  # force the same mtime
    assert os.path.getsize(p) == key1[1]
    key2, mapped2 = _resident.load_table(p)
    assert key2 != key1
    # the first mapping still holds the first version's bytes
    v1 = np.stack(mapped.column("vector").to_numpy(zero_copy_only=False))
    v2 = np.stack(mapped2.column("vector").to_numpy(zero_copy_only=False))
    np.testing.assert_array_equal(v1, x1)
    np.testing.assert_array_equal(v2, x2)
    assert arrow.file_version(p) == key2[1:]
    assert not [f for f in os.listdir(os.path.dirname(p)) if f.endswith(".tmp")]


def test_chunk_values_honours_offsets():
    x = np.arange(40, dtype=np.float32)
    arr = pa.FixedSizeListArray.from_arrays(pa.array(x), list_size=4)
    sl = arr.slice(3, 4)
    v = engine._chunk_values(sl, np.dtype(np.float32))
    np.testing.assert_array_equal(v, x.reshape(10, 4)[3:7])
    t = io_torch.from_arrow(sl)
    np.testing.assert_array_equal(t.numpy(), x.reshape(10, 4)[3:7])


def test_chunk_values_null_slots():
    """A null slot with stored values is staged like any row (the reference's
    from_dlpack ignores the list's validity); nulls inside the values raise
    the reference's ArrowTypeError (tests/golden g7_nulls), from staging and
    from io.torch.from_arrow alike."""
    x = np.arange(40, dtype=np.float32)
    mask = pa.array([False, True] + [False] * 8)
    arr = pa.FixedSizeListArray.from_arrays(pa.array(x), list_size=4, mask=mask)
    assert arr.null_count == 1
    np.testing.assert_array_equal(engine._chunk_values(arr, np.dtype(np.float32)),
                                  x.reshape(10, 4))
    child = pa.array([[1.0, 2.0], None, [3.0, 4.0]], type=pa.list_(pa.float32(), 2))
    assert child.values.null_count == 2
    with pytest.raises(pa.ArrowTypeError, match="DLPack on arrays with no nulls"):
        engine._chunk_values(child, np.dtype(np.float32))
    with pytest.raises(pa.ArrowTypeError, match="DLPack on arrays with no nulls"):
        io_torch.from_arrow(child)
    # a slice that excludes the null-valued slot stages
    np.testing.assert_array_equal(engine._chunk_values(child.slice(2, 1), np.dtype(np.float32)),
                                  [[3.0, 4.0]])


def test_target_normalisation_matches_index_py():
    t = pa.list_(pa.float32(), D)
    q = np.arange(D, dtype=np.float32)
    for target in (q, torch.from_numpy(q), pa.array(q), pa.chunked_array([pa.array(q)]),
                   pa.scalar(q, type=t)):
        np.testing.assert_array_equal(index._target_values(target, t)[0], q)
    with pytest.raises(pa.ArrowInvalid):
        index._target_values(np.zeros(D + 1, np.float32), t)
    # fp16 column: the query takes the column's value type (index.py:111)
    t16 = pa.list_(pa.float16(), D)
    q16 = index._target_values(q / 3, t16)[0]
    np.testing.assert_array_equal(q16, (q / 3).astype(np.float16).astype(np.float32))


def test_filter_mask_equals_arrow_filter(tmp_path):
    t, _ = make_source(str(tmp_path), "f")
    expr = ((pc.field("id") > 2000) & (pc.field("id") < 2100)) | (pc.field("id") < 10)
    m = index._filter_mask(t, expr)
    np.testing.assert_array_equal(np.nonzero(m)[0], t.filter(expr).column("id").to_numpy())


def test_take_rows_is_chunk_aware_and_ordered(tmp_path):
    t, _ = make_source(str(tmp_path), "g", n=5500, chunk=700)
    rows = np.array([5499, 0, 701, 700, 3333, 699, 12, 4200])
    got = index.take_rows(t, rows)
    assert got.equals(t.take(pa.array(rows)))
    assert index.take_rows(t, np.zeros(0, np.int64)).num_rows == 0


def test_bitmap_layout():
    m = np.random.RandomState(0).rand(101) < 0.4
    words = engine.bitmap(m)
    assert words.dtype == np.uint32 and words.size == 4
    for r in range(101):
        assert ((int(words[r >> 5]) >> (r & 31)) & 1) == m[r]
    np.testing.assert_array_equal(words, O.bitmap(m))


def test_unknown_metric_is_value_error():
    with pytest.raises(ValueError):
        fenix_amd.io.coder.metric_id("manhattan")


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_search_fails_loudly_without_gpu(tmp_path):
    root = str(tmp_path)
    make_source(root, "s")
    q = O.fill_normal(1, D, 1)[0]
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        index.call(root, None, "s", "vector", target=q, metric="l2", maxval=5)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        fenix_amd.io.coder.distance(torch.from_numpy(q), torch.from_numpy(O.fill_normal(5, D, 2)),
                                    "l2")


def test_call_argument_errors(tmp_path):
    root = str(tmp_path)
    make_source(root, "s")
    q = O.fill_normal(1, D, 1)[0]
    with pytest.raises(AssertionError):  # index.py:131
        index.call(root, None, "s", "vector", target=q, metric=None, maxval=5)
    with pytest.raises(ValueError):  # coder.py:50
        index.call(root, None, "s", "vector", target=q, metric="hamming", maxval=5)
    with pytest.raises(FileNotFoundError):  # coder.load of a missing coding (coder.py:73)
        index.call(root, "code", "s", "vector", target=q, metric="l2", maxval=5, probes=4)
    with pytest.raises(pa.ArrowInvalid):  # index.py:111 length check
        index.call(root, None, "s", "vector", target=q[:-1], metric="l2", maxval=5)


def test_flight_client_asserts_metric():
    f = fenix_amd.Flight(host="127.0.0.1", port=1)
    with pytest.raises(AssertionError):  # flight.py:256
        f.search(target=np.zeros(D, np.float32), source="s", column="vector", metric="bad")


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_flight_table_admin_without_gpu(tmp_path):
    """make_table / read_table / drop_table / remove need no GPU (flight.py:34-60)."""
    port = _free_port()
    server = fenix_amd.Server(str(tmp_path / "root"), host="127.0.0.1", port=port)
    try:
        client = fenix_amd.Flight(host="127.0.0.1", port=port)
        src, _ = make_source(str(tmp_path / "tmp"), "x")
        client.make_table("t/x", src.to_reader())
        got = client.read_table("t/x").read_all()
        assert got == src
        sel = client.read_table("t/x", select=["id"], filter=pc.field("id") < 5).read_all()
        assert sel.column_names == ["id"] and sel.num_rows == 5
        desc = pickle.dumps({"name": "t/x"})
        assert desc  # the action body format is a pickled dict (flight.py:79-81)
        client.drop_table("t/x")
        assert not os.path.exists(tmp_path / "root" / "sources" / "t" / "x.arrow")
        client.remove()
        assert not os.path.exists(tmp_path / "root")
    finally:
        server.shutdown()


def test_coding_file_roundtrip_and_udf(tmp_path):
    """coder.load (coder.py:68-91) without a GPU: the file format loads with
    weights_only=True, the UDF ``name`` is registered with the reference's
    signature, list/drop work; a file holding a pickled pa.DataType (what the
    reference writes) is refused instead of unpickled."""
    import torch

    from fenix_amd.io import coder

    root = str(tmp_path)
    name = "cpu/l2"
    vt = pa.list_(pa.float32(), 8)
    os.makedirs(os.path.join(root, coder.LOCATION, "cpu"))
    cfg = {"metric": "l2", "codebook_size": 4, "num_codebooks": 2, "batch_size": 16,
           "num_epochs": 1}
    t = torch.arange(64, dtype=torch.float32).reshape(2, 4, 8)
    with open(coder._path(root, name), "wb") as f:
        torch.save({"tensor": t, "column": coder._type_bytes(vt), "config": cfg}, f)
    c = coder.load(root, name)
    assert c["column"] == vt and c["config"] == cfg
    assert torch.equal(c["tensor"], t)
    assert name in pc.list_functions()
    fn = pc.get_function(name)
    assert fn.arity == 2
    assert list(coder.list(root)) == [name]
    with open(coder._path(root, "cpu/bad"), "wb") as f:
        torch.save({"tensor": t, "column": vt, "config": cfg}, f)
    with pytest.raises(ValueError):
        coder.load(root, "cpu/bad")
    coder.drop(root, name)
    assert list(coder.list(root)) == ["cpu/bad"]


def test_index_files_list_and_drop(tmp_path):
    root = str(tmp_path)
    for src, col, name in [("a/b", "vector", "c/l2"), ("t", "v", "dot")]:
        p = index._index_path(root, name, src, col)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        fenix_amd.io.arrow.make(p, pa.RecordBatchReader.from_batches(
            pa.schema({index.CODE_COL: pa.int64()}),
            [pa.record_batch([pa.array([1, 2], pa.int64())], names=[index.CODE_COL])]))
    assert sorted(index.list(root)) == ["a/b/vector/c/l2", "t/v/dot"]
    index.drop(root, "dot", "t", "v")
    assert list(index.list(root)) == ["a/b/vector/c/l2"]


def test_launcher_cli_help():
    """fenix_amd.launch mirrors src/fenix/launch.py (root, --host, --port)."""
    import subprocess
    import sys

    out = subprocess.run([sys.executable, "-m", "fenix_amd.launch", "--help"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0
    for opt in ("--host", "--port", "--devices"):
        assert opt in out.stdout
