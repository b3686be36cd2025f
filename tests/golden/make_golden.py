"""Generate golden vectors from the reference implementation (nrlugg/fenix).

Run ONLY in the build container, where the reference checkout exists:

    python tests/golden/make_golden.py [--only-g6 | --only-g7]

It imports fenix from /root/reference/src (Python 3.10 needs the
``typing.Self`` shim: fenix/flight.py:5 imports it, fenix wants >= 3.11),
writes synthetic corpora with the reference's own writer (io.table.make,
src/fenix/io/table/table.py:24-26 -> io/arrow/arrow.py:11-21), and records
what the reference returns from

* ``fenix.io.index.call``  (src/fenix/io/index/index.py:81-170), and
* ``fenix.Flight.search``  (src/fenix/flight.py:242-288) against an
  in-process ``fenix.Server`` (flight.py:17-77) over loopback gRPC.

Only OUTPUTS are committed (``tests/golden/*.npz``): the row ids (the ``id``
column = global row number), the ``__DISTANCE__`` values, the result schema,
and a SHA-256 of each corpus so the tests can prove they regenerated the same
bytes with ``oracle.fill_normal``.  No reference source is copied.
"""

from __future__ import annotations

import hashlib
import json
import os
import socket
import sys
import tempfile
import typing

import numpy as np
import pyarrow as pa

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.oracle import fill_normal  # noqa: E402

METRICS = ["l2", "euclidean", "cosine", "inner_product", "dot"]


def _import_fenix():
    import typing_extensions

    typing.Self = typing_extensions.Self  # fenix/flight.py:5 (Python >= 3.11 API)
    sys.path.insert(0, "/root/reference/src")
    import fenix  # noqa: F401
    import fenix.io.index  # noqa: F401

    return fenix


def _batches(x: np.ndarray, chunk: int):
    d = x.shape[1]
    vt = pa.list_(pa.from_numpy_dtype(x.dtype), list_size=d)
    schema = pa.schema({"id": pa.int64(), "vector": vt})
    out = []
    for s in range(0, x.shape[0], chunk):
        part = x[s : s + chunk]
        arr = pa.FixedSizeListArray.from_arrays(pa.array(part.ravel()), list_size=d)
        ids = pa.array(np.arange(s, s + part.shape[0], dtype=np.int64))
        out.append(pa.record_batch([ids, arr], names=["id", "vector"]))
    return schema, out


def _sha(x: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def direct_case(fenix, root, name, x, chunk, queries, ks, metrics=METRICS, meta=None):
    schema, batches = _batches(x, chunk)
    fenix.io.table.make(root, name, pa.RecordBatchReader.from_batches(schema, batches))
    rec = {}
    for metric in metrics:
        for k in ks:
            ids = np.full((len(queries), k), -1, dtype=np.int64)
            dist = np.full((len(queries), k), np.nan, dtype=np.float32)
            for i, q in enumerate(queries):
                t = fenix.io.index.call(
                    root, None, name, "vector", target=q.astype(np.float32), metric=metric,
                    maxval=k,
                )
                ids[i, : t.num_rows] = t.column("id").to_numpy()
                dist[i, : t.num_rows] = t.column("__DISTANCE__").to_numpy()
                rec["schema"] = str(t.schema)
            rec[f"{metric}_k{k}_ids"] = ids
            rec[f"{metric}_k{k}_dist"] = dist
    return rec


def g6_fp16(fenix, root) -> dict:
    """G6: a 1536-d float16 column (configs[4]'s dtype and width).  The
    reference's fp16 path works up to select_k (which crashes on a halffloat
    key in pyarrow 25): with maxval=None it returns the UDF's own
    per-chunk distances (index.py:133-159 -> coder.py:38-50 in ATen half
    arithmetic) for every row, as halffloat (index.py:150-158, 165).  The
    target is passed as float16: index.py:111's pa.scalar(target, type=...)
    does not cast a float32 array to a halffloat list."""
    n, d = 3000 + 111, 1536
    x = fill_normal(n, d, seed=13, dtype=np.float16)
    q = fill_normal(4, d, seed=14).astype(np.float16)
    schema, batches = _batches(x, 1000)
    fenix.io.table.make(root, "g6_fp16", pa.RecordBatchReader.from_batches(schema, batches))
    rec = {}
    metrics = ["l2", "cosine", "inner_product"]
    for metric in metrics:
        out = np.empty((len(q), n), dtype=np.float16)
        for i, qv in enumerate(q):
            t = fenix.io.index.call(root, None, "g6_fp16", "vector", target=qv, metric=metric)
            assert t.schema.field("__DISTANCE__").type == pa.float16()
            np.testing.assert_array_equal(t.column("id").to_numpy(), np.arange(n))
            out[i] = t.column("__DISTANCE__").to_numpy()
            rec["schema"] = str(t.schema)
        rec[f"{metric}_all_dist"] = out
    meta = dict(kind="direct_full_table_fp16", n=n, d=d, seed=13, qseed=14, nq=4, chunk=1000,
                cluster=0, dtype="float16", sha256=_sha(x), metrics=metrics)
    np.savez_compressed(os.path.join(HERE, "g6_fp16.npz"), meta=json.dumps(meta), **rec)
    return meta


G7_NULLS = [0, 3, 17, 999, 1000, 1777, 2499]


def g7_corpus():
    """G7's corpus: fill_normal rows, row 17 = query 0 and row 1777 = query 1
    + 0.01 (so null rows rank first), and the null slots G7_NULLS."""
    n, d = 2500, 64
    x = fill_normal(n, d, seed=15)
    q = fill_normal(3, d, seed=16)
    x[17] = q[0]
    x[1777] = q[1] + np.float32(0.01)
    return x, q


def g7_nulls(fenix, root) -> dict:
    """G7: null embedding slots (index.py:161-170 + io/torch/torch.py:6-10).

    (a) the parent list array carries the validity bitmap and the child
    values stay intact (FixedSizeListArray.from_arrays(values, mask=...)):
    the reference scans a null slot's stored values like any other row
    (from_dlpack of the child ignores the parent's validity), ranks it, and
    the result's vector column is null there (Table.take keeps validity).
    Recorded for maxval 10 (select path), None and 5000 > rows (whole table
    in row order), with each result row's vector validity.
    (b) nulls in the child values (a null slot built from Python None): the
    UDF's from_dlpack raises; the error type and message are recorded."""
    x, q = g7_corpus()
    n, d = x.shape
    mask = np.zeros(n, dtype=bool)
    mask[G7_NULLS] = True
    vt = pa.list_(pa.float32(), d)
    schema = pa.schema({"id": pa.int64(), "vector": vt})
    batches = []
    for s in range(0, n, 1000):
        e = min(n, s + 1000)
        arr = pa.FixedSizeListArray.from_arrays(pa.array(x[s:e].ravel()), list_size=d,
                                                mask=pa.array(mask[s:e]))
        batches.append(pa.record_batch([pa.array(np.arange(s, e, dtype=np.int64)), arr],
                                       names=["id", "vector"]))
    fenix.io.table.make(root, "g7_nulls", pa.RecordBatchReader.from_batches(schema, batches))
    rec = {}
    metrics = ["l2", "cosine", "inner_product"]
    for metric in metrics:
        for mv in (10, None, 5000):
            tag = f"{metric}_{'all' if mv is None else mv}"
            rows = n if mv is None or mv >= n else mv
            ids = np.empty((len(q), rows), dtype=np.int64)
            dist = np.empty((len(q), rows), dtype=np.float32)
            null = np.empty((len(q), rows), dtype=bool)
            for i, qv in enumerate(q):
                t = fenix.io.index.call(root, None, "g7_nulls", "vector", target=qv,
                                        metric=metric, maxval=mv)
                ids[i] = t.column("id").to_numpy()
                dist[i] = t.column("__DISTANCE__").to_numpy()
                null[i] = t.column("vector").is_null().to_numpy(zero_copy_only=False)
                rec["schema"] = str(t.schema)
            rec[f"{tag}_ids"], rec[f"{tag}_dist"], rec[f"{tag}_null"] = ids, dist, null
    # (b) child-level nulls
    rows_py = [None if m else [float(v) for v in r] for r, m in zip(x[:1000], mask[:1000])]
    arr = pa.array(rows_py, type=vt)
    b = pa.record_batch([pa.array(np.arange(1000, dtype=np.int64)), arr], names=["id", "vector"])
    fenix.io.table.make(root, "g7_child_nulls", pa.RecordBatchReader.from_batches(schema, [b]))
    try:
        fenix.io.index.call(root, None, "g7_child_nulls", "vector", target=q[0], metric="l2",
                            maxval=10)
        child_error = ""
    except Exception as e:  # recorded, not raised: this is the expected outcome
        child_error = f"{type(e).__name__}: {e}"
    meta = dict(kind="direct_nulls", n=n, d=d, seed=15, qseed=16, nq=3, chunk=1000, cluster=0,
                nulls=G7_NULLS, planted={"17": "q0", "1777": "q1 + 0.01"}, sha256=_sha(x),
                metrics=metrics, maxvals=[10, None, 5000], child_nulls_error=child_error)
    np.savez_compressed(os.path.join(HERE, "g7_nulls.npz"), meta=json.dumps(meta), **rec)
    return meta


def main() -> None:
    fenix = _import_fenix()
    root = tempfile.mkdtemp(prefix="fenix_golden_")
    manifest = {}
    only = {"--only-g6": ("g6_fp16", g6_fp16), "--only-g7": ("g7_nulls", g7_nulls)}
    for flag, (name, fn) in only.items():
        if flag in sys.argv:  # add one case to an existing manifest
            with open(os.path.join(HERE, "MANIFEST.json")) as f:
                manifest = json.load(f)
            manifest[name] = fn(fenix, root)
            with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
                json.dump(manifest, f, indent=1, sort_keys=True)
            print("wrote", name)
            return

    # G1: generic N(0,1)-like corpora, ragged last chunk (8192 = 8*1000 + 192)
    for d in (128, 768):
        x = fill_normal(8192, d, seed=0)
        q = fill_normal(8, d, seed=1)
        rec = direct_case(fenix, root, f"g1_d{d}", x, 1000, q, ks=(10, 100))
        meta = dict(kind="direct", n=8192, d=d, seed=0, qseed=1, nq=8, chunk=1000,
                    cluster=0, sha256=_sha(x), ks=[10, 100], metrics=METRICS)
        np.savez_compressed(os.path.join(HERE, f"g1_d{d}.npz"), meta=json.dumps(meta), **rec)
        manifest[f"g1_d{d}"] = meta

    # G2: exact duplicates (every row twice): fenix pins only the tie SET.
    base = fill_normal(1024, 64, seed=5)
    x = np.concatenate([base, base])
    q = fill_normal(4, 64, seed=6)
    rec = direct_case(fenix, root, "g2_ties", x, 1000, q, ks=(10,), metrics=["l2", "inner_product", "cosine"])
    meta = dict(kind="direct", n=2048, d=64, seed=5, qseed=6, nq=4, chunk=1000, cluster=0,
                duplicate=True, sha256=_sha(x), ks=[10], metrics=["l2", "inner_product", "cosine"])
    np.savez_compressed(os.path.join(HERE, "g2_ties.npz"), meta=json.dumps(meta), **rec)
    manifest["g2_ties"] = meta

    # G3: tail chunk of 12 rows (<= 25 rows: torch.cdist takes the direct path)
    x = fill_normal(1012, 128, seed=9)
    q = fill_normal(4, 128, seed=10)
    rec = direct_case(fenix, root, "g3_tail", x, 1000, q, ks=(10, 1012))
    meta = dict(kind="direct", n=1012, d=128, seed=9, qseed=10, nq=4, chunk=1000, cluster=0,
                sha256=_sha(x), ks=[10, 1012], metrics=METRICS)
    np.savez_compressed(os.path.join(HERE, "g3_tail.npz"), meta=json.dumps(meta), **rec)
    manifest["g3_tail"] = meta

    # G4: Flight end to end on the reference test distribution
    # (tests/test_flight.py:17-35: per-1000-row batch x + 10 * x[0]).
    n, d = 20_000, 256
    x = fill_normal(n, d, seed=11, cluster=1000)
    q = fill_normal(4, d, seed=12)
    port = _free_port()
    server = fenix.Server(os.path.join(root, "flight"), host="127.0.0.1", port=port)
    try:
        flight = fenix.Flight(host="127.0.0.1", port=port)
        schema, batches = _batches(x, 1000)
        flight.make_table("g4/table", pa.RecordBatchReader.from_batches(schema, batches))
        rec = {}
        for metric in METRICS:
            k = 10
            ids = np.full((len(q), k), -1, dtype=np.int64)
            dist = np.full((len(q), k), np.nan, dtype=np.float32)
            for i, qv in enumerate(q):
                t = flight.search(target=qv, source="g4/table", column="vector", metric=metric,
                                  maxval=k)
                ids[i] = t.column("id").to_numpy()
                dist[i] = t.column("__DISTANCE__").to_numpy()
                rec["schema"] = str(t.schema)
            rec[f"{metric}_k{k}_ids"] = ids
            rec[f"{metric}_k{k}_dist"] = dist
        # maxval=None: whole table in original row order (index.py:165)
        t = flight.search(target=q[0], source="g4/table", column="vector", metric="l2")
        rec["l2_all_dist"] = t.column("__DISTANCE__").to_numpy()
        rec["l2_all_ids"] = t.column("id").to_numpy()
        del flight
    finally:
        server.shutdown()
    meta = dict(kind="flight", n=n, d=d, seed=11, qseed=12, nq=4, chunk=1000, cluster=1000,
                sha256=_sha(x), ks=[10], metrics=METRICS)
    np.savez_compressed(os.path.join(HERE, "g4_flight.npz"), meta=json.dumps(meta), **rec)
    manifest["g4_flight"] = meta

    manifest["g6_fp16"] = g6_fp16(fenix, root)
    manifest["g7_nulls"] = g7_nulls(fenix, root)

    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", sorted(manifest))


if __name__ == "__main__":
    main()
