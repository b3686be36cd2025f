"""``call`` — the search entry point — and the coded index, on the GPU.

Drop-in for src/fenix/io/index/index.py of the reference.

``call(root, coding, source, column, target, metric, select, filter, maxval,
probes)`` (index.py:81-170, the function ``Server.do_exchange`` invokes,
flight.py:74).  Same signature, argument meaning, output schema and error
behaviour:

* source: name or list of names under ``<root>/sources`` (index.py:93-97); a
  ``pa.Table`` is also accepted (the reference leaves ``data`` unbound there,
  index.py:93-99, an UnboundLocalError);
* target: Array / ChunkedArray / FixedSizeListScalar / ndarray / Tensor,
  normalised and cast to the column's value type exactly as index.py:101-111
  (``pa.scalar(target, type=column type)``: a wrong length raises
  ``ArrowInvalid``);
* ``coding`` given: the table is joined with its ``__CODED_ID__`` column
  (``load``, index.py:19-34); with ``probes`` the metric defaults to the
  coding's and only rows whose code is among the ``probes`` composites
  nearest the target are searched (index.py:113-126) — the probe set is
  computed on the GPU (fx_code_probe) and turned into a row bitmap there
  (fx_code_mask, AND the filter), which the masked scan consumes without
  loading the excluded rows;
* ``select`` default = every column, then ``__DISTANCE__`` appended
  (index.py:128-129); ``assert metric is not None`` (index.py:131); an unknown
  metric raises ``ValueError()`` (coder.py:50);
* ``filter`` (pc.Expression) restricts the rows before the scan (index.py:161);
* if ``maxval is not None and rows > maxval``: the ``maxval`` nearest rows,
  ascending by distance (index.py:165-168, select_k_unstable), here with the
  deterministic (distance, row) tie-break; otherwise every row in table order
  with its distance (index.py:165 not taken);
* the result is one chunk (``combine_chunks``, index.py:170); ``__DISTANCE__``
  has the column's value type (the UDF's output type, index.py:153-159).

``make`` / ``load`` / ``list`` / ``drop`` (index.py:19-78): index files
``<root>/indexes/<source>/<column>/<name>.arrow`` holding one int64
``__CODED_ID__`` per row, written in the source's batch layout; ``make``
encodes the HBM-resident column with fx_code_assign (MFMA nearest codeword per
codebook) instead of the per-batch pyarrow UDF (index.py:46-49).

What changes underneath: the corpus column is resident in HBM (engine.CACHE)
instead of re-read and scanned per chunk by a Python UDF, top-k is fused into
the gfx950 scan, and only the k winning rows are gathered (chunk-aware, no
``Table.take`` over the whole chunked vector column, index.py:166).
"""

from __future__ import annotations

import os
import threading
from typing import Iterator, List, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import torch
from torch import Tensor

from .. import engine as _engine
from . import _resident, arrow, coder, table

CODE_COL: str = "__CODED_ID__"
DIST_COL: str = "__DISTANCE__"
LOCATION: str = "indexes"


def _quint8_target(target, type: pa.DataType) -> np.ndarray:
    """A quint8 tensor column (ex/arrow/quint8) is searched with a float target
    of prod(shape) values (only the corpus is coded); a wrong length raises
    ArrowInvalid like index.py:111's pa.scalar."""
    if isinstance(target, pa.ChunkedArray):
        target = target.combine_chunks()
    if isinstance(target, pa.ExtensionScalar):
        target = target.to_numpy().dequantize()
    elif isinstance(target, pa.Scalar):
        target = target.values.to_numpy(zero_copy_only=False)
    elif isinstance(target, pa.Array):
        target = target.to_numpy(zero_copy_only=False)
    elif isinstance(target, Tensor):
        target = target.numpy()
    values = np.array(target, dtype=np.float32).ravel()
    d = _engine.list_size(type)
    if values.size != d:
        raise pa.ArrowInvalid(f"target has {values.size} values, the column {d}")
    return values.reshape(1, -1)


def _dist_type(type: pa.DataType) -> pa.DataType:
    """__DISTANCE__ has the column's value type (index.py:153-159); float32 for quint8."""
    return pa.float32() if isinstance(type, pa.ExtensionType) else type.value_type


def _target_values(target, type: pa.DataType) -> np.ndarray:
    """index.py:101-111: normalise the target and cast it to the column type."""
    if isinstance(type, pa.ExtensionType):
        return _quint8_target(target, type)
    if isinstance(target, pa.ChunkedArray):
        target = target.combine_chunks()
    if isinstance(target, pa.Array):
        target = target.to_numpy(zero_copy_only=False)
    if isinstance(target, Tensor):
        target = target.numpy()
    if isinstance(target, np.ndarray):
        if pa.types.is_float16(type.value_type):
            target = np.asarray(target).astype(np.float16)
        target = pa.scalar(target, type=type)
    if not isinstance(target, pa.FixedSizeListScalar):
        raise TypeError(f"unsupported target type {type(target)}")
    if target.type != type:
        target = target.cast(type)
    values = target.values.to_numpy(zero_copy_only=False)
    return np.array(values, dtype=np.float32).reshape(1, -1)  # writable copy


def _filter_mask(data: pa.Table, filter: pc.Expression) -> np.ndarray:
    """Evaluate the row predicate of index.py:161 into a bool mask (nulls drop)."""
    import pyarrow.dataset as ds

    m = ds.dataset(data).to_table(columns={"__m__": filter}).column("__m__")
    return m.fill_null(False).to_numpy(zero_copy_only=False).astype(bool)


def _take_chunked(col: pa.ChunkedArray, rows: np.ndarray) -> pa.Array:
    """Gather ``rows`` of a chunked column without concatenating it first."""
    lens = np.fromiter((len(c) for c in col.chunks), dtype=np.int64, count=col.num_chunks)
    starts = np.concatenate([[0], np.cumsum(lens)])
    ci = np.searchsorted(starts, rows, side="right") - 1
    order = np.argsort(ci, kind="stable")
    pieces = []
    for c in np.unique(ci):
        sel = order[ci[order] == c]
        pieces.append(col.chunk(int(c)).take(pa.array(rows[sel] - starts[c])))
    if not pieces:
        return pa.array([], type=col.type)
    cat = pa.concat_arrays(pieces)
    return cat.take(pa.array(np.argsort(order, kind="stable")))


def take_rows(data: pa.Table, rows: np.ndarray) -> pa.Table:
    rows = np.asarray(rows, dtype=np.int64)
    cols = [_take_chunked(data.column(i), rows) for i in range(data.num_columns)]
    return pa.Table.from_arrays(cols, schema=data.schema)


def _gather_vectors(shards, rows: np.ndarray, type: pa.DataType,
                    null: np.ndarray | None = None,
                    values: np.ndarray | None = None) -> pa.Array:
    """The k winning embeddings, read back from their HBM shards (they are the
    stored Arrow values, staged verbatim) instead of gathered from Arrow
    chunks (index.py:166's take): one H2D of (result position, local row)
    pairs per device, an ``index_select`` per shard placed by ``index_copy_``
    into one result buffer on the first shard's device (other devices' rows
    travel there peer to peer), and ONE D2H into pinned memory with one
    synchronisation — not a round trip per shard (configs[4]'s 8 shards:
    0.63 -> 0.41 ms, profiles/r05_profile_call_cfg4_{before,after}.json,
    DESIGN §6.2).  ``null``: which
    result rows are null slots of the column; their stored values are
    gathered like any other (they were scanned) and the slot stays null, as
    index.py:166's ``take`` keeps validity (tests/golden g7_nulls).
    ``values``: the rows' stored values, already gathered on the device
    behind the search (engine.search_host, one D2H with the distances); only
    the Arrow array is built then."""
    d = _engine.list_size(type)
    _, tdt, ndt = _engine.value_dtype(type)
    m = rows.size
    if values is not None:
        out = np.ascontiguousarray(values).view(ndt).reshape(m, d)
    elif m == 0 or not shards:
        out = np.empty((m, d), dtype=ndt)
    else:
        bases = np.array([s.row_base for s in shards], dtype=np.int64)
        sizes_n = np.array([s.n for s in shards], dtype=np.int64)
        if np.any(np.diff(bases) < 0):
            raise ValueError("_gather_vectors: shards must be in row order")
        which = np.searchsorted(bases, rows, side="right") - 1
        if np.any(which < 0) or np.any(rows - bases[np.maximum(which, 0)] >= sizes_n[which]):
            raise ValueError("_gather_vectors: a result row lies outside every shard")
        dev0 = shards[0].data.device
        with torch.cuda.device(dev0):
            acc = torch.empty((m, d), dtype=shards[0].data.dtype, device=dev0)
            by_dev = {}
            for i, s in enumerate(shards):
                by_dev.setdefault(s.data.device, []).append(i)
            for dev, idx in by_dev.items():
                # (position in the result, local row) of every row this device holds
                pos = [np.nonzero(which == i)[0] for i in idx]
                sizes = [p.size for p in pos]
                if not sum(sizes):
                    continue
                pairs = np.empty((2, sum(sizes)), dtype=np.int64)
                pairs[0] = np.concatenate(pos)
                pairs[1] = rows[pairs[0]] - np.repeat(bases[idx], sizes)
                with torch.cuda.device(dev):
                    pd = torch.from_numpy(pairs).to(dev)
                    off = 0
                    for i, c in zip(idx, sizes):
                        if c:
                            g = shards[i].data.index_select(0, pd[1, off : off + c])
                            p = pd[0, off : off + c]
                            if dev != dev0:
                                g, p = g.to(dev0), p.to(dev0)
                            acc.index_copy_(0, p, g)
                        off += c
                    if dev != dev0:  # the peer copies above read on this device's stream
                        torch.cuda.current_stream(dev0).wait_stream(torch.cuda.current_stream(dev))
            host = torch.empty((m, d), dtype=acc.dtype, pin_memory=True)
            host.copy_(acc, non_blocking=True)
            torch.cuda.current_stream(dev0).synchronize()
        out = host.numpy().view(ndt)
    mask = pa.array(null) if null is not None and null.any() else None
    lists = pa.FixedSizeListArray.from_arrays(pa.array(out.ravel()), list_size=d, mask=mask)
    if isinstance(type, pa.ExtensionType):  # quint8 codes: same type, same parameters
        return pa.ExtensionArray.from_storage(type, lists.cast(type.storage_type))
    return lists.cast(type)


def _null_mask(col: pa.ChunkedArray) -> np.ndarray:
    """bool[rows]: which slots of ``col`` are null."""
    return pc.is_null(col).to_numpy(zero_copy_only=False).astype(bool)


def _take_columns(data: pa.Table, cols: List[str], rows: np.ndarray, column: str, shards,
                  version, values: np.ndarray | None = None) -> pa.Table:
    """select(cols).take(rows) without Table.take's concatenation of the whole
    chunked vector column (index.py:166; 0.75 s per 1M x 768 measured);
    ``values``: the vector column's rows, gathered on the device already."""
    arrays = []
    for c in cols:
        col = data.column(c)
        if c == column:
            null = None
            if (col.null_count if version is None else _resident.null_count(version, c, col)):
                null = (_resident.null_mask(version, c, col) if version is not None
                        else _null_mask(col))[rows]
            arrays.append(_gather_vectors(shards, rows, col.type, null, values))
        elif version is None:
            arrays.append(_take_chunked(col, rows))
        else:
            arrays.append(_resident.combined(version, c, col).take(pa.array(rows)))
    return pa.Table.from_arrays(arrays, schema=pa.schema([data.schema.field(c) for c in cols],
                                                         metadata=data.schema.metadata))


_register_lock = threading.Lock()


def register_distance(metric: str, type: pa.DataType) -> str:
    """Register (once) the pyarrow scalar UDF ``distance:{metric}:{T}:{D}``.

    The reference registers it lazily inside ``call`` (index.py:133-159):
    ``(x: fixed_size_list<T>[D] array, q: same-type scalar) -> T array``, one
    ``coder.distance`` per Arrow chunk.  ``call`` here does not need it (the
    scan fuses distance + top-k), but code that invokes the function through
    ``pc.call_function`` keeps working: each chunk is evaluated by the GPU
    distance kernel (fx_knn_distances).  Returns the function name.
    """
    coder.metric_id(metric)
    _engine.value_dtype(type)
    func = f"distance:{metric}:{type.value_type}:{type.list_size}"
    with _register_lock:
        if func in pc.list_functions():
            return func

        def dist(ctx: pc.UdfContext, x: pa.FixedSizeListArray,
                 q: pa.FixedSizeListScalar) -> pa.Array:
            from . import torch as io_torch

            xv = io_torch.from_arrow(x)
            qv = torch.from_numpy(_target_values(q, type))
            out = coder.distance(qv, xv, metric)[0]
            return pa.array(out.numpy(), type=type.value_type)

        pc.register_scalar_function(
            dist,
            func,
            {"summary": "fenix distance (GPU)", "description": "coder.py:38-50 on gfx950"},
            {"x": type, "q": type},
            type.value_type,
        )
    return func


def _index_path(root: str, name: str, source: str, column: str) -> str:
    return os.path.join(root, LOCATION, source, column, name + ".arrow")


def load(root: str, name: str, source: str | Sequence[str], column: str) -> pa.Table:
    """index.py:19-34: the source table(s) with their ``__CODED_ID__`` column."""
    if isinstance(source, str):
        coder.load(root, name)

        path = _index_path(root, name, source, column)

        return table.join(table.load(root, source), arrow.load(path), axis=1)

    assert isinstance(source, Sequence) and not isinstance(source, str)
    return table.join(*[load(root, name, s, column) for s in source])


def _encode(root: str, source: str, column: str, code: coder.Coding) -> tuple:
    """Composite code of every row of one source: fx_code_assign over its HBM
    shards.  -> (source table, int64 codes)."""
    _, t = _resident.load_table(table.path(root, source))
    parts = [(table.path(root, source), t)]
    out = np.zeros(t.num_rows, dtype=np.int64)
    m = coder.metric_id(code["config"]["metric"])
    for s, _, start in _resident.shards(parts, column, _engine.devices()):
        dev = s.data.device
        with torch.cuda.device(dev):
            _, c, _ = _engine.Engine.get(dev).code_assign(s.data, code["tensor"], m)
            out[start : start + s.n] = c.cpu().numpy()
    return t, out


def make(root: str, name: str, source: str | Sequence[str], column: str) -> pa.Table:
    """index.py:37-65: encode the source(s) with the coding ``name`` and write
    the code column, one record batch per source batch."""
    if isinstance(source, str):
        path = _index_path(root, name, source, column)

        os.makedirs(os.path.dirname(path), exist_ok=True)

        code = coder.load(root, name)
        t, codes = _encode(root, source, column, code)

        def record_batch_generator():
            start = 0
            for batch in t.to_batches():
                n = batch.num_rows
                yield pa.record_batch([pa.array(codes[start : start + n])], names=[CODE_COL])
                start += n

        arrow.make(
            path,
            pa.RecordBatchReader.from_batches(
                pa.schema({CODE_COL: pa.int64()}),
                record_batch_generator(),
            ),
        )

        return load(root, name, source, column)

    assert isinstance(source, Sequence) and not isinstance(source, str)
    return table.join(*[make(root, name, s, column) for s in source])


def list(root: str) -> Iterator[str]:
    """index.py:68-71: index files as ``<source>/<column>/<name>``."""
    base = os.path.join(root, LOCATION)
    for dirpath, _, files in os.walk(base):
        for f in sorted(files):
            if f.endswith(".arrow"):
                rel = os.path.relpath(os.path.join(dirpath, f), base)
                yield rel.removesuffix(".arrow")


def drop(root: str, name: str, source: str, column: str) -> None:
    path = _index_path(root, name, source, column)

    if os.path.exists(path):
        os.unlink(path)


def _unpack(words: torch.Tensor, n: int) -> np.ndarray:
    w = words.cpu().numpy().view(np.uint8)
    return np.unpackbits(w, bitorder="little")[:n].astype(bool)


def _probe_masks(code: coder.Coding, q: np.ndarray, probes: int, shard_info, code_parts,
                 masks):
    """index.py:113-126 on the device: the ``probes`` composites nearest the
    target (with the coding's metric, as pc.call_function(coding, ...) does),
    then per shard bit r = code[r] in that set AND the filter bit.
    -> (per-shard masks, per-shard kept rows, kept-row total, lazy host mask)."""
    nb = int(code["config"]["num_codebooks"])
    ks = int(code["config"]["codebook_size"])
    total = ks**nb
    if probes > total:
        raise RuntimeError("selected index k out of range")  # torch.topk in coder.call
    dev0 = shard_info[0][0].data.device if shard_info else _engine.devices()[0]
    with torch.cuda.device(dev0):
        eng0 = _engine.Engine.get(dev0)
        cw = code["tensor"].to(dev0, torch.float32).contiguous()
        qd = torch.from_numpy(q).to(dev0)
        d = eng0.distances(_engine.Shard(cw.reshape(nb * ks, -1), 0), qd,
                           coder.metric_id(code["config"]["metric"]))
        _, _, sel = eng0.code_probe(d.reshape(1, nb, ks), int(probes), sel=True)
    out, counts = [], []
    for i, (s, src, start) in enumerate(shard_info):
        dev = s.data.device
        with torch.cuda.device(dev):
            key, t = code_parts[src]
            rc = _resident.code_column(key, t, CODE_COL, dev)[start : start + s.n]
            mk, cnt = _engine.Engine.get(dev).code_mask(
                rc, sel[0].to(dev), total, masks[i] if masks is not None else None)
        out.append(mk)
        counts.append(cnt)
    counts = [int(c.item()) for c in counts]
    n_rows = sum(counts)

    def host() -> np.ndarray:
        if not out:
            return np.zeros(0, dtype=bool)
        return np.concatenate([_unpack(mk, s.n) for mk, (s, _, _) in zip(out, shard_info)])

    return out, counts, n_rows, host


def call(
    root: str,
    coding: str | None,
    source: str | Sequence[str] | pa.Table,
    column: str,
    target: pa.Array | pa.ChunkedArray | pa.FixedSizeListScalar | np.ndarray | Tensor,
    metric: str | None = None,
    select: Sequence[str] | None = None,
    filter: pc.Expression | None = None,
    maxval: int | None = None,
    probes: int | None = None,
) -> pa.Table:
    code_parts = None
    if isinstance(source, pa.Table):
        data, parts, version = source, [(None, source)], None
    else:
        names = [source] if isinstance(source, str) else [*source]
        data, parts, version = _resident.sources(root, names)
        if coding is not None:
            coder.load(root, coding)
            code_parts = [_resident.load_table(_index_path(root, coding, s, column))
                          for s in names]
            data = table.join(*[table.join(t, it, axis=1)
                                for (_, t), (_, it) in zip(parts, code_parts)])
            version = version + tuple(k for k, _ in code_parts)

    type = data.schema.field(column).type
    q = _target_values(target, type)

    code = None
    if coding is not None and probes is not None:
        code = coder.load(root, coding)

        if metric is None:
            metric = code["config"]["metric"]

    select = [*select] if select is not None else data.column_names
    select = select + [DIST_COL]

    assert metric is not None

    m = coder.metric_id(metric)
    _engine.value_dtype(type)

    fmask = _filter_mask(data, filter) if filter is not None else None
    shard_info = _resident.shards(parts, column, _engine.devices())
    shards = [s for s, _, _ in shard_info]
    masks = None
    if fmask is not None:
        masks = [_engine.device_mask(fmask[s.row_base : s.row_base + s.n], s.data.device)
                 for s in shards]
    if code is not None:
        if code_parts is None:
            raise ValueError("a probe search needs named sources with an index")
        masks, counts, n_rows, host_mask = _probe_masks(code, q, probes, shard_info, code_parts,
                                                         masks)
    else:
        n_rows = int(fmask.sum()) if fmask is not None else data.num_rows
        host_mask = (lambda: fmask) if fmask is not None else None
        counts = [int(fmask[s.row_base : s.row_base + s.n].sum()) for s in shards] \
            if fmask is not None else None

    qt = torch.from_numpy(q)
    base_cols = [c for c in dict.fromkeys(select) if c != DIST_COL]

    if maxval is not None and n_rows > maxval:
        # the k winning vectors are gathered on the device behind the scan and
        # come back with the distances (one synchronisation)
        dist, rows, vecs = _engine.search_host(shards, qt, m, int(maxval), masks, counts,
                                               gather=column in base_cols)
        dist, rows = dist[0], rows[0]
        keep = rows >= 0
        dist, rows = dist[keep], rows[keep]
        vecs = vecs[0][keep] if vecs is not None else None
        out = _take_columns(data, base_cols, rows, column, shards, version, vecs)
    else:
        dist = _engine.distances_all(shards, qt, m, masks)[0]
        out = data.select(base_cols)
        if host_mask is not None:
            hm = host_mask()
            out = out.filter(pa.array(hm))
            dist = dist[hm]
    dt = _dist_type(type)
    out = out.append_column(DIST_COL, pa.array(dist.astype(dt.to_pandas_dtype()), type=dt))
    return out.select(select).combine_chunks()
