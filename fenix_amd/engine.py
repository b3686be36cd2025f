"""Device-resident corpus shards and the kernel launch wrappers.

This is the MI355X replacement for the per-call corpus handling of the
reference's ``io.index.call`` (src/fenix/io/index/index.py:81-170):

* the reference re-opens the Arrow IPC file on every search (index.py:97 ->
  table.py:12-21 -> arrow.py:6-8) and hands every chunk to a Python UDF that
  runs ``coder.distance`` on the CPU (index.py:137-162);
* here the embedding column is staged ONCE into HBM (``stage_column``), keyed
  by (path, file version, column, device) so a rewrite by ``do_put`` restages it
  (``CorpusCache``), and every search is one fused scan + merge on the GPU
  (``Engine.search`` -> ``fx_knn_search`` / ``fx_topk_merge``).

PyTorch is used for device memory, streams and copies only; all arithmetic is
in the HIP library.  Nothing here falls back to the CPU.
"""

from __future__ import annotations

import ctypes
import os
import threading
import warnings
import weakref
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa
import torch

from . import _lib, coalesce

_PINNED_CHUNK = 256 << 20  # bytes per pinned staging buffer


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError(
            "fenix_amd requires a ROCm GPU (torch.cuda.is_available() is False); "
            "there is no CPU fallback"
        )


def _is_quint8(t: pa.DataType) -> bool:
    return isinstance(t, pa.ExtensionType) and t.extension_name == "tensor::qint8"


def list_size(t: pa.DataType) -> int:
    return (t.storage_type if isinstance(t, pa.ExtensionType) else t).list_size


def qparams(t: pa.DataType) -> Tuple[float, int]:
    """(scale, zero point) of a quint8 tensor column (ex/arrow/quint8); (1, 0) otherwise."""
    if _is_quint8(t):
        return float(t.scale), int(t.shift)
    return 1.0, 0


def value_dtype(t: pa.DataType) -> Tuple[int, torch.dtype, np.dtype]:
    """fixed_size_list<float32|float16>[D] or a quint8 tensor column ->
    (C-ABI dtype, torch dtype, numpy dtype)."""
    if _is_quint8(t):
        return _lib.DTYPE_QU8, torch.uint8, np.dtype(np.uint8)
    if not pa.types.is_fixed_size_list(t):
        raise TypeError(f"embedding column must be fixed_size_list<float>[D], got {t}")
    v = t.value_type
    if pa.types.is_float32(v):
        return _lib.DTYPE_F32, torch.float32, np.dtype(np.float32)
    if pa.types.is_float16(v):
        return _lib.DTYPE_F16, torch.float16, np.dtype(np.float16)
    raise NotImplementedError(f"fenix_amd scans float32/float16 embeddings, got {v}")


def _chunk_values(chunk: pa.FixedSizeListArray, np_dtype: np.dtype) -> np.ndarray:
    """Zero-copy [len, D] view of the STORED values of one chunk.

    Like the reference's ``io.torch.from_arrow`` (src/fenix/io/torch/torch.py:6-10)
    validity is ignored (a null slot's stored values are scanned), but unlike it
    the parent's array offset is honoured (from_arrow reads ``.values`` from
    element 0 even for a sliced array).  Nulls inside the VALUES (a null slot
    built from a Python ``None``) raise what the reference's ``from_dlpack``
    raises there, ``ArrowTypeError`` (tests/golden g7_nulls); a null slot whose
    values are stored (validity on the list array only) is scanned.
    """
    if isinstance(chunk, pa.ExtensionArray):
        chunk = chunk.storage
    d = chunk.type.list_size
    vals = chunk.values
    if vals.null_count and vals.slice(chunk.offset * d, len(chunk) * d).null_count:
        raise pa.ArrowTypeError("Can only use DLPack on arrays with no nulls.")
    buf = vals.buffers()[1]
    start = (vals.offset + chunk.offset * d) * np_dtype.itemsize
    count = len(chunk) * d
    return np.frombuffer(buf, dtype=np_dtype, count=count, offset=start).reshape(len(chunk), d)


def stage_column(col: pa.ChunkedArray, device: torch.device) -> torch.Tensor:
    """Copy an Arrow fixed_size_list column into one contiguous [n, D] HBM tensor
    through pinned bounce buffers (one H2D copy per ~256 MB, not per chunk)."""
    _, tdt, ndt = value_dtype(col.type)
    d = list_size(col.type)
    n = len(col)
    out = torch.empty((n, d), dtype=tdt, device=device)
    if n == 0:
        return out
    row_bytes = d * ndt.itemsize
    rows_per_buf = max(1, _PINNED_CHUNK // row_bytes)
    bufs = [torch.empty((rows_per_buf, d), dtype=tdt, pin_memory=True) for _ in range(2)]
    events = [None, None]
    stream = torch.cuda.current_stream(device)
    slot, fill, dst = 0, 0, 0
    host = bufs[0].numpy()

    def flush(slot: int, fill: int, dst: int) -> None:
        out[dst : dst + fill].copy_(bufs[slot][:fill], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        events[slot] = ev

    for chunk in col.chunks:
        view = _chunk_values(chunk, ndt)
        pos = 0
        while pos < view.shape[0]:
            take = min(rows_per_buf - fill, view.shape[0] - pos)
            host[fill : fill + take] = view[pos : pos + take]
            fill += take
            pos += take
            if fill == rows_per_buf:
                flush(slot, fill, dst)
                dst += fill
                slot ^= 1
                fill = 0
                if events[slot] is not None:
                    events[slot].synchronize()
                host = bufs[slot].numpy()
    if fill:
        flush(slot, fill, dst)
    torch.cuda.current_stream(device).synchronize()
    return out


@dataclass
class Shard:
    """One contiguous row range of the searched table, resident in HBM."""

    data: torch.Tensor  # [n, D] float32 / float16 / uint8 (quint8 codes)
    row_base: int  # global row of local row 0 (multi-source numbering, table.py:19-21)
    scale: float = 1.0  # quint8: value = scale * (code - zero_point)
    zero_point: int = 0

    @property
    def n(self) -> int:
        return int(self.data.shape[0])

    @property
    def d(self) -> int:
        return int(self.data.shape[1])

    @property
    def dtype_id(self) -> int:
        if self.data.dtype == torch.uint8:
            return _lib.DTYPE_QU8
        return _lib.DTYPE_F32 if self.data.dtype == torch.float32 else _lib.DTYPE_F16

    def corpus(self) -> "_lib.Corpus":
        """struct fx_corpus for the _ex entry points."""
        return _lib.Corpus(self.data.data_ptr(), self.dtype_id, self.n, self.d, self.row_base,
                           self.scale, self.zero_point)


@dataclass
class Piece:
    """The part of one staged column that lives on one device."""

    device: torch.device
    data: torch.Tensor  # [rows, D]
    start: int  # first row of the column held here


@dataclass
class ScanState:
    """What ``Engine.scan`` hands to ``Engine.reduce``: the workspace and the
    filter image (None: the scan read none) with its width in bits."""

    ws: torch.Tensor
    image: Optional[torch.Tensor]
    rowinfo: Optional[torch.Tensor]
    bits: int


@dataclass
class _Entry:
    key: tuple
    table: pa.Table
    pieces: List[Piece]


def devices() -> List[torch.device]:
    """Devices a server process shards its corpora over.

    ``FENIX_AMD_DEVICES``: comma-separated ordinals, or ``all``; default: the
    current device only.  Repeating an ordinal (``0,0``) is allowed and makes
    several shards share one GPU (used to exercise the multi-device path on a
    single-GPU machine)."""
    require_gpu()
    env = os.environ.get("FENIX_AMD_DEVICES", "").strip()
    if env == "all":
        return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    if env:
        return [torch.device("cuda", int(v)) for v in env.split(",") if v.strip()]
    single = os.environ.get("FENIX_AMD_DEVICE")
    return [torch.device("cuda", int(single) if single else torch.cuda.current_device())]


def stage_sharded(col: pa.ChunkedArray, devs: Sequence[torch.device]) -> List[Piece]:
    """Row-range shards of one column over ``devs`` (SURVEY §8(e) partitioning)."""
    from .distributed import shard_rows

    pieces = []
    for i, dev in enumerate(devs):
        start, count = shard_rows(len(col), len(devs), i)
        with torch.cuda.device(dev):
            pieces.append(Piece(dev, stage_column(col.slice(start, count), dev), start))
    return pieces


def _budget_bytes(dev: int) -> int:
    """HBM the resident caches may hold on device ``dev``.

    ``FENIX_AMD_HBM_BUDGET``: bytes (an integer), or a fraction of the device's
    memory (a number <= 1); default 0.85 of it, the rest left to workspaces,
    query batches and the caller's own tensors."""
    env = os.environ.get("FENIX_AMD_HBM_BUDGET", "").strip()
    total = torch.cuda.get_device_properties(dev).total_memory
    if env:
        v = float(env)
        return int(v * total) if v <= 1.0 else int(v)
    return int(0.85 * total)


class Residency:
    """LRU accounting of the HBM held by the resident caches: staged corpus
    shards (``CorpusCache``) and filter images (``Engine.filter_image``).

    The reference holds nothing between calls (it re-maps the Arrow file per
    search, src/fenix/io/index/index.py:97); a server keeping tables resident
    must bound them.  Before a cache allocates, ``reserve`` evicts least-
    recently-used entries until the new bytes fit the device's budget:
    filter images first (rebuilt in ~10 ms, and a search is correct without
    one), then corpus entries (restaged from the Arrow file on their next
    search).  An entry in use by a running search keeps its tensors alive
    through that search's own references; eviction only drops the cache's."""

    IMAGE, CORPUS = 0, 1

    def __init__(self) -> None:
        self._lock = threading.RLock()
        # key -> (kind, {device index: bytes}, evict callback); order = LRU first
        self._items: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.evictions = 0

    def used(self, dev: int) -> int:
        with self._lock:
            return sum(b.get(dev, 0) for _, b, _ in self._items.values())

    def add(self, key: tuple, kind: int, nbytes: Dict[int, int], evict) -> None:
        with self._lock:
            self._items[key] = (kind, dict(nbytes), evict)
            self._items.move_to_end(key)

    def touch(self, key: tuple) -> None:
        with self._lock:
            if key in self._items:
                self._items.move_to_end(key)

    def remove(self, key: tuple) -> None:
        with self._lock:
            self._items.pop(key, None)

    def reserve(self, need: Dict[int, int], keep: Sequence[tuple] = (),
                kinds: Sequence[int] = (0, 1)) -> bool:
        """Evict entries of ``kinds`` (LRU first, images before corpora) until
        ``need`` more bytes fit every listed device's budget; False when they
        cannot.  A filter image reserves with ``kinds=(IMAGE,)``: an optional
        image never evicts a corpus (it could be the one it is built for).
        The victims' callbacks run after this object's lock is released (they
        take their cache's lock)."""
        victims = []
        ok = True
        with self._lock:
            for dev, extra in need.items():
                budget = _budget_bytes(dev)
                used = self.used(dev)
                for kind in [k for k in (self.IMAGE, self.CORPUS) if k in kinds]:
                    for key in [k for k, v in self._items.items()
                                if v[0] == kind and v[1].get(dev, 0) > 0 and k not in keep]:
                        if used + extra <= budget:
                            break
                        item = self._items.pop(key)
                        used -= item[1].get(dev, 0)
                        victims.append(item)
                ok = ok and used + extra <= budget
        for item in victims:
            self.evictions += 1
            item[2]()
        return ok

    def evict(self, key: tuple) -> None:
        with self._lock:
            item = self._items.pop(key, None)
        if item is not None:
            self.evictions += 1
            item[2]()

    def evict_all(self, kind: Optional[int] = None) -> None:
        with self._lock:
            keys = [k for k, v in self._items.items() if kind is None or v[0] == kind]
        for k in keys:
            self.evict(k)


RESIDENT = Residency()


def _with_oom_retry(fn):
    """Run ``fn``; on a device out-of-memory error evict every cached image and
    corpus once, release torch's cached blocks and run it again."""
    try:
        return fn()
    except torch.cuda.OutOfMemoryError:
        RESIDENT.evict_all()
        torch.cuda.empty_cache()
        return fn()


class CorpusCache:
    """HBM-resident embedding columns keyed by (path, file version, column,
    devices), within the devices' HBM budgets (``Residency``)."""

    def __init__(self) -> None:
        # re-entrant: staging may evict this cache's own older entries
        self._lock = threading.RLock()
        self._entries: Dict[tuple, _Entry] = {}

    @staticmethod
    def _key(path: str, column: str, devs: Sequence[torch.device]) -> tuple:
        from .io.arrow import file_version

        return (os.path.abspath(path), file_version(path), column, tuple(str(d) for d in devs))

    def get(self, path: str, table: pa.Table, column: str,
            devs: Sequence[torch.device]) -> _Entry:
        key = self._key(path, column, devs)
        rkey = ("corpus", id(self)) + key
        with self._lock:
            hit = self._entries.get(key)
            if hit is not None:
                RESIDENT.touch(rkey)
                return hit
            # drop stale versions of the same file/column/devices
            for k in [k for k in self._entries if k[0] == key[0] and k[2:] == key[2:]]:
                self._drop(k)
            col = table.column(column)
            need = self._bytes(col, devs)
            RESIDENT.reserve(need)
            entry = _Entry(key, table, _with_oom_retry(lambda: stage_sharded(col, devs)))
            self._entries[key] = entry
            RESIDENT.add(rkey, Residency.CORPUS, need, lambda: self._evicted(key))
            return entry

    @staticmethod
    def _bytes(col: pa.ChunkedArray, devs: Sequence[torch.device]) -> Dict[int, int]:
        from .distributed import shard_rows

        _, _, ndt = value_dtype(col.type)
        row = list_size(col.type) * ndt.itemsize
        need: Dict[int, int] = {}
        for i, dev in enumerate(devs):
            _, count = shard_rows(len(col), len(devs), i)
            need[dev.index] = need.get(dev.index, 0) + count * row
        return need

    def _evicted(self, key: tuple) -> None:
        with self._lock:
            self._entries.pop(key, None)

    def _drop(self, key: tuple) -> None:
        self._entries.pop(key, None)
        RESIDENT.remove(("corpus", id(self)) + key)

    def __contains__(self, key: tuple) -> bool:
        return key in self._entries

    def clear(self) -> None:
        with self._lock:
            for k in list(self._entries):
                self._drop(k)


CACHE = CorpusCache()


class Engine:
    """Launches the HIP kernels on one device; one instance per device."""

    _instances: Dict[int, "Engine"] = {}
    _ilock = threading.Lock()

    def __init__(self, device: torch.device) -> None:
        self.device = device
        self.lock = threading.Lock()
        self._ws: Optional[torch.Tensor] = None
        # fp16 filter images of f32 corpora, by id of the corpus tensor:
        # (signature, image, rowinfo); dropped when the tensor is collected
        self._images: Dict[int, tuple] = {}

    @classmethod
    def get(cls, device: Optional[torch.device] = None) -> "Engine":
        require_gpu()
        _lib.load()
        if device is None:
            env = os.environ.get("FENIX_AMD_DEVICE")
            idx = int(env) if env is not None else torch.cuda.current_device()
            device = torch.device("cuda", idx)
        with cls._ilock:
            eng = cls._instances.get(device.index)
            if eng is None:
                eng = cls(device)
                cls._instances[device.index] = eng
            return eng

    def _workspace(self, nbytes: int) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=self.device)
        return self._ws

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def filter_image(self, shard: Shard, nq: int, k: int, metric: int, build: bool = True
                     ) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor], int]:
        """The filter image of an f32 (or, int8 images, f16) shard for a search that runs the batched
        filter (fx_filter_image_used): (image, rowinfo, bits), bits 8
        (fx_filter_image8, the default) or 16 (fx_filter_image) as the library
        option "filter_image" says, built on first use and kept while the
        corpus tensor lives and is unmodified; (None, None, 0) when the search
        does not read one, when the option is 0, or when the HBM budget
        (``Residency``) cannot hold it without evicting a corpus.  The filter only
        selects candidates, which are rescored from the f32 rows, so results
        never depend on whether or which image is used.

        Invariant: an image is valid only while its corpus is unchanged.
        Staleness is detected through the tensor's identity, data pointer,
        shape and torch version counter, which every torch write and
        ``Engine.fill`` bump; a writer that bypasses torch (a raw pointer
        through ctypes, DLPack, another library) must call
        ``invalidate_image`` afterwards.

        The image is built on the caller's current stream; a search on another
        stream waits for the build through an event recorded after it, and the
        image is recorded on that stream, so an eviction while the search runs
        cannot hand its memory to another allocation early."""
        none = (None, None, 0)
        bits = _lib.get_option("filter_image")
        # int8 images serve f32 and f16 corpora, fp16 images f32 ones
        if ((shard.dtype_id != _lib.DTYPE_F32
             and not (bits == 8 and shard.dtype_id == _lib.DTYPE_F16)) or bits not in (8, 16)
                or not _lib.filter_image_used(shard.n, shard.d, shard.dtype_id, nq, k, metric)):
            return none
        t = shard.data
        # an unaligned corpus takes the scan's scalar-load variant, never the
        # batched filter (fx_filter_image_used assumes 16-B aligned rows)
        if not t.is_contiguous() or t.data_ptr() % 16 != 0:
            return none
        key = id(t)
        rkey = ("image", self.device.index, key)
        sig = (t.data_ptr(), tuple(t.shape), t._version, bits)
        hit = self._images.get(key)
        if hit is not None and hit[0] == sig:
            RESIDENT.touch(rkey)
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(hit[3])
            hit[1].record_stream(cur)
            hit[2].record_stream(cur)
            return hit[1], hit[2], bits
        if not build:  # (reduce: only the image its scan used, never a new one)
            return none
        self.invalidate_image(t)  # a stale image: free it before building the new one
        n, d = shard.n, shard.d
        L = _lib.load()
        size_fn = L.fx_filter_image8_bytes if bits == 8 else L.fx_filter_image_bytes
        ib, rb = ctypes.c_size_t(0), ctypes.c_size_t(0)
        _lib.check(size_fn(n, d, ctypes.byref(ib), ctypes.byref(rb)))
        need = ib.value + rb.value
        if not RESIDENT.reserve({self.device.index: need}, kinds=(Residency.IMAGE,)):
            return none
        free, _ = torch.cuda.mem_get_info(self.device)
        cached = torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
        if need + (1 << 30) > free + cached:
            return none
        try:
            img = torch.empty((ib.value,), dtype=torch.uint8, device=self.device)
            info = torch.empty((rb.value // 4,), dtype=torch.float32, device=self.device)
        except torch.cuda.OutOfMemoryError:
            return none  # the f32 filter (no image) is always correct
        if bits == 8:
            _lib.check(L.fx_filter_image8_typed(_ptr(t), shard.dtype_id, n, d, _ptr(img),
                                                _ptr(info), self._stream()))
        else:
            _lib.check(L.fx_filter_image(_ptr(t), n, d, _ptr(img), _ptr(info), self._stream()))
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._images[key] = (sig, img, info, ev)
        RESIDENT.add(rkey, Residency.IMAGE, {self.device.index: need},
                     lambda: self._images.pop(key, None))
        weakref.finalize(t, self._drop_image, key)
        return img, info, bits

    def clear_images(self) -> None:
        """Drop every filter image this engine holds."""
        for key in list(self._images):
            self._drop_image(key)

    def invalidate_image(self, t: torch.Tensor) -> None:
        """Drop the filter image of corpus tensor ``t`` (for writers that
        modify it behind torch's version counter)."""
        self._drop_image(id(t))

    def _drop_image(self, key: int) -> None:
        self._images.pop(key, None)
        RESIDENT.remove(("image", self.device.index, key))

    def search_shard(self, shard: Shard, queries: torch.Tensor, metric: int, k: int,
                     mask: Optional[torch.Tensor], out_dist: torch.Tensor,
                     out_row: torch.Tensor) -> None:
        """fx_knn_search on one shard.  queries [nq, D] f32 on device; caller holds lock."""
        nq = queries.shape[0]
        if shard.dtype_id == _lib.DTYPE_QU8:
            self._search_ex(shard, None, -1, queries, metric, k, mask, out_dist, out_row)
            return
        img, info, bits = self.filter_image(shard, nq, k, metric)
        ws = self._workspace(_lib.knn_workspace_bytes(shard.n, shard.d, shard.dtype_id, nq, k,
                                                      img8=bits == 8))
        self._hold(shard.data)
        L = _lib.load()
        _lib.check(
            (L.fx_knn_search_img8 if bits == 8 else L.fx_knn_search_img)(
                _ptr(shard.data), shard.dtype_id, shard.n, shard.d, shard.row_base,
                _ptr(img), _ptr(info), _ptr(queries), nq, metric, k, _ptr(mask), _ptr(ws),
                ws.numel(), _ptr(out_dist), _ptr(out_row), self._stream(),
            )
        )

    def _search_ex(self, shard: Shard, rows: Optional[torch.Tensor], nrows: int,
                   queries: torch.Tensor, metric: int, k: int, mask: Optional[torch.Tensor],
                   out_dist: torch.Tensor, out_row: torch.Tensor) -> None:
        """fx_knn_search_ex (any dtype incl. quint8 codes, optional row list); caller holds lock."""
        c = shard.corpus()
        nq = queries.shape[0]
        ws = self._workspace(_lib.search_ex_workspace_bytes(c, nrows, nq, k))
        self._hold(shard.data)
        _lib.check(_lib.load().fx_knn_search_ex(
            ctypes.byref(c), _ptr(rows), nrows, _ptr(queries), nq, metric, k, _ptr(mask),
            _ptr(ws), ws.numel(), _ptr(out_dist), _ptr(out_row), self._stream()))

    def _hold(self, *tensors: Optional[torch.Tensor]) -> None:
        """Record the current stream on cached tensors a launch reads (corpus
        shards, filter images): if a cache evicts them while the kernels run on
        a stream other than the one they were allocated on, the caching
        allocator waits for this stream before reusing their memory."""
        cur = torch.cuda.current_stream(self.device)
        for t in tensors:
            if t is not None and t.is_cuda:
                t.record_stream(cur)

    def scan(self, shard: Shard, queries: torch.Tensor, metric: int, k: int,
             mask: Optional[torch.Tensor] = None) -> "ScanState":
        """Phase 1 of search_shard (fx_knn_scan / fx_knn_scan_img8): returns the
        state ``reduce`` completes — the workspace and the exact filter image
        (and its width) the scan planned with, held until the reduce, so the
        pair never plans differently (an image evicted or rebuilt in between
        would make fx_knn_reduce read a filter workspace as scan lists)."""
        nq = queries.shape[0]
        img, info, bits = self.filter_image(shard, nq, k, metric)
        ws = self._workspace(_lib.knn_workspace_bytes(shard.n, shard.d, shard.dtype_id, nq, k,
                                                      img8=bits == 8))
        self._hold(shard.data)
        L = _lib.load()
        _lib.check(
            (L.fx_knn_scan_img8 if bits == 8 else L.fx_knn_scan_img)(
                _ptr(shard.data), shard.dtype_id, shard.n, shard.d, shard.row_base,
                _ptr(img), _ptr(info), _ptr(queries), nq, metric, k, _ptr(mask), _ptr(ws),
                ws.numel(), self._stream(),
            )
        )
        return ScanState(ws, img, info, bits)

    def reduce(self, shard: Shard, queries: torch.Tensor, metric: int, k: int, state: "ScanState",
               out_dist: torch.Tensor, out_row: torch.Tensor,
               mask: Optional[torch.Tensor] = None) -> None:
        """Phase 2 of search_shard (fx_knn_reduce), same arguments as scan plus
        its state.  A scan that received an int8 filter image is completed by
        fx_knn_reduce_img8 with that same image (the library may have planned
        a single query through the filter)."""
        nq = queries.shape[0]
        ws = state.ws
        L = _lib.load()
        if state.bits == 8 and state.image is not None:
            _lib.check(L.fx_knn_reduce_img8(
                _ptr(shard.data), shard.dtype_id, shard.n, shard.d, shard.row_base,
                _ptr(state.image), _ptr(queries), nq, metric, k, _ptr(mask), _ptr(ws), ws.numel(),
                _ptr(out_dist), _ptr(out_row), self._stream()))
            return
        _lib.check(
            L.fx_knn_reduce(
                _ptr(shard.data), shard.dtype_id, shard.n, shard.d, shard.row_base,
                _ptr(queries), nq, metric, k, _ptr(mask), _ptr(ws), ws.numel(),
                _ptr(out_dist), _ptr(out_row), self._stream(),
            )
        )

    def filter_counts(self, shard: Shard, nq: int, metric: int, k: int,
                      state: "ScanState") -> Tuple[Optional[np.ndarray], int]:
        """fx_knn_filter_counts after ``scan``: each query's final candidate
        count (> cap: the exact scan recomputed it) and the capacity; (None,
        -1) when the scan did not run the filter.  Synchronises (tests, tools)."""
        out = torch.zeros(nq, dtype=torch.int32, device=self.device)
        cap = ctypes.c_int64(0)
        _lib.check(_lib.load().fx_knn_filter_counts(
            _ptr(shard.data), shard.dtype_id, shard.n, shard.d, nq, metric, k,
            1 if (state.bits == 8 and state.image is not None) else 0, _ptr(state.ws),
            state.ws.numel(), _ptr(out), ctypes.byref(cap), self._stream()))
        if cap.value < 0:
            return None, -1
        return out.cpu().numpy().view(np.uint32), int(cap.value)

    def merge(self, dist: torch.Tensor, row: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """fx_topk_merge of [nq, parts, kin] sorted lists -> [nq, k]."""
        nq, parts, kin = dist.shape
        nbytes = _lib.merge_workspace_bytes(nq, parts, kin, k)
        ws = self._workspace(nbytes)
        od = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        orow = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        # contiguous copies are held in locals until the merge is queued: a
        # temporary freed before the launch could be handed to the next
        # allocation (the row copy) and be read as distances
        dist = dist.contiguous()
        row = row.contiguous()
        _lib.check(
            _lib.load().fx_topk_merge(
                _ptr(dist), _ptr(row), nq, parts, kin, k, _ptr(ws),
                ws.numel(), _ptr(od), _ptr(orow), self._stream(),
            )
        )
        return od, orow

    def compact(self, mask: torch.Tensor, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """fx_mask_compact: (ascending int32 rows [n capacity], count [1] int64); caller holds lock."""
        rows = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        cnt = torch.empty(1, dtype=torch.int64, device=self.device)
        ws = self._workspace(_lib.compact_workspace_bytes(n))
        _lib.check(_lib.load().fx_mask_compact(_ptr(mask), n, _ptr(ws), ws.numel(), _ptr(rows),
                                               _ptr(cnt), self._stream()))
        return rows, cnt

    def search_rows(self, shard: Shard, rows: torch.Tensor, nrows: int, queries: torch.Tensor,
                    metric: int, k: int, out_dist: torch.Tensor, out_row: torch.Tensor) -> None:
        """fx_knn_search_rows over the listed local rows; caller holds lock."""
        nq = queries.shape[0]
        if shard.dtype_id == _lib.DTYPE_QU8:
            self._search_ex(shard, rows, nrows, queries, metric, k, None, out_dist, out_row)
            return
        ws = self._workspace(_lib.search_rows_workspace_bytes(nrows, shard.d, shard.dtype_id, nq, k))
        self._hold(shard.data)
        _lib.check(_lib.load().fx_knn_search_rows(
            _ptr(shard.data), shard.dtype_id, shard.n, shard.d, shard.row_base, _ptr(rows), nrows,
            _ptr(queries), nq, metric, k, _ptr(ws), ws.numel(), _ptr(out_dist), _ptr(out_row),
            self._stream()))

    # a mask keeping less than this fraction of a shard is compacted to a row
    # list, so the scan reads only the kept rows (a masked scan still walks all)
    SPARSE = 0.5

    def _search_one(self, shard: Shard, queries: torch.Tensor, metric: int, k: int,
                    mask: Optional[torch.Tensor], count: Optional[int], out_dist: torch.Tensor,
                    out_row: torch.Tensor) -> None:
        if mask is not None and count is not None and count < self.SPARSE * shard.n:
            if count == 0:
                out_dist.fill_(float("nan"))
                out_row.fill_(-1)
                return
            rows, _ = self.compact(mask, shard.n)
            self.search_rows(shard, rows, int(count), queries, metric, k, out_dist, out_row)
            return
        self.search_shard(shard, queries, metric, k, mask, out_dist, out_row)

    # several exact-scan shards on this device share one merge tree
    # (fx_knn_search_shards); False: a merge per shard, then one over them
    ONE_MERGE = True

    def _one_merge(self, shards: Sequence[Shard], nq: int, k: int, metric: int,
                   masks: Optional[Sequence[Optional[torch.Tensor]]]) -> bool:
        """fx_knn_search_shards applies: a single query whose every shard
        takes the exact scan (no filter image, k within the fused scan's),
        no masks (a mask may pick the row-list scan per shard), one d and
        dtype."""
        if not self.ONE_MERGE or nq != 1 or k > _lib.max_k():
            return False
        if masks is not None and any(m is not None for m in masks):
            return False
        d, dt = shards[0].d, shards[0].dtype_id
        for s in shards:
            if s.d != d or s.dtype_id != dt or s.n < 1:
                return False
            if dt != _lib.DTYPE_QU8 and _lib.filter_image_used(s.n, s.d, dt, nq, k, metric):
                return False
        return True

    def _search_shards(self, shards: Sequence[Shard], queries: torch.Tensor, metric: int, k: int,
                       out_dist: torch.Tensor, out_row: torch.Tensor) -> None:
        """fx_knn_search_shards: every shard's scan into one list buffer, one
        merge; caller holds lock."""
        arr = (_lib.Corpus * len(shards))(*[s.corpus() for s in shards])
        key = ("shards", self.device.index, queries.shape[0], k,
               tuple((s.n, s.d, s.dtype_id, s.data.data_ptr() % 16 == 0) for s in shards))
        ws = self._workspace(_lib._planned(
            key, lambda: _lib.search_shards_workspace_bytes(arr, queries.shape[0], k)))
        self._hold(*[s.data for s in shards])
        _lib.check(_lib.load().fx_knn_search_shards(
            arr, len(shards), _ptr(queries), queries.shape[0], metric, k, None, _ptr(ws),
            ws.numel(), _ptr(out_dist), _ptr(out_row), self._stream()))

    def search(self, shards: Sequence[Shard], queries: torch.Tensor, metric: int, k: int,
               masks: Optional[Sequence[Optional[torch.Tensor]]] = None,
               counts: Optional[Sequence[Optional[int]]] = None,
               out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
               ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Exact top-k over several shards (sources): per-shard scan, then merge.
        ``counts`` (optional): rows each mask keeps, to pick the row-list scan.
        ``out`` (one shard only): the (dist [nq, k] f32, row [nq, k] i64)
        tensors on this device to write into (search_host's packed result)."""
        queries = _to_device(queries, self.device)
        nq = queries.shape[0]
        mask_of = (lambda i: masks[i]) if masks else (lambda i: None)
        count_of = (lambda i: counts[i]) if counts else (lambda i: None)
        if out is not None and len(shards) != 1:
            raise ValueError("Engine.search: out= needs exactly one shard")
        with self.lock:
            if len(shards) == 1:
                od, orow = out if out is not None else (
                    torch.empty((nq, k), dtype=torch.float32, device=self.device),
                    torch.empty((nq, k), dtype=torch.int64, device=self.device))
                self._search_one(shards[0], queries, metric, k, mask_of(0), count_of(0), od, orow)
                return od, orow
            if self._one_merge(shards, nq, k, metric, masks):
                od = torch.empty((nq, k), dtype=torch.float32, device=self.device)
                orow = torch.empty((nq, k), dtype=torch.int64, device=self.device)
                self._search_shards(shards, queries, metric, k, od, orow)
                return od, orow
            pd = torch.empty((nq, len(shards), k), dtype=torch.float32, device=self.device)
            pr = torch.empty((nq, len(shards), k), dtype=torch.int64, device=self.device)
            for i, sh in enumerate(shards):
                td = torch.empty((nq, k), dtype=torch.float32, device=self.device)
                tr = torch.empty((nq, k), dtype=torch.int64, device=self.device)
                self._search_one(sh, queries, metric, k, mask_of(i), count_of(i), td, tr)
                pd[:, i] = td
                pr[:, i] = tr
            return self.merge(pd, pr, k)

    def distances(self, shard: Shard, queries: torch.Tensor, metric: int,
                  mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        queries = queries.to(self.device, torch.float32).contiguous()
        out = torch.empty((queries.shape[0], shard.n), dtype=torch.float32, device=self.device)
        with self.lock:
            if shard.dtype_id == _lib.DTYPE_QU8:
                c = shard.corpus()
                _lib.check(_lib.load().fx_knn_distances_ex(
                    ctypes.byref(c), _ptr(queries), queries.shape[0], metric, _ptr(mask),
                    _ptr(out), self._stream()))
                return out
            _lib.check(
                _lib.load().fx_knn_distances(
                    _ptr(shard.data), shard.dtype_id, shard.n, shard.d, _ptr(queries),
                    queries.shape[0], metric, _ptr(mask), _ptr(out), self._stream(),
                )
            )
        return out

    # ------------------------------------------------------------ coded index
    def row_sqnorms(self, x: torch.Tensor) -> torch.Tensor:
        """fx_row_sqnorms: [n] f32 sum of squares of each row of x [n, D]."""
        out = torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
        dt = _lib.DTYPE_F32 if x.dtype == torch.float32 else _lib.DTYPE_F16
        with self.lock:
            _lib.check(_lib.load().fx_row_sqnorms(_ptr(x), dt, x.shape[0], x.shape[1], _ptr(out),
                                                  self._stream()))
        return out

    def code_assign(self, x: torch.Tensor, codewords: torch.Tensor, metric: int,
                    index: bool = False, code: bool = True, dist: bool = False
                    ) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor],
                               Optional[torch.Tensor]]:
        """fx_code_assign: nearest codeword of every row of x [n, D] (f32/f16, on
        this device) in every codebook of codewords [nb, ks, D] (f32).  Returns
        (index [n, nb] int32, code [n] int64, dist [n, nb] f32), each or None."""
        nb, ks, d = codewords.shape
        n = x.shape[0]
        cw = codewords.to(self.device, torch.float32).contiguous()
        dt = _lib.DTYPE_F32 if x.dtype == torch.float32 else _lib.DTYPE_F16
        oi = torch.empty((n, nb), dtype=torch.int32, device=self.device) if index else None
        oc = torch.empty(n, dtype=torch.int64, device=self.device) if code else None
        od = torch.empty((n, nb), dtype=torch.float32, device=self.device) if dist else None
        with self.lock:
            ws = self._workspace(_lib.code_assign_workspace_bytes(n, d, nb, ks))
            _lib.check(_lib.load().fx_code_assign(
                _ptr(x), dt, n, d, _ptr(cw), nb, ks, metric, _ptr(ws), ws.numel(), _ptr(oi),
                _ptr(oc), _ptr(od), self._stream()))
        return oi, oc, od

    def kmeans_step(self, sample: torch.Tensor, codewords: torch.Tensor, metric: int) -> None:
        """fx_kmeans_step: sample [nb, bs, D] (f32/f16), codewords [nb, ks, D] f32
        contiguous on this device, updated in place (coder.py:53-65 under vmap)."""
        nb, bs, d = sample.shape
        ks = codewords.shape[1]
        if not (codewords.is_contiguous() and codewords.dtype == torch.float32
                and codewords.device == self.device):
            raise ValueError("codewords must be a contiguous float32 tensor on the device")
        dt = _lib.DTYPE_F32 if sample.dtype == torch.float32 else _lib.DTYPE_F16
        with self.lock:
            ws = self._workspace(_lib.kmeans_workspace_bytes(nb, bs, d, ks))
            _lib.check(_lib.load().fx_kmeans_step(
                _ptr(sample), dt, nb, bs, d, _ptr(codewords), ks, metric, _ptr(ws), ws.numel(),
                self._stream()))

    def code_probe(self, cw_dist: torch.Tensor, probes: int, sel: bool = True
                   ) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
        """fx_code_probe: cw_dist [nq, nb, ks] f32 -> (codes [nq, probes] int64,
        scores [nq, probes] f32, selected-code bitmap [nq, words] int32 or None)."""
        nq, nb, ks = cw_dist.shape
        cd = cw_dist.to(self.device, torch.float32).contiguous()
        codes = torch.empty((nq, probes), dtype=torch.int64, device=self.device)
        scores = torch.empty((nq, probes), dtype=torch.float32, device=self.device)
        bits = None
        if sel:
            words = (ks**nb + 31) // 32
            bits = torch.empty((nq, words), dtype=torch.int32, device=self.device)
        with self.lock:
            ws = self._workspace(_lib.code_probe_workspace_bytes(nq, nb, ks))
            _lib.check(_lib.load().fx_code_probe(
                _ptr(cd), nq, nb, ks, probes, _ptr(ws), ws.numel(), _ptr(codes), _ptr(scores),
                _ptr(bits), self._stream()))
        return codes, scores, bits

    def code_mask(self, row_code: torch.Tensor, sel: torch.Tensor, ncodes: int,
                  filter: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """fx_code_mask: (bitmap [ceil(n/32)] int32, kept-row count [1] int64)."""
        n = row_code.shape[0]
        out = torch.empty(max(1, (n + 31) // 32), dtype=torch.int32, device=self.device)
        cnt = torch.empty(1, dtype=torch.int64, device=self.device)
        with self.lock:
            _lib.check(_lib.load().fx_code_mask(
                _ptr(row_code), n, _ptr(sel), ncodes, _ptr(filter), _ptr(out), _ptr(cnt),
                self._stream()))
        return out, cnt

    def fill(self, out: torch.Tensor, seed: int, row_base: int = 0, cluster: int = 0) -> None:
        """Synthetic corpus (bit-identical to oracle.fill_normal) written in place."""
        dt = _lib.DTYPE_F32 if out.dtype == torch.float32 else _lib.DTYPE_F16
        n, d = out.shape
        _lib.check(
            _lib.load().fx_fill_normal(_ptr(out), dt, n, d, seed, row_base, cluster, self._stream())
        )
        # written behind torch's back: bump the version counter that cached
        # derived data (filter images) is keyed on
        torch.autograd.graph.increment_version(out)


def _to_device(queries: torch.Tensor, device: torch.device) -> torch.Tensor:
    """Queries as contiguous float32 on ``device``.  A host tensor goes
    through a pinned buffer with an asynchronous copy on the current stream
    (a pageable H2D blocks the host for ~15-20 us before the search can be
    queued; the caching host allocator keeps the buffer until the copy ran)."""
    if queries.device == device and queries.dtype == torch.float32:
        return queries.contiguous()
    if queries.device.type == "cpu":
        staged = torch.empty(queries.shape, dtype=torch.float32, pin_memory=True)
        staged.copy_(queries)
        return staged.to(device, non_blocking=True)
    return queries.to(device, torch.float32).contiguous()


def bitmap(mask: np.ndarray) -> np.ndarray:
    """bool[n] -> uint32 words, bit r of word r>>5 (the C ABI mask format)."""
    mask = np.asarray(mask, dtype=bool).ravel()
    words = (mask.size + 31) // 32
    padded = np.zeros(words * 32, dtype=bool)
    padded[: mask.size] = mask
    return np.packbits(padded, bitorder="little").view("<u4").astype(np.uint32)


def device_mask(mask: Optional[np.ndarray], device: torch.device) -> Optional[torch.Tensor]:
    if mask is None:
        return None
    words = bitmap(mask)
    return torch.from_numpy(words.view(np.int32)).to(device)


def search_all(shards: Sequence[Shard], queries: torch.Tensor, metric: int, k: int,
               masks: Optional[Sequence[Optional[torch.Tensor]]] = None,
               counts: Optional[Sequence[Optional[int]]] = None,
               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact top-k over shards that may live on several devices.

    A single unfiltered query goes through the serving coalescer
    (``fenix_amd.coalesce``): concurrent requests over the same shards run as
    one batch (returned on the host, shape [1, k]).  Everything else, and
    every batch, runs ``_search_all``."""
    if (queries.shape[0] == 1 and masks is None and counts is None and coalesce.enabled()
            and k <= _lib.load().fx_max_k()):
        key = (tuple((id(s.data), s.data.data_ptr(), s.n, s.row_base) for s in shards), metric)

        def run(qs: np.ndarray, kk: int) -> Tuple[np.ndarray, np.ndarray]:
            d, r = _search_all(shards, torch.from_numpy(qs), metric, kk)
            return d.cpu().numpy(), r.cpu().numpy()

        d, r = coalesce.default().search(key, run, queries.cpu().numpy(), k)
        return torch.from_numpy(d), torch.from_numpy(r)
    return _search_all(shards, queries, metric, k, masks, counts)


def gather_rows(shards: Sequence[Shard], rows: torch.Tensor) -> Optional[torch.Tensor]:
    """The stored values of result rows, gathered on the device that holds
    ``rows`` ([nq, K] int64 global row numbers, -1 = empty slot) ->
    [nq, K, D] in the shards' dtype, or None when a shard lives on another
    device (the caller then gathers on the host side, io.index._gather_vectors).

    Queued on the stream right behind the search that produced ``rows``, so
    the host enqueues it while the device still scans and the winning rows
    come back with the distances in one D2H (index.py:166's take).  Empty
    slots and rows outside every shard read a clamped row; the caller drops
    the first and rejects the second (``check_rows``)."""
    dev = rows.device
    shards = [s for s in shards if s.n > 0]  # (an empty shard holds no result row)
    if not shards or any(s.data.device != dev for s in shards):
        return None
    nq, kk = rows.shape
    flat = rows.reshape(-1)
    with torch.cuda.device(dev):
        if len(shards) == 1:
            s = shards[0]
            # (row_base 0, a table's first shard: one clamp launch, not a
            # subtraction and a clamp, ~5 us of the served search's tail)
            local = (flat.clamp(0, max(s.n - 1, 0)) if s.row_base == 0
                     else (flat - s.row_base).clamp_(0, max(s.n - 1, 0)))
            return s.data.index_select(0, local).view(nq, kk, s.d)
        bases = torch.tensor([s.row_base for s in shards], dtype=torch.int64).to(
            dev, non_blocking=True)
        which = torch.searchsorted(bases, flat, right=True) - 1
        out = None
        for i, s in enumerate(shards):
            g = s.data.index_select(0, (flat - s.row_base).clamp_(0, max(s.n - 1, 0)))
            out = g if out is None else torch.where((which == i).unsqueeze(1), g, out)
        return out.view(nq, kk, shards[0].d)


def check_rows(shards: Sequence[Shard], rows: np.ndarray) -> None:
    """Every non-empty result row lies inside a shard, the shards in row order
    (the assumption of gather_rows and io.index._gather_vectors)."""
    if len(shards) == 1:  # (the common case, a few us)
        s = shards[0]
        lo, hi = int(rows.min(initial=0)), int(rows.max(initial=-1))
        if (lo < 0 and lo != -1) or (hi >= 0 and (int(rows[rows >= 0].min()) < s.row_base
                                                  or hi >= s.row_base + s.n)):
            raise ValueError("a result row lies outside every shard")
        return
    bases = np.array([s.row_base for s in shards], dtype=np.int64)
    ns = np.array([s.n for s in shards], dtype=np.int64)
    if np.any(np.diff(bases) < 0):
        raise ValueError("shards must be in row order")
    r = rows[rows >= 0]
    which = np.searchsorted(bases, r, side="right") - 1
    if np.any(which < 0) or np.any(r - bases[np.maximum(which, 0)] >= ns[np.maximum(which, 0)]):
        raise ValueError("a result row lies outside every shard")


def _to_host(*ts: torch.Tensor) -> Tuple[np.ndarray, ...]:
    """Device tensors -> host arrays: one pinned D2H each on the current
    stream of their device, ONE synchronisation."""
    outs = []
    for t in ts:
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        outs.append(h)
    torch.cuda.current_stream(ts[0].device).synchronize()
    return tuple(h.numpy() for h in outs)


def _search_packed(shard: Shard, queries: torch.Tensor, metric: int, k: int,
                   masks=None, counts=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """One shard's search with the k winning rows gathered behind it, all
    three results written into ONE device buffer [rows i64 | dist f32 | pad |
    vectors] and brought back with ONE D2H and one synchronisation (three
    copies of a served search's tail were ~15 us of it,
    profiles/r06_flight_cfg1_host_gap.txt).  Same results as _search_all +
    gather_rows + _to_host."""
    dev = shard.data.device
    nq = queries.shape[0]
    m = nq * k
    esz = shard.data.element_size()
    off_d = 8 * m
    off_v = (off_d + 4 * m + 15) // 16 * 16
    total = off_v + m * shard.d * esz
    with torch.cuda.device(dev):
        packed = torch.empty(total, dtype=torch.uint8, device=dev)
        orow = packed[:off_d].view(torch.int64).view(nq, k)
        od = packed[off_d:off_d + 4 * m].view(torch.float32).view(nq, k)
        vecs = packed[off_v:].view(shard.data.dtype).view(m, shard.d)
        Engine.get(dev).search([shard], queries, metric, k, masks, counts, out=(od, orow))
        flat = orow.reshape(-1)
        local = (flat.clamp(0, max(shard.n - 1, 0)) if shard.row_base == 0
                 else (flat - shard.row_base).clamp_(0, max(shard.n - 1, 0)))
        torch.index_select(shard.data, 0, local, out=vecs)
        host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
        host.copy_(packed, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
    hb = host.numpy()
    return (hb[off_d:off_d + 4 * m].view(np.float32).reshape(nq, k),
            hb[:off_d].view(np.int64).reshape(nq, k),
            hb[off_v:].view(_np_dtype(shard.data.dtype)).reshape(nq, k, shard.d))


def _np_dtype(dt: torch.dtype):
    return {torch.float32: np.float32, torch.float16: np.float16, torch.uint8: np.uint8}[dt]


def search_host(shards: Sequence[Shard], queries: torch.Tensor, metric: int, k: int,
                masks: Optional[Sequence[Optional[torch.Tensor]]] = None,
                counts: Optional[Sequence[Optional[int]]] = None, gather: bool = False,
                ) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
    """``search_all`` with the results on the host — what io.index.call
    needs: (dist [nq, k] f32, rows [nq, k] i64, vectors [nq, k, D] or None).

    With ``gather`` the result rows' stored values are gathered on the
    device behind the search (``gather_rows``) and come back with the
    distances and rows in one synchronisation (None when the shards span
    devices).  A single unfiltered query goes through the serving coalescer
    like ``search_all``."""
    def run(qs: torch.Tensor, kk: int, ms=None, cs=None) -> Tuple[np.ndarray, ...]:
        if gather and len(shards) == 1 and shards[0].n > 0:
            return _search_packed(shards[0], qs, metric, kk, ms, cs)
        d, r = _search_all(shards, qs, metric, kk, ms, cs)
        v = gather_rows(shards, r) if gather else None
        if v is None:
            return _to_host(d, r)
        with torch.cuda.device(r.device):
            return _to_host(d, r, v)

    if (queries.shape[0] == 1 and masks is None and counts is None and coalesce.enabled()
            and k <= _lib.load().fx_max_k()):
        key = (tuple((id(s.data), s.data.data_ptr(), s.n, s.row_base) for s in shards), metric,
               gather)
        parts = coalesce.default().search(key, lambda qs, kk: run(torch.from_numpy(qs), kk),
                                          queries.cpu().numpy(), k)
    else:
        parts = run(queries, k, masks, counts)
    if len(parts) == 3:
        check_rows(shards, parts[1])
        return parts
    return parts[0], parts[1], None


# how many multi-device searches gathered their lists each way (bench.py, tests)
GATHERS: Dict[str, int] = {"rccl": 0, "p2p": 0}
_GATHERS_LOCK = threading.Lock()

# Every grouped RCCL exchange of this process is enqueued under this one lock
# (DESIGN §4).  Flight handlers run on concurrent gRPC threads
# (reference: src/fenix/flight.py:62-77), and an fx_allgather_topk enqueues one
# collective per device (ncclGroupStart … ncclAllGather × ndev … ncclGroupEnd,
# comm.hip).  Two such enqueues that interleave can order collectives A, B on
# device 0 and B, A on device 1; each RCCL kernel waits for its peers, so both
# hang.  One lock for the whole process (not one per communicator) also orders
# exchanges of communicators over overlapping device sets, which share the
# devices' streams.
COLLECTIVE_LOCK = threading.Lock()


def gather_mode(devs: Sequence[torch.device]) -> str:
    """How ``_search_all`` gathers per-device top-k lists: ``rccl`` (one
    grouped RCCL all-gather over xGMI, fx_allgather_topk: SURVEY §8(e)'s
    exchange, the default for distinct devices) or ``p2p`` (a peer copy per
    device to the first one; the only choice when an ordinal repeats, since
    RCCL takes one rank per device).  ``FENIX_AMD_GATHER`` overrides."""
    env = os.environ.get("FENIX_AMD_GATHER", "").strip()
    distinct = len({d.index for d in devs}) == len(devs)
    if env == "p2p" or not distinct:
        return "p2p"
    if env in ("", "rccl"):
        return "rccl"
    raise ValueError(f"FENIX_AMD_GATHER={env!r}: expected rccl or p2p")


def _search_all(shards: Sequence[Shard], queries: torch.Tensor, metric: int, k: int,
                masks: Optional[Sequence[Optional[torch.Tensor]]] = None,
                counts: Optional[Sequence[Optional[int]]] = None,
                ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact top-k over shards that may live on several devices.

    Each device's shards are searched by that device's Engine.  No library
    call waits for the host (the batched path's overflow fallback is gated on
    the device, fx_knn_reduce), so this loop queues every device's scan and
    merge back to back and the devices scan concurrently.  The per-device
    [nq, k] results are then exchanged as ``gather_mode`` says: one RCCL
    all-gather over xGMI (distinct devices) or peer copies to the first
    device, and merged there by fx_topk_merge.  (The one-process-per-GPU
    path uses torch.distributed's RCCL all-gather, distributed.py.)
    """
    groups: Dict[torch.device, List[int]] = {}
    for i, s in enumerate(shards):
        groups.setdefault(s.data.device, []).append(i)
    per = []
    for dev, idx in groups.items():
        with torch.cuda.device(dev):
            eng = Engine.get(dev)
            ms = [masks[i] for i in idx] if masks is not None else None
            cs = [counts[i] for i in idx] if counts is not None else None
            per.append(eng.search([shards[i] for i in idx], queries, metric, k, ms, cs))
    if len(per) == 1:
        return per[0]
    devs = list(groups)
    if gather_mode(devs) == "rccl":
        comm = DeviceComm.get_or_none(devs)
        if comm is not None:
            with _GATHERS_LOCK:
                GATHERS["rccl"] += 1
            return comm.gather_merge(per, k)
    with _GATHERS_LOCK:
        GATHERS["p2p"] += 1
    dev0 = next(iter(groups))
    with torch.cuda.device(dev0):
        eng0 = Engine.get(dev0)
        dd = torch.stack([d.to(dev0) for d, _ in per], dim=1)
        rr = torch.stack([r.to(dev0) for _, r in per], dim=1)
        with eng0.lock:
            return eng0.merge(dd, rr, k)


class DeviceComm:
    """fx_comm_init_all over distinct devices (one RCCL rank each), cached.

    ``gather_merge`` all-gathers every device's [nq, k] top-k with one grouped
    fx_allgather_topk and merges on the first device.  ``_search_all`` uses
    it for distinct devices unless FENIX_AMD_GATHER=p2p (``gather_mode``).

    The collective is enqueued under ``COLLECTIVE_LOCK``, so concurrent
    searches reach every device's stream in one order.  A device set whose
    communicator cannot be created (no RCCL, ncclCommInitAll failing) is
    remembered, and ``get_or_none`` returns None for it, so ``_search_all``
    takes the peer-copy path instead of failing every search."""

    _cache: Dict[tuple, "DeviceComm"] = {}
    _failed: Dict[tuple, str] = {}
    _clock = threading.Lock()

    def __init__(self, devs: Sequence[torch.device]) -> None:
        self.devs = list(devs)
        ids = (ctypes.c_int * len(devs))(*[d.index for d in devs])
        handle = ctypes.c_void_p()
        _lib.check(_lib.load().fx_comm_init_all(len(devs), ids, ctypes.byref(handle)))
        self.handle = handle

    @classmethod
    def get(cls, devs: Sequence[torch.device]) -> "DeviceComm":
        key = tuple(d.index for d in devs)
        with cls._clock:
            c = cls._cache.get(key)
            if c is None:
                c = cls(devs)
                cls._cache[key] = c
            return c

    @classmethod
    def get_or_none(cls, devs: Sequence[torch.device]) -> Optional["DeviceComm"]:
        """``get``, or None (with one warning per device set) when the
        communicator cannot be created."""
        key = tuple(d.index for d in devs)
        if key in cls._failed:
            return None
        try:
            return cls.get(devs)
        except (RuntimeError, OSError) as e:
            with cls._clock:
                first = key not in cls._failed
                cls._failed[key] = str(e)
            if first:
                warnings.warn(f"RCCL communicator over devices {key} unavailable ({e}); "
                              "gathering top-k lists by peer copies", RuntimeWarning)
            return None

    def close(self) -> None:
        if self.handle:
            _lib.check(_lib.load().fx_comm_destroy(self.handle))
            self.handle = None

    def allgather(self, per: Sequence[Tuple[torch.Tensor, torch.Tensor]]
                  ) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        """per[i] = (dist [nq, k] f32, row [nq, k] i64) on devs[i] ->
        [(dist [ndev, nq, k], row [ndev, nq, k])] on every device."""
        n = len(self.devs)
        nq, k = per[0][0].shape
        outs = [(torch.empty((n, nq, k), dtype=torch.float32, device=dv),
                 torch.empty((n, nq, k), dtype=torch.int64, device=dv)) for dv in self.devs]
        P = ctypes.c_void_p * n
        # keep the contiguous sources alive until the collective is queued
        srcs = [(d.contiguous(), r.contiguous()) for d, r in per]
        src_d = P(*[d.data_ptr() for d, _ in srcs])
        src_r = P(*[r.data_ptr() for _, r in srcs])
        dst_d = P(*[d.data_ptr() for d, _ in outs])
        dst_r = P(*[r.data_ptr() for _, r in outs])
        streams = P(*[torch.cuda.current_stream(dv).cuda_stream for dv in self.devs])
        with COLLECTIVE_LOCK:
            _lib.check(_lib.load().fx_allgather_topk(self.handle, src_d, src_r, nq, k,
                                                     dst_d, dst_r, streams))
        return outs

    def gather_merge(self, per, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        d, r = self.allgather(per)[0]
        dev0 = self.devs[0]
        with torch.cuda.device(dev0):
            eng0 = Engine.get(dev0)
            with eng0.lock:
                return eng0.merge(d.permute(1, 0, 2), r.permute(1, 0, 2), k)


def distances_all(shards: Sequence[Shard], queries: torch.Tensor, metric: int,
                  masks: Optional[Sequence[Optional[torch.Tensor]]] = None) -> np.ndarray:
    """[nq, sum of shard rows] distances, shards concatenated in order."""
    outs = []
    for i, s in enumerate(shards):
        dev = s.data.device
        with torch.cuda.device(dev):
            m = masks[i] if masks is not None else None
            outs.append(Engine.get(dev).distances(s, queries, metric, m))
    if not outs:
        return np.zeros((queries.shape[0], 0), np.float32)
    return np.concatenate([o.cpu().numpy() for o in outs], axis=1)
