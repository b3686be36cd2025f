"""Arrow IPC stream files — the on-disk corpus format the scan reads.

Mirrors src/fenix/io/arrow/arrow.py:6-21 of the reference: ``load`` memory-maps
an IPC *stream* file (zero-copy) and ``make`` writes one record batch per
incoming batch (so client batch size = chunk size).
"""

from __future__ import annotations

import itertools
import os
import threading

import pyarrow as pa

from ..ex.arrow import quint8 as _quint8  # noqa: F401  (registers "tensor::qint8" for IPC reads)


_gen_lock = threading.Lock()
_GEN: dict = {}  # abspath -> generation, bumped by every make() of this process
_tmp_ids = itertools.count()


def file_version(path: str) -> tuple:
    """(size, mtime_ns, inode, generation) of ``path``: the key every cache of
    a file's contents (mmap'd tables, HBM shards, codings) is stamped with.
    ``make`` replaces files atomically (new inode) and bumps the generation,
    so a rewrite with the same size inside one mtime tick is still seen."""
    # stat and generation read under the lock ``replace`` holds across the
    # rename and the bump: a reader never pairs the new file with the old
    # generation (which would restage the corpus once more after the bump)
    with _gen_lock:
        st = os.stat(path)
        gen = _GEN.get(os.path.abspath(path), 0)
    return (st.st_size, st.st_mtime_ns, st.st_ino, gen)


def load(path: str) -> pa.Table:
    with pa.memory_map(path, "rb") as source:
        return pa.ipc.open_stream(source).read_all()


def make(path: str, data: pa.RecordBatchReader) -> pa.Table:
    assert path.endswith(".arrow")

    os.makedirs(os.path.dirname(path), exist_ok=True)

    # Written next to the target and renamed over it: tables already mapped
    # by a search (the resident caches keep their mmaps across calls) stay
    # valid, where the reference's in-place OSFile(path, "wb") truncates them.
    tmp = temp_path(path)
    try:
        with pa.OSFile(tmp, "wb") as sink:
            with pa.ipc.new_stream(sink, data.schema) as writer:
                for batch in data:
                    writer.write_batch(batch)
    except BaseException:
        if os.path.exists(tmp):
            os.remove(tmp)
        raise
    replace(tmp, path)

    return load(path)


def temp_path(path: str) -> str:
    """A fresh file name next to ``path`` for an atomic rewrite (see ``replace``)."""
    return f"{path}.{os.getpid()}.{next(_tmp_ids)}.tmp"


def replace(tmp: str, path: str) -> None:
    """Rename a fully written ``tmp`` over ``path`` and bump its generation."""
    with _gen_lock:
        os.replace(tmp, path)
        key = os.path.abspath(path)
        _GEN[key] = _GEN.get(key, 0) + 1
