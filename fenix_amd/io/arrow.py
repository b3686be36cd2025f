"""Arrow IPC stream files — the on-disk corpus format the scan reads.

Mirrors src/fenix/io/arrow/arrow.py:6-21 of the reference: ``load`` memory-maps
an IPC *stream* file (zero-copy) and ``make`` writes one record batch per
incoming batch (so client batch size = chunk size).
"""

from __future__ import annotations

import os

import pyarrow as pa

from ..ex.arrow import quint8 as _quint8  # noqa: F401  (registers "tensor::qint8" for IPC reads)


def load(path: str) -> pa.Table:
    with pa.memory_map(path, "rb") as source:
        return pa.ipc.open_stream(source).read_all()


def make(path: str, data: pa.RecordBatchReader) -> pa.Table:
    assert path.endswith(".arrow")

    os.makedirs(os.path.dirname(path), exist_ok=True)

    with pa.OSFile(path, "wb") as sink:
        with pa.ipc.new_stream(sink, data.schema) as writer:
            for batch in data:
                writer.write_batch(batch)

    return load(path)
