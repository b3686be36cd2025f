"""Named tables under ``<root>/sources/<name>.arrow``.

Mirrors src/fenix/io/table/table.py:9-56 of the reference (load / make / join /
list / drop).  ``join(axis=0)`` concatenates sources row-wise: global row
numbers of a multi-source search run across the sources in the given order
(table.py:19-21,35), which is the ``row_base`` of each device shard.
"""

from __future__ import annotations

import os
from typing import Iterator, Literal, Sequence

import pyarrow as pa

from . import arrow

LOCATION: str = "sources"


def path(root: str, name: str) -> str:
    return os.path.join(root, LOCATION, name + ".arrow")


def load(root: str, name: str | Sequence[str]) -> pa.Table:
    if isinstance(name, str):
        return arrow.load(path(root, name))

    assert isinstance(name, Sequence) and not isinstance(name, str)
    return join(*[load(root, n) for n in name])


def make(root: str, name: str, data: pa.RecordBatchReader) -> pa.Table:
    return arrow.make(path(root, name), data)


def join(*data: pa.Table, axis: Literal[0, 1] = 0) -> pa.Table:
    if len(data) == 1:
        return data[0]

    if axis == 0:
        return pa.concat_tables(data)
    if axis == 1:
        return pa.table({c: t.column(c) for t in data for c in t.column_names})
    raise ValueError()


def list(root: str) -> Iterator[str]:
    base = os.path.join(root, LOCATION)
    for dirpath, _, files in os.walk(base):
        for f in sorted(files):
            if f.endswith(".arrow"):
                rel = os.path.relpath(os.path.join(dirpath, f), base)
                yield rel.removesuffix(".arrow")


def drop(root: str, name: str) -> None:
    p = path(root, name)

    if os.path.exists(p):
        os.unlink(p)
