"""Arrow Flight server and client — the drop-in API surface of the search path.

Mirrors src/fenix/flight.py of the reference:

* ``Server(root, host, port)`` (flight.py:17-134): ``do_put`` ingests a table
  (:34-44), ``do_get`` streams one (:46-60), ``do_exchange`` is the search
  (:62-77, unpickles the descriptor dict and the pickled filter, reads the
  ``target`` column, calls ``io.index.call`` and streams the result), and
  ``do_action`` runs the pickled-dict admin actions (:79-134).
* ``Flight(host, port)`` (flight.py:137-292): ``make_table``, ``read_table``,
  ``drop_table``, ``search`` (:242-288: metric assert, pickled descriptor,
  ``pa.table({"target": ...})`` over ``do_exchange``) and ``remove``.

The wire format (descriptor dict, ``target`` column, result schema, action
names and their pickled bodies) is unchanged, so a reference client can talk
to this server and vice versa.  Only ``search`` / ``do_exchange`` / ``do_put``
are on the accelerated path; the admin surface is kept for drop-in use and
written here as tables: server actions dispatch through ``Server._ACTIONS``,
the read options that ``read_table`` sets before a ``do_get`` live in one
locked dict (``Server._read_opts``, not attributes of the server object), and
the client issues every action through ``Flight._action``.
``io.index.call`` underneath runs on the GPU (fenix_amd.io.index), as do the
coded-index actions (``make-coder``, ``make-index``, ``drop-index``,
:82-101: k-means training, table encoding and probe search, io.coder /
io.index).  ``drop-index`` removes the coding and every index file built
with it; the reference's loop (:88-93) takes the basename of each index path
and then splits it on "/", so it never removes an index whose name contains
"/" and raises ValueError for one that does not.
"""

from __future__ import annotations

import functools
import os
import pickle
import shutil
import threading
from typing import Iterator, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pyarrow.flight as fl
from pydantic.dataclasses import dataclass
from typing_extensions import Self

from . import io


class Server(fl.FlightServerBase):
    # read_table's per-read options, set and cleared by "set-*" / "del-*"
    # actions around a do_get (flight.py:105-131 of the reference); the value
    # of each lives under the action body's key of the same name
    _READ_OPTS = ("coding", "column", "filter", "select")

    def __init__(self, root: str, host: str = "0.0.0.0", port: int = 9001) -> None:
        self.root = os.path.abspath(root)
        self.grpc = f"grpc://{host}:{port}"
        self._opts_lock = threading.Lock()
        self._read_opts: dict = {}

        super().__init__(location=self.grpc)

    def get_flight_info(
        self, ctx: fl.ServerCallContext, descriptor: fl.FlightDescriptor
    ) -> fl.FlightInfo:
        raise NotImplementedError()

    def list_flights(
        self, ctx: fl.ServerCallContext, criteria: bytes
    ) -> Iterator[fl.FlightDescriptor]:
        raise NotImplementedError()

    def do_put(
        self,
        ctx: fl.ServerCallContext,
        descriptor: fl.FlightDescriptor,
        reader: fl.MetadataRecordBatchReader,
        writer: fl.FlightMetadataWriter,
    ) -> None:
        # an atomic rewrite bumps the file version: the HBM copy is restaged
        io.table.make(self.root, descriptor.path[0].decode(), reader.to_reader())

    def do_get(self, ctx: fl.ServerCallContext, ticket: fl.Ticket):
        sources = ticket.ticket.decode().split(":")
        with self._opts_lock:
            opts = dict(self._read_opts)
        if "coding" in opts and "column" in opts:
            data = io.index.load(self.root, opts["coding"], sources, opts["column"])
        else:
            data = io.table.load(self.root, sources)
        for key, apply in (("filter", pa.Table.filter), ("select", pa.Table.select)):
            if key in opts:
                data = apply(data, opts[key])
        return fl.GeneratorStream(data.schema, data.to_reader())

    def do_exchange(
        self,
        ctx: fl.ServerCallContext,
        descriptor: fl.FlightDescriptor,
        reader: fl.MetadataRecordBatchReader,
        writer: fl.MetadataRecordBatchWriter,
    ) -> None:
        config = pickle.loads(descriptor.command)
        config["target"] = reader.read_all().column("target").combine_chunks()
        config["filter"] = pickle.loads(config["filter"])

        data = io.index.call(self.root, **config)

        writer.begin(data.schema)
        writer.write_table(data)

    # ------------------------------------------------------------- actions
    def _drop_index(self, name: str) -> None:
        io.coder.drop(self.root, name)
        for path in io.index.list(self.root):
            if path.endswith("/" + name):
                os.unlink(os.path.join(self.root, io.index.LOCATION, path + ".arrow"))

    _ACTIONS = {
        "make-coder": lambda self, b: io.coder.make(self.root, **b),
        "make-index": lambda self, b: io.index.make(self.root, **b),
        "drop-index": lambda self, b: self._drop_index(**b),
        "drop-table": lambda self, b: io.table.drop(self.root, **b),
        "remove": lambda self, b: shutil.rmtree(self.root),
    }

    def do_action(self, ctx: fl.ServerCallContext, action: fl.Action) -> None:
        verb, _, key = action.type.partition("-")
        handler = self._ACTIONS.get(action.type)
        if handler is None and not (verb in ("set", "del") and key in self._READ_OPTS):
            raise ValueError()
        body = pickle.loads(action.body.to_pybytes())
        if handler is not None:
            handler(self, body)
            return
        with self._opts_lock:
            if verb == "set":
                self._read_opts[key] = body[key]
            else:
                self._read_opts.pop(key, None)


# the metric names Flight.search accepts (coder.py:38-50 and their aliases)
METRICS = frozenset({"cosine", "dot", "inner_product", "l2", "euclidean"})


@dataclass(frozen=True)
class Flight:
    host: str = "0.0.0.0"
    port: int = 9001

    @functools.cached_property
    def conn(self) -> fl.FlightClient:
        return fl.connect(f"grpc://{self.host}:{self.port}")

    def __del__(self) -> None:
        if "conn" in self.__dict__:
            self.conn.close()

    def _action(self, action: str, **body) -> Self:
        """One admin action: its name and a pickled dict body (the reference's
        wire format)."""
        self.conn.do_action(fl.Action(action, pickle.dumps(body)))
        return self

    def make_table(self, name: str, data: pa.RecordBatchReader) -> Self:
        writer, _ = self.conn.do_put(fl.FlightDescriptor.for_path(name), data.schema)
        with writer:
            for batch in data:
                writer.write_batch(batch)
        return self

    def read_table(
        self,
        source: str | Sequence[str],
        coding: str | None = None,
        column: str | None = None,
        select: Sequence[str] | None = None,
        filter: pc.Expression | None = None,
    ) -> pa.RecordBatchReader:
        opts = {"select": select, "filter": filter}
        if coding is not None and column is not None:
            opts.update(coding=coding, column=column)
        for key, value in opts.items():
            if value is not None:
                self._action(f"set-{key}", **{key: value})
        names = source if isinstance(source, str) else ":".join(source)
        reader = self.conn.do_get(fl.Ticket(names)).to_reader()
        for key in ("coding", "column", "select", "filter"):
            self._action(f"del-{key}")
        return reader

    def drop_table(self, name: str) -> Self:
        return self._action("drop-table", name=name)

    def make_index(
        self, name: str, source: str | Sequence[str], column: str, config: dict
    ) -> Self:
        self._action("make-coder", name=name, source=source, column=column, config=config)
        return self.sync_index(name, source, column)

    def sync_index(self, name: str, source: str | Sequence[str], column: str) -> Self:
        return self._action("make-index", name=name, source=source, column=column)

    def drop_index(self, name: str) -> Self:
        return self._action("drop-index", name=name)

    def search(
        self,
        target,  # pa.Array | pa.ChunkedArray | pa.FixedSizeListScalar | np.ndarray | Tensor
        source: str | Sequence[str],
        column: str,
        metric: str,
        coding: str | None = None,
        select: Sequence[str] | None = None,
        filter: pc.Expression | None = None,
        maxval: int | None = None,
        probes: int | None = None,
    ) -> pa.Table:
        """The drop-in search (flight.py:242-288 of the reference): the same
        assert, descriptor dict (filter pickled twice) and ``target`` table."""
        assert metric in METRICS

        command = {"coding": coding, "source": source, "column": column, "metric": metric,
                   "select": select, "filter": pickle.dumps(filter), "maxval": maxval,
                   "probes": probes}
        if type(target).__module__.split(".")[0] == "torch":  # Tensor, without importing torch
            target = target.numpy()
        if isinstance(target, np.ndarray):
            target = pa.array(target)
        table = pa.table({"target": target})

        writer, reader = self.conn.do_exchange(
            fl.FlightDescriptor.for_command(pickle.dumps(command)))
        with writer:
            writer.begin(table.schema)
            writer.write_table(table)
            writer.done_writing()
            # the same table as the reference's reader.read_all() (flight.py:288),
            # read through the RecordBatchReader interface: FlightStreamReader.read_all
            # costs ~1-2 ms more per call (tools/bench_flight.py --read-all)
            return reader.to_reader().read_all()

    def remove(self) -> Self:
        return self._action("remove")
