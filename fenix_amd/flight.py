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

The wire format (descriptor dict, ``target`` column, result schema) is
unchanged, so a reference client can talk to this server and vice versa.
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
    def __init__(self, root: str, host: str = "0.0.0.0", port: int = 9001) -> None:
        self.root = os.path.abspath(root)
        self.grpc = f"grpc://{host}:{port}"
        self._attr_lock = threading.Lock()

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
        name = descriptor.path[0].decode()
        data = reader.to_reader()

        # rewriting the file changes its (size, mtime): the HBM copy is restaged
        io.table.make(self.root, name, data)

    def do_get(self, ctx: fl.ServerCallContext, ticket: fl.Ticket):
        source = ticket.ticket.decode().split(":")

        if hasattr(self, "coding") and hasattr(self, "column"):
            data = io.index.load(self.root, self.coding, source, self.column)
        else:
            data = io.table.load(self.root, source)

        if hasattr(self, "filter"):
            data = data.filter(self.filter)

        if hasattr(self, "select"):
            data = data.select(self.select)

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

    def do_action(self, ctx: fl.ServerCallContext, action: fl.Action) -> None:
        config = pickle.loads(action.body.to_pybytes())

        match action.type:
            case "make-coder":
                io.coder.make(self.root, **config)

            case "make-index":
                io.index.make(self.root, **config)

            case "drop-index":
                io.coder.drop(self.root, **config)

                suffix = "/" + config["name"]
                for path in io.index.list(self.root):
                    if path.endswith(suffix):
                        os.unlink(os.path.join(self.root, io.index.LOCATION, path + ".arrow"))

            case "drop-table":
                io.table.drop(self.root, **config)

            case "remove":
                shutil.rmtree(self.root)

            case "set-coding":
                self.coding = config["coding"]

            case "del-coding":
                if hasattr(self, "coding"):
                    delattr(self, "coding")

            case "set-column":
                self.column = config["column"]

            case "del-column":
                if hasattr(self, "column"):
                    delattr(self, "column")

            case "set-filter":
                self.filter = config["filter"]

            case "del-filter":
                if hasattr(self, "filter"):
                    delattr(self, "filter")

            case "set-select":
                self.select = config["select"]

            case "del-select":
                if hasattr(self, "select"):
                    delattr(self, "select")

            case _:
                raise ValueError()


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

    def make_table(self, name: str, data: pa.RecordBatchReader) -> Self:
        descriptor = fl.FlightDescriptor.for_path(name)

        writer, reader = self.conn.do_put(descriptor, data.schema)

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
        if coding is not None and column is not None:
            self.conn.do_action(fl.Action("set-coding", pickle.dumps({"coding": coding})))
            self.conn.do_action(fl.Action("set-column", pickle.dumps({"column": column})))

        if select is not None:
            self.conn.do_action(fl.Action("set-select", pickle.dumps({"select": select})))

        if filter is not None:
            self.conn.do_action(fl.Action("set-filter", pickle.dumps({"filter": filter})))

        source = ":".join(source) if not isinstance(source, str) else source
        ticket = fl.Ticket(source)
        reader = self.conn.do_get(ticket).to_reader()

        self.conn.do_action(fl.Action("del-coding", pickle.dumps({})))
        self.conn.do_action(fl.Action("del-column", pickle.dumps({})))
        self.conn.do_action(fl.Action("del-select", pickle.dumps({})))
        self.conn.do_action(fl.Action("del-filter", pickle.dumps({})))

        return reader

    def drop_table(self, name: str) -> Self:
        self.conn.do_action(fl.Action("drop-table", pickle.dumps({"name": name})))

        return self

    def make_index(
        self, name: str, source: str | Sequence[str], column: str, config: dict
    ) -> Self:
        self.conn.do_action(
            fl.Action(
                "make-coder",
                pickle.dumps({"name": name, "source": source, "column": column, "config": config}),
            )
        )

        return self.sync_index(name, source, column)

    def sync_index(self, name: str, source: str | Sequence[str], column: str) -> Self:
        self.conn.do_action(
            fl.Action(
                "make-index",
                pickle.dumps({"name": name, "source": source, "column": column}),
            )
        )

        return self

    def drop_index(self, name: str) -> Self:
        self.conn.do_action(
            fl.Action("drop-index", pickle.dumps({"name": name})),
        )

        return self

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
        METRICS: set[str] = {"cosine", "dot", "inner_product", "l2", "euclidean"}

        assert metric in METRICS

        descriptor = fl.FlightDescriptor.for_command(
            pickle.dumps(
                {
                    "coding": coding,
                    "source": source,
                    "column": column,
                    "metric": metric,
                    "select": select,
                    "filter": pickle.dumps(filter),
                    "maxval": maxval,
                    "probes": probes,
                }
            )
        )

        if type(target).__module__.split(".")[0] == "torch":  # Tensor, without importing torch
            target = target.numpy()

        if isinstance(target, np.ndarray):
            target = pa.array(target)

        target = pa.table({"target": target})

        writer, reader = self.conn.do_exchange(descriptor)

        with writer:
            writer.begin(target.schema)
            writer.write_table(target)
            writer.done_writing()

            return reader.read_all()

    def remove(self) -> Self:
        self.conn.do_action(fl.Action("remove", pickle.dumps({})))
        return self
