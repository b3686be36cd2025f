"""Server launcher — mirrors src/fenix/launch.py of the reference
(``python -m fenix_amd.launch ROOT --host H --port P``), plus the device
list the server shards its tables over (``--devices all`` or ``0,1,2``; sets
FENIX_AMD_DEVICES, see engine.devices) and an optional warm start that stages
named sources into HBM before the first request."""

from __future__ import annotations

import logging
import os
from typing import List, Optional

import typer

logging.basicConfig()
LOGGER = logging.getLogger("fenix")
LOGGER.setLevel(level=logging.INFO)


def launch(root: str, host: str = "0.0.0.0", port: int = 9001,
           devices: Optional[str] = typer.Option(None, help="'all' or ordinals '0,1,...'"),
           preload: Optional[List[str]] = typer.Option(None, help="source:column to stage")):
    if devices:
        os.environ["FENIX_AMD_DEVICES"] = devices
    from .flight import Server

    server = Server(root, host, port)
    for item in preload or []:
        from .engine import CACHE, devices as _devices
        from .io import table

        name, column = item.rsplit(":", 1)
        t = table.load(server.root, name)
        CACHE.get(table.path(server.root, name), t, column, _devices())
        LOGGER.info(f" staged {name}:{column} ({t.num_rows} rows)")

    LOGGER.info(f" Server started at {server.grpc}")

    server.serve()


def main() -> None:
    typer.run(launch)


if __name__ == "__main__":
    main()
