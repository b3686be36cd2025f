"""``fenix_amd.io`` — same module layout as the reference's ``fenix.io``
(src/fenix/io/__init__.py:1): arrow, table, torch, coder, index (brute-force
search and the coded multi-codebook index).  The random batch loader
(io/batch) is not part of the search path and is not provided.

Submodules load on first use (PEP 562), so a process that only uses the
Flight client never imports torch or the HIP library: an ``import torch`` in a
client process was measured to raise every Flight round trip from ~2 ms to
~12-15 ms."""

import importlib

_SUBMODULES = ("arrow", "coder", "index", "table", "torch")


def __getattr__(name):
    if name in _SUBMODULES:
        mod = importlib.import_module(f"{__name__}.{name}")
        globals()[name] = mod
        return mod
    raise AttributeError(name)


def __dir__():
    return sorted(list(globals()) + list(_SUBMODULES))
