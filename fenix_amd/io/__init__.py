"""``fenix_amd.io`` — same module layout as the reference's ``fenix.io``
(src/fenix/io/__init__.py:1): arrow, table, torch, coder, index.  The coded
(product-quantised) index and the random batch loader are outside the MI355X
hot path and are not provided."""

from . import arrow, coder, index, table, torch  # noqa: F401
