"""``fenix_amd.ex`` — Arrow extension types (src/fenix/ex of the reference).

Only the quint8 tensor type is provided: it is the one the search path can
scan (1-byte codes dequantised in the scan's registers)."""

from . import arrow  # noqa: F401
