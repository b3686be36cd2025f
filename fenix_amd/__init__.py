"""fenix_amd — MI355X (gfx950) brute-force kNN engine behind fenix's search API.

Import surface mirrors the reference's ``fenix`` package
(src/fenix/__init__.py:1-2): ``io``, ``Flight``, ``Server``.
"""

from . import io
from .flight import Flight, Server

__version__ = "0.1.0"
__all__ = ["io", "Flight", "Server"]
