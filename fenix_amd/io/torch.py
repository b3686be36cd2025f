"""Arrow ``FixedSizeList`` -> ``torch.Tensor`` bridge.

Mirrors src/fenix/io/torch/torch.py:6-10 (DLPack, zero-copy).  One deliberate
fix: the reference reads ``x.values`` from element 0 and so ignores the parent
array's offset (a sliced array returns the wrong rows); this
version slices the values to the array's own rows.
"""

from __future__ import annotations

import pyarrow as pa
import torch
from torch import Tensor


def from_arrow(x: pa.FixedSizeListArray | pa.FixedSizeListScalar) -> Tensor:
    if isinstance(x, pa.FixedSizeListScalar):
        return torch.from_dlpack(x.values)

    d = x.type.list_size
    values = x.values.slice(x.offset * d, len(x) * d)
    return torch.from_dlpack(values).view(-1, d)
