"""Per-tensor affine quint8 tensor columns — mirrors
src/fenix/ex/arrow/quint8/quint8.py of the reference.

* ``QUInt8NDArray`` (quint8.py:11-54): uint8 codes + ``scale`` + ``shift``
  (zero point); ``quantize`` = torch.quantize_per_tensor_dynamic(x, quint8,
  reduce_range=True) (codes 0..127, the reference's call, :24-29);
  ``dequantize`` = scale * (codes - shift) in float32 (:53-54).
* ``QUInt8TensorType`` (:56-84): Arrow extension type ``"tensor::qint8"``
  over ``fixed_size_list<uint8>[prod(shape)]``, its parameters serialized as a
  msgpack map {shape, scale, shift} (the reference uses msgspec, which writes
  the same msgpack; msgpack-python is used here).  Registered with pyarrow on
  import, so IPC files written through Flight read back as this type.
* ``QUInt8TensorArray`` / ``QUInt8TensorScalar`` (:87-176), ``from_numpy`` /
  ``from_torch`` (:179-184).

Search: a column of this type is staged to HBM as its 1-byte codes and
scanned by the same fused kernel with the codes dequantised in registers
(fx_knn_search_ex, FX_DTYPE_QU8): 768 bytes per 768-d row instead of 3 072.
The reference cannot search such a column (io.torch.from_arrow reads
``.values``, which an ExtensionArray does not have).
"""

from __future__ import annotations

from typing import Sequence, Type

from typing import TYPE_CHECKING

import msgpack
import numpy as np
import pyarrow as pa
from numpy.typing import ArrayLike, NDArray

if TYPE_CHECKING:
    from torch import Tensor

EXTENSION_NAME = "tensor::qint8"


def _torch():
    import torch  # lazily: registering the type (io.arrow) must not pull torch into clients

    return torch


def _quantize(tensor: Tensor) -> Tensor:
    torch = _torch()
    if not tensor.is_quantized:
        tensor = torch.quantize_per_tensor_dynamic(tensor, dtype=torch.quint8, reduce_range=True)
    return tensor


class QUInt8NDArray(np.ndarray):
    scale: float
    shift: int

    def __new__(cls, array: NDArray[np.uint8], scale: float, shift: int) -> "QUInt8NDArray":
        q = np.asarray(array, dtype=np.uint8).view(cls)
        q.scale = scale
        q.shift = shift
        return q

    def __array_finalize__(self, obj) -> None:
        self.scale = getattr(obj, "scale", 1.0)
        self.shift = getattr(obj, "shift", 0)

    @staticmethod
    def from_torch(tensor: Tensor) -> "QUInt8NDArray":
        tensor = _quantize(tensor)
        return QUInt8NDArray(tensor.int_repr().numpy(), tensor.q_scale(), tensor.q_zero_point())

    def to_torch(self) -> Tensor:
        torch = _torch()
        return torch._make_per_tensor_quantized_tensor(
            torch.from_numpy(np.ascontiguousarray(self.view(np.ndarray))), self.scale, self.shift
        )

    @staticmethod
    def quantize(array: ArrayLike) -> "QUInt8NDArray":
        return QUInt8NDArray.from_torch(_torch().from_numpy(np.asarray(array, dtype=np.float32)))

    def dequantize(self) -> NDArray[np.float32]:
        return self.scale * (self.astype(np.float32).view(np.ndarray) - self.shift)


class QUInt8TensorType(pa.ExtensionType):
    def __init__(self, shape: Sequence[int], scale: float, shift: int) -> None:
        self.shape = tuple(int(s) for s in shape)
        self.scale = float(scale)
        self.shift = int(shift)
        super().__init__(pa.list_(pa.uint8(), int(np.prod(self.shape))), EXTENSION_NAME)

    def __arrow_ext_serialize__(self) -> bytes:
        return msgpack.packb({"shape": list(self.shape), "scale": self.scale,
                              "shift": self.shift})

    @classmethod
    def __arrow_ext_deserialize__(cls, storage_type: pa.DataType,
                                  serialized: bytes) -> "QUInt8TensorType":
        return QUInt8TensorType(**msgpack.unpackb(serialized))

    def __arrow_ext_class__(self) -> Type["QUInt8TensorArray"]:
        return QUInt8TensorArray

    def __arrow_ext_scalar_class__(self) -> Type["QUInt8TensorScalar"]:
        return QUInt8TensorScalar

    def __reduce__(self):
        return QUInt8TensorType, (self.shape, self.scale, self.shift)


class QUInt8TensorArray(pa.ExtensionArray):
    @staticmethod
    def from_torch(tensor: Tensor) -> "QUInt8TensorArray":
        tensor = _quantize(tensor)
        batch, shape = tensor.shape[0], tensor.shape[1:]
        codes = np.ascontiguousarray(tensor.int_repr().numpy()).reshape(-1)
        storage = pa.FixedSizeListArray.from_arrays(pa.array(codes, pa.uint8()),
                                                    int(np.prod(shape)))
        assert len(storage) == batch
        return pa.ExtensionArray.from_storage(
            QUInt8TensorType(shape, tensor.q_scale(), tensor.q_zero_point()), storage
        )

    @staticmethod
    def from_numpy(tensor: np.ndarray) -> "QUInt8TensorArray":
        if isinstance(tensor, QUInt8NDArray):
            return QUInt8TensorArray.from_torch(tensor.to_torch())
        return QUInt8TensorArray.from_numpy(QUInt8NDArray.quantize(tensor))

    def codes(self) -> NDArray[np.uint8]:
        """[len, prod(shape)] uint8 view of the stored codes (offset-aware)."""
        st = self.storage
        d = st.type.list_size
        vals = st.values
        buf = vals.buffers()[1]
        start = vals.offset + st.offset * d
        return np.frombuffer(buf, dtype=np.uint8, count=len(st) * d, offset=start).reshape(-1, d)

    def to_torch(self) -> Tensor:
        torch = _torch()
        codes = torch.from_numpy(self.codes().copy()).view(len(self), *self.type.shape)
        return torch._make_per_tensor_quantized_tensor(codes, self.type.scale, self.type.shift)

    def to_numpy(self) -> QUInt8NDArray:
        return QUInt8NDArray.from_torch(self.to_torch())


class QUInt8TensorScalar(pa.ExtensionScalar):
    @staticmethod
    def from_torch(tensor: Tensor) -> "QUInt8TensorScalar":
        tensor = _quantize(tensor)
        value = pa.scalar(tensor.int_repr().reshape(-1).numpy(),
                          pa.list_(pa.uint8(), int(np.prod(tensor.shape))))
        return pa.ExtensionScalar.from_storage(
            QUInt8TensorType(tensor.shape, tensor.q_scale(), tensor.q_zero_point()), value
        )

    @staticmethod
    def from_numpy(tensor: np.ndarray) -> "QUInt8TensorScalar":
        if isinstance(tensor, QUInt8NDArray):
            return QUInt8TensorScalar.from_torch(tensor.to_torch())
        return QUInt8TensorScalar.from_torch(_torch().from_numpy(np.asarray(tensor, np.float32)))

    def to_torch(self) -> Tensor:
        torch = _torch()
        codes = torch.from_numpy(np.asarray(self.value.values.to_numpy(), np.uint8).copy())
        return torch._make_per_tensor_quantized_tensor(codes.view(*self.type.shape),
                                                       self.type.scale, self.type.shift)

    def to_numpy(self) -> QUInt8NDArray:
        return QUInt8NDArray(self.value.values.to_numpy().reshape(*self.type.shape),
                             self.type.scale, self.type.shift)


def from_numpy(tensor: np.ndarray) -> QUInt8TensorArray:
    return QUInt8TensorArray.from_numpy(tensor)


def from_torch(tensor: Tensor) -> QUInt8TensorArray:
    return QUInt8TensorArray.from_torch(tensor)


def is_quint8(t: pa.DataType) -> bool:
    return isinstance(t, pa.ExtensionType) and t.extension_name == EXTENSION_NAME


try:
    pa.register_extension_type(QUInt8TensorType((1,), 1.0, 0))
except pa.ArrowKeyError:  # already registered (module reloaded)
    pass
