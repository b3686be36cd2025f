"""The quint8 tensor column type (fenix_amd/ex/arrow/quint8.py), CPU only.

The reference module (src/fenix/ex/arrow/quint8/quint8.py) does not import in
this container (it needs msgspec, which is not installed), so parity is
anchored on the library call it makes: torch.quantize_per_tensor_dynamic(x,
torch.quint8, reduce_range=True) (quint8.py:24-29, 91-96) and its own
dequantize formula (quint8.py:53-54, restated in oracle.dequantize)."""

from __future__ import annotations

import msgpack
import numpy as np
import pyarrow as pa
import torch

from fenix_amd.ex.arrow import quint8 as Q
from fenix_amd.io import table
from oracle import oracle as O


def test_quantize_is_torch_dynamic_reduce_range():
    x = O.fill_normal(500, 24, seed=3, cluster=50)
    a = Q.from_numpy(x)
    t = torch.quantize_per_tensor_dynamic(torch.from_numpy(x), torch.quint8, reduce_range=True)
    np.testing.assert_array_equal(a.codes(), t.int_repr().numpy())
    assert a.type.scale == t.q_scale() and a.type.shift == t.q_zero_point()
    assert a.codes().max() <= 127  # reduce_range: 7-bit codes
    assert a.type.shape == (24,) and a.type.storage_type == pa.list_(pa.uint8(), 24)


def test_dequantize_matches_reference_formula_and_torch():
    x = O.fill_normal(300, 16, seed=4)
    a = Q.from_numpy(x)
    deq = a.to_numpy().dequantize()
    np.testing.assert_array_equal(deq, O.dequantize(a.codes(), a.type.scale, a.type.shift))
    tq = torch.quantize_per_tensor_dynamic(torch.from_numpy(x), torch.quint8, reduce_range=True)
    np.testing.assert_allclose(deq, tq.dequantize().numpy(), rtol=0, atol=1e-6)
    assert np.abs(deq - x).max() <= a.type.scale / 2 + 1e-6


def test_extension_serialization_is_msgpack_map():
    t = Q.QUInt8TensorType((4, 8), 0.125, 7)
    raw = t.__arrow_ext_serialize__()
    assert msgpack.unpackb(raw) == {"shape": [4, 8], "scale": 0.125, "shift": 7}
    back = Q.QUInt8TensorType.__arrow_ext_deserialize__(t.storage_type, raw)
    assert back == t or (back.shape, back.scale, back.shift) == (t.shape, t.scale, t.shift)


def test_ipc_roundtrip_through_table_files(tmp_path):
    x = O.fill_normal(2500, 32, seed=5)
    a = Q.from_numpy(x)
    ids = pa.array(np.arange(2500, dtype=np.int64))
    src = pa.table({"id": ids, "vector": a})
    table.make(str(tmp_path), "q/t", src.to_reader(max_chunksize=1000))
    back = table.load(str(tmp_path), "q/t")
    col = back.column("vector")
    assert Q.is_quint8(col.type)
    assert (col.type.scale, col.type.shift) == (a.type.scale, a.type.shift)
    got = np.concatenate([c.codes() for c in col.chunks])
    np.testing.assert_array_equal(got, a.codes())


def test_scalar_and_array_conversions():
    x = O.fill_normal(6, 10, seed=6)
    arr = Q.from_torch(torch.from_numpy(x))
    tt = arr.to_torch()
    assert tt.is_quantized and tuple(tt.shape) == (6, 10)
    s = Q.QUInt8TensorScalar.from_numpy(x[0])
    assert s.type.shape == (10,)
    np.testing.assert_allclose(s.to_numpy().dequantize(), x[0], atol=s.type.scale)
    nd = Q.QUInt8NDArray.quantize(x)
    again = Q.QUInt8TensorArray.from_numpy(nd)
    np.testing.assert_array_equal(again.codes(), nd.view(np.ndarray))
