"""Streaming GGUF v3 writer.

Tensors are declared up front (name, ggml type, shape) and their bytes are then
streamed in declaration order, so a multi-GB synthetic model never has to sit
in memory. Shapes follow ggml order: ``shape[0]`` is the
innermost (row) dimension, e.g. ``token_embd.weight`` is ``[n_embd, n_vocab]``.
"""
from __future__ import annotations

import struct
from typing import Any, BinaryIO, Dict, List, Sequence, Tuple

import numpy as np

from .constants import GGUF_DEFAULT_ALIGNMENT, GGUF_MAGIC, GGUF_VERSION, GGMLType, GGUFValueType, tensor_nbytes


def _pack_str(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


_SCALAR_FMT = {
    GGUFValueType.UINT8: "<B", GGUFValueType.INT8: "<b", GGUFValueType.UINT16: "<H",
    GGUFValueType.INT16: "<h", GGUFValueType.UINT32: "<I", GGUFValueType.INT32: "<i",
    GGUFValueType.FLOAT32: "<f", GGUFValueType.BOOL: "<?", GGUFValueType.UINT64: "<Q",
    GGUFValueType.INT64: "<q", GGUFValueType.FLOAT64: "<d",
}


def _infer_type(v: Any) -> GGUFValueType:
    if isinstance(v, bool):
        return GGUFValueType.BOOL
    if isinstance(v, int):
        return GGUFValueType.UINT32 if 0 <= v < 2 ** 32 else GGUFValueType.INT64
    if isinstance(v, float):
        return GGUFValueType.FLOAT32
    if isinstance(v, str):
        return GGUFValueType.STRING
    if isinstance(v, (list, tuple, np.ndarray)):
        return GGUFValueType.ARRAY
    raise TypeError(type(v))


def _pack_value(v: Any, vtype: GGUFValueType, elem_type: GGUFValueType | None = None) -> bytes:
    if vtype == GGUFValueType.STRING:
        return _pack_str(v)
    if vtype == GGUFValueType.ARRAY:
        seq = list(v) if not isinstance(v, np.ndarray) else v
        if elem_type is None:
            elem_type = _infer_type(seq[0]) if len(seq) else GGUFValueType.INT32
            if elem_type == GGUFValueType.UINT32 and any((isinstance(x, int) and x < 0) for x in seq):
                elem_type = GGUFValueType.INT32
        head = struct.pack("<IQ", int(elem_type), len(seq))
        if elem_type == GGUFValueType.STRING:
            return head + b"".join(_pack_str(s) for s in seq)
        np_t = {GGUFValueType.INT32: np.int32, GGUFValueType.UINT32: np.uint32,
                GGUFValueType.FLOAT32: np.float32, GGUFValueType.INT64: np.int64,
                GGUFValueType.UINT64: np.uint64, GGUFValueType.UINT8: np.uint8,
                GGUFValueType.INT8: np.int8, GGUFValueType.FLOAT64: np.float64,
                GGUFValueType.BOOL: np.bool_, GGUFValueType.INT16: np.int16,
                GGUFValueType.UINT16: np.uint16}[elem_type]
        return head + np.asarray(seq, dtype=np_t).tobytes()
    return struct.pack(_SCALAR_FMT[vtype], v)


class GGUFWriter:
    def __init__(self, path: str, alignment: int = GGUF_DEFAULT_ALIGNMENT):
        self.path = path
        self.alignment = alignment
        self.kv: List[Tuple[str, GGUFValueType, Any, GGUFValueType | None]] = []
        self.tensors: List[Tuple[str, int, Tuple[int, ...], int]] = []  # name, type, shape, nbytes
        self._fh: BinaryIO | None = None
        self._next = 0
        self._offsets: List[int] = []

    # ---- metadata
    def add(self, key: str, value: Any, vtype: GGUFValueType | None = None,
            elem_type: GGUFValueType | None = None):
        self.kv.append((key, vtype if vtype is not None else _infer_type(value), value, elem_type))

    def add_dict(self, d: Dict[str, Any]):
        for k, v in d.items():
            self.add(k, v)

    # ---- tensors
    def declare_tensor(self, name: str, ggml_type: int, shape: Sequence[int]):
        n = int(np.prod(shape))
        self.tensors.append((name, int(ggml_type), tuple(int(s) for s in shape), tensor_nbytes(ggml_type, n)))

    def _align(self, off: int) -> int:
        a = self.alignment
        return (off + a - 1) // a * a

    def begin(self):
        if not any(k == "general.alignment" for k, *_ in self.kv) and self.alignment != GGUF_DEFAULT_ALIGNMENT:
            self.add("general.alignment", self.alignment, GGUFValueType.UINT32)
        fh = open(self.path, "wb")
        fh.write(struct.pack("<IIQQ", GGUF_MAGIC, GGUF_VERSION, len(self.tensors), len(self.kv)))
        for key, vtype, val, et in self.kv:
            fh.write(_pack_str(key) + struct.pack("<I", int(vtype)) + _pack_value(val, vtype, et))
        off = 0
        for name, t, shape, nbytes in self.tensors:
            off = self._align(off)
            self._offsets.append(off)
            fh.write(_pack_str(name) + struct.pack("<I", len(shape)))
            fh.write(struct.pack(f"<{len(shape)}Q", *shape))
            fh.write(struct.pack("<IQ", t, off))
            off += nbytes
        pos = fh.tell()
        fh.write(b"\0" * (self._align(pos) - pos))
        self._data_start = fh.tell()
        self._fh = fh
        self._idx = 0

    def write_tensor_data(self, data):
        """Write the bytes of the next declared tensor (in declaration order)."""
        assert self._fh is not None
        name, t, shape, nbytes = self.tensors[self._idx]
        buf = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        assert buf.size == nbytes, (name, buf.size, nbytes)
        cur = self._fh.tell() - self._data_start
        target = self._offsets[self._idx]
        assert cur <= target
        self._fh.write(b"\0" * (target - cur))
        self._fh.write(memoryview(buf))
        self._idx += 1

    def close(self):
        if self._fh is not None:
            assert self._idx == len(self.tensors), "not every declared tensor was written"
            self._fh.close()
            self._fh = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if exc[0] is None:
            self.close()
        elif self._fh is not None:
            self._fh.close()
