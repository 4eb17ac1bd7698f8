"""Pure-Python GGUF v3 reader (numpy memmap, zero-copy tensor views).

Used by tooling, tests and the torch reference model. The serving engine
parses the file natively (csrc/runtime/gguf.cpp); ``tests/test_gguf.py`` checks
that both agree.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Any, Dict, List, Tuple

import numpy as np

from .constants import GGUF_DEFAULT_ALIGNMENT, GGUF_MAGIC, GGMLType, GGUFValueType, tensor_nbytes
from .quants import dequantize

_SCALAR = {
    GGUFValueType.UINT8: ("<B", 1), GGUFValueType.INT8: ("<b", 1), GGUFValueType.UINT16: ("<H", 2),
    GGUFValueType.INT16: ("<h", 2), GGUFValueType.UINT32: ("<I", 4), GGUFValueType.INT32: ("<i", 4),
    GGUFValueType.FLOAT32: ("<f", 4), GGUFValueType.BOOL: ("<?", 1), GGUFValueType.UINT64: ("<Q", 8),
    GGUFValueType.INT64: ("<q", 8), GGUFValueType.FLOAT64: ("<d", 8),
}
_NP = {GGUFValueType.UINT8: np.uint8, GGUFValueType.INT8: np.int8, GGUFValueType.UINT16: np.uint16,
       GGUFValueType.INT16: np.int16, GGUFValueType.UINT32: np.uint32, GGUFValueType.INT32: np.int32,
       GGUFValueType.FLOAT32: np.float32, GGUFValueType.BOOL: np.bool_, GGUFValueType.UINT64: np.uint64,
       GGUFValueType.INT64: np.int64, GGUFValueType.FLOAT64: np.float64}


@dataclass
class TensorInfo:
    name: str
    shape: Tuple[int, ...]  # ggml order (shape[0] innermost)
    ggml_type: int
    offset: int             # absolute file offset
    nbytes: int

    @property
    def n_elements(self) -> int:
        return int(np.prod(self.shape))


class GGUFReader:
    def __init__(self, path: str):
        self.path = path
        self._mm = np.memmap(path, dtype=np.uint8, mode="r")
        self._pos = 0
        magic, self.version, n_tensors, n_kv = struct.unpack_from("<IIQQ", self._mm, 0)
        if magic != GGUF_MAGIC:
            raise ValueError(f"{path}: not a GGUF file")
        if self.version not in (2, 3):
            raise ValueError(f"{path}: unsupported GGUF version {self.version}")
        self._pos = 24
        self.metadata: Dict[str, Any] = {}
        for _ in range(n_kv):
            key = self._str()
            vtype = GGUFValueType(self._u32())
            self.metadata[key] = self._value(vtype)
        infos = []
        for _ in range(n_tensors):
            name = self._str()
            nd = self._u32()
            shape = struct.unpack_from(f"<{nd}Q", self._mm, self._pos)
            self._pos += 8 * nd
            t = self._u32()
            off = struct.unpack_from("<Q", self._mm, self._pos)[0]
            self._pos += 8
            infos.append((name, tuple(int(s) for s in shape), t, off))
        align = int(self.metadata.get("general.alignment", GGUF_DEFAULT_ALIGNMENT))
        self.data_offset = (self._pos + align - 1) // align * align
        self.tensors: Dict[str, TensorInfo] = {}
        self.tensor_order: List[str] = []
        for name, shape, t, off in infos:
            n = int(np.prod(shape))
            self.tensors[name] = TensorInfo(name, shape, t, self.data_offset + off, tensor_nbytes(t, n))
            self.tensor_order.append(name)

    # ---- primitive decoding
    def _u32(self) -> int:
        v = struct.unpack_from("<I", self._mm, self._pos)[0]
        self._pos += 4
        return v

    def _u64(self) -> int:
        v = struct.unpack_from("<Q", self._mm, self._pos)[0]
        self._pos += 8
        return v

    def _str(self) -> str:
        n = self._u64()
        s = bytes(self._mm[self._pos:self._pos + n]).decode("utf-8", errors="replace")
        self._pos += n
        return s

    def _value(self, vtype: GGUFValueType):
        if vtype == GGUFValueType.STRING:
            return self._str()
        if vtype == GGUFValueType.ARRAY:
            et = GGUFValueType(self._u32())
            n = self._u64()
            if et == GGUFValueType.STRING:
                return [self._str() for _ in range(n)]
            if et == GGUFValueType.ARRAY:
                return [self._value(et) for _ in range(n)]
            dt = np.dtype(_NP[et]).newbyteorder("<")
            arr = np.frombuffer(self._mm, dtype=dt, count=n, offset=self._pos).copy()
            self._pos += n * dt.itemsize
            return arr.tolist()
        fmt, size = _SCALAR[vtype]
        v = struct.unpack_from(fmt, self._mm, self._pos)[0]
        self._pos += size
        return v

    # ---- tensor access
    def raw(self, name: str) -> np.ndarray:
        ti = self.tensors[name]
        return self._mm[ti.offset:ti.offset + ti.nbytes]

    def dequant(self, name: str, arith: str = "f32") -> np.ndarray:
        """float32 array in row-major numpy order (reverse of ggml shape)."""
        ti = self.tensors[name]
        return dequantize(np.asarray(self.raw(name)), ti.ggml_type, ti.n_elements, arith=arith).reshape(ti.shape[::-1])

    def get(self, key: str, default=None):
        return self.metadata.get(key, default)
