"""Minimal UBJSON (draft 12) reader/writer for XGBoost ``.ubj`` models.

xgboost >= 1.6 saves models as UBJSON by default: the same document as its
JSON model, with numbers big-endian and arrays usually in the optimised
``[$<type>#<count>`` form.  Decoded arrays of numbers come back as numpy
arrays so large models parse quickly.
"""
from __future__ import annotations

import struct
from typing import Any, Tuple

import numpy as np

_NUM = {
    b"i": (">i1", 1), b"U": (">u1", 1), b"I": (">i2", 2), b"l": (">i4", 4),
    b"L": (">i8", 8), b"d": (">f4", 4), b"D": (">f8", 8),
}


class UBJSONError(ValueError):
    pass


class _Dec:
    def __init__(self, buf: bytes):
        self.b = buf
        self.p = 0

    def byte(self) -> bytes:
        if self.p >= len(self.b):
            raise UBJSONError("truncated UBJSON")
        c = self.b[self.p:self.p + 1]
        self.p += 1
        return c

    def marker(self) -> bytes:
        c = self.byte()
        while c == b"N":
            c = self.byte()
        return c

    def number(self, t: bytes):
        dt, n = _NUM[t]
        if self.p + n > len(self.b):
            raise UBJSONError("truncated UBJSON number")
        v = np.frombuffer(self.b, dtype=dt, count=1, offset=self.p)[0]
        self.p += n
        return v.item()

    def length(self) -> int:
        t = self.marker()
        if t not in _NUM or t in (b"d", b"D"):
            raise UBJSONError("bad length type %r" % t)
        n = int(self.number(t))
        if n < 0:
            raise UBJSONError("negative length")
        return n

    def string(self) -> str:
        n = self.length()
        s = self.b[self.p:self.p + n]
        self.p += n
        return s.decode("utf-8")

    def value(self, t: bytes = None) -> Any:
        t = t or self.marker()
        if t in _NUM:
            return self.number(t)
        if t == b"S" or t == b"H":
            return self.string()
        if t == b"C":
            return self.byte().decode()
        if t == b"T":
            return True
        if t == b"F":
            return False
        if t == b"Z":
            return None
        if t == b"[":
            return self.array()
        if t == b"{":
            return self.obj()
        raise UBJSONError("unknown UBJSON marker %r at %d" % (t, self.p - 1))

    def _container_header(self) -> Tuple[bytes, int]:
        typ, cnt = None, -1
        if self.b[self.p:self.p + 1] == b"$":
            self.p += 1
            typ = self.byte()
        if self.b[self.p:self.p + 1] == b"#":
            self.p += 1
            cnt = self.length()
        if typ is not None and cnt < 0:
            raise UBJSONError("typed container without count")
        return typ, cnt

    def array(self):
        typ, cnt = self._container_header()
        if typ in _NUM and cnt >= 0:
            dt, n = _NUM[typ]
            if self.p + n * cnt > len(self.b):
                raise UBJSONError("truncated UBJSON array")
            a = np.frombuffer(self.b, dtype=dt, count=cnt, offset=self.p)
            self.p += n * cnt
            return a.astype(dt[1:])          # native byte order
        if cnt >= 0:
            return [self.value(typ) for _ in range(cnt)]
        out = []
        while True:
            t = self.marker()
            if t == b"]":
                return out
            out.append(self.value(t))

    def obj(self):
        typ, cnt = self._container_header()
        out = {}
        if cnt >= 0:
            for _ in range(cnt):
                k = self.string()
                out[k] = self.value(typ)
            return out
        while True:
            if self.b[self.p:self.p + 1] == b"}":
                self.p += 1
                return out
            k = self.string()
            out[k] = self.value()


def loads(buf: bytes) -> Any:
    d = _Dec(buf)
    v = d.value()
    return v


# ------------------------------------------------------------------ writer
def _len(n: int) -> bytes:
    return b"l" + struct.pack(">i", n) if n > 255 else b"U" + struct.pack(">B", n)


def dumps(v: Any) -> bytes:
    """Encode python / numpy values; numeric arrays use the optimised form."""
    if isinstance(v, dict):
        out = [b"{"]
        for k, x in v.items():
            kb = str(k).encode()
            out += [_len(len(kb)), kb, dumps(x)]
        out.append(b"}")
        return b"".join(out)
    if isinstance(v, np.ndarray):
        if v.dtype.kind == "f":
            t, dt = (b"d", ">f4") if v.dtype == np.float32 else (b"D", ">f8")
        elif v.dtype.kind in "iu":
            t, dt = (b"l", ">i4") if v.dtype.itemsize <= 4 else (b"L", ">i8")
        elif v.dtype.kind == "b":
            t, dt = b"U", ">u1"
        else:
            return dumps(v.tolist())
        return b"[$" + t + b"#" + _len(v.size) + np.ascontiguousarray(v, dtype=dt).tobytes()
    if isinstance(v, (list, tuple)):
        return b"[" + b"".join(dumps(x) for x in v) + b"]"
    if isinstance(v, bool):
        return b"T" if v else b"F"
    if v is None:
        return b"Z"
    if isinstance(v, (int, np.integer)):
        return b"L" + struct.pack(">q", int(v))
    if isinstance(v, (float, np.floating)):
        return b"D" + struct.pack(">d", float(v))
    if isinstance(v, str):
        b = v.encode()
        return b"S" + _len(len(b)) + b
    raise UBJSONError(f"cannot encode {type(v)}")
