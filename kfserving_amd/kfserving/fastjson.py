"""ctypes binding of libkfserve.so (include/kfserve.h): the native v1 body
parser.  ``parse_instances(body)`` returns the float64 matrix that
``np.asarray(json.loads(body)["instances"], dtype=np.float64)`` would give
for bodies of the form ``{"instances": [[...], ...]}``, or None when the body
is outside that subset (the caller then takes the json.loads path, which keeps
the reference's behaviour and error messages, handlers/http.py:66-74)."""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import numpy as np

# KFSERVE_LIB: another build of the same library, e.g. the AddressSanitizer
# build (__graft_entry__.build_host(asan=True), tests/test_asan_fuzz.py)
_LIB_PATH = os.environ.get("KFSERVE_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libkfserve.so")
_lib = None
_lock = threading.Lock()

KF_PARSED, KF_FALLBACK, KF_ERR_SPACE = 1, 0, -1


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None or path is not None:
            p = path or _LIB_PATH
            if not os.path.exists(p):
                raise RuntimeError(f"{p} not found: build it with "
                                   "`python -c 'import __graft_entry__ as g; g.build()'`")
            lib = ctypes.CDLL(p)
            lib.kf_parse_instances.restype = ctypes.c_int
            lib.kf_parse_instances.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p,
                                               ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                               ctypes.POINTER(ctypes.c_int64)]
            lib.kf_parse_instances_mt.restype = ctypes.c_int
            lib.kf_parse_instances_mt.argtypes = lib.kf_parse_instances.argtypes + [ctypes.c_int32]
            _lib = lib
        return _lib


class JsonInstances(np.ndarray):
    """A float64 [rows, cols] matrix decoded from a JSON ``instances`` list.

    Marks the origin so the plugins apply the same conversion they apply to a
    Python list (e.g. xgboost's DMatrix(list): 0 means missing), not the one
    for an ndarray argument."""


# host threads for bodies of >= 1 MB (kf_parse_instances_mt); the serving box
# gives a process a share of its cores, so a fixed small count
PARSE_THREADS = max(1, min(8, int(os.environ.get("KF_PARSE_THREADS", "8"))))


def parse_instances(body: bytes, threads: Optional[int] = None) -> Optional[JsonInstances]:
    lib = load_library()
    n = len(body)
    # a number takes >= 1 byte plus a separator: (n + 1) // 2 values always fit
    out = np.empty((n + 1) // 2, dtype=np.float64)
    rows, cols = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = lib.kf_parse_instances_mt(body, n, out.ctypes.data, out.size, ctypes.byref(rows),
                                   ctypes.byref(cols), PARSE_THREADS if threads is None else threads)
    if rc != KF_PARSED:
        return None
    r, c = rows.value, cols.value
    return out[:r * c].reshape(r, c).view(JsonInstances)
