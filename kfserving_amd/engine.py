"""ctypes binding of libtreeinfer.so (include/treeinfer.h).

This is the Python side of the drop-in boundary: the plugins call
:meth:`DeviceForest.predict` where the reference called the third-party
library's own ctypes binding (``Booster.predict`` at
python/xgbserver/xgbserver/model.py:47 and python/lgbserver/lgbserver/model.py:51,
``estimator.predict`` at python/sklearnserver/sklearnserver/model.py:50).

There is no CPU fallback: if the HIP library is missing or the device call
fails, a :class:`TreeInferError` is raised.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Sequence

import numpy as np

from .forest import (Forest, OUT_CONTRIB, OUT_LEAF, OUT_MARGIN, OUT_PREDICT, TI_F32, TI_F64,
                     TI_I32)

ABI_VERSION = 4
_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.environ.get("TREEINFER_LIB", os.path.join(_LIB_DIR, "libtreeinfer.so"))

EXPORTED_SYMBOLS = (
    "ti_forest_create", "ti_forest_destroy", "ti_forest_get_info", "ti_output_shape",
    "ti_predict", "ti_predict_device", "ti_transform_device", "ti_last_error", "ti_device_count",
    "ti_abi_version", "ti_forest_set_option",
)

# ti_forest_set_option options (include/treeinfer.h)
OPT_SHAP_TABLE_ROWS = 1
OPT_SHAP_TABLE_MB = 2
OPT_HOST_REGISTER = 3


class TreeInferError(RuntimeError):
    """A libtreeinfer call failed (carries the library's last-error text)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"libtreeinfer error {code}: {message}")
        self.code = code


class _ForestDesc(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("n_trees", ctypes.c_int32),
        ("n_features", ctypes.c_int32),
        ("n_groups", ctypes.c_int32),
        ("leaf_width", ctypes.c_int32),
        ("accum_dtype", ctypes.c_int32),
        ("base_first", ctypes.c_int32),
        ("lgb_zero_map", ctypes.c_int32),
        ("n_nodes", ctypes.c_int64),
        ("tree_offset", ctypes.c_void_p),
        ("tree_group", ctypes.c_void_p),
        ("feature", ctypes.c_void_p),
        ("threshold", ctypes.c_void_p),
        ("flags", ctypes.c_void_p),
        ("left", ctypes.c_void_p),
        ("right", ctypes.c_void_p),
        ("leaf_id", ctypes.c_void_p),
        ("leaf_value", ctypes.c_void_p),
        ("base_margin", ctypes.c_void_p),
        ("average_divisor", ctypes.c_double),
        ("transform", ctypes.c_int32),
        ("reserved0", ctypes.c_int32),
        ("transform_param", ctypes.c_double),
        ("n_cat_words", ctypes.c_int64),
        ("cat_bits", ctypes.c_void_p),
        ("cat_offset", ctypes.c_void_p),
        ("cat_nwords", ctypes.c_void_p),
        ("cover", ctypes.c_void_p),
    ]


class _ForestInfo(ctypes.Structure):
    _fields_ = [
        ("layout", ctypes.c_int32),
        ("depth", ctypes.c_int32),
        ("n_trees", ctypes.c_int32),
        ("n_groups", ctypes.c_int32),
        ("n_features", ctypes.c_int32),
        ("n_devices", ctypes.c_int32),
        ("device_bytes", ctypes.c_int64),
        ("tree_stride_bytes", ctypes.c_int64),
        ("walk", ctypes.c_int32),
        ("bin_bits", ctypes.c_int32),
        ("tree_ilp", ctypes.c_int32),
        ("n_stages", ctypes.c_int32),
        ("top_depth", ctypes.c_int32),
        ("bottom", ctypes.c_int32),
        ("shap_table", ctypes.c_int32),
        ("reserved1", ctypes.c_int32),
        ("shap_table_bytes", ctypes.c_int64),
        ("shap_table_build_ms", ctypes.c_double),
    ]


_lib = None
_lib_lock = threading.Lock()


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libtreeinfer.so once; raise loudly if it is missing."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise TreeInferError(-1, f"{p} not found: build it with "
                                     "`python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(p)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        lib.ti_abi_version.restype = i32
        lib.ti_abi_version.argtypes = []
        lib.ti_last_error.restype = ctypes.c_char_p
        lib.ti_last_error.argtypes = []
        lib.ti_device_count.restype = ctypes.c_int
        lib.ti_device_count.argtypes = [ctypes.POINTER(i32)]
        lib.ti_forest_create.restype = ctypes.c_int
        lib.ti_forest_create.argtypes = [ctypes.POINTER(_ForestDesc), ctypes.POINTER(i32), i32,
                                         ctypes.POINTER(vp)]
        lib.ti_forest_destroy.restype = ctypes.c_int
        lib.ti_forest_destroy.argtypes = [vp]
        lib.ti_forest_get_info.restype = ctypes.c_int
        lib.ti_forest_get_info.argtypes = [vp, ctypes.POINTER(_ForestInfo)]
        lib.ti_output_shape.restype = ctypes.c_int
        lib.ti_output_shape.argtypes = [vp, i32, i64, ctypes.POINTER(i64), ctypes.POINTER(i32)]
        lib.ti_predict.restype = ctypes.c_int
        lib.ti_predict.argtypes = [vp, vp, i32, i64, i32, i64, i32, vp, i64]
        lib.ti_predict_device.restype = ctypes.c_int
        lib.ti_predict_device.argtypes = [vp, i32, vp, i32, i64, i32, i64, i32, vp, i64, vp]
        lib.ti_forest_set_option.restype = ctypes.c_int
        lib.ti_forest_set_option.argtypes = [vp, i32, i64]
        lib.ti_transform_device.restype = ctypes.c_int
        lib.ti_transform_device.argtypes = [vp, i32, vp, i64, vp, i64, vp]
        if lib.ti_abi_version() != ABI_VERSION:
            raise TreeInferError(-1, f"ABI mismatch: library {lib.ti_abi_version()}, "
                                     f"binding {ABI_VERSION}")
        if path is None:
            _lib = lib
        return lib


def _check(lib, rc: int) -> None:
    if rc != 0:
        msg = lib.ti_last_error()
        raise TreeInferError(rc, msg.decode("utf-8", "replace") if msg else "unknown error")


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int32(0)
    _check(lib, lib.ti_device_count(ctypes.byref(n)))
    return int(n.value)


def default_devices() -> Sequence[int]:
    """Devices a server process drives: $TREEINFER_DEVICES or all visible."""
    env = os.environ.get("TREEINFER_DEVICES")
    if env:
        return [int(x) for x in env.split(",") if x.strip()]
    return list(range(device_count()))


def prepare_input(forest: Forest, X) -> np.ndarray:
    """Convert X the way the library being replaced converts it.

    XGBoost's DMatrix and sklearn's check_array make float32; LightGBM
    keeps float32 input as float32 and reads anything else as float64.
    """
    X = np.asarray(X)
    if X.ndim == 1:
        X = X.reshape(1, -1)
    if X.ndim != 2:
        raise ValueError(f"expected a 2-D input, got shape {X.shape}")
    if forest.input_dtype == TI_F64 and X.dtype != np.float32:
        return np.ascontiguousarray(X, dtype=np.float64)
    return np.ascontiguousarray(X, dtype=np.float32)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class DeviceForest:
    """A forest resident on one or more GPUs (a ``ti_forest*`` handle)."""

    def __init__(self, forest: Forest, devices: Optional[Sequence[int]] = None):
        self.forest = forest.contiguous()
        self.forest.validate()
        self._lib = load_library()
        devs = list(devices) if devices is not None else list(default_devices())
        if not devs:
            raise TreeInferError(-2, "no HIP device visible")
        self.devices = devs
        f = self.forest
        desc = _ForestDesc()
        desc.abi_version = ABI_VERSION
        desc.n_trees = f.n_trees
        desc.n_features = f.n_features
        desc.n_groups = f.n_groups
        desc.leaf_width = f.leaf_width
        desc.accum_dtype = f.accum_dtype
        desc.base_first = 1 if f.base_first else 0
        desc.lgb_zero_map = 1 if f.lgb_zero_map else 0
        desc.n_nodes = f.n_nodes
        desc.tree_offset = _ptr(f.tree_offset)
        desc.tree_group = _ptr(f.tree_group)
        desc.feature = _ptr(f.feature)
        desc.threshold = _ptr(f.threshold)
        desc.flags = _ptr(f.flags)
        desc.left = _ptr(f.left)
        desc.right = _ptr(f.right)
        desc.leaf_id = _ptr(f.leaf_id)
        desc.leaf_value = _ptr(f.leaf_value)
        desc.base_margin = _ptr(f.base_margin)
        desc.average_divisor = float(f.average_divisor)
        desc.transform = int(f.transform)
        desc.transform_param = float(f.transform_param)
        if f.cat_bits is not None:
            desc.n_cat_words = int(f.cat_bits.shape[0])
            desc.cat_bits = _ptr(f.cat_bits) if f.cat_bits.size else None
            desc.cat_offset = _ptr(f.cat_offset)
            desc.cat_nwords = _ptr(f.cat_nwords)
        if f.cover is not None:
            desc.cover = _ptr(f.cover)
        dev_arr = (ctypes.c_int32 * len(devs))(*devs)
        handle = ctypes.c_void_p()
        _check(self._lib, self._lib.ti_forest_create(ctypes.byref(desc), dev_arr, len(devs),
                                                     ctypes.byref(handle)))
        self._handle = handle

    # ------------------------------------------------------------------ info
    def info(self) -> dict:
        inf = _ForestInfo()
        _check(self._lib, self._lib.ti_forest_get_info(self._handle, ctypes.byref(inf)))
        return {k: getattr(inf, k) for k, _ in _ForestInfo._fields_}

    def set_option(self, option: int, value: int) -> None:
        """ti_forest_set_option: speed knobs that never change results
        (OPT_SHAP_TABLE_ROWS, OPT_SHAP_TABLE_MB, OPT_HOST_REGISTER)."""
        _check(self._lib, self._lib.ti_forest_set_option(self._handle, option, int(value)))

    def output_shape(self, kind: int, n_rows: int):
        n = ctypes.c_int64()
        dt = ctypes.c_int32()
        _check(self._lib, self._lib.ti_output_shape(self._handle, kind, n_rows, ctypes.byref(n),
                                                    ctypes.byref(dt)))
        return int(n.value), int(dt.value)

    # --------------------------------------------------------------- predict
    def prepare_input(self, X) -> np.ndarray:
        return prepare_input(self.forest, X)

    def predict(self, X, kind: int = OUT_PREDICT) -> np.ndarray:
        X = self.prepare_input(X)
        rows, cols = X.shape
        width = self.forest.output_width(kind)
        out = np.empty(rows * width, dtype=self.forest.output_dtype(kind))
        xdt = TI_F32 if X.dtype == np.float32 else TI_F64
        if rows:
            _check(self._lib, self._lib.ti_predict(self._handle, _ptr(X), xdt, rows, cols, cols,
                                                   kind, _ptr(out), out.shape[0]))
        if width == 1 and kind != OUT_LEAF:
            return out
        return out.reshape(rows, width)

    def predict_device(self, x_ptr: int, x_dtype: int, n_rows: int, n_cols: int,
                       row_stride: int, kind: int, out_ptr: int, out_len: int,
                       slot: int = 0, stream: int = 0) -> None:
        """Enqueue a predict on device-resident buffers (no synchronisation)."""
        _check(self._lib, self._lib.ti_predict_device(self._handle, slot, x_ptr, x_dtype, n_rows,
                                                      n_cols, row_stride, kind, out_ptr, out_len,
                                                      stream or None))

    def transform_device(self, margin_ptr: int, n_rows: int, out_ptr: int, out_len: int,
                         slot: int = 0, stream: int = 0) -> None:
        """Enqueue the output transform over [n_rows, n_groups] device margins
        (ti_transform_device; the tree-sharded mode's last step)."""
        _check(self._lib, self._lib.ti_transform_device(self._handle, slot, margin_ptr, n_rows,
                                                        out_ptr, out_len, stream or None))

    def close(self) -> None:
        if getattr(self, "_handle", None) is not None and self._handle.value:
            self._lib.ti_forest_destroy(self._handle)
            self._handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["DeviceForest", "TreeInferError", "prepare_input", "load_library", "device_count", "default_devices",
           "OPT_SHAP_TABLE_ROWS", "OPT_SHAP_TABLE_MB",
           "EXPORTED_SYMBOLS", "OUT_MARGIN", "OUT_PREDICT", "OUT_LEAF", "OUT_CONTRIB", "TI_F32", "TI_F64",
           "TI_I32"]
