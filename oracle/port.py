"""ctypes wrapper of oracle/c/tree_port.c -- TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py).  Used by bench.py's cpu_baseline leg and tests."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libtreeport.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-C", _HERE, "build/libtreeport.so"], check=True,
                   stdout=subprocess.DEVNULL)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.port_num_threads.restype = ctypes.c_int
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def num_threads() -> int:
    return int(lib().port_num_threads())


def xgb_predict(trees, tree_info, n_groups, base_margin, n_features, X, sigmoid=False,
                nthread=0):
    """trees: list of RegTree dicts (cleft, cright, sindex, value)."""
    L = lib()
    sizes = [len(t["cleft"]) for t in trees]
    off = np.zeros(len(trees) + 1, dtype=np.int64)
    np.cumsum(sizes, out=off[1:])
    cl = np.ascontiguousarray(np.concatenate([t["cleft"] for t in trees]), dtype=np.int32)
    cr = np.ascontiguousarray(np.concatenate([t["cright"] for t in trees]), dtype=np.int32)
    si = np.ascontiguousarray(np.concatenate([t["sindex"] for t in trees]), dtype=np.uint32)
    val = np.ascontiguousarray(np.concatenate([t["value"] for t in trees]), dtype=np.float32)
    ti = np.ascontiguousarray(tree_info, dtype=np.int32)
    X = np.ascontiguousarray(X, dtype=np.float32)
    out = np.empty((X.shape[0], n_groups), dtype=np.float32)
    f = L.port_xgb_predict
    f.restype = ctypes.c_int
    rc = f(ctypes.c_int32(len(trees)), _p(off), _p(cl), _p(cr), _p(si), _p(val), _p(ti),
           ctypes.c_int32(n_groups), ctypes.c_float(base_margin), ctypes.c_int32(n_features),
           _p(X), ctypes.c_int64(X.shape[0]), ctypes.c_int32(X.shape[1]),
           ctypes.c_int32(1 if sigmoid else 0), _p(out), ctypes.c_int32(nthread))
    if rc:
        raise RuntimeError("port_xgb_predict failed")
    return out


def lgb_predict_raw(trees, n_groups, n_features, X, nthread=0):
    """trees: list of LightGBM tree dicts (split_feature, threshold, decision_type,
    left_child, right_child, leaf_value)."""
    L = lib()
    nl = np.array([len(t["leaf_value"]) for t in trees], dtype=np.int32)
    ni = np.array([len(t["split_feature"]) for t in trees], dtype=np.int64)
    noff = np.zeros(len(trees) + 1, dtype=np.int64)
    np.cumsum(ni, out=noff[1:])
    loff = np.zeros(len(trees) + 1, dtype=np.int64)
    np.cumsum(nl, out=loff[1:])

    def cat(key, dt):
        parts = [np.asarray(t[key]) for t in trees if len(t[key])]
        return np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros(1), dtype=dt)

    sf = cat("split_feature", np.int32)
    th = cat("threshold", np.float64)
    dt = cat("decision_type", np.int8)
    lc = cat("left_child", np.int32)
    rc_ = cat("right_child", np.int32)
    lv = cat("leaf_value", np.float64)
    X = np.ascontiguousarray(X, dtype=np.float64)
    out = np.empty((X.shape[0], n_groups), dtype=np.float64)
    f = L.port_lgb_predict
    f.restype = ctypes.c_int
    rc = f(ctypes.c_int32(len(trees)), _p(noff), _p(loff), _p(sf), _p(th), _p(dt), _p(lc),
           _p(rc_), _p(lv), _p(nl), ctypes.c_int32(n_groups), ctypes.c_int32(n_features),
           _p(X), ctypes.c_int64(X.shape[0]), ctypes.c_int32(X.shape[1]), _p(out),
           ctypes.c_int32(nthread))
    if rc:
        raise RuntimeError("port_lgb_predict failed")
    return out


def sk_predict(trees, value_width, n_features, X, average=True, nthread=0):
    """trees: list of sklearn tree-array dicts (see kfserving_amd sklearn_format)."""
    L = lib()
    sizes = [len(t["children_left"]) for t in trees]
    off = np.zeros(len(trees) + 1, dtype=np.int64)
    np.cumsum(sizes, out=off[1:])

    def cat(key, dt):
        return np.ascontiguousarray(np.concatenate([np.asarray(t[key]) for t in trees]), dtype=dt)

    cl = cat("children_left", np.int32)
    cr = cat("children_right", np.int32)
    ft = cat("feature", np.int32)
    th = cat("threshold", np.float64)
    mg = cat("missing_go_to_left", np.uint8)
    val = np.ascontiguousarray(np.concatenate(
        [np.asarray(t["value"])[:, 0, :value_width] for t in trees]), dtype=np.float64)
    X = np.ascontiguousarray(X, dtype=np.float32)
    out = np.empty((X.shape[0], value_width), dtype=np.float64)
    f = L.port_sk_predict
    f.restype = ctypes.c_int
    f(ctypes.c_int32(len(trees)), _p(off), _p(cl), _p(cr), _p(ft), _p(th), _p(mg), _p(val),
      ctypes.c_int32(value_width), ctypes.c_int32(n_features), _p(X),
      ctypes.c_int64(X.shape[0]), ctypes.c_int32(X.shape[1]), _p(out),
      ctypes.c_int32(1 if average else 0), ctypes.c_int32(nthread))
    return out


def tree_shap(f, X, nthread=0):
    """TreeSHAP contributions of a canonical Forest (oracle/c/shap_port.c),
    [rows, K * (F + 1)] float64 -- the same layout as TI_OUTPUT_CONTRIB."""
    if f.cover is None:
        raise ValueError("forest has no node covers")
    L = lib()
    fn = L.port_tree_shap
    fn.restype = ctypes.c_int
    X = np.ascontiguousarray(X, dtype=np.float64)
    out = np.empty((X.shape[0], f.n_groups * (f.n_features + 1)), dtype=np.float64)
    arrs = [np.ascontiguousarray(a, dtype=dt) for a, dt in (
        (f.tree_offset, np.int64), (f.tree_group, np.int32), (f.feature, np.int32),
        (f.threshold, np.float64), (f.flags, np.uint8), (f.left, np.int32),
        (f.right, np.int32), (f.leaf_value, np.float64), (f.cover, np.float64),
        (f.base_margin, np.float64))]
    rc = fn(ctypes.c_int32(f.n_trees), *[_p(a) for a in arrs[:9]],
            ctypes.c_int32(f.leaf_width), ctypes.c_int32(f.n_groups),
            ctypes.c_int32(f.n_features), _p(arrs[9]), ctypes.c_double(f.average_divisor),
            ctypes.c_int32(1 if f.lgb_zero_map else 0), ctypes.c_int32(int(f.depths().max())),
            _p(X), ctypes.c_int64(X.shape[0]), ctypes.c_int32(X.shape[1]), _p(out),
            ctypes.c_int32(nthread))
    if rc:
        raise MemoryError("port_tree_shap failed")
    return out
