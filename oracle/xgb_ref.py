"""xgboost 0.82 predict restatement -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows the call at python/xgbserver/xgbserver/model.py:46-47
(``xgb.DMatrix(request["instances"], nthread)`` then ``Booster.predict``) and
the model load at :38-39.  Upstream algorithm (xgboost 0.82, not vendored in
/root/reference), restated here:

* learner.cc  Learner::Load: LearnerModelParam (136 B), objective name,
  booster name, GBTreeModelParam (160 B), per tree TreeParam (148 B) + Node
  (20 B: parent, cleft, cright, sindex[bit31 = default_left], float
  split/leaf) + RTreeNodeStat (16 B), tree_info (int32 per tree), then the
  attribute table.  The 1.x ``binf`` file is the same body after a 4-byte
  magic with major/minor version words in the LearnerModelParam.
* tree_model.h  RegTree::GetNext: missing -> default child, else
  ``fvalue < split_cond`` -> left.
* cpu_predictor.cc  PredValue/PredLoopSpecalize: psum = 0.0f; psum +=
  leaf for trees of the group in order; preds[row, g] (= base_margin) += psum.
* DMatrix from a numpy array (missing = NaN): NaN entries are missing.
  From a python list (model.py:46) 0.82 builds ``scipy.sparse.csr_matrix``:
  zeros are dropped (missing) and NaN stays a present value (never < split,
  so it goes right).
* objectives: binary:logistic / reg:logistic 1/(1+exp(-x)) in float;
  multi:softprob softmax (float max, double sum); multi:softmax first argmax.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List

import numpy as np


@dataclass
class XGBRefTree:
    cleft: np.ndarray
    cright: np.ndarray
    sindex: np.ndarray
    value: np.ndarray   # float32 split condition or leaf value


@dataclass
class XGBRefModel:
    base_score: float
    num_feature: int
    num_class: int
    num_output_group: int
    objective: str
    major_version: int
    trees: List[XGBRefTree]
    tree_info: np.ndarray


def read_xgb_binary(path: str) -> XGBRefModel:
    """Sequential reader of the xgboost legacy / binf binary (node by node)."""
    with open(path, "rb") as fh:
        buf = fh.read()
    off = 4 if buf[:4] == b"binf" else 0

    def rd(fmt):
        nonlocal off
        vals = struct.unpack_from(fmt, buf, off)
        off += struct.calcsize(fmt)
        return vals

    base_score, num_feature, num_class, _extra, _evals, major, _minor = rd("<fIiiiii")
    off += 136 - 28
    (n,) = rd("<Q")
    objective = buf[off:off + n].decode()
    off += n
    (n,) = rd("<Q")
    booster = buf[off:off + n].decode()
    off += n
    assert booster == "gbtree", booster
    num_trees, _roots, _nf, _pad, _pbuf, num_output_group, _slv = rd("<iiiiqii")
    off += 160 - 32
    trees = []
    for _ in range(num_trees):
        _nr, num_nodes, _nd, _md, _tnf, _tslv = rd("<6i")
        off += 148 - 24
        cl, cr, si, val = [], [], [], []
        for _i in range(num_nodes):
            _parent, c_l, c_r, s_i, info = rd("<iiiIf")
            cl.append(c_l)
            cr.append(c_r)
            si.append(s_i)
            val.append(info)
        off += 16 * num_nodes
        trees.append(XGBRefTree(np.array(cl, np.int64), np.array(cr, np.int64),
                                np.array(si, np.uint64), np.array(val, np.float32)))
    tree_info = np.array(rd(f"<{num_trees}i"), dtype=np.int64)
    return XGBRefModel(base_score, num_feature, num_class, num_output_group, objective, major,
                       trees, tree_info)


def base_margin(m: XGBRefModel) -> np.float32:
    """0.x stores base_score in margin space; 1.x applies ProbToMargin."""
    b = np.float32(m.base_score)
    if m.major_version < 1:
        return b
    if m.objective in ("binary:logistic", "reg:logistic", "binary:logitraw"):
        return np.float32(-np.log(np.float32(1) / b - np.float32(1)))
    if m.objective in ("count:poisson", "reg:gamma", "reg:tweedie"):
        return np.float32(np.log(b))
    return b


def n_groups(m: XGBRefModel) -> int:
    return max(1, m.num_output_group, m.num_class)


def leaf_index(m: XGBRefModel, X: np.ndarray, missing: str = "nan") -> np.ndarray:
    """Leaf node id per (row, tree): RegTree::GetLeafIndex for every tree."""
    X = np.asarray(X, dtype=np.float32)
    rows = X.shape[0]
    out = np.zeros((rows, len(m.trees)), dtype=np.int64)
    for t, tr in enumerate(m.trees):
        nid = np.zeros(rows, dtype=np.int64)
        while True:
            internal = tr.cleft[nid] != -1
            if not internal.any():
                break
            idx = np.nonzero(internal)[0]
            n = nid[idx]
            f = (tr.sindex[n] & 0x7FFFFFFF).astype(np.int64)
            v = np.where(f < X.shape[1], X[idx, np.minimum(f, X.shape[1] - 1)], np.float32(np.nan))
            if missing == "csr":
                # python-list input: csr_matrix drops zeros; NaN is a present value
                is_missing = v == 0
            else:
                is_missing = np.isnan(v)
            default_left = (tr.sindex[n] >> 31) != 0
            go_left = np.where(is_missing, default_left, v < tr.value[n])
            nid[idx] = np.where(go_left, tr.cleft[n], tr.cright[n])
        out[:, t] = nid
    return out


def predict(m: XGBRefModel, X: np.ndarray, output_margin: bool = False, pred_leaf: bool = False,
            missing: str = "nan") -> np.ndarray:
    leaves = leaf_index(m, X, missing)
    if pred_leaf:
        return leaves.astype(np.float32)
    rows = leaves.shape[0]
    K = n_groups(m)
    margin = np.empty((rows, K), dtype=np.float32)
    for g in range(K):
        psum = np.zeros(rows, dtype=np.float32)
        for t, tr in enumerate(m.trees):
            if m.tree_info[t] == g:
                psum = psum + tr.value[leaves[:, t]]          # float32 + float32
        margin[:, g] = base_margin(m) + psum                   # preds(base) += psum
    if output_margin:
        return margin if K > 1 else margin[:, 0]
    return transform(m.objective, margin)


def transform(objective: str, margin: np.ndarray) -> np.ndarray:
    K = margin.shape[1]
    if objective in ("binary:logistic", "reg:logistic"):
        p = np.float32(1) / (np.float32(1) + np.exp(-margin))
        return p if K > 1 else p[:, 0]
    if objective == "multi:softmax":
        return np.argmax(margin, axis=1).astype(np.float32)     # first maximum
    if objective == "multi:softprob":
        wmax = margin.max(axis=1, keepdims=True)
        e = np.exp(margin - wmax).astype(np.float32)
        wsum = e.astype(np.float64).sum(axis=1, keepdims=True)
        return (e / wsum.astype(np.float32)).astype(np.float32)
    if objective == "binary:hinge":
        return np.where(margin > 0, np.float32(1), np.float32(0))[:, 0]
    if objective in ("count:poisson", "reg:gamma", "reg:tweedie"):
        return np.exp(margin)[:, 0]
    return margin if K > 1 else margin[:, 0]


def from_raw_trees(trees, tree_info, num_feature, num_class, base_score, objective,
                   major_version: int = 0) -> XGBRefModel:
    """Build a reference model from RegTree arrays (synthetic models)."""
    rt = [XGBRefTree(np.asarray(t["cleft"], np.int64), np.asarray(t["cright"], np.int64),
                     np.asarray(t["sindex"], np.uint64), np.asarray(t["value"], np.float32))
          for t in trees]
    return XGBRefModel(base_score, num_feature, num_class, max(1, num_class), objective,
                       major_version, rt, np.asarray(tree_info, np.int64))
