"""lightgbm 2.3.1 predict restatement -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows python/lgbserver/lgbserver/model.py:44-54 (one DataFrame per
``inputs`` element with ``columns=booster.feature_name()``, concatenated, then
``Booster.predict``) and the load at :36-42.  Upstream algorithm (lightgbm
2.3.1, not vendored in /root/reference), restated:

* text model v3: header ``key=value`` lines, ``Tree=i`` blocks with
  split_feature / threshold / decision_type / left_child / right_child /
  leaf_value (fixture python/lgbserver/lgbserver/example_model/model/model.bst:1-28).
* predictor.hpp: a dense row keeps entries with |x| > kZeroThreshold (1e-35f)
  or NaN, everything else reads 0.0.
* tree.h Tree::CategoricalDecision (decision_type bit 0): int_fval =
  static_cast<int>(fval) -- on x86 a NaN or out-of-range value converts to
  INT_MIN, so it goes right like any negative value; otherwise left iff bit
  int_fval is set in the node's bitset cat_threshold[cat_boundaries[c] ..
  cat_boundaries[c+1]) with c = (int)threshold (Common::FindInBitset).
* tree.h Tree::NumericalDecision: missing type = (decision_type >> 2) & 3;
  NaN with type != NaN becomes 0.0; (Zero and IsZero(x)) or (NaN and isnan(x))
  -> default child (decision_type bit 1 = default left); else x <= threshold.
* gbdt.cpp GBDT::PredictRaw: output[k] = 0; output[k] += tree(i*K + k) in
  order; average_output divides by the iteration count; ConvertOutput:
  multiclass softmax (double), binary 1/(1+exp(-sigmoid*x)).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List

import numpy as np

K_ZERO_THRESHOLD = float(np.float32(1e-35))


@dataclass
class LGBRefTree:
    num_leaves: int
    split_feature: np.ndarray
    threshold: np.ndarray
    decision_type: np.ndarray
    left_child: np.ndarray
    right_child: np.ndarray
    leaf_value: np.ndarray
    cat_boundaries: np.ndarray = None
    cat_threshold: np.ndarray = None


@dataclass
class LGBRefModel:
    header: Dict[str, str]
    average_output: bool
    trees: List[LGBRefTree]

    @property
    def num_tree_per_iteration(self) -> int:
        return int(self.header.get("num_tree_per_iteration", "1"))

    @property
    def feature_names(self) -> List[str]:
        return self.header.get("feature_names", "").split()

    @property
    def objective(self) -> str:
        return self.header.get("objective", "")


def read_lgb_text(path: str) -> LGBRefModel:
    header: Dict[str, str] = {}
    average = False
    trees: List[LGBRefTree] = []
    block = None
    with open(path) as fh:
        for raw in fh:
            line = raw.rstrip("\n")
            if line.startswith("Tree="):
                block = {}
                continue
            if line == "end of trees":
                break
            if block is None:
                if "=" in line:
                    k, v = line.split("=", 1)
                    header[k] = v
                elif line.strip() == "average_output":
                    average = True
                continue
            if "=" in line:
                k, v = line.split("=", 1)
                block[k] = v
            elif line == "" and "leaf_value" in block and "shrinkage" in block:
                trees.append(_tree(block))
                block = {}
    return LGBRefModel(header, average, trees)


def _tree(b: Dict[str, str]) -> LGBRefTree:
    nl = int(b["num_leaves"])

    def ints(k):
        return np.array([int(x) for x in b.get(k, "").split()], dtype=np.int64)

    def flts(k):
        return np.array([float(x) for x in b.get(k, "").split()], dtype=np.float64)

    return LGBRefTree(nl, ints("split_feature"), flts("threshold"), ints("decision_type"),
                      ints("left_child"), ints("right_child"), flts("leaf_value"),
                      ints("cat_boundaries"), ints("cat_threshold").astype(np.uint32))


def x86_int(fval: np.ndarray) -> np.ndarray:
    """static_cast<int>(double) as cvttsd2si computes it: truncation, and
    INT_MIN for NaN or anything outside the int range."""
    fval = np.asarray(fval, dtype=np.float64)
    bad = np.isnan(fval) | (fval >= 2147483648.0) | (fval <= -2147483649.0)
    return np.where(bad, np.iinfo(np.int32).min, np.trunc(np.where(bad, 0, fval))).astype(np.int64)


def categorical_left(tr: LGBRefTree, node: np.ndarray, fval: np.ndarray) -> np.ndarray:
    iv = x86_int(fval)
    c = tr.threshold[node].astype(np.int64)
    lo = tr.cat_boundaries[c]
    nw = tr.cat_boundaries[c + 1] - lo
    word = np.where(iv >= 0, iv // 32, 0)
    ok = (iv >= 0) & (word < nw)
    w = tr.cat_threshold[np.where(ok, lo + word, 0)].astype(np.int64)
    return ok & (((w >> np.where(ok, iv % 32, 0)) & 1) == 1)


def from_raw_trees(trees, n_features: int, objective: str, num_class: int = 1) -> LGBRefModel:
    header = {"num_class": str(num_class),
              "num_tree_per_iteration": str(num_class if num_class > 1 else 1),
              "max_feature_idx": str(n_features - 1), "objective": objective,
              "feature_names": " ".join(f"Column_{j}" for j in range(n_features))}
    rt = [LGBRefTree(len(t["leaf_value"]), np.asarray(t["split_feature"], np.int64),
                     np.asarray(t["threshold"], np.float64),
                     np.asarray(t["decision_type"], np.int64),
                     np.asarray(t["left_child"], np.int64), np.asarray(t["right_child"], np.int64),
                     np.asarray(t["leaf_value"], np.float64),
                     np.asarray(t.get("cat_boundaries", []), np.int64),
                     np.asarray(t.get("cat_threshold", []), np.uint32)) for t in trees]
    return LGBRefModel(header, False, rt)


def rows_from_inputs(model: LGBRefModel, inputs) -> np.ndarray:
    """pd.DataFrame(input, columns=feature_name()) per element, pd.concat:
    columns selected by name, absent columns NaN, extra keys dropped."""
    names = model.feature_names
    blocks = []
    for inp in inputs:
        cols = []
        n = None
        for name in names:
            v = inp.get(name)
            if v is None:
                cols.append(None)
                continue
            vals = list(v.values()) if isinstance(v, dict) else list(v)
            n = len(vals)
            cols.append(np.asarray(vals, dtype=np.float64))
        n = n or 0
        blocks.append(np.stack([c if c is not None else np.full(n, np.nan) for c in cols], axis=1)
                      if names else np.zeros((n, 0)))
    return np.concatenate(blocks, axis=0)


def leaf_index(model: LGBRefModel, X: np.ndarray) -> np.ndarray:
    X = np.asarray(X, dtype=np.float64)
    X = np.where((np.abs(X) > K_ZERO_THRESHOLD) | np.isnan(X), X, 0.0)   # predictor row fill
    rows = X.shape[0]
    out = np.zeros((rows, len(model.trees)), dtype=np.int64)
    for t, tr in enumerate(model.trees):
        if tr.num_leaves <= 1:
            continue
        node = np.zeros(rows, dtype=np.int64)
        while True:
            act = node >= 0
            if not act.any():
                break
            idx = np.nonzero(act)[0]
            n = node[idx]
            raw = X[idx, tr.split_feature[n]]
            dt = tr.decision_type[n]
            mt = (dt >> 2) & 3
            fval = np.where(np.isnan(raw) & (mt != 2), 0.0, raw)
            is_zero = (fval >= -K_ZERO_THRESHOLD) & (fval <= K_ZERO_THRESHOLD)
            to_default = ((mt == 1) & is_zero) | ((mt == 2) & np.isnan(fval))
            default_left = (dt & 2) != 0
            go_left = np.where(to_default, default_left, fval <= tr.threshold[n])
            cat = (dt & 1) != 0
            if cat.any():
                go_left = np.where(cat, categorical_left(tr, n, raw), go_left)
            node[idx] = np.where(go_left, tr.left_child[n], tr.right_child[n])
        out[:, t] = ~node
    return out


def predict(model: LGBRefModel, X: np.ndarray, raw_score: bool = False,
            pred_leaf: bool = False) -> np.ndarray:
    leaves = leaf_index(model, X)
    if pred_leaf:
        return leaves
    rows = leaves.shape[0]
    K = model.num_tree_per_iteration
    score = np.zeros((rows, K), dtype=np.float64)
    for t, tr in enumerate(model.trees):
        score[:, t % K] += tr.leaf_value[leaves[:, t]]
    if model.average_output:
        score /= len(model.trees) // K
    if not raw_score:
        score = convert_output(model.objective, score)
    return score if K > 1 else score[:, 0]


def convert_output(objective: str, score: np.ndarray) -> np.ndarray:
    parts = objective.split()
    name = parts[0] if parts else ""
    kv = dict(p.split(":", 1) for p in parts[1:] if ":" in p)
    if name == "multiclass":
        wmax = score.max(axis=1, keepdims=True)
        e = np.exp(score - wmax)
        return e / e.sum(axis=1, keepdims=True)
    if name in ("binary", "multiclassova"):
        s = float(kv.get("sigmoid", 1.0))
        return 1.0 / (1.0 + np.exp(-s * score))
    if name in ("poisson", "gamma", "tweedie"):
        return np.exp(score)
    return score
