"""sklearn tree-ensemble predict restatement -- TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py).

Follows python/sklearnserver/sklearnserver/model.py:43-54
(``np.array(instances)`` -> ``self._model.predict``) against the installed
sklearn 1.7.2:

* sklearn/tree/_tree.pyx:979-997 ``_apply_dense``: X as float32; NaN ->
  ``missing_go_to_left``; else ``X_i_node_feature <= node.threshold``
  (float32 promoted to float64).
* sklearn/ensemble/_forest.py:723-736 ``_accumulate_prediction``: out +=
  per-tree prediction, estimator order (n_jobs=1); :1083 ``y_hat /=
  len(estimators_)``; :921-962 classifier probabilities averaged the same
  way; :882-919 ``classes_.take(argmax(proba))``.
"""
from __future__ import annotations

from typing import List

import numpy as np


def apply(trees: List[dict], X: np.ndarray) -> np.ndarray:
    """Leaf node id per (row, tree)."""
    X32 = np.asarray(X, dtype=np.float32)
    rows = X32.shape[0]
    out = np.zeros((rows, len(trees)), dtype=np.int64)
    for t, tr in enumerate(trees):
        cl, cr = tr["children_left"], tr["children_right"]
        feat, thr, mgl = tr["feature"], tr["threshold"], tr["missing_go_to_left"]
        node = np.zeros(rows, dtype=np.int64)
        while True:
            act = cl[node] != -1
            if not act.any():
                break
            idx = np.nonzero(act)[0]
            n = node[idx]
            x = X32[idx, feat[n]]
            go_left = np.where(np.isnan(x), mgl[n] != 0, x.astype(np.float64) <= thr[n])
            node[idx] = np.where(go_left, cl[n], cr[n])
        out[:, t] = node
    return out


def predict_regressor(trees: List[dict], X: np.ndarray, average: bool = True) -> np.ndarray:
    leaves = apply(trees, X)
    y = np.zeros(leaves.shape[0], dtype=np.float64)
    for t, tr in enumerate(trees):
        y += tr["value"][leaves[:, t], 0, 0]
    if average:
        y /= len(trees)
    return y


def predict_proba(trees: List[dict], X: np.ndarray, n_classes: int,
                  average: bool = True) -> np.ndarray:
    leaves = apply(trees, X)
    p = np.zeros((leaves.shape[0], n_classes), dtype=np.float64)
    for t, tr in enumerate(trees):
        p += tr["value"][leaves[:, t], 0, :n_classes]
    if average:
        p /= len(trees)
    return p


def predict_classifier(trees: List[dict], X: np.ndarray, classes: np.ndarray,
                       average: bool = True) -> np.ndarray:
    p = predict_proba(trees, X, len(classes), average)
    return np.asarray(classes).take(np.argmax(p, axis=1), axis=0)
