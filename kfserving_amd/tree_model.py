"""Shared GPU plumbing of the three tree plugins.

The reference loads the model *before* ``KFServer.start`` forks its workers
(python/xgbserver/xgbserver/__main__.py:37-46, kfserver.py:99), so the parsed
forest must stay a plain host object until the first predict in each worker
process: :class:`GPUForestMixin` creates the device replica lazily
(post-fork), once, under a lock.  Input conversion helpers reproduce how each
library turns a JSON request into a feature matrix.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence

import numpy as np

from .engine import DeviceForest, prepare_input
from .forest import OUT_CONTRIB, OUT_PREDICT, Forest


class GPUForestMixin:
    # KFServer may hand predict() the natively decoded float64 matrix
    # (kfserving.fastjson.JsonInstances) instead of a list of lists
    accepts_array_instances = True
    _forest: Optional[Forest] = None
    _device_forest: Optional[DeviceForest] = None
    devices: Optional[Sequence[int]] = None

    def _set_forest(self, forest: Forest) -> None:
        self._forest = forest
        self._device_forest = None
        if not hasattr(self, "_dev_lock"):
            self._dev_lock = threading.Lock()

    def device_forest(self) -> DeviceForest:
        dfo = self._device_forest
        if dfo is None:
            if not hasattr(self, "_dev_lock"):
                self._dev_lock = threading.Lock()
            with self._dev_lock:
                if self._device_forest is None:
                    if self._forest is None:
                        raise RuntimeError("model is not loaded")
                    self._device_forest = DeviceForest(self._forest, self.devices)
                dfo = self._device_forest
        return dfo

    def predict_matrix(self, X: np.ndarray, kind: int = OUT_PREDICT) -> np.ndarray:
        return self.device_forest().predict(X, kind)

    # V2 tensors (kfserving.v2): a [rows, features] numeric matrix, read with
    # the numpy-argument semantics of each library (NaN = missing)
    def tensor_matrix(self, X: np.ndarray) -> np.ndarray:
        return X

    def predict_tensor(self, X: np.ndarray) -> np.ndarray:
        return self.predict_matrix(self.tensor_matrix(X))

    def predict_tensor_batched(self, X: np.ndarray) -> Dict:
        """KFServer's batcher, kind "tensor": one predict over the rows of
        every V2 request of a batch."""
        try:
            return {"predictions": self.predict_tensor(X)}
        except Exception as e:
            raise Exception("Failed to predict %s" % e)

    # KFServer's native batcher (kfserving_amd.batcher.native.NativeModelBatcher):
    # each request is converted here exactly as predict / predict_batched /
    # predict_tensor convert it, and its rows of the batch's output become its
    # predictions as those methods return them
    native_batching = True

    def native_rows(self, chunk, kind: str) -> np.ndarray:
        if kind == "inputs":          # already batch_inputs' float64 matrix
            X = chunk
        elif kind == "tensor":
            X = self.tensor_matrix(chunk)
        else:
            X = self.request_matrix({"instances": chunk})
        return prepare_input(self._forest, X)

    def native_request(self, chunk, kind: str):
        """(matrix, kb_submit_convert transform) for one request: by default
        the converted rows of native_rows, copied as they are."""
        return self.native_rows(chunk, kind), 0

    def native_predictions(self, out: np.ndarray, kind: str):
        return out if kind == "tensor" else out.tolist()

    def explain(self, request: Dict) -> Dict:
        """The ``:explain`` route (kfserver.py:79-82 in the reference, which
        forwards to an explainer service; kfmodel.py:106-122) answered in
        process: TreeSHAP feature contributions computed on the GPU
        (libtreeinfer TI_OUTPUT_CONTRIB), shaped like xgboost's
        ``predict(pred_contribs=True)``: [rows, F + 1] for one output group,
        [rows, K, F + 1] for K groups; the last column is the bias (base
        margin + expected tree output).  The request is parsed exactly as
        ``predict`` parses it (``request_matrix``)."""
        try:
            X = self.request_matrix(request)
            f = self._forest
            c = self.predict_matrix(X, OUT_CONTRIB)
            if f.n_groups > 1:
                c = c.reshape(c.shape[0], f.n_groups, f.n_features + 1)
            return {"explanations": c.tolist()}
        except Exception as e:
            raise Exception("Failed to explain %s" % e)


def xgb_matrix_from_list(instances) -> np.ndarray:
    """``xgb.DMatrix(list)`` as xgboost 0.82 builds it (xgbserver/model.py:46).

    A python list goes through ``scipy.sparse.csr_matrix(data)``: zeros are not
    stored (missing -> default child) while NaN is stored as a value, which never
    satisfies ``x < split`` (always the right child).  Encoded for the canonical
    kernel as 0 -> NaN (missing) and NaN -> +inf (right at every split).
    """
    X = np.asarray(instances, dtype=np.float64)
    if X.ndim == 1:
        X = X.reshape(1, -1)
    if X.ndim != 2:
        raise ValueError(f"expected a list of rows, got shape {X.shape}")
    absent = X == 0
    present_nan = np.isnan(X)
    X32 = X.astype(np.float32)
    X32[absent] = np.nan
    X32[present_nan] = np.inf
    return X32


def _numeric_column(values) -> bool:
    """Whether pandas types the column as a number or bool dtype: all bool
    (no None), or int / float with None allowed beside at least one number.
    Mixed bool / number and bool + None columns are object dtype, which
    lightgbm's dtype check rejects: those take the pandas path."""
    n_bool = n_num = n_none = 0
    for v in values:
        if v is None:
            n_none += 1
        elif isinstance(v, bool):
            n_bool += 1
        elif isinstance(v, (int, float)):
            n_num += 1
        else:
            return False
    if n_bool:
        return n_num == 0 and n_none == 0
    return n_num > 0 or len(values) == 0


def lgb_matrix_from_inputs(inputs: List[dict], feature_names: List[str]) -> np.ndarray:
    """``pd.concat([pd.DataFrame(i, columns=booster.feature_name()) ...])`` then
    lightgbm's float conversion (lgbserver/model.py:46-51): columns chosen by
    name, absent columns NaN, extra keys dropped, float64."""
    fast = []
    for inp in inputs:
        # the fast path takes only what pandas would type as numbers: lists of
        # bool / int / float (None allowed beside numbers, where pandas infers
        # float); anything else (numeric strings, all-None columns, objects)
        # goes through pandas, which applies lightgbm's dtype check
        if not isinstance(inp, dict) or not all(
                isinstance(v, (list, tuple)) and _numeric_column(v) for k, v in inp.items()
                if k in feature_names):
            fast = None
            break
        n = {len(inp[k]) for k in feature_names if k in inp}
        if len(n) > 1:
            fast = None
            break
        rows = n.pop() if n else 0
        cols = [np.asarray(inp[k], dtype=np.float64) if k in inp else np.full(rows, np.nan)
                for k in feature_names]
        fast.append(np.stack(cols, axis=1) if cols else np.zeros((rows, 0)))
    if fast is not None:
        return np.concatenate(fast, axis=0) if fast else np.zeros((0, len(feature_names)))
    import pandas as pd
    df = pd.concat([pd.DataFrame(i, columns=feature_names) for i in inputs], axis=0)
    for dt in df.dtypes:
        if not (np.issubdtype(dt, np.number) or dt == bool):
            raise ValueError("DataFrame.dtypes for data must be int, float or bool")
    return df.to_numpy(dtype=np.float64)
