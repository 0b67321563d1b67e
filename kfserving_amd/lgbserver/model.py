"""LightGBMModel -- GPU drop-in for python/lgbserver/lgbserver/model.py:25-54.

Same constructor (name, model_dir, nthread, booster=None) and ``inputs``
request format: one DataFrame per element with ``columns=feature_name()``,
rows concatenated (:46-50), then one libtreeinfer call in float64 where the
reference called ``Booster.predict`` (:51).
"""
import os
from typing import Dict

import numpy as np

from ..formats.lightgbm_format import load_lightgbm_model
from ..forest import Forest
from ..kfserving.kfmodel import KFModel
from ..kfserving.storage import Storage
from ..tree_model import GPUForestMixin, lgb_matrix_from_inputs

BOOSTER_FILE = "model.bst"


class LightGBMModel(GPUForestMixin, KFModel):
    def __init__(self, name: str, model_dir: str, nthread: int, booster: Forest = None):
        super().__init__(name)
        self.name = name
        self.model_dir = model_dir
        self.nthread = nthread
        if booster is not None:
            self._set_forest(booster)
            self.ready = True

    def load(self) -> bool:
        model_file = os.path.join(Storage.download(self.model_dir), BOOSTER_FILE)
        self._set_forest(load_lightgbm_model(model_file))
        self.ready = True
        return self.ready

    def feature_name(self):
        names = self._forest.feature_names
        return list(names) if names else [f"Column_{j}" for j in range(self._forest.n_features)]

    def request_matrix(self, request: Dict) -> np.ndarray:
        return lgb_matrix_from_inputs(request["inputs"], self.feature_name())

    def tensor_matrix(self, X: np.ndarray) -> np.ndarray:
        """A V2 tensor's columns in the booster's feature order, float64 (as
        ``Booster.predict(ndarray)`` reads them)."""
        X = np.asarray(X, dtype=np.float64)
        n = self._forest.n_features
        if X.ndim != 2 or X.shape[1] != n:
            raise ValueError("The number of features in data (%d) is not the same as it was "
                             "in training data (%d)." % (X.shape[-1], n))
        return X

    def predict(self, request: Dict) -> Dict:
        try:
            result = self.predict_matrix(self.request_matrix(request))
            return {"predictions": result.tolist()}
        except Exception as e:
            raise Exception("Failed to predict %s" % e)

    # the native HTTP front end (kfhttp.h) reads batched v1 {"inputs": ...}
    # bodies of this model itself (kf_parse_inputs: columns by these names, the
    # subset lgb_matrix_from_inputs takes without pandas), rows as they are
    native_v1_transform = 0

    def native_v1_names(self):
        return self.feature_name()

    # V2 tensors: tensor_matrix reads the columns in the booster's order as
    # float64 (FP32 data widened exactly), the plain cast of the native route
    native_v2_transform = 0

    # KFServer's in-process batcher (kfserving_amd.batcher.ModelBatcher, kind
    # "inputs"): one request's rows as the float64 matrix its columns select,
    # then one predict over the concatenated rows of a batch
    def batch_inputs(self, request: Dict) -> np.ndarray:
        X = self.request_matrix(request)
        if X.shape[0] == 0:
            raise ValueError("no rows in the request")
        return X

    def predict_batched(self, X: np.ndarray) -> Dict:
        try:
            return {"predictions": self.predict_matrix(X).tolist()}
        except Exception as e:
            raise Exception("Failed to predict %s" % e)
