"""XGBoostModel -- GPU drop-in for python/xgbserver/xgbserver/model.py:24-50.

Same constructor (name, model_dir, nthread, booster=None), same ``load`` /
``predict`` contract and response shape; ``Booster.predict`` on a DMatrix
(:46-47) becomes one libtreeinfer call.  ``nthread`` is accepted for CLI and
repository compatibility; the device, not host threads, runs the trees.
"""
import os
from typing import Dict

import numpy as np

from ..formats.xgboost_format import load_xgboost_model
from ..forest import Forest
from ..kfserving.fastjson import JsonInstances
from ..kfserving.kfmodel import KFModel
from ..kfserving.storage import Storage
from ..tree_model import GPUForestMixin, xgb_matrix_from_list

BOOSTER_FILE = "model.bst"


class XGBoostModel(GPUForestMixin, KFModel):
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
        self._set_forest(load_xgboost_model(model_file))
        self.ready = True
        return self.ready

    def request_matrix(self, request: Dict) -> np.ndarray:
        instances = request["instances"]
        if isinstance(instances, np.ndarray) and not isinstance(instances, JsonInstances):
            return self.tensor_matrix(instances)  # DMatrix(ndarray): NaN = missing
        return xgb_matrix_from_list(instances)    # DMatrix(list) semantics (JSON rows)

    def tensor_matrix(self, X: np.ndarray) -> np.ndarray:
        # DMatrix(ndarray) stores float32: a float64 array is rounded first
        # (comparing the double against the split would differ from xgboost
        # for doubles that round onto the float32 threshold)
        X = np.asarray(X)
        if X.ndim == 1:
            X = X.reshape(1, -1)
        return X if X.dtype == np.float32 else X.astype(np.float32)

    # the native HTTP front end answers batched v1 :predict bodies of this
    # model itself, with DMatrix(list)'s element rule (kfbatch.h KB_IN_XGB_LIST)
    native_v1_transform = 1
    # ... and its V2 tensor requests (FP32 / FP64 JSON data, kh_add_v2_tensor_predict):
    # tensor_matrix is the plain float32 cast the native batcher applies
    native_v2_transform = 0

    def native_request(self, chunk, kind: str):
        # a natively decoded JSON list: DMatrix(list)'s rule (0 missing, NaN
        # right) and the float32 cast are applied by the native batcher while
        # it copies the rows (KB_IN_XGB_LIST), the conversion
        # xgb_matrix_from_list makes in numpy
        if kind == "instances" and isinstance(chunk, JsonInstances) and chunk.ndim == 2:
            return np.asarray(chunk), 1
        return super().native_request(chunk, kind)

    def predict(self, request: Dict) -> Dict:
        try:
            result = self.predict_matrix(self.request_matrix(request))
            return {"predictions": result.tolist()}
        except Exception as e:
            raise Exception("Failed to predict %s" % e)
