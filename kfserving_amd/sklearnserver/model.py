"""SKLearnModel -- GPU drop-in for python/sklearnserver/sklearnserver/model.py:25-54.

Same constructor (name, model_dir) and ``instances`` request format.  ``load``
finds model.joblib / .pkl / .pickle like the reference (:21-41; these files
are the user's own model, loaded with joblib exactly as the reference does)
or the pickle-free ``model.npz`` tree-array export, and flattens a
RandomForest / ExtraTrees / DecisionTree estimator; ``predict`` runs the
trees through libtreeinfer where the reference called ``_model.predict``.
"""
import os
from typing import Dict

import numpy as np

from ..formats.sklearn_format import forest_from_sklearn, load_tree_arrays
from ..kfserving.kfmodel import KFModel
from ..kfserving.storage import Storage
from ..engine import prepare_input
from ..tree_model import GPUForestMixin

MODEL_BASENAME = "model"
MODEL_EXTENSIONS = [".joblib", ".pkl", ".pickle"]
ARRAYS_EXTENSION = ".npz"


class SKLearnModel(GPUForestMixin, KFModel):  # pylint:disable=c-extension-no-member
    def __init__(self, name: str, model_dir: str):
        super().__init__(name)
        self.name = name
        self.model_dir = model_dir
        self.ready = False

    def load(self) -> bool:
        model_path = Storage.download(self.model_dir)
        paths = [os.path.join(model_path, MODEL_BASENAME + ext) for ext in MODEL_EXTENSIONS]
        for path in paths:
            if os.path.exists(path):
                import joblib
                self._set_forest(forest_from_sklearn(joblib.load(path)))
                self.ready = True
                break
        if not self.ready:
            npz = os.path.join(model_path, MODEL_BASENAME + ARRAYS_EXTENSION)
            if os.path.exists(npz):
                self._set_forest(load_tree_arrays(npz))
                self.ready = True
        return self.ready

    def _array(self, request: Dict) -> np.ndarray:
        instances = request["instances"]
        try:
            return np.array(instances)
        except Exception as e:
            raise Exception(
                "Failed to initialize NumPy array from inputs: %s, %s" % (e, instances))

    def request_matrix(self, request: Dict) -> np.ndarray:
        """sklearn's validate_data checks on the ``instances`` array."""
        f = self._forest
        X = np.asarray(self._array(request), dtype=np.float64)
        if X.ndim != 2:
            raise ValueError("Expected 2D array, got %dD array instead" % X.ndim)
        if X.shape[1] != f.n_features:
            raise ValueError("X has %d features, but %s is expecting %d features as input."
                             % (X.shape[1], f.objective, f.n_features))
        if not f.meta.get("allow_nan", True) and np.isnan(X).any():
            raise ValueError("Input X contains NaN.")   # GradientBoosting: validate_data
        # sklearn converts to float32 (DTYPE) before its finiteness check, so a
        # finite float64 beyond the float32 range is rejected like infinity
        with np.errstate(over="ignore"):
            X32 = X.astype(np.float32)
        if np.isinf(X32).any():
            raise ValueError("Input X contains infinity or a value too large for "
                             "dtype('float32').")
        return X

    def predict_tensor(self, X: np.ndarray) -> np.ndarray:
        """A V2 tensor through the same checks and label mapping as predict."""
        f = self._forest
        result = self.predict_matrix(self.request_matrix({"instances": X}))
        classes = f.meta.get("classes")
        if classes is not None:
            result = np.asarray(classes).take(result.astype(np.int64), axis=0)
        return result

    @property
    def native_v1_transform(self):
        """The native HTTP route's element rule and checks (kfhttp.h): the
        float32 cast; a value that overflows it, or a NaN the estimator
        rejects, sends the request to predict's own checks."""
        f = self._forest
        if f is None:
            return None
        return (1 << 8) | (0 if f.meta.get("allow_nan", True) else (1 << 9))

    @property
    def native_v2_transform(self):
        """V2 tensors take request_matrix's checks and float32 cast too
        (native_rows), so regressors answer them natively with the same flags;
        a classifier's labels come back as a typed tensor, which the
        application encodes."""
        f = self._forest
        if f is None or f.meta.get("classes") is not None:
            return None
        return self.native_v1_transform

    def native_v1_labels(self):
        """A classifier's labels as its predict renders them
        (classes.take(index).tolist() -> json.dumps), for the native route."""
        import json
        classes = self._forest.meta.get("classes")
        if classes is None:
            return None
        return [json.dumps(c) for c in np.asarray(classes).tolist()]

    def native_rows(self, chunk, kind: str) -> np.ndarray:
        # the same checks for V2 tensors and instances (predict_tensor)
        X = chunk if kind == "inputs" else self.request_matrix({"instances": chunk})
        return prepare_input(self._forest, X)

    def native_predictions(self, out: np.ndarray, kind: str):
        classes = self._forest.meta.get("classes")
        if classes is not None:
            out = np.asarray(classes).take(out.astype(np.int64), axis=0)
        return out if kind == "tensor" else out.tolist()

    def predict(self, request: Dict) -> Dict:
        inputs = self._array(request)
        try:
            f = self._forest
            result = self.predict_matrix(self.request_matrix({"instances": inputs}))
            classes = f.meta.get("classes")
            if classes is not None:
                result = np.asarray(classes).take(result.astype(np.int64), axis=0)
            return {"predictions": result.tolist()}
        except Exception as e:
            raise Exception("Failed to predict %s" % e)
