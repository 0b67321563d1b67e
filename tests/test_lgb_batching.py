"""lgbserver ``inputs`` requests through the in-process batcher (SURVEY.md
8(f1)): the Go batcher only reads ``instances`` and rejects these with 400
(pkg/batcher/handler.go:229-241); here each request's inputs become the
float64 matrix its columns select by feature name and the batch predicts the
concatenated rows once.  CPU: the device call is replaced by the canonical
numpy evaluator; the -m gpu twin is tests/test_gpu_server.py."""
import json
import os
import shutil
import threading

import numpy as np
import pytest

from kfserving_amd.forest import OUT_PREDICT
from kfserving_amd.kfserving import KFServer
from tests import canon_eval
from tests.test_server import _Running


def _lgb_model(golden, tmp_path, stub=True):
    from kfserving_amd.lgbserver import LightGBMModel
    d = tmp_path / "m"
    d.mkdir()
    shutil.copy(os.path.join(golden, "lgb_iris_v3.txt"), str(d / "model.bst"))
    model = LightGBMModel("lightgbm", str(d), 1)
    model.load()
    if stub:
        model.predict_matrix = lambda X, kind=OUT_PREDICT: canon_eval.predict(model._forest, X, kind)
    return model


def _requests(n, seed=0):
    """n lgbserver bodies of 1-3 rows, columns in shuffled order, an extra key
    the model ignores (lgbserver/test_model.py:43-47), a missing column (NaN)."""
    rng = np.random.default_rng(seed)
    names = ["sepal_length_(cm)", "sepal_width_(cm)", "petal_length_(cm)", "petal_width_(cm)"]
    out = []
    for i in range(n):
        rows = int(rng.integers(1, 4))
        cols = {k: rng.uniform(0, 7, rows).round(2).tolist() for k in names}
        if i % 3 == 0:
            cols["x"] = [1.0] * rows
        if i % 4 == 1:
            del cols[names[2]]
        keys = list(cols)
        rng.shuffle(keys)
        out.append({"inputs": [{k: cols[k] for k in keys}]})
    return out


def _want(model, req):
    X = model.request_matrix(req)
    return canon_eval.predict(model._forest, X, OUT_PREDICT)


def run_batched(model, n=12):
    server = KFServer(max_batchsize=64, max_latency_ms=200)
    server.register_model(model)
    s = _Running(server)
    reqs = _requests(n)
    results = [None] * n

    def one(i):
        results[i] = s.fetch("/v1/models/lightgbm:predict", "POST", json.dumps(reqs[i]).encode())
    th = [threading.Thread(target=one, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    s.stop()
    return reqs, results


def test_lgb_inputs_batched_cpu(golden, tmp_path):
    model = _lgb_model(golden, tmp_path)
    reqs, results = run_batched(model)
    bodies = [json.loads(b) for _, _, b in results]
    assert all(c == 200 for c, _, _ in results)
    assert len({b["batchId"] for b in bodies}) < len(bodies)       # requests shared batches
    for req, b in zip(reqs, bodies):
        assert b["message"] == ""
        assert np.array_equal(np.array(b["predictions"]), _want(model, req))


def test_lgb_inputs_batch_errors(golden, tmp_path):
    model = _lgb_model(golden, tmp_path)
    server = KFServer(max_batchsize=64, max_latency_ms=20)
    server.register_model(model)
    s = _Running(server)
    # a column of strings: lightgbm's dtype check, 500 as the reference answers
    code, _, out = s.fetch("/v1/models/lightgbm:predict", "POST",
                           b'{"inputs": [{"sepal_length_(cm)": ["a"]}]}')
    assert code == 500 and b"Failed to predict" in out
    code, _, out = s.fetch("/v1/models/lightgbm:predict", "POST", b'{"inputs": 3}')
    assert code == 400
    s.stop()


def test_lgb_matrix_mixed_bool_columns_follow_pandas():
    """Columns pandas types as object (bool mixed with numbers, bool beside
    None) take the pandas path and are rejected by lightgbm's dtype check;
    all-bool and number + None columns are numeric."""
    from kfserving_amd.tree_model import lgb_matrix_from_inputs
    names = ["a", "b"]
    for bad in ([True, 1], [True, None], [1, False]):
        with pytest.raises(ValueError):
            lgb_matrix_from_inputs([{"a": bad, "b": [1.0, 2.0]}], names)
    X = lgb_matrix_from_inputs([{"a": [True, False], "b": [1, None]}], names)
    np.testing.assert_array_equal(X, np.array([[1.0, 1.0], [0.0, np.nan]]))
