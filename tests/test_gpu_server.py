"""End to end on the GPU: HTTP v1 :predict -> KFServer -> plugin -> libtreeinfer,
with the reference fixtures and known answers (test/e2e/predictor/*)."""
import json
import os
import shutil

import numpy as np
import pytest

from kfserving_amd.kfserving import KFServer
from tests.test_server import _Running

pytestmark = pytest.mark.gpu


def _dir(golden, tmp_path, src, dst):
    d = tmp_path / "m"
    d.mkdir()
    shutil.copy(os.path.join(golden, src), str(d / dst))
    return str(d)


def test_xgbserver_http_known_answer(golden, tmp_path):
    from kfserving_amd.xgbserver import XGBoostModel, XGBoostModelRepository
    model = XGBoostModel("xgboost-iris", _dir(golden, tmp_path, "xgb_iris_legacy_082.bst",
                                              "model.bst"), 1)
    model.load()
    server = KFServer(registered_models=XGBoostModelRepository(str(tmp_path)))
    server.register_model(model)
    s = _Running(server)
    with open(os.path.join(golden, "iris_input.json"), "rb") as fh:
        body = fh.read()
    code, hdrs, out = s.fetch("/v1/models/xgboost-iris:predict", "POST", body)
    assert code == 200 and json.loads(out)["predictions"] == [1, 1]   # test_xgboost.py:67-68
    assert out == b'{"predictions": [1.0, 1.0]}'                      # v1alpha2 README:103
    s.stop()


def test_lgbserver_http_known_answer(golden, tmp_path):
    from kfserving_amd.lgbserver import LightGBMModel
    model = LightGBMModel("lightgbm", _dir(golden, tmp_path, "lgb_iris_v3.txt", "model.bst"), 1)
    model.load()
    server = KFServer(workers=1)
    server.register_model(model)
    s = _Running(server)
    with open(os.path.join(golden, "iris_input_v3.json"), "rb") as fh:
        code, _, out = s.fetch("/v1/models/lightgbm:predict", "POST", fh.read())
    assert code == 200 and json.loads(out)["predictions"][0][0] > 0.5  # test_lightgbm.py:65-67
    s.stop()


def test_sklearnserver_http_and_batcher(golden, tmp_path):
    from kfserving_amd.sklearnserver import SKLearnModel
    from oracle import sk_ref
    from tests.test_oracle import _sk_trees
    model = SKLearnModel("sk", _dir(golden, tmp_path, "sk_rf_reg_model.npz", "model.npz"))
    assert model.load()
    server = KFServer(max_batchsize=64, max_latency_ms=20)
    server.register_model(model)
    s = _Running(server)
    g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
    X = np.nan_to_num(g["X"][:8]).astype(np.float64)
    trees, _ = _sk_trees(os.path.join(golden, "sk_rf_reg_model.npz"))
    want = sk_ref.predict_regressor(trees, X)
    code, _, out = s.fetch("/v1/models/sk:predict", "POST",
                           json.dumps({"instances": X.tolist()}).encode())
    res = json.loads(out)
    assert code == 200 and res["message"] == "" and res["batchId"]
    assert np.array_equal(np.array(res["predictions"]), want)
    s.stop()


def test_lgbserver_inputs_batched_gpu(golden, tmp_path):
    """Concurrent lgbserver ``inputs`` requests share a batch (one batchId per
    batch) and each gets lgb_ref.predict on its own rows."""
    from oracle import lgb_ref
    from tests.test_lgb_batching import _lgb_model, run_batched
    model = _lgb_model(golden, tmp_path, stub=False)
    reqs, results = run_batched(model)
    m = lgb_ref.read_lgb_text(os.path.join(golden, "lgb_iris_v3.txt"))
    bodies = [json.loads(b) for _, _, b in results]
    assert all(c == 200 for c, _, _ in results)
    assert len({b["batchId"] for b in bodies}) < len(bodies)
    for req, b in zip(reqs, bodies):
        X = model.request_matrix(req)
        np.testing.assert_allclose(np.array(b["predictions"]), lgb_ref.predict(m, X),
                                   rtol=1e-5, atol=0)
        assert np.array_equal(np.argmax(b["predictions"], axis=1),
                              np.argmax(lgb_ref.predict(m, X), axis=1))


def test_c1_iris_32_single_row_requests_one_batch(golden, tmp_path):
    """BASELINE config C1 as named: 32 concurrent single-row Iris v1 :predict
    requests through xgbserver (the reference's legacy 0.82 fixture) with
    --max_batchsize 32 are answered from ONE batch (one batchId:
    test/e2e/batcher/test_batcher.py:71-78), and every answer is the
    oracle's label for its row -- the reference's known answers among them
    (X[0] -> 0, xgbserver/test_model.py:42-44; the e2e rows -> 1,
    test/e2e/predictor/test_xgboost.py:67-68)."""
    import threading
    from sklearn.datasets import load_iris
    from kfserving_amd.xgbserver import XGBoostModel, XGBoostModelRepository
    from oracle import xgb_ref
    path = _dir(golden, tmp_path, "xgb_iris_legacy_082.bst", "model.bst")
    model = XGBoostModel("xgboost-iris", path, 1)
    assert model.load()
    server = KFServer(registered_models=XGBoostModelRepository(str(tmp_path)),
                      max_batchsize=32, max_latency_ms=5000)
    server.register_model(model)
    s = _Running(server)
    X = load_iris()["data"]
    with open(os.path.join(golden, "iris_input.json")) as fh:
        e2e = json.load(fh)["instances"]
    rows = [X[0].tolist()] + e2e + [X[i].tolist() for i in range(5, 150, 5)][:29]
    assert len(rows) == 32
    ref = xgb_ref.read_xgb_binary(os.path.join(path, "model.bst"))
    want = xgb_ref.predict(ref, np.asarray(rows, dtype=np.float32))
    out = [None] * 32
    start = threading.Barrier(32)

    def one(i):
        start.wait()
        out[i] = s.fetch("/v1/models/xgboost-iris:predict", "POST",
                         json.dumps({"instances": [rows[i]]}).encode())

    th = [threading.Thread(target=one, args=(i,)) for i in range(32)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    s.stop()
    bodies = []
    for code, _, body in out:
        assert code == 200
        bodies.append(json.loads(body))
    assert len({b["batchId"] for b in bodies}) == 1 and bodies[0]["batchId"]
    got = [b["predictions"][0] for b in bodies]
    assert got == [float(w) for w in want]
    assert got[0] == 0 and got[1] == 1 and got[2] == 1        # the reference's known answers
