"""The native HTTP front end (include/kfhttp.h) in front of the GPU: xgbserver
with the C2 forest (500 depth-8 trees, 28 features) answers batched v1
:predict requests natively through the native batcher and libtreeinfer; the
bytes of every answer equal those of the asyncio server (KF_NATIVE_HTTP off)
on the same requests, and the probabilities are the oracle's.  The CPU twin
is tests/test_native_http.py."""
import json
import os
import re
import sys
import time

import numpy as np
import pytest

from kfserving_amd.kfserving import KFServer
from tests.test_server import _Running

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

pytestmark = pytest.mark.gpu


def _norm(b: bytes) -> bytes:
    return re.sub(rb'"batchId": "[0-9a-f-]{36}"', b'"batchId": "ID"', b)


def test_native_http_c2_bytes_equal_python_server(tmp_path):
    import bench_serving as bs
    from kfserving_amd.xgbserver import XGBoostModel
    from oracle import xgb_ref
    bs.write_c2_model(str(tmp_path))
    runs = []
    for native in (True, False):
        m = XGBoostModel("model", str(tmp_path), 1)
        assert m.load()
        srv = KFServer(max_batchsize=65536, max_latency_ms=3)
        srv.native_http = native
        srv.register_model(m)
        runs.append(_Running(srv))
    nat, py = runs
    t0 = time.time()
    while nat.server.front_end is None and time.time() - t0 < 60:
        time.sleep(0.05)
    ref = xgb_ref.read_xgb_binary(os.path.join(str(tmp_path), "model.bst"))
    rng = np.random.default_rng(8)
    try:
        assert nat.server.front_end is not None and "model" in nat.server.front_end.routes
        for i in range(24):
            X = rng.standard_normal((int(rng.integers(1, 65)), 28)).astype(np.float32)
            X[rng.random(X.shape) < 0.05] = 0.0          # DMatrix(list): missing
            body = json.dumps({"instances": X.tolist()}).encode()
            # every other body on /v2/.../infer, which takes a v1 body as :predict
            path = "/v1/models/model:predict" if i % 2 == 0 else "/v2/models/model/infer"
            a = nat.fetch(path, "POST", body)
            b = py.fetch(path, "POST", body)
            assert a[0] == b[0] == 200 and a[1] == b[1]
            assert _norm(a[2]) == _norm(b[2])
            got = np.asarray(json.loads(a[2])["predictions"])
            Xo = X.copy()
            Xo[X == 0] = np.nan
            np.testing.assert_allclose(got, xgb_ref.predict(ref, Xo), rtol=1e-5, atol=0)
        st = nat.server.front_end.stats()
        assert st["native_requests"] >= 24
    finally:
        nat.stop()
        py.stop()


def test_native_http_c2_large_bodies(tmp_path):
    """v1 bodies of 2.4 and 38 MB (4,096 and 65,536 rows) take the native
    route on the GPU (the threaded parser on the IO thread): the bytes equal
    the asyncio server's, no request reaches the application, and the
    probabilities are the oracle's."""
    import bench_serving as bs
    from kfserving_amd.xgbserver import XGBoostModel
    from oracle import xgb_ref
    bs.write_c2_model(str(tmp_path))
    runs = []
    for native in (True, False):
        m = XGBoostModel("model", str(tmp_path), 1)
        assert m.load()
        srv = KFServer(max_batchsize=65536, max_latency_ms=3)
        srv.native_http = native
        srv.register_model(m)
        runs.append(_Running(srv))
    nat, py = runs
    t0 = time.time()
    while nat.server.front_end is None and time.time() - t0 < 60:
        time.sleep(0.05)
    ref = xgb_ref.read_xgb_binary(os.path.join(str(tmp_path), "model.bst"))
    rng = np.random.default_rng(11)
    try:
        small = json.dumps({"instances": rng.standard_normal((4, 28)).tolist()}).encode()
        assert nat.fetch("/v1/models/model:predict", "POST", small)[0] == 200   # the route
        assert "model" in nat.server.front_end.routes
        before = nat.server.front_end.stats()
        for rows in (4096, 65536):
            X = rng.standard_normal((rows, 28)).astype(np.float32)
            X[rng.random(X.shape) < 0.02] = 0.0           # DMatrix(list): missing
            body = json.dumps({"instances": X.tolist()}).encode()
            a = nat.fetch("/v1/models/model:predict", "POST", body)
            b = py.fetch("/v1/models/model:predict", "POST", body)
            assert a[0] == b[0] == 200 and a[1] == b[1]
            assert _norm(a[2]) == _norm(b[2])
            got = np.asarray(json.loads(a[2])["predictions"])
            Xo = X.copy()
            Xo[X == 0] = np.nan
            np.testing.assert_allclose(got[:2000], xgb_ref.predict(ref, Xo[:2000]), rtol=1e-5, atol=0)
        st = nat.server.front_end.stats()
        assert st["native_requests"] - before["native_requests"] == 2
        assert st["python_requests"] == before["python_requests"]
    finally:
        nat.stop()
        py.stop()


def test_native_http_c2_v2_tensors(tmp_path):
    """V2 tensor requests (FP32 / FP64 JSON data) on the C2 forest: after the
    first (which makes the model's tensor batcher), each is answered on the
    native route; the bytes equal the asyncio server's and the probabilities
    are the oracle's (the float32 rows as DMatrix(ndarray) holds them)."""
    import bench_serving as bs
    from kfserving_amd.xgbserver import XGBoostModel
    from oracle import xgb_ref
    bs.write_c2_model(str(tmp_path))
    runs = []
    for native in (True, False):
        m = XGBoostModel("model", str(tmp_path), 1)
        assert m.load()
        srv = KFServer(max_batchsize=65536, max_latency_ms=3)
        srv.native_http = native
        srv.register_model(m)
        runs.append(_Running(srv))
    nat, py = runs
    t0 = time.time()
    while nat.server.front_end is None and time.time() - t0 < 60:
        time.sleep(0.05)
    ref = xgb_ref.read_xgb_binary(os.path.join(str(tmp_path), "model.bst"))
    rng = np.random.default_rng(12)
    path = "/v2/models/model/infer"
    try:
        first = bs.body_of(rng.standard_normal((3, 28)).astype(np.float32), "v2")
        assert nat.fetch(path, "POST", first)[0] == 200
        fe = nat.server.front_end
        assert "v2:model" in fe.routes
        before = fe.stats()
        for i in range(16):
            rows = int(rng.integers(1, 65))
            X = rng.standard_normal((rows, 28))
            X[rng.random(X.shape) < 0.03] = np.nan
            dt = "FP32" if i % 2 == 0 else "FP64"
            req = {"inputs": [{"name": "x", "shape": [rows, 28], "datatype": dt,
                               "data": X.reshape(-1).tolist() if i % 4 < 2 else X.tolist()}]}
            if i % 3 == 0:
                req["id"] = f"r{i}"
            body = json.dumps(req).encode()
            a = nat.fetch(path, "POST", body)
            b = py.fetch(path, "POST", body)
            assert a[0] == b[0] == 200 and a[1] == b[1] and a[2] == b[2]
            out = json.loads(a[2])["outputs"][0]
            assert out["datatype"] == "FP32" and out["shape"] == [rows]
            np.testing.assert_allclose(np.asarray(out["data"]),
                                       xgb_ref.predict(ref, X.astype(np.float32)), rtol=1e-5,
                                       atol=0)
        st = fe.stats()
        assert st["native_requests"] - before["native_requests"] == 16
        assert st["python_requests"] == before["python_requests"]
        # the binary tensor extension, in and out
        X = rng.standard_normal((40, 28)).astype(np.float32)
        head = json.dumps({"inputs": [{"name": "x", "shape": [40, 28], "datatype": "FP32",
                                       "parameters": {"binary_data_size": X.nbytes}}],
                           "parameters": {"binary_data_output": True}}).encode()
        hdr = {"Inference-Header-Content-Length": str(len(head))}
        a = nat.fetch(path, "POST", head + X.tobytes(), hdr)
        b = py.fetch(path, "POST", head + X.tobytes(), hdr)
        assert a[0] == b[0] == 200 and a[1] == b[1] and a[2] == b[2]
        n = int(a[1]["Inference-Header-Content-Length"])
        got = np.frombuffer(a[2][n:], dtype="<f4")
        np.testing.assert_allclose(got, xgb_ref.predict(ref, X), rtol=1e-5, atol=0)
        assert fe.stats()["native_requests"] - st["native_requests"] == 1
    finally:
        nat.stop()
        py.stop()
