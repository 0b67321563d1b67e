"""V2 inference protocol tensors on /v2/models/<name>/infer (kfserving.v2):
JSON and binary tensor data in and out, the error object, the v1 fallback on
the same route, and V2 requests coalesced by the in-process batcher.  The
model is a numpy stand-in for a tree plugin (the GPU plugins: test_gpu_v2)."""
import json
import struct
import threading

import numpy as np
import pytest

from kfserving_amd.kfserving import KFModel, KFModelRepository, KFServer, v2
from tests.test_server import _Running


class RowSum(KFModel):
    """Takes matrices like the tree plugins (accepts_array_instances) and
    answers sum(row) * 2 in the input's float type."""
    accepts_array_instances = True

    def __init__(self, name="m"):
        super().__init__(name)
        self.ready = True
        self.batches = []

    def predict_tensor(self, X):
        self.batches.append(X.shape[0])
        return (X.sum(axis=1) * 2).astype(X.dtype)

    def predict_tensor_batched(self, X):
        return {"predictions": self.predict_tensor(X)}

    def predict(self, request):
        return {"predictions": [sum(r) * 2 for r in request["instances"]]}


@pytest.fixture
def serve():
    running = []

    def start(server):
        r = _Running(server)
        running.append(r)
        return r
    yield start
    for r in running:
        r.stop()


def _binary_request(X, out_binary=True, name="input-0"):
    dt = v2.NAMES[X.dtype]
    raw = np.ascontiguousarray(X).astype(X.dtype.newbyteorder("<")).tobytes()
    head = {"id": "7", "inputs": [{"name": name, "shape": list(X.shape), "datatype": dt,
                                   "parameters": {"binary_data_size": len(raw)}}]}
    if out_binary:
        head["outputs"] = [{"name": "predict", "parameters": {"binary_data": True}}]
    hb = json.dumps(head).encode()
    return hb + raw, {"Inference-Header-Content-Length": str(len(hb)),
                      "Content-Type": "application/octet-stream"}


def _split_response(hdrs, body):
    n = int(hdrs["Inference-Header-Content-Length"])
    return json.loads(body[:n]), body[n:]


@pytest.mark.parametrize("batch", [0, 16])
def test_v2_json_tensor(serve, batch):
    server = KFServer(registered_models=KFModelRepository(), max_batchsize=batch,
                      max_latency_ms=5)
    server.register_model(RowSum())
    s = serve(server)
    req = {"id": "42", "inputs": [{"name": "x", "shape": [2, 3], "datatype": "FP64",
                                   "data": [[1, 2, 3], [4, 5, 6.5]]}]}
    code, hdrs, out = s.fetch("/v2/models/m/infer", "POST", json.dumps(req).encode())
    assert code == 200, out
    r = json.loads(out)
    assert r == {"model_name": "m", "id": "42", "outputs": [
        {"name": "predict", "shape": [2], "datatype": "FP64", "data": [12.0, 31.0]}]}
    # flat data, FP32, a named output, integer tensors read as float64
    req = {"inputs": [{"name": "x", "shape": [1, 4], "datatype": "INT32", "data": [1, 2, 3, 4]}],
           "outputs": [{"name": "score"}]}
    code, _, out = s.fetch("/v2/models/m/infer", "POST", json.dumps(req).encode())
    r = json.loads(out)
    assert code == 200 and r["outputs"] == [{"name": "score", "shape": [1], "datatype": "FP64",
                                             "data": [20.0]}] and "id" not in r


@pytest.mark.parametrize("batch", [0, 16])
def test_v2_binary_tensor_in_and_out(serve, batch):
    server = KFServer(registered_models=KFModelRepository(), max_batchsize=batch,
                      max_latency_ms=5)
    server.register_model(RowSum())
    s = serve(server)
    X = np.random.default_rng(0).standard_normal((300, 28)).astype(np.float32)
    body, hdrs = _binary_request(X)
    code, rh, out = s.fetch("/v2/models/m/infer", "POST", body, hdrs)
    assert code == 200, out
    head, raw = _split_response(rh, out)
    assert rh["Content-Type"] == "application/octet-stream"
    assert head["id"] == "7" and head["model_name"] == "m"
    o = head["outputs"][0]
    assert o["datatype"] == "FP32" and o["shape"] == [300] and "data" not in o
    assert o["parameters"]["binary_data_size"] == len(raw) == 300 * 4
    assert np.array_equal(np.frombuffer(raw, "<f4"), (X.sum(axis=1) * 2).astype(np.float32))
    # binary in, JSON out
    body, hdrs = _binary_request(X[:3], out_binary=False)
    code, rh, out = s.fetch("/v2/models/m/infer", "POST", body, hdrs)
    o = json.loads(out)["outputs"][0]
    assert code == 200 and o["data"] == (X[:3].sum(axis=1) * 2).astype(np.float32).tolist()


def test_v2_v1_body_and_errors(serve):
    server = KFServer(registered_models=KFModelRepository())
    server.register_model(RowSum())
    s = serve(server)
    # the reference routes v1 bodies here too (kfserver.py:77-78)
    code, _, out = s.fetch("/v2/models/m/infer", "POST", b'{"instances": [[1, 2]]}')
    assert code == 200 and json.loads(out) == {"predictions": [6]}
    bad = [
        ({"inputs": [{"name": "x", "shape": [2, 2], "datatype": "FP32", "data": [1, 2, 3]}]},
         "3 values for shape [2, 2]"),
        ({"inputs": [{"name": "x", "shape": [1, 1], "datatype": "BYTES", "data": ["a"]}]},
         "unsupported datatype"),
        ({"inputs": [{"name": "x", "shape": [1, 2], "datatype": "FP32", "data": [1, 2]},
                     {"name": "y", "shape": [1, 2], "datatype": "FP32", "data": [1, 2]}]},
         "one input tensor"),
        ({"inputs": [{"name": "x", "shape": [1, 2, 2], "datatype": "FP32",
                      "data": [1, 2, 3, 4]}]}, "[rows, features]"),
        ({"inputs": [{"name": "x", "shape": [-1, 2], "datatype": "FP32", "data": [1, 2]}]},
         "non-negative"),
        ({"inputs": [{"name": "x", "shape": [1, 2], "datatype": "FP32", "data": ["a", 2]}]},
         "not FP32"),
    ]
    for req, msg in bad:
        code, hdrs, out = s.fetch("/v2/models/m/infer", "POST", json.dumps(req).encode())
        assert code == 400 and msg in json.loads(out)["error"], (req, out)
        assert hdrs["Content-Type"] == "application/json"
    # binary sizes that do not add up
    X = np.ones((2, 2), np.float32)
    body, hdrs = _binary_request(X)
    code, _, out = s.fetch("/v2/models/m/infer", "POST", body + b"\0\0\0\0", hdrs)
    assert code == 400 and "belong to no input" in json.loads(out)["error"]
    code, _, out = s.fetch("/v2/models/m/infer", "POST", body[:-4], hdrs)
    assert code == 400 and "binary_data_size" in json.loads(out)["error"]
    hdrs["Inference-Header-Content-Length"] = str(len(body) + 1)
    code, _, out = s.fetch("/v2/models/m/infer", "POST", body, hdrs)
    assert code == 400 and "exceeds the body" in json.loads(out)["error"]
    code, _, _ = s.fetch("/v2/models/nope/infer", "POST",
                         json.dumps(bad[0][0]).encode())
    assert code == 404


def test_v2_requests_share_batches(serve):
    server = KFServer(registered_models=KFModelRepository(), max_batchsize=64,
                      max_latency_ms=50)
    model = RowSum()
    model._forest = _Width(5)            # the tensor batcher takes the model's own width
    server.register_model(model)
    s = serve(server)
    rng = np.random.default_rng(3)
    Xs = [rng.standard_normal((int(rng.integers(1, 9)), 5)) for _ in range(12)]
    res = [None] * len(Xs)

    def one(i):
        body, hdrs = _binary_request(Xs[i])
        res[i] = s.fetch("/v2/models/m/infer", "POST", body, hdrs)
    th = [threading.Thread(target=one, args=(i,)) for i in range(len(Xs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for X, (code, rh, out) in zip(Xs, res):
        assert code == 200
        _, raw = _split_response(rh, out)
        assert np.array_equal(np.frombuffer(raw, "<f8"), X.sum(axis=1) * 2)
    assert len(model.batches) < len(Xs)                 # coalesced
    assert sum(model.batches) == sum(X.shape[0] for X in Xs)


class _Width:
    def __init__(self, n):
        self.n_features = n


def test_v2_model_without_width_is_not_batched(serve):
    """a model that states no width gets no tensor batcher, so
    requests of different widths never share (and fail) one batch."""
    server = KFServer(registered_models=KFModelRepository(), max_batchsize=64,
                      max_latency_ms=50)
    model = RowSum()
    server.register_model(model)
    s = serve(server)
    rng = np.random.default_rng(4)
    Xs = [rng.standard_normal((2, w)) for w in (3, 4, 3, 6, 5, 3)]
    res = [None] * len(Xs)

    def one(i):
        body, hdrs = _binary_request(Xs[i])
        res[i] = s.fetch("/v2/models/m/infer", "POST", body, hdrs)
    th = [threading.Thread(target=one, args=(i,)) for i in range(len(Xs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for X, (code, rh, out) in zip(Xs, res):
        assert code == 200, out
        _, raw = _split_response(rh, out)
        assert np.array_equal(np.frombuffer(raw, "<f8"), X.sum(axis=1) * 2)
    assert model.batches == [2] * len(Xs)               # each request alone


def test_v2_decode_units():
    req = {"inputs": [{"name": "a", "shape": [2], "datatype": "UINT8",
                       "parameters": {"binary_data_size": 2}},
                      {"name": "b", "shape": [3], "datatype": "BOOL", "data": [True, False, True]},
                      {"name": "c", "shape": [1], "datatype": "FP16",
                       "parameters": {"binary_data_size": 2}}]}
    tail = bytes([7, 9]) + struct.pack("<e", 1.5)
    got = v2.decode_inputs(req, tail)
    assert [n for n, _ in got] == ["a", "b", "c"]
    assert got[0][1].tolist() == [7, 9] and got[1][1].tolist() == [True, False, True]
    assert got[2][1].dtype == np.float16 and float(got[2][1][0]) == 1.5
    assert v2.feature_matrix([("c", np.float16([1, 2]))]).dtype == np.float32
    assert v2.feature_matrix([("c", np.int64([1, 2]))]).dtype == np.float64
    assert not v2.is_tensor_request({"inputs": [{"a": [1]}]})      # lgbserver rows stay v1
    assert v2.is_tensor_request({"inputs": [{"name": "x", "shape": [1], "datatype": "FP32"}]})


def test_v2_decode_errors_are_v2_errors():
    """Every malformed tensor is a V2Error (400), never an escaping numpy
    error: out-of-range integers, a non-int binary size, a bool
    shape entry, a shape whose product overflows int64."""
    cases = [
        ({"inputs": [{"name": "x", "shape": [1], "datatype": "UINT8", "data": [-1]}]}, b""),
        ({"inputs": [{"name": "x", "shape": [1], "datatype": "INT8", "data": [1000]}]}, b""),
        ({"inputs": [{"name": "x", "shape": [2], "datatype": "FP32",
                      "parameters": {"binary_data_size": 8.0}}]}, b"\0" * 8),
        ({"inputs": [{"name": "x", "shape": [2], "datatype": "FP32",
                      "parameters": {"binary_data_size": True}}]}, b"\0" * 8),
        ({"inputs": [{"name": "x", "shape": [True], "datatype": "FP32", "data": [1.0]}]}, b""),
        ({"inputs": [{"name": "x", "shape": [1 << 40, 1 << 40], "datatype": "FP32",
                      "data": [1.0]}]}, b""),
    ]
    for req, tail in cases:
        with pytest.raises(v2.V2Error):
            v2.decode_inputs(req, tail)


def test_v2_tensor_widths_do_not_grow_batchers(serve):
    """requests of any width are answered, but only the model's own
    width is batched; other widths are predicted alone, so a client cannot
    create a batcher per width."""
    class Forest:
        n_features = 3

    m = RowSum()
    m._forest = Forest()
    server = KFServer(registered_models=KFModelRepository(), max_batchsize=16, max_latency_ms=5)
    server.register_model(m)
    apps = []
    make = server.create_application
    server.create_application = lambda: apps.append(make()) or apps[-1]
    s = serve(server)
    for w in (3, 2, 5, 7, 3, 11):
        req = {"inputs": [{"name": "x", "shape": [1, w], "datatype": "FP64", "data": [1.0] * w}]}
        code, _, out = s.fetch("/v2/models/m/infer", "POST", json.dumps(req).encode())
        assert code == 200, out
        assert json.loads(out)["outputs"][0]["data"] == [2.0 * w]
    assert [k for k in apps[0]._batchers if "tensor" in k] == [("m", "tensor")]
