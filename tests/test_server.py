"""Server contract tests, modelled on python/kfserving/test/test_server.py:51-236
(DummyModel echo, liveness, health, exact predict bytes + content type,
list, load/unload 200/503/404, model-not-ready 503) -- over a real socket."""
import asyncio
import http.client
import json
import threading

import pytest

from kfserving_amd.kfserving import HTTPError, KFModel, KFModelRepository, KFServer


class DummyModel(KFModel):
    def __init__(self, name):
        super().__init__(name)
        self.name = name
        self.ready = False

    def load(self):
        self.ready = True

    async def predict(self, request):
        return {"predictions": request["instances"]}

    async def explain(self, request):
        return {"predictions": request["instances"]}


class SyncModel(KFModel):
    def __init__(self, name):
        super().__init__(name)
        self.ready = True
        self.calls = 0

    def predict(self, request):
        self.calls += 1
        if request["instances"] == ["boom"]:
            raise Exception("Failed to predict boom")
        return {"predictions": [[v * 2 for v in row] for row in request["instances"]]}


class DummyKFModelRepository(KFModelRepository):
    def __init__(self, test_load_success):
        super().__init__(models_dir="/tmp")
        self.test_load_success = test_load_success

    async def load(self, name):
        if self.test_load_success:
            model = DummyModel(name)
            model.load()
            self.update(model)
        return self.test_load_success


class _Running:
    def __init__(self, server):
        self.server = server
        self.loop = asyncio.new_event_loop()
        server.http_port = 0
        sock = server.bind("127.0.0.1")
        self.port = server.http_port
        self.thread = threading.Thread(target=self._run, args=(sock,), daemon=True)
        self.thread.start()

    def _run(self, sock):
        asyncio.set_event_loop(self.loop)
        try:
            self.loop.run_until_complete(self.server.serve(sock))
        except asyncio.CancelledError:
            pass

    def fetch(self, path, method="GET", body=None, headers=None):
        conn = http.client.HTTPConnection("127.0.0.1", self.port, timeout=30)
        conn.request(method, path, body=body, headers=headers or {})
        r = conn.getresponse()
        data = r.read()
        conn.close()
        return r.status, dict(r.getheaders()), data

    def stop(self):
        for t in asyncio.all_tasks(self.loop):
            self.loop.call_soon_threadsafe(t.cancel)
        self.thread.join(timeout=5)


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


def test_liveness_model_predict_list(serve):
    server = KFServer(registered_models=KFModelRepository())
    model = DummyModel("TestModel")
    model.load()
    server.register_model(model)
    s = serve(server)
    assert s.fetch("/")[0] == 200 and s.fetch("/")[2] == b"Alive"
    assert s.fetch("/v2/health/live")[0] == 200
    assert s.fetch("/v1/models/TestModel")[0] == 200
    code, hdrs, body = s.fetch("/v1/models/TestModel:predict", "POST", b'{"instances":[[1,2]]}')
    assert code == 200
    assert body == b'{"predictions": [[1, 2]]}'                     # test_server.py:156
    assert hdrs["Content-Type"] == "application/json; charset=UTF-8"  # test_server.py:157
    code, _, body = s.fetch("/v2/models/TestModel/infer", "POST", b'{"instances":[[1,2]]}')
    assert code == 200 and body == b'{"predictions": [[1, 2]]}'
    code, _, body = s.fetch("/v1/models/TestModel:explain", "POST", b'{"instances":[[1,2]]}')
    assert code == 200 and body == b'{"predictions": [[1, 2]]}'
    assert s.fetch("/v1/models") == (200, s.fetch("/v1/models")[1], b'["TestModel"]')


def test_predict_errors(serve):
    server = KFServer(registered_models=KFModelRepository())
    server.register_model(SyncModel("m"))
    s = serve(server)
    assert s.fetch("/v1/models/nope:predict", "POST", b'{}')[0] == 404
    assert s.fetch("/v1/models/m:predict", "POST", b'{not json')[0] == 400
    assert s.fetch("/v1/models/m:predict", "POST", b'{"instances": 3}')[0] == 400
    assert s.fetch("/v1/models/m:predict", "POST", b'{"instances": ["boom"]}')[0] == 500
    code, _, body = s.fetch("/v1/models/m:predict", "POST", b'{"instances": [[1, 2]]}')
    assert code == 200 and json.loads(body) == {"predictions": [[2, 4]]}
    assert s.fetch("/v1/models/m:predict", "GET")[0] == 405


def test_cloudevent_structured_unwrap(serve):
    server = KFServer(registered_models=KFModelRepository())
    m = DummyModel("TestModel")
    m.load()
    server.register_model(m)
    s = serve(server)
    event = {"specversion": "1.0", "id": "1", "source": "x", "type": "t",
             "time": "2021-01-01T00:00:00Z", "data": {"instances": [[1, 2]]}}
    code, _, body = s.fetch("/v1/models/TestModel:predict", "POST", json.dumps(event).encode(),
                            {"Content-Type": "application/cloudevents+json"})
    assert code == 200 and body == b'{"predictions": [[1, 2]]}'


def test_load_unload(serve):
    s = serve(KFServer(registered_models=DummyKFModelRepository(test_load_success=True)))
    code, _, body = s.fetch("/v2/repository/models/model/load", "POST", b"")
    assert code == 200 and body == b'{"name": "model", "load": true}'
    code, _, body = s.fetch("/v2/repository/models/model/unload", "POST", b"")
    assert code == 200 and body == b'{"name": "model", "unload": true}'


def test_load_unload_failure(serve):
    s = serve(KFServer(registered_models=DummyKFModelRepository(test_load_success=False)))
    assert s.fetch("/v2/repository/models/model/load", "POST", b"")[0] == 503
    assert s.fetch("/v2/repository/models/model/unload", "POST", b"")[0] == 404


def test_model_not_ready(serve):
    server = KFServer(registered_models=KFModelRepository())
    server.register_model(DummyModel("TestModel"))
    s = serve(server)
    code, _, body = s.fetch("/v1/models/TestModel")
    assert code == 503 and b"503: Model with name TestModel is not ready." in body


def test_keepalive_and_chunked(serve):
    server = KFServer(registered_models=KFModelRepository())
    server.register_model(SyncModel("m"))
    s = serve(server)
    conn = http.client.HTTPConnection("127.0.0.1", s.port, timeout=30)
    for i in range(3):
        conn.request("POST", "/v1/models/m:predict", body=iter([b'{"instances": ', b'[[%d]]}' % i]),
                     headers={"Transfer-Encoding": "chunked"}, encode_chunked=True)
        r = conn.getresponse()
        assert r.status == 200 and json.loads(r.read()) == {"predictions": [[2 * i]]}
    conn.close()


def test_in_process_batcher_route(serve):
    server = KFServer(registered_models=KFModelRepository(), max_batchsize=8, max_latency_ms=50)
    model = SyncModel("m")
    server.register_model(model)
    s = serve(server)
    results = []

    def one(i):
        results.append(s.fetch("/v1/models/m:predict", "POST",
                               json.dumps({"instances": [[i]]}).encode()))
    th = [threading.Thread(target=one, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    bodies = [json.loads(b) for c, _, b in results]
    assert all(c == 200 for c, _, _ in results)
    assert len({b["batchId"] for b in bodies}) < 8          # requests shared batches
    for b in bodies:
        assert b["message"] == "" and len(b["predictions"]) == 1
    assert sorted(b["predictions"][0][0] for b in bodies) == [2 * i for i in range(8)]


def test_httperror_reason():
    e = HTTPError(404, "x")
    assert e.status_code == 404 and e.reason == "x"


# ------------------------------------------------ native body decode (fast path)
class ArrayModel(KFModel):
    """Takes the natively decoded matrix, like the tree plugins; predicts a
    row checksum through the DMatrix(list) conversion (0 -> missing)."""
    accepts_array_instances = True

    def __init__(self, name):
        super().__init__(name)
        self.ready = True
        self.seen = []

    def predict(self, request):
        import numpy as np
        from kfserving_amd.tree_model import xgb_matrix_from_list
        inst = request["instances"]
        self.seen.append(type(inst).__name__)
        X = xgb_matrix_from_list(inst)
        return {"predictions": np.nan_to_num(X, nan=-7.0).sum(axis=1).tolist()}


class CustomPre(ArrayModel):
    def preprocess(self, request):
        assert isinstance(request["instances"], list)
        return request


FAST_BODIES = [
    b'{"instances": [[1, 2.5, 0, -0.0], [3, 4, 5e-3, NaN]]}',
    b'{ "instances" : [ [0.1,0.2 ,0.30000000000000004,1e22] ] }',
    b'{"instances": [[Infinity, -Infinity, 7, 123456789012345678]]}',
    b'{"instances": [[1, 2], [3]]}',                 # ragged: json.loads path
    b'{"instances": [[1, 2]], "signature_name": "x"}',
    b'{"instances": []}',
    b'{"instances": [[1, 2]',                        # malformed: 400 either way
]


@pytest.mark.parametrize("batch", [0, 4])
def test_fast_json_bytes_match_json_loads_path(serve, batch):
    outs = {}
    for fast in (True, False):
        server = KFServer(registered_models=KFModelRepository(), fast_json=fast,
                          max_batchsize=batch, max_latency_ms=5)
        model = ArrayModel("m")
        server.register_model(model)
        s = serve(server)
        outs[fast] = [s.fetch("/v1/models/m:predict", "POST", b) for b in FAST_BODIES]
        if fast:
            assert "JsonInstances" in model.seen
        else:
            assert "JsonInstances" not in model.seen
    for (c1, h1, b1), (c2, h2, b2) in zip(outs[True], outs[False]):
        if batch and c1 == 200:   # batchId is random
            b1, b2 = json.loads(b1), json.loads(b2)
            if isinstance(b1, dict):
                b1.pop("batchId", None)
                b2.pop("batchId", None)
        assert (c1, b1) == (c2, b2)
        assert h1["Content-Type"] == h2["Content-Type"]


def test_fast_json_not_for_custom_preprocess_or_plain_models(serve):
    server = KFServer(registered_models=KFModelRepository())
    m1, m2 = CustomPre("c"), SyncModel("s")
    server.register_model(m1)
    server.register_model(m2)
    s = serve(server)
    code, _, body = s.fetch("/v1/models/c:predict", "POST", b'{"instances": [[1, 2]]}')
    assert code == 200 and m1.seen == ["list"]
    code, _, body = s.fetch("/v1/models/s:predict", "POST", b'{"instances": [[1, 2]]}')
    assert code == 200 and json.loads(body) == {"predictions": [[2, 4]]}


# ------------------------------------------------ binary-mode CloudEvents
# The request a cloudevents ``to_binary(dummy_cloud_event(data, set_contenttype=True))``
# makes (python/kfserving/test/test_server.py:35-48), sent as tornado's test
# client sends it (POST bodies default to application/x-www-form-urlencoded).
CE_HEADERS = {
    "ce-specversion": "1.0",
    "ce-id": "36077800-0c23-4f38-a0b4-01f4369f670a",
    "ce-source": "https://example.com/event-producer",
    "ce-type": "com.example.sampletype1",
    "ce-time": "2021-01-28T21:04:43.144141+00:00",
    "ce-content-type": "application/json",
    "Content-Type": "application/x-www-form-urlencoded",
}


class RawBytesModel(KFModel):
    """Like the reference's DummyAvroCEModel: its own preprocess keeps the
    binary event's attributes and raw bytes (here: echoes their length)."""

    def __init__(self, name):
        super().__init__(name)
        self.ready = True

    def preprocess(self, request):
        from kfserving_amd.kfserving.cloudevent import CloudEvent
        assert isinstance(request, CloudEvent)
        a = request._attributes
        assert a["specversion"] == "1.0" and a["source"] == "https://example.com/event-producer"
        assert a["type"] == "com.example.sampletype1"
        assert a["datacontenttype"] == "application/x-www-form-urlencoded"
        assert a["content-type"] == "application/json"
        return request.data

    async def predict(self, request):
        return {"predictions": [[len(request), request[:1].decode("latin-1")]]}


def _check_ce_response(code, hdrs, body, want_body):
    assert code == 200
    assert body == want_body
    h = {k.lower(): v for k, v in hdrs.items()}
    assert h["content-type"] == "application/x-www-form-urlencoded"
    assert h["ce-specversion"] == "1.0"
    assert h["ce-id"] == "36077800-0c23-4f38-a0b4-01f4369f670a"
    assert h["ce-source"] == "https://example.com/event-producer"
    assert h["ce-type"] == "com.example.sampletype1"
    assert h["ce-datacontenttype"] == "application/x-www-form-urlencoded"
    assert h["ce-time"] > "2021-01-28T21:04:43.144141+00:00"


@pytest.mark.parametrize("batch", [0, 4])
def test_cloudevent_binary(serve, batch):
    """test_server.py:262-297 (binary dict / bytes data) and :299-303 (bad JSON,
    bad UTF-8: 400 with the decoder's message)."""
    server = KFServer(registered_models=KFModelRepository(), max_batchsize=batch,
                      max_latency_ms=5)
    m = DummyModel("TestModel")
    m.load()
    server.register_model(m)
    s = serve(server)
    for body in (json.dumps({"instances": [[1, 2]]}).encode(), b'{"instances":[[1,2]]}'):
        code, hdrs, out = s.fetch("/v1/models/TestModel:predict", "POST", body, CE_HEADERS)
        if batch:
            out = json.loads(out)
            assert out["predictions"] == [[1, 2]] and out["batchId"]
            out = b'{"predictions": [[1, 2]]}'
        _check_ce_response(code, hdrs, out, b'{"predictions": [[1, 2]]}')
    code, _, out = s.fetch("/v1/models/TestModel:predict", "POST", b"{", CE_HEADERS)
    assert code == 400
    assert b"Unrecognized request format: Expecting property name enclosed in double quotes" in out
    code, _, out = s.fetch("/v1/models/TestModel:predict", "POST", b"0\x80\x80\x06World!\x00\x00",
                           CE_HEADERS)
    assert code == 400
    assert (b"Unrecognized request format: 'utf-8' codec can't decode byte 0x80 in position 1: "
            b"invalid start byte") in out
    # missing a required attribute: not a binary event at all -> JSON path
    hdrs = {k: v for k, v in CE_HEADERS.items() if k != "ce-id"}
    code, _, out = s.fetch("/v1/models/TestModel:predict", "POST", b'{"instances":[[3]]}', hdrs)
    assert code == 200 and json.loads(out)["predictions"] == [[3]]
    # a bad specversion
    hdrs = dict(CE_HEADERS, **{"ce-specversion": "9.9"})
    code, _, out = s.fetch("/v1/models/TestModel:predict", "POST", b'{"instances":[[3]]}', hdrs)
    assert code == 400 and b"Cloud Event Exceptions" in out


def test_cloudevent_binary_raw_bytes(serve):
    """test_server.py:314-341 with the Avro payload replaced by raw bytes the
    model's own preprocess keeps (avro is not installed here)."""
    server = KFServer(registered_models=KFModelRepository())
    server.register_model(RawBytesModel("TestModel"))
    s = serve(server)
    data = b"\x06foo\x02\x00\x02\x08pink"
    code, hdrs, out = s.fetch("/v1/models/TestModel:predict", "POST", data, CE_HEADERS)
    _check_ce_response(code, hdrs, out, b'{"predictions": [[12, "\\u0006"]]}')


class FailingRepository(KFModelRepository):
    def __init__(self, msg):
        super().__init__(models_dir="/tmp")
        self.msg = msg

    async def load(self, name):
        raise RuntimeError(self.msg)


@pytest.mark.parametrize("msg", ["bad\r\nX-Injected: 1", "café ☃ unicode"])
def test_error_reason_is_sanitised(serve, msg):
    """A load error text with CR/LF or non-latin-1 characters still gives one
    well-formed 500 response (no header injection, no dropped connection)."""
    s = serve(KFServer(registered_models=FailingRepository(msg)))
    conn = http.client.HTTPConnection("127.0.0.1", s.port, timeout=30)
    conn.request("POST", "/v2/repository/models/m/load", body=b"")
    r = conn.getresponse()
    body = r.read()
    assert r.status == 500
    assert r.getheader("X-Injected") is None
    assert "\n" not in r.reason and "\r" not in r.reason
    assert msg.encode("utf-8") in body
    # the connection is still usable
    conn.request("GET", "/")
    r = conn.getresponse()
    assert r.status == 200 and r.read() == b"Alive"
    conn.close()
