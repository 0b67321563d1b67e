"""The native HTTP front end (include/kfhttp.h, libkfserve.so), CPU only:
every response must be the Python server's bytes for the same request
(python/kfserving/test/test_server.py's byte contracts are the reference's).
The xgbserver model's device call is replaced by the canonical numpy
evaluator, so the native route's batches go through the native batcher to a
Python model behind the same function pointer; the -m gpu twin is
tests/test_gpu_native_http.py."""
import http.client
import json
import os
import re
import shutil
import socket
import struct
import time

import numpy as np
import pytest

from kfserving_amd.forest import OUT_PREDICT
from kfserving_amd.kfserving import KFServer
from kfserving_amd.kfserving.native_http import EXPORTED_SYMBOLS, load_library, repr_double
from tests import canon_eval
from tests.test_server import _Running

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_declares_the_binding_symbols():
    import subprocess
    src = open(os.path.join(ROOT, "include", "kfhttp.h")).read()
    names = sorted(set(re.findall(r"^\s*(?:int|int32_t)\s+(kh_\w+)\(", src, re.M)))
    assert names == sorted(EXPORTED_SYMBOLS)
    lib = load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True,
                         text=True, check=True).stdout
    assert set(names) <= set(re.findall(r"\bT (kh_\w+)", out))


def test_repr_double_matches_python():
    rng = np.random.default_rng(1)
    vals = [0.0, -0.0, 1.0, -1.0, 0.5, 0.1, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5,
            0.0001234, 123456789012345678.0, 5e-324, 1.7976931348623157e308, 2.5e-7,
            float("nan"), float("inf"), float("-inf"), 100.0, 1e22, 1e21, 0.001, 12.5]
    vals += list(rng.standard_normal(2000) * 10.0 ** rng.integers(-30, 30, 2000))
    vals += [float(np.float32(v)) for v in rng.standard_normal(2000)]
    vals += [float(v) for v in rng.uniform(0, 1, 500).astype(np.float32)]
    for v in vals:
        assert repr_double(v) == json.dumps(v), v


def _xgb_model(golden, tmp_path, name="xgboost-iris"):
    from kfserving_amd.xgbserver import XGBoostModel
    d = tmp_path / name
    d.mkdir(parents=True)
    shutil.copy(os.path.join(golden, "xgb_iris_legacy_082.bst"), str(d / "model.bst"))
    m = XGBoostModel(name, str(d), 1)
    m.load()
    m.predict_matrix = lambda X, kind=OUT_PREDICT: canon_eval.predict(m._forest, X, kind)
    return m


def _servers(golden, tmp_path, **kw):
    """The same model behind the native front end and behind the Python server."""
    out = []
    for native in (True, False):
        srv = KFServer(max_batchsize=kw.get("batch", 64), max_latency_ms=kw.get("lat", 3))
        srv.native_http = native
        srv.register_model(_xgb_model(golden, tmp_path / ("n" if native else "p")))
        out.append(_Running(srv))
    _wait_front_end(out[0])
    return out


def _wait_front_end(running, timeout=30.0):
    """serve() installs the native front end on the server's thread."""
    t0 = time.time()
    while running.server.front_end is None and time.time() - t0 < timeout:
        time.sleep(0.02)
    assert running.server.front_end is not None, "native front end did not start"


def _raw(port, data: bytes, timeout=10.0) -> bytes:
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    s.sendall(data)
    chunks = []
    try:
        while True:
            b = s.recv(65536)
            if not b:
                break
            chunks.append(b)
    except socket.timeout:
        pass
    s.close()
    return b"".join(chunks)


def _norm(b: bytes) -> bytes:
    return re.sub(rb'"batchId": "[0-9a-f-]{36}"', b'"batchId": "ID"', b)


def _iris_bodies():
    from sklearn.datasets import load_iris
    X = load_iris()["data"]
    rng = np.random.default_rng(0)
    bodies = []
    for i in range(12):
        rows = X[rng.integers(0, 150, int(rng.integers(1, 9)))].tolist()
        if i % 4 == 1:
            rows[0][1] = 0            # DMatrix(list): 0 is missing
        bodies.append(json.dumps({"instances": rows}).encode())
    bodies.append(b'{"instances": [[6.8, 2.8, 4.8, 1.4], [6.0, 3.4, 4.5, 1.6]]}')
    bodies.append(b'{ "instances" : [ [ NaN, 1e-3, -0.0, Infinity ] ] }')
    return bodies


def test_native_predict_bytes_equal_python_server(golden, tmp_path):
    nat, py = _servers(golden, tmp_path)
    try:
        fe = nat.server.front_end
        assert fe is not None and "xgboost-iris" in fe.routes
        for body in _iris_bodies():
            a = nat.fetch("/v1/models/xgboost-iris:predict", "POST", body)
            b = py.fetch("/v1/models/xgboost-iris:predict", "POST", body)
            assert a[0] == b[0] == 200
            assert {k: v for k, v in a[1].items()} == {k: v for k, v in b[1].items()}
            assert _norm(a[2]) == _norm(b[2])
            assert json.loads(a[2])["batchId"]
            # /v2/.../infer answers a v1 body as :predict (ref kfserver.py:77-78)
            a = nat.fetch("/v2/models/xgboost-iris/infer", "POST", body)
            b = py.fetch("/v2/models/xgboost-iris/infer", "POST", body)
            assert (a[0], dict(a[1].items())) == (b[0], dict(b[1].items()))
            assert _norm(a[2]) == _norm(b[2])
        st = fe.stats()
        assert st["native_requests"] >= 28 and st["python_requests"] == 0
    finally:
        nat.stop()
        py.stop()


def test_fallback_routes_and_errors_equal_python_server(golden, tmp_path):
    nat, py = _servers(golden, tmp_path)
    cases = [
        ("/", "GET", None, {}),
        ("/v1/models", "GET", None, {}),
        ("/v1/models/xgboost-iris", "GET", None, {}),
        ("/v1/models/nope", "GET", None, {}),
        ("/v1/models/nope:predict", "POST", b'{"instances": [[1, 2, 3, 4]]}', {}),
        ("/v1/models/xgboost-iris:predict", "POST", b'{"instances": 3}', {}),
        ("/v1/models/xgboost-iris:predict", "POST", b'not json', {}),
        ("/v1/models/xgboost-iris:predict", "POST", b'{"instances": [[1, 2, 3]]}', {}),
        ("/v1/models/xgboost-iris:predict", "GET", None, {}),
        ("/v1/models/xgboost-iris:predict?x=1", "POST", b'{"instances": [[1, 2, 3, 4]]}', {}),
        ("/v2/models/xgboost-iris/infer", "POST",
         json.dumps({"inputs": [{"name": "x", "shape": [1, 4], "datatype": "FP32",
                                 "data": [1, 2, 3, 4]}]}).encode(), {}),
        ("/v1/models/xgboost-iris:predict", "POST", b'{"instances": [[1, 2, 3, 4]]}',
         {"ce-specversion": "1.0", "ce-source": "s", "ce-type": "t", "ce-id": "1",
          "content-type": "application/json"}),
        ("/v2/models/xgboost-iris/infer", "POST", b'{"instances": [[1, 2, 3, 4]]}',
         {"Inference-Header-Content-Length": "29"}),
        ("/v2/models/xgboost-iris/infer", "POST", b'{"instances": [[1, 2, 3, 4]]}',
         {"Inference-Header-Content-Length": "12"}),
        ("/v2/models/nope/infer", "POST", b'{"instances": [[1, 2, 3, 4]]}', {}),
        ("/v2/models/xgboost-iris/infer", "GET", None, {}),
    ]
    try:
        for path, method, body, hdrs in cases:
            a = nat.fetch(path, method, body, hdrs)
            b = py.fetch(path, method, body, hdrs)
            a_h = {k: v for k, v in a[1].items() if k.lower() not in ("ce-time", "ce-id")}
            b_h = {k: v for k, v in b[1].items() if k.lower() not in ("ce-time", "ce-id")}
            assert (a[0], a_h) == (b[0], b_h), (path, method)
            assert _norm(a[2]) == _norm(b[2]), (path, method, a[2], b[2])
        assert nat.server.front_end.stats()["python_requests"] >= len(cases) - 1
    finally:
        nat.stop()
        py.stop()


def test_malformed_requests_and_framing(golden, tmp_path):
    """400 / 413 pages and closes, chunked bodies, keep-alive, pipelining and
    Connection: close, byte for byte as the Python server."""
    nat, py = _servers(golden, tmp_path)
    body = b'{"instances": [[6.8, 2.8, 4.8, 1.4]]}'
    req = (b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nHost: x\r\n"
           b"Content-Length: %d\r\n\r\n" % len(body)) + body
    chunked = (b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nHost: x\r\n"
               b"Transfer-Encoding: chunked\r\n\r\n" + b"%x\r\n" % 10 + body[:10] + b"\r\n" +
               b"%x;ext=1\r\n" % (len(body) - 10) + body[10:] + b"\r\n0\r\n\r\n")
    close = req.replace(b"Host: x\r\n", b"Host: x\r\nConnection: close\r\n")
    http10 = req.replace(b"HTTP/1.1\r\n", b"HTTP/1.0\r\n", 1)
    cases = [
        b"GARBAGE\r\n\r\n",
        b"GET / HTTP/1.1 extra\r\n\r\n",
        b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nContent-Length: abc\r\n\r\n",
        b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nContent-Length: 999999999999\r\n\r\n",
        chunked + close,          # a chunked request, then one that closes
        req + req + close,        # three pipelined requests on one connection
        http10,                   # HTTP/1.0: no keep-alive
        close,
    ]
    # a 3 MB body in 4 KB chunks (arrives over many reads; the threaded parser
    # and the application answer it), then one that closes
    rows = [[6.8, 2.8, 4.8, 1.4], [5.0, 3.4, 1.5, 0.2]] * 70000
    big = json.dumps({"instances": rows}).encode()
    assert len(big) > 3_000_000
    parts = [big[i:i + 4096] for i in range(0, len(big), 4096)]
    big_chunked = (b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nHost: x\r\n"
                   b"Transfer-Encoding: chunked\r\n\r\n" +
                   b"".join(b"%x\r\n" % len(p) + p + b"\r\n" for p in parts) + b"0\r\n\r\n")
    cases.append(big_chunked + close)
    try:
        for data in cases:
            a = _raw(nat.port, data, timeout=3)
            b = _raw(py.port, data, timeout=3)
            assert _norm(a) == _norm(b), (data[:60], a[:300], b[:300])
            assert a.startswith(b"HTTP/1.1 ")
    finally:
        nat.stop()
        py.stop()


def _raw_parts(port, parts, delay=0.0, shut=True, timeout=10.0) -> bytes:
    """Send `parts` with `delay` between them (each a separate read on the
    server), half-close (SHUT_WR) if `shut`, then read until the server closes."""
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    for p in parts:
        s.sendall(p)
        if delay:
            time.sleep(delay)
    if shut:
        s.shutdown(socket.SHUT_WR)
    chunks = []
    try:
        while True:
            b = s.recv(65536)
            if not b:
                break
            chunks.append(b)
    except socket.timeout:
        pass
    s.close()
    return b"".join(chunks)


def test_half_close_answers_every_pipelined_request(golden, tmp_path):
    """a client that pipelines requests and then shuts its side
    (SHUT_WR) gets every complete request answered, in order, then the close;
    a request cut short by the EOF is answered 400 (the Python server's
    IncompleteReadError); bytes equal to the asyncio server's."""
    nat, py = _servers(golden, tmp_path)
    bodies = _iris_bodies()[:3]
    reqs = [(b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nHost: x\r\n"
             b"Content-Length: %d\r\n\r\n" % len(b)) + b for b in bodies]
    get = b"GET /v1/models/xgboost-iris HTTP/1.1\r\nHost: x\r\n\r\n"
    cases = [
        [b"".join(reqs)],                           # three keep-alive requests, then EOF
        [reqs[0], get, reqs[1]],                    # native, application, native
        [reqs[0] + reqs[1][:-7]],                   # the second body cut by the EOF: 400
    ]
    try:
        for parts in cases:
            a = _raw_parts(nat.port, parts, delay=0.05)
            b = _raw_parts(py.port, parts, delay=0.05)
            assert _norm(a) == _norm(b), (a[-400:], b[-400:])
        a = _raw_parts(nat.port, cases[0])
        assert a.count(b"HTTP/1.1 200 OK") == 3
        a = _raw_parts(nat.port, cases[2])
        assert a.count(b"HTTP/1.1 200 OK") == 1 and b"HTTP/1.1 400 Bad Request" in a
        # cut inside the headers: the asyncio server's readline hands the
        # fragment on as a header line and the application answers the
        # body-less request; the native parser answers 400 (documented in
        # DESIGN.md section 7)
        a = _raw_parts(nat.port, [reqs[0] + reqs[1][:40]])
        assert a.count(b"HTTP/1.1 200 OK") == 1 and a.endswith(b"400: Bad Request</body></html>")
    finally:
        nat.stop()
        py.stop()


def test_chunked_body_resumes_across_reads(golden, tmp_path):
    """an incomplete chunked body keeps its parse state between
    reads.  Bodies split at every kind of boundary (inside a chunk-size line,
    inside chunk data, between data and its CRLF, inside the last-chunk
    line) arrive over many reads and are answered as the Python server
    answers them; a body of 200k one-byte chunks sent in 100 pieces finishes
    quickly (the resumed parse is linear in the chunks)."""
    nat, py = _servers(golden, tmp_path)
    body = b'{"instances": [[6.8, 2.8, 4.8, 1.4], [5.0, 3.4, 1.5, 0.2]]}'
    head = (b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nHost: x\r\n"
            b"Transfer-Encoding: chunked\r\n\r\n")
    framed = b"".join(b"%x\r\n" % 3 + body[i:i + 3] + b"\r\n"
                      for i in range(0, len(body), 3)) + b"0\r\n\r\n"
    msg = head + framed
    try:
        for step in (1, 2, 5, 7, 11):
            parts = [msg[i:i + step] for i in range(0, len(msg), step)][:40]
            parts.append(msg[sum(len(p) for p in parts):])
            a = _raw_parts(nat.port, parts, delay=0.002)
            b = _raw_parts(py.port, parts, delay=0.002)
            assert _norm(a) == _norm(b) and a.startswith(b"HTTP/1.1 200 OK"), (step, a[:200])
        rows = [[6.8, 2.8, 4.8, 1.4]] * 9200
        big = json.dumps({"instances": rows}).encode()
        assert len(big) > 200_000
        framed = b"".join(b"1\r\n" + big[i:i + 1] + b"\r\n" for i in range(len(big))) + b"0\r\n\r\n"
        data = head + framed
        n = 100
        parts = [data[i * len(data) // n:(i + 1) * len(data) // n] for i in range(n)]
        t0 = time.time()
        a = _raw_parts(nat.port, parts, delay=0.002, timeout=60)
        took = time.time() - t0
        assert a.startswith(b"HTTP/1.1 200 OK") and len(json.loads(a.split(b"\r\n\r\n", 1)[1])
                                                       ["predictions"]) == 9200
        assert took < 20, took
    finally:
        nat.stop()
        py.stop()


def _rss_bytes() -> int:
    with open("/proc/self/statm") as fh:
        return int(fh.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")


def test_pipelined_bytes_behind_a_busy_request_are_bounded(golden, tmp_path):
    """while a request is being answered the front end stops
    reading once kMaxPipelined (2 MiB) of unparsed bytes wait behind it, so a
    client pipelining 96 MB behind a slow request does not grow the server's
    memory; reading resumes after the answer (here the garbage behind it is
    then a 400 and a close)."""
    import threading
    nat, py = _servers(golden, tmp_path)
    py.stop()
    m = nat.server.registered_models.get_model("xgboost-iris")
    fast = m.predict_matrix

    def slow(X, kind=OUT_PREDICT):
        time.sleep(3.0)
        return fast(X, kind)
    m.predict_matrix = slow
    body = b'{"instances": [[6.8, 2.8, 4.8, 1.4]]}'
    req = (b"POST /v1/models/xgboost-iris:predict HTTP/1.1\r\nHost: x\r\n"
           b"Content-Length: %d\r\n\r\n" % len(body)) + body
    junk = b"x" * (96 << 20)
    s = socket.create_connection(("127.0.0.1", nat.port), timeout=30)
    got = []

    def send():
        try:
            s.sendall(req)
            s.sendall(junk)
        except OSError:
            pass
    rss0 = _rss_bytes()
    th = threading.Thread(target=send, daemon=True)
    th.start()
    try:
        time.sleep(1.5)             # the request is on the batcher; bytes pile up behind it
        grown = _rss_bytes() - rss0
        assert grown < (24 << 20), grown
        assert th.is_alive()        # the sender is blocked: the server stopped reading
        try:
            while True:
                b = s.recv(65536)
                if not b:
                    break
                got.append(b)
        except (socket.timeout, ConnectionResetError):
            pass
        out = b"".join(got)
        assert out.startswith(b"HTTP/1.1 200 OK")          # the slow request is answered
        assert b"HTTP/1.1 400 Bad Request" in out          # then the garbage line: 400
    finally:
        s.close()
        th.join(timeout=10)
        m.predict_matrix = fast
        nat.stop()


def test_concurrent_connections_share_batches(golden, tmp_path):
    """Many connections at once: one batch answers several requests (one
    batchId), every answer is the evaluator's for its own rows."""
    import threading
    from sklearn.datasets import load_iris
    nat, py = _servers(golden, tmp_path, lat=20)
    X = load_iris()["data"]
    model = _xgb_model(golden, tmp_path / "ref")
    out = [None] * 48
    start = threading.Barrier(48)

    def one(i):
        rows = X[i:i + 1 + i % 3].tolist()
        start.wait()
        out[i] = (rows, nat.fetch("/v1/models/xgboost-iris:predict", "POST",
                                  json.dumps({"instances": rows}).encode()))
    th = [threading.Thread(target=one, args=(i,)) for i in range(48)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    try:
        ids = set()
        for rows, (code, _, body) in out:
            assert code == 200
            res = json.loads(body)
            ids.add(res["batchId"])
            want = model.predict({"instances": rows})["predictions"]
            assert res["predictions"] == want
        assert len(ids) < 48
    finally:
        nat.stop()
        py.stop()


def test_reload_moves_the_route_to_the_new_batcher(golden, tmp_path):
    """A reload through the repository route (/v2/repository/models/<m>/load)
    retires the model's batchers: the native route is removed before its
    batcher stops, the next request goes through the application, which makes
    the new model's batcher, and the route comes back on it."""
    from kfserving_amd.kfserving.kfmodel_repository import KFModelRepository

    class Repo(KFModelRepository):
        def load(self, name):
            self.update(_xgb_model(golden, tmp_path / f"reload{len(loads)}"))
            loads.append(name)
            return True
    loads = []
    srv = KFServer(max_batchsize=64, max_latency_ms=3, registered_models=Repo())
    srv.register_model(_xgb_model(golden, tmp_path / "first"))
    nat = _Running(srv)
    _wait_front_end(nat)
    body = b'{"instances": [[6.8, 2.8, 4.8, 1.4]]}'
    try:
        fe = srv.front_end
        m0 = srv.registered_models.get_model("xgboost-iris")
        first = nat.fetch("/v1/models/xgboost-iris:predict", "POST", body)
        code, _, out = nat.fetch("/v2/repository/models/xgboost-iris/load", "POST", b"")
        assert code == 200 and loads == ["xgboost-iris"]
        assert "xgboost-iris" not in fe.routes
        m1 = srv.registered_models.get_model("xgboost-iris")
        assert m1 is not m0
        code, _, out = nat.fetch("/v1/models/xgboost-iris:predict", "POST", body)
        assert code == 200 and _norm(out) == _norm(first[2])
        nb = fe.app._batchers[("xgboost-iris", "instances")]
        assert nb.model is m1 and fe.routes["xgboost-iris"].value == nb._nb._h.value
        n0 = fe.stats()["native_requests"]
        assert nat.fetch("/v1/models/xgboost-iris:predict", "POST", body)[0] == 200
        assert fe.stats()["native_requests"] == n0 + 1
        # the V2 tensor route follows its batcher through a reload too
        tb = _v2([[6.8, 2.8, 4.8, 1.4]], [1, 4], "FP32")
        v2p = "/v2/models/xgboost-iris/infer"
        first_v2 = nat.fetch(v2p, "POST", tb)
        assert first_v2[0] == 200 and "v2:xgboost-iris" in fe.routes
        assert nat.fetch("/v2/repository/models/xgboost-iris/load", "POST", b"")[0] == 200
        assert "v2:xgboost-iris" not in fe.routes
        again = nat.fetch(v2p, "POST", tb)                  # through the application
        assert again[0] == 200 and again[2] == first_v2[2]
        tnb = fe.app._batchers[("xgboost-iris", "tensor")]
        assert fe.routes["v2:xgboost-iris"].value == tnb._nb._h.value
        n1 = fe.stats()["native_requests"]
        assert nat.fetch(v2p, "POST", tb)[2] == first_v2[2]
        assert fe.stats()["native_requests"] == n1 + 1
    finally:
        nat.stop()


def test_sklearn_regressor_route_and_its_checks(golden, tmp_path):
    """sklearnserver regressors get a native route too: the float32 cast,
    and a body the model's own checks reject (a value beyond float32, an
    infinity, a NaN for an estimator without missing-value support) is
    answered by the application, byte for byte as the asyncio server."""
    from kfserving_amd.sklearnserver import SKLearnModel

    def model(sub, allow_nan=True):
        d = tmp_path / sub
        d.mkdir(parents=True)
        shutil.copy(os.path.join(golden, "sk_rf_reg_model.npz"), str(d / "model.npz"))
        m = SKLearnModel("sk", str(d))
        assert m.load()
        m._forest.meta["allow_nan"] = allow_nan
        m.predict_matrix = lambda X, kind=OUT_PREDICT: canon_eval.predict(m._forest, X, kind)
        return m
    g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
    X = np.nan_to_num(g["X"][:6]).astype(np.float64)
    F = X.shape[1]
    for allow_nan in (True, False):
        runs = []
        for native in (True, False):
            srv = KFServer(max_batchsize=64, max_latency_ms=3)
            srv.native_http = native
            srv.register_model(model(f"{allow_nan}{native}", allow_nan))
            runs.append(_Running(srv))
        nat, py = runs
        _wait_front_end(nat)
        try:
            assert "sk" in nat.server.front_end.routes
            bodies = [json.dumps({"instances": X[:k].tolist()}).encode() for k in (1, 3, 6)]
            bad = X[:2].tolist()
            bad[1][0] = 1e39
            bodies.append(json.dumps({"instances": bad}).encode())
            bodies.append(json.dumps({"instances": [[float("inf")] * F]}).encode())
            bodies.append(json.dumps({"instances": [[float("nan")] + [0.5] * (F - 1)]}).encode())
            for body in bodies:
                a = nat.fetch("/v1/models/sk:predict", "POST", body)
                b = py.fetch("/v1/models/sk:predict", "POST", body)
                assert a[0] == b[0] and a[1] == b[1] and _norm(a[2]) == _norm(b[2]), body[:80]
            st = nat.server.front_end.stats()
            assert st["native_requests"] >= 3 and st["python_requests"] >= 2
        finally:
            nat.stop()
            py.stop()


def test_sklearn_classifier_route_answers_labels(golden, tmp_path):
    """A classifier's native route answers class labels, rendered as its
    predict renders classes.take(index).tolist() (numeric and string
    labels), byte for byte as the asyncio server."""
    from kfserving_amd.sklearnserver import SKLearnModel
    g = np.load(os.path.join(golden, "sk_rf_clf.npz"))
    X = np.nan_to_num(g["X"][:8]).astype(np.float64)
    for labels in (None, np.array(["setosa", "versiécolor", 'vir"ginica', "x", "y"])):
        runs = []
        for native in (True, False):
            d = tmp_path / f"{labels is None}{native}"
            d.mkdir(parents=True)
            shutil.copy(os.path.join(golden, "sk_rf_clf_model.npz"), str(d / "model.npz"))
            m = SKLearnModel("clf", str(d))
            assert m.load()
            if labels is not None:
                k = len(m._forest.meta["classes"])
                m._forest.meta["classes"] = labels[:k]
            m.predict_matrix = (lambda mm: lambda X, kind=OUT_PREDICT:
                                canon_eval.predict(mm._forest, X, kind))(m)
            srv = KFServer(max_batchsize=64, max_latency_ms=3)
            srv.native_http = native
            srv.register_model(m)
            runs.append(_Running(srv))
        nat, py = runs
        _wait_front_end(nat)
        try:
            assert "clf" in nat.server.front_end.routes
            for k in (1, 3, 8):
                body = json.dumps({"instances": X[:k].tolist()}).encode()
                a = nat.fetch("/v1/models/clf:predict", "POST", body)
                b = py.fetch("/v1/models/clf:predict", "POST", body)
                assert a[0] == b[0] == 200 and _norm(a[2]) == _norm(b[2]), (a[2], b[2])
            assert nat.server.front_end.stats()["native_requests"] >= 3
        finally:
            nat.stop()
            py.stop()


def test_lgbserver_inputs_route_bytes_equal_python_server(golden, tmp_path):
    """lgbserver's {"inputs": [...]} bodies on the native route
    (kf_parse_inputs): columns by name, absent columns NaN, dropped keys of
    any shape, nulls, boolean columns -- and every body outside that subset
    (booleans mixed with numbers, all-null or string columns, duplicate or
    escaped keys, unequal columns, no rows, non-object elements) answered by
    the application; bytes identical to the asyncio server."""
    from tests.test_lgb_batching import _lgb_model
    runs = []
    for native in (True, False):
        srv = KFServer(max_batchsize=64, max_latency_ms=3)
        srv.native_http = native
        (tmp_path / ("n" if native else "p")).mkdir()
        srv.register_model(_lgb_model(golden, tmp_path / ("n" if native else "p")))
        runs.append(_Running(srv))
    nat, py = runs
    _wait_front_end(nat)
    names = ["sepal_length_(cm)", "sepal_width_(cm)", "petal_length_(cm)", "petal_width_(cm)"]
    a, b, c, d = names
    bodies = [
        {"inputs": [{a: [5.1, 6.2], b: [3.5, 2.9], c: [1.4, 4.3], d: [0.2, 1.3]}]},
        {"inputs": [{d: [1.8], c: [5.0], a: [6.3], b: [2.5], "x": [1, 2, 3]}]},
        {"inputs": [{a: [5.0, 5.5], c: [1.0, None]}, {b: [3.0], d: [0.1]}]},
        {"inputs": [{a: [True, False], b: [1, 2], c: [0, 0], d: [2, 3],
                     "meta": {"k": ["s", {"n": None}], "t": True}}]},
        {"inputs": [{a: [1e-320, -0.0], b: [1e300, 3], c: [float("nan"), 2], d: [4, 5]}]},
        {"inputs": [{a: [True, 1.0], b: [1.0, 2.0]}]},            # bool mixed: pandas
        {"inputs": [{a: [None, None], b: [1.0, 2.0]}]},           # all-null column
        {"inputs": [{a: ["1.0"], b: [1.0]}]},                     # strings
        {"inputs": [{a: [1.0, 2.0], b: [1.0]}]},                  # unequal lengths
        {"inputs": [{"x": [1.0]}]},                               # no rows
        {"inputs": []},
        {"inputs": [3]},
        {"inputs": 3},
    ]
    raw = [
        b'{"inputs": [{"sepal_length_(cm)": [1.0], "sepal_length_(cm)": [2.0]}]}',
        b'{"inputs": [{"sepal_length_\\u0028cm)": [1.0]}]}',
        b'{"inputs": [{"sepal_length_(cm)": [12345678901234567890123], "sepal_width_(cm)": [1]}]}',
    ]
    try:
        assert "lightgbm" in nat.server.front_end.routes
        for body in [json.dumps(x).encode() for x in bodies] + raw:
            x = nat.fetch("/v1/models/lightgbm:predict", "POST", body)
            y = py.fetch("/v1/models/lightgbm:predict", "POST", body)
            assert x[0] == y[0] and x[1] == y[1] and _norm(x[2]) == _norm(y[2]), (body, x, y)
        st = nat.server.front_end.stats()
        assert st["native_requests"] >= 5 and st["python_requests"] >= 8
    finally:
        nat.stop()
        py.stop()


def test_create_failure_closes_what_it_opened(tmp_path):
    """kh_create on a descriptor epoll cannot watch (a regular file) fails
    with -3 and leaves no descriptor of its own open."""
    import ctypes
    from kfserving_amd.kfserving.native_http import KH_ABI_VERSION, KhConfig
    lib = load_library()
    p = tmp_path / "f"
    p.write_bytes(b"x")
    with open(p, "rb") as fh:
        before = len(os.listdir("/proc/self/fd"))
        cfg = KhConfig(abi_version=KH_ABI_VERSION, listen_fd=fh.fileno(), io_threads=4,
                       max_body_bytes=0)
        h = ctypes.c_void_p()
        for _ in range(5):
            assert lib.kh_create(ctypes.byref(cfg), ctypes.byref(h)) == -3
        assert not h.value
        assert len(os.listdir("/proc/self/fd")) == before


def test_large_bodies_take_the_native_route(golden, tmp_path):
    """Bodies of >= 1 MB are parsed natively on the IO thread with the
    threaded parser (kf_parse_instances_mt, KF_PARSE_THREADS as the
    application's fastjson) and answered natively: the bytes equal the
    asyncio server's, and no request reaches the application."""
    from sklearn.datasets import load_iris
    nat, py = _servers(golden, tmp_path, batch=65536)
    X = load_iris()["data"]
    rng = np.random.default_rng(4)
    try:
        fe = nat.server.front_end
        for n in (50_000, 120_000):
            rows = X[rng.integers(0, 150, n)].tolist()
            rows[7][2] = 0                       # DMatrix(list): 0 is missing
            body = json.dumps({"instances": rows}).encode()
            assert len(body) >= 1 << 20
            a = nat.fetch("/v1/models/xgboost-iris:predict", "POST", body)
            b = py.fetch("/v1/models/xgboost-iris:predict", "POST", body)
            assert a[0] == b[0] == 200 and dict(a[1].items()) == dict(b[1].items())
            assert _norm(a[2]) == _norm(b[2])
        st = fe.stats()
        assert st["native_requests"] >= 2 and st["python_requests"] == 0
    finally:
        nat.stop()
        py.stop()


def test_v2_tensor_route_bytes_equal_python_server(golden, tmp_path):
    """V2 tensor requests (/v2/models/<name>/infer, JSON data) of xgbserver
    take the native route once the application has made the model's tensor
    batcher: FP32 / FP64, flat or row-nested data, a [F] tensor as one row,
    an id echoed, JSON's NaN / Infinity and integers; every other V2 request
    (outputs, parameters, other datatypes, ragged data, a size or width that
    does not match, an escaped id) is the application's.  Bytes equal the
    asyncio server's throughout."""
    nat, py = _servers(golden, tmp_path)
    rng = np.random.default_rng(9)
    X = rng.uniform(0, 7, (6, 4)).round(3)

    def t(data, shape, dt="FP32", **extra):
        body = {"inputs": [{"name": "x", "shape": shape, "datatype": dt, "data": data}]}
        body.update(extra)
        return json.dumps(body).encode()
    native = [
        t(X.reshape(-1).tolist(), [6, 4]),
        t(X.tolist(), [6, 4], "FP64", id="req-17"),
        t(X[0].tolist(), [4]),
        t([[1, 2.5, 0, 3], [4, 5, 6, 7]], [2, 4], "FP64"),
        b'{"id": "q", "inputs": [{"data": [NaN, 1.0, Infinity, -Infinity], "datatype": "FP32",'
        b' "shape": [1, 4], "name": "in"}]}',
        t((X * 1e30).reshape(-1).tolist(), [6, 4], "FP32"),       # float32 overflow: inf
        t(X.reshape(-1).tolist(), [6, 4], parameters={"binary_data_output": True}),
        t(X.reshape(-1).tolist(), [6, 4], parameters={"binary_data_output": False}, id="b"),
    ]
    fallback = [
        t(X.reshape(-1).tolist(), [6, 4], outputs=[{"name": "predict"}]),
        t(X.reshape(-1).tolist(), [6, 4], parameters={"binary_data_output": 1}),
        t([1, 2, 3, 4], [1, 4], "INT32"),
        t([[1, 2, 3, 4], [5, 6, 7]], [2, 4]),
        t(X.reshape(-1).tolist(), [5, 4]),
        t(X[:, :3].reshape(-1).tolist(), [6, 3]),
        t(X[0].tolist(), [4], id="été"),
        t([], [0, 4]),
        b'{"inputs": [{"name": "x", "shape": [1, 4], "datatype": "FP32", "data": [1, 2, 3, 4]},'
        b' {"name": "y", "shape": [1, 4], "datatype": "FP32", "data": [1, 2, 3, 4]}]}',
    ]
    path = "/v2/models/xgboost-iris/infer"
    try:
        fe = nat.server.front_end
        # the first tensor request makes the tensor batcher: the route follows
        for body in [native[0]] + native + fallback:
            a = nat.fetch(path, "POST", body)
            b = py.fetch(path, "POST", body)
            assert (a[0], dict(a[1].items())) == (b[0], dict(b[1].items())), (body[:90], a, b)
            assert a[2] == b[2], (body[:90], a[2][:300], b[2][:300])
        assert "v2:xgboost-iris" in fe.routes
        st = fe.stats()
        assert st["python_requests"] == 1 + len(fallback), st
        assert st["native_requests"] == len(native), st
        # the binary tensor extension (Inference-Header-Content-Length): input
        # and output natively; a size that does not match, or bytes no input
        # claims, are the application's
        def binreq(Xb, dt, size=None, extra=b"", **top):
            raw = Xb.astype(np.float32 if dt == "FP32" else np.float64).tobytes()
            req = {"inputs": [{"name": "x", "shape": list(Xb.shape), "datatype": dt,
                               "parameters": {"binary_data_size": size or len(raw)}}]}
            req.update(top)
            head = json.dumps(req).encode()
            return head + raw + extra, {"Inference-Header-Content-Length": str(len(head))}
        bin_native = [binreq(X, "FP32"), binreq(X, "FP64", id="k"),
                      binreq(X[:2], "FP32", parameters={"binary_data_output": True}),
                      (t(X.tolist(), [6, 4]), {"Inference-Header-Content-Length":
                                               str(len(t(X.tolist(), [6, 4])))})]
        bin_fallback = [binreq(X, "FP32", size=12), binreq(X, "FP32", extra=b"xx"),
                        (t(X.tolist(), [6, 4]), {"Inference-Header-Content-Length": "abc"}),
                        (t(X.tolist(), [6, 4]), {"Inference-Header-Content-Length": "99999"})]
        n0 = fe.stats()
        for body, hdr in bin_native + bin_fallback:
            a = nat.fetch(path, "POST", body, hdr)
            b = py.fetch(path, "POST", body, hdr)
            assert (a[0], dict(a[1].items()), a[2]) == (b[0], dict(b[1].items()), b[2]), \
                (body[:90], a[:2], b[:2])
        n1 = fe.stats()
        assert n1["native_requests"] - n0["native_requests"] == len(bin_native)
        assert n1["python_requests"] - n0["python_requests"] == len(bin_fallback)
    finally:
        nat.stop()
        py.stop()


def _v2(data, shape, dt="FP64", **extra):
    body = {"inputs": [{"name": "x", "shape": shape, "datatype": dt, "data": data}]}
    body.update(extra)
    return json.dumps(body).encode()


def _v2_pairs(nat, py, path, bodies):
    for body in bodies:
        a = nat.fetch(path, "POST", body)
        b = py.fetch(path, "POST", body)
        assert (a[0], dict(a[1].items()), a[2]) == (b[0], dict(b[1].items()), b[2]), \
            (body[:90], a, b)


def test_v2_tensor_route_lgbserver_and_sklearn_regressor(golden, tmp_path):
    """The V2 tensor route of lgbserver (float64 columns in booster order,
    FP64 output) and of a sklearn regressor (the float32 cast with its
    checks: a value beyond float32 or a NaN it rejects goes to the
    application), byte for byte as the asyncio server."""
    from tests.test_lgb_batching import _lgb_model
    from kfserving_amd.sklearnserver import SKLearnModel
    # lgbserver
    runs = []
    for native in (True, False):
        srv = KFServer(max_batchsize=64, max_latency_ms=3)
        srv.native_http = native
        (tmp_path / ("ln" if native else "lp")).mkdir()
        srv.register_model(_lgb_model(golden, tmp_path / ("ln" if native else "lp")))
        runs.append(_Running(srv))
    nat, py = runs
    _wait_front_end(nat)
    name = nat.server.front_end.app.models.get_models()[0].name
    path = f"/v2/models/{name}/infer"
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 7, (5, 4)).round(2)
    try:
        _v2_pairs(nat, py, path, [_v2(X.tolist(), [5, 4])])     # makes the tensor batcher
        before = nat.server.front_end.stats()
        _v2_pairs(nat, py, path, [_v2(X.reshape(-1).tolist(), [5, 4]),
                                  _v2(X[1].tolist(), [4], "FP32", id="a"),
                                  _v2([[float("nan"), 1, 2, 3]], [1, 4], "FP64")])
        st = nat.server.front_end.stats()
        assert st["native_requests"] - before["native_requests"] == 3
        assert f"v2:{name}" in nat.server.front_end.routes
    finally:
        nat.stop()
        py.stop()
    # a sklearn regressor without missing-value support
    g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
    Xs = np.nan_to_num(g["X"][:4]).astype(np.float64)
    F = Xs.shape[1]
    runs = []
    for native in (True, False):
        d = tmp_path / f"sk{native}"
        d.mkdir()
        shutil.copy(os.path.join(golden, "sk_rf_reg_model.npz"), str(d / "model.npz"))
        m = SKLearnModel("sk", str(d))
        assert m.load()
        m._forest.meta["allow_nan"] = False
        m.predict_matrix = lambda X, kind=OUT_PREDICT, m=m: canon_eval.predict(m._forest, X, kind)
        srv = KFServer(max_batchsize=64, max_latency_ms=3)
        srv.native_http = native
        srv.register_model(m)
        runs.append(_Running(srv))
    nat, py = runs
    _wait_front_end(nat)
    path = "/v2/models/sk/infer"
    bad = Xs[:2].copy()
    bad[1, 0] = 1e39
    try:
        _v2_pairs(nat, py, path, [_v2(Xs.tolist(), [4, F])])
        before = nat.server.front_end.stats()
        _v2_pairs(nat, py, path, [_v2(Xs.reshape(-1).tolist(), [4, F], "FP32"),
                                  _v2(Xs[0].tolist(), [F], id="one")])
        mid = nat.server.front_end.stats()
        assert mid["native_requests"] - before["native_requests"] == 2
        _v2_pairs(nat, py, path, [_v2(bad.tolist(), [2, F]),                       # > float32
                                  _v2([[float("nan")] + [0.5] * (F - 1)], [1, F])])  # NaN
        st = nat.server.front_end.stats()
        assert st["python_requests"] - mid["python_requests"] == 2
    finally:
        nat.stop()
        py.stop()


def test_lgbserver_large_inputs_body_native(golden, tmp_path):
    """An lgbserver {"inputs": ...} body of more than 1 MB also takes the
    native route (kf_parse_inputs on the IO thread), bytes equal to the
    asyncio server's."""
    from tests.test_lgb_batching import _lgb_model
    runs = []
    for native in (True, False):
        srv = KFServer(max_batchsize=1 << 16, max_latency_ms=3)
        srv.native_http = native
        (tmp_path / ("n" if native else "p")).mkdir()
        srv.register_model(_lgb_model(golden, tmp_path / ("n" if native else "p")))
        runs.append(_Running(srv))
    nat, py = runs
    _wait_front_end(nat)
    names = ["sepal_length_(cm)", "sepal_width_(cm)", "petal_length_(cm)", "petal_width_(cm)"]
    rng = np.random.default_rng(5)
    cols = {n: rng.uniform(0, 7, 45000).round(4).tolist() for n in names}
    body = json.dumps({"inputs": [cols]}).encode()
    assert len(body) > 1 << 20
    name = nat.server.front_end.app.models.get_models()[0].name
    path = f"/v1/models/{name}:predict"
    try:
        small = json.dumps({"inputs": [{n: [1.0] for n in names}]}).encode()
        assert nat.fetch(path, "POST", small)[0] == 200                 # the route
        before = nat.server.front_end.stats()
        a = nat.fetch(path, "POST", body)
        b = py.fetch(path, "POST", body)
        assert a[0] == b[0] == 200 and dict(a[1].items()) == dict(b[1].items())
        assert _norm(a[2]) == _norm(b[2])
        st = nat.server.front_end.stats()
        assert st["native_requests"] - before["native_requests"] == 1
        assert st["python_requests"] == before["python_requests"]
    finally:
        nat.stop()
        py.stop()
