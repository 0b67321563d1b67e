"""KFServer -- the v1/v2 model-server front end (mirror of
python/kfserving/kfserving/kfserver.py:30-196 and handlers/http.py:27-112).

Same CLI flags (--http_port 8080 --grpc_port 8081 --max_buffer_size
104857600 --workers 1), the same ten routes (kfserver.py:61-87), status codes
(404 unknown model, 503 not ready, 400 malformed body, 500 predict failure)
and response bytes: dict bodies are ``json.dumps`` with
``Content-Type: application/json; charset=UTF-8`` (test_server.py:151-157),
string bodies ``text/html; charset=UTF-8``, errors tornado's
``<html><title>CODE: REASON</title>...`` page with the reason in the status line.

tornado is not available here, so the transport is a small asyncio HTTP/1.1
server (keep-alive, Content-Length and chunked request bodies).  Like
``HTTPServer.start(workers)`` (kfserver.py:99) it binds first and then forks
``workers`` processes that share the listening socket; models are loaded
before the fork and their GPU state is created lazily in each worker.
A synchronous ``predict`` runs in a worker thread (the GPU call releases the
GIL) instead of blocking the event loop as the tornado handler does
(http.py:79); an optional in-process batcher (kfserving_amd.batcher) can be
put in front of ``:predict``.
"""
from __future__ import annotations

import argparse
import asyncio
import gc
import inspect
import json
import logging
import os
import re
import socket
import sys
from concurrent.futures import ThreadPoolExecutor
from http import HTTPStatus
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import cloudevent, fastjson, v2
from .errors import HTTPError
from .kfmodel import KFModel
from .kfmodel_repository import KFModelRepository

DEFAULT_HTTP_PORT = 8080
DEFAULT_GRPC_PORT = 8081
DEFAULT_MAX_BUFFER_SIZE = 104857600

parser = argparse.ArgumentParser(add_help=False)
parser.add_argument('--http_port', default=DEFAULT_HTTP_PORT, type=int,
                    help='The HTTP Port listened to by the model server.')
parser.add_argument('--grpc_port', default=DEFAULT_GRPC_PORT, type=int,
                    help='The GRPC Port listened to by the model server.')
parser.add_argument('--max_buffer_size', default=DEFAULT_MAX_BUFFER_SIZE, type=int,
                    help='The max buffer size for tornado.')
parser.add_argument('--workers', default=1, type=int,
                    help='The number of works to fork')
parser.add_argument('--max_batchsize', default=0, type=int,
                    help='Enable the in-process batcher with this many rows per batch (0 = off).')
parser.add_argument('--max_latency_ms', default=5000, type=int,
                    help='Batcher flush latency in milliseconds.')
parser.add_argument('--http_io_threads', default=4, type=int,
                    help='IO threads of the native HTTP front end per worker process.')
parser.add_argument('--no_fast_json', action='store_true',
                    help='Decode every body with json.loads (no native v1 parser).')
args, _ = parser.parse_known_args()

JSON_CT = "application/json; charset=UTF-8"
HTML_CT = "text/html; charset=UTF-8"

Response = Tuple[int, str, Dict[str, str], bytes]


def _json_body(obj) -> bytes:
    # tornado.escape.json_encode
    return json.dumps(obj).replace("</", "<\\/").encode("utf-8")


def _ok(body, content_type=None) -> Response:
    if isinstance(body, (dict, list)) and content_type is None:
        return 200, "OK", {"Content-Type": JSON_CT}, _json_body(body)
    if isinstance(body, str):
        return 200, "OK", {"Content-Type": content_type or HTML_CT}, body.encode("utf-8")
    return 200, "OK", {"Content-Type": content_type or HTML_CT}, bytes(body)


def tune_gc() -> None:
    """Move the loaded models / parsed forests to the permanent generation and
    make young-generation collections rarer: with thousands of in-flight
    request futures, default gen-2 pauses reached 300 ms at p99 (measured in
    bench.py's batched-latency leg at 10k requests/s; 8 ms with this).

    Also shorten the interpreter's GIL switch interval (5 ms by default) to
    0.5 ms: a predict thread returning from ti_predict (which drops the GIL)
    waits for the event loop's thread to hand the GIL back, up to one switch
    interval, and that wait sat in the tail of every batch's latency."""
    gc.collect()
    gc.freeze()
    gc.set_threshold(50_000, 50, 100)
    sys.setswitchinterval(min(sys.getswitchinterval(), 0.0005))


def gpu_count_without_init() -> int:
    """GPUs the KFD driver exposes, counted from sysfs (no HIP call: the
    workers fork after this and must initialise HIP themselves)."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "gpu_id")) as fh:
                    n += int(fh.read().strip() or 0) != 0
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if vis:
        n = min(n, len([v for v in vis.split(",") if v.strip()]))
    return n


def pin_worker_device(index: int, workers: int) -> None:
    """With several pre-forked workers and several GPUs, worker i drives GPU
    i mod n (its forest replica lives there) unless TREEINFER_DEVICES says
    otherwise; a single worker keeps every GPU and row-shards each batch."""
    if workers <= 1 or os.environ.get("TREEINFER_DEVICES"):
        return
    n = gpu_count_without_init()
    if n > 1:
        os.environ["TREEINFER_DEVICES"] = str(index % n)


def status_reason(reason: str) -> str:
    """The reason phrase as it may stand in a status line: CR / LF (which
    would split the response) become spaces; characters outside latin-1 are
    replaced when the line is encoded (_serialize).  The full text stays in the
    error page body (UTF-8)."""
    return reason.replace("\r", " ").replace("\n", " ")


def error_response(code: int, reason: str) -> Response:
    page = "<html><title>%d: %s</title><body>%d: %s</body></html>" % (code, reason, code, reason)
    return code, status_reason(reason), {"Content-Type": HTML_CT}, page.encode("utf-8")


class Application:
    """Route table + handlers, independent of the socket transport."""

    def __init__(self, models: KFModelRepository, executor: Optional[ThreadPoolExecutor] = None,
                 batcher_factory=None, fast_json: bool = True):
        self.models = models
        # native v1 body decode (libkfserve.so) for models that take the
        # decoded matrix (accepts_array_instances); loaded here so a missing
        # library fails at start-up, not on the first request
        self.fast_json = fast_json
        if fast_json:
            fastjson.load_library()
        self.executor = executor or ThreadPoolExecutor(max_workers=8)
        self._batchers = {}
        self._batcher_factory = batcher_factory
        self.batcher_listeners = []
        name = r"([a-zA-Z0-9_-]+)"
        self.routes = [
            (re.compile(r"^/$"), self.liveness),
            (re.compile(r"^/v2/health/live$"), self.liveness),
            (re.compile(r"^/v1/models$"), self.list_models),
            (re.compile(r"^/v2/models$"), self.list_models),
            (re.compile(rf"^/v1/models/{name}$"), self.health),
            (re.compile(rf"^/v2/models/{name}/status$"), self.health),
            (re.compile(rf"^/v1/models/{name}:predict$"), self.predict),
            (re.compile(rf"^/v2/models/{name}/infer$"), self.infer),
            (re.compile(rf"^/v1/models/{name}:explain$"), self.explain),
            (re.compile(rf"^/v2/models/{name}/explain$"), self.explain),
            (re.compile(rf"^/v2/repository/models/{name}/load$"), self.load),
            (re.compile(rf"^/v2/repository/models/{name}/unload$"), self.unload),
        ]
        self._methods = {self.liveness: "GET", self.list_models: "GET", self.health: "GET",
                         self.predict: "POST", self.infer: "POST", self.explain: "POST",
                         self.load: "POST", self.unload: "POST"}

    async def handle(self, method: str, path: str, headers: Dict[str, str], body: bytes) -> Response:
        path = path.split("?", 1)[0]
        for rx, fn in self.routes:
            m = rx.match(path)
            if m is None:
                continue
            if method != self._methods[fn]:
                return error_response(405, "Method Not Allowed")
            try:
                return await fn(headers, body, *m.groups())
            except HTTPError as e:
                return error_response(e.status_code, e.reason)
            except Exception as e:   # tornado: uncaught handler exception -> 500
                logging.exception("request failed: %s", e)
                return error_response(500, "Internal Server Error")
        return error_response(404, "Not Found")

    # ------------------------------------------------------------ handlers
    async def liveness(self, headers, body):
        return _ok("Alive")

    async def list_models(self, headers, body):
        return _ok(json.dumps([ob.name for ob in self.models.get_models()]))

    async def health(self, headers, body, name):
        model = self.models.get_model(name)
        if model is None:
            raise HTTPError(404, "Model with name %s does not exist." % name)
        if not model.ready:
            raise HTTPError(503, "Model with name %s is not ready." % name)
        return _ok(json.dumps({"name": model.name, "ready": model.ready}))

    def get_model(self, name: str):
        model = self.models.get_model(name)
        if model is None:
            raise HTTPError(HTTPStatus.NOT_FOUND, "Model with name %s does not exist." % name)
        if not model.ready:
            model.load()
        return model

    @staticmethod
    def validate(request):
        if isinstance(request, dict):
            inst = request.get("instances")
            if ("instances" in request and not isinstance(inst, list)
                    and not isinstance(inst, fastjson.JsonInstances)) or \
               ("inputs" in request and not isinstance(request["inputs"], list)):
                raise HTTPError(HTTPStatus.BAD_REQUEST,
                                "Expected \"instances\" or \"inputs\" to be a list")
        return request

    async def _call(self, fn, request):
        if inspect.iscoroutinefunction(fn):
            return await fn(request)
        return await asyncio.get_running_loop().run_in_executor(self.executor, fn, request)

    async def predict(self, headers, body, name):
        if cloudevent.has_binary_headers(headers):
            return await self._predict_binary_ce(headers, body, name)
        X = fastjson.parse_instances(body) if self.fast_json else None
        if X is None:
            try:
                request = json.loads(body)
            except (json.JSONDecodeError, UnicodeDecodeError) as e:
                raise HTTPError(HTTPStatus.BAD_REQUEST, "Unrecognized request format: %s" % e)
        model = self.get_model(name)
        if X is not None:
            # the decoded matrix goes only to models that take it and keep the
            # base preprocess (identity for this body shape); others get lists
            if getattr(model, "accepts_array_instances", False) and \
                    type(model).preprocess is KFModel.preprocess:
                request = {"instances": X}
            else:
                request = json.loads(body)
        request = model.preprocess(request)
        request = self.validate(request)
        return _ok(await self._predict_request(model, name, request))

    async def infer(self, headers, body, name):
        """``/v2/models/<name>/infer`` (ref kfserver.py:77-78 routes it to the
        v1 handler).  V2 tensor bodies -- JSON ``data`` or the binary
        tensor-data extension -- are decoded into a matrix and answered as a
        V2 inference response (kfserving.v2); any other body takes the v1
        path unchanged.  Malformed tensor requests get 400 with
        ``{"error": ...}`` (required_api.md:326-340)."""
        def bad(msg):
            return 400, "Bad Request", {"Content-Type": "application/json"}, v2.error_body(msg)
        try:
            head, tail = v2.split_body(headers, body)
        except v2.V2Error as e:
            return bad(str(e))
        # a tensor request names a datatype; v1 bodies skip the second decode
        req = v2.parse_header(head) if (tail or b'"datatype"' in head) else None
        if req is None:
            if tail:
                return bad("binary tensor data without a V2 inference request header")
            return await self.predict(headers, body, name)
        model = self.get_model(name)
        if not getattr(model, "accepts_array_instances", False):
            # a generic KFModel gets the request dict as the reference passes it
            return _ok(await self._predict_request(model, name, self.validate(req)))
        try:
            X = v2.feature_matrix(v2.decode_inputs(req, tail))
        except v2.V2Error as e:
            return bad(str(e))
        forest = getattr(model, "_forest", None)
        width = getattr(forest, "n_features", None)
        if self._batcher_factory is not None and width is not None and X.shape[1] == width:
            # one tensor batcher per model, for requests of the model's own
            # width; a request of another width (fewer columns read as missing,
            # as the libraries read them) is predicted alone, so a client's
            # widths can neither fail a batch of well-formed requests nor grow
            # the batcher table.  A model that does not state its width is not
            # batched: requests of different widths could share a batch
            batcher = self._batcher_for(model, name, "tensor")
            response = await batcher.submit(X)
            if response.get("predictions") is None:
                raise HTTPError(500, response.get("message") or "Failed to predict")
            result = np.asarray(response["predictions"])
        else:
            try:
                result = await self._call(model.predict_tensor, X)
            except Exception as e:
                raise HTTPError(500, "Failed to predict %s" % e)
        hdrs, payload = v2.encode_response(name, req, np.asarray(result))
        return 200, "OK", hdrs, payload

    def _batcher_for(self, model, name: str, kind: str):
        """One batcher per model and request kind, made on first use; a model
        object replaced under the same name (a reload) gets a new one.
        Listeners (the native HTTP front end) hear of every batcher made and
        retired: ``listener(event, name, kind, batcher)``."""
        key = (name, kind)
        batcher = self._batchers.get(key)
        if batcher is None or batcher.model is not model:
            if batcher is not None:
                self._retire(key, batcher)
            batcher = self._batcher_factory(model, self._call, kind)
            self._batchers[key] = batcher
            for fn in self.batcher_listeners:
                fn("create", name, kind, batcher)
        return batcher

    def _retire(self, key, batcher) -> None:
        for fn in self.batcher_listeners:   # before it stops: nothing may submit to it
            fn("retire", key[0], key[1], batcher)
        # a native batcher owns threads and an eventfd: it answers what it
        # holds, then stops (the asyncio batcher needs nothing)
        aclose = getattr(batcher, "aclose", None)
        if aclose is not None:
            asyncio.ensure_future(aclose())

    def retire_batchers(self, name: str) -> None:
        for key in [k for k in self._batchers if k[0] == name]:
            self._retire(key, self._batchers.pop(key))

    async def _predict_request(self, model, name, request):
        """predict -> postprocess, through the batcher when one is configured:
        ``instances`` as they are, lgbserver ``inputs`` as the float64 matrix
        their columns select (``batch_inputs``), one batcher per model and
        request kind."""
        if self._batcher_factory is not None and isinstance(request, dict):
            chunk, kind = None, None
            if "instances" in request:
                chunk, kind = request["instances"], "instances"
            elif "inputs" in request and hasattr(model, "batch_inputs"):
                try:
                    chunk, kind = model.batch_inputs(request), "inputs"
                except Exception as e:
                    raise HTTPError(500, "Failed to predict %s" % e)
            if kind is not None:
                batcher = self._batcher_for(model, name, kind)
                response = await batcher.submit(chunk)
                return model.postprocess(response)
        response = await self._call(model.predict, request)
        return model.postprocess(response)

    async def _predict_binary_ce(self, headers, body, name):
        """Binary-mode CloudEvent in, binary-mode CloudEvent out
        (handlers/http.py:55-66, 81-91)."""
        try:
            event = cloudevent.from_binary_http(headers, body)
        except cloudevent.CloudEventError as e:
            raise HTTPError(HTTPStatus.BAD_REQUEST, "Cloud Event Exceptions: %s" % e)
        model = self.get_model(name)
        request = self.validate(model.preprocess(event))
        response = await self._predict_request(model, name, request)
        hdrs, payload = cloudevent.to_binary_http(event, response)
        hdrs.setdefault("Content-Type", HTML_CT)    # tornado's default for written bytes
        return 200, "OK", hdrs, payload

    async def explain(self, headers, body, name):
        model = self.get_model(name)
        try:
            request = json.loads(body)
        except (json.JSONDecodeError, UnicodeDecodeError) as e:
            raise HTTPError(HTTPStatus.BAD_REQUEST, "Unrecognized request format: %s" % e)
        request = model.preprocess(request)
        request = self.validate(request)
        response = await self._call(model.explain, request)
        return _ok(model.postprocess(response))

    async def load(self, headers, body, name):
        try:
            fn = self.models.load
            if inspect.iscoroutinefunction(fn):
                await fn(name)
            else:
                fn(name)
        except Exception:
            ex_type, ex_value, _ = sys.exc_info()
            raise HTTPError(500, f"Model with name {name} is not ready. "
                                 f"Error type: {ex_type} error msg: {ex_value}")
        # the repository may hold a new model object now: its batchers (and
        # the native front end's route on them) are made afresh on the next request
        self.retire_batchers(name)
        if not self.models.is_model_ready(name):
            raise HTTPError(503, f"Model with name {name} is not ready.")
        return _ok(json.dumps({"name": name, "load": True}))

    async def unload(self, headers, body, name):
        try:
            self.models.unload(name)
            self.retire_batchers(name)
        except KeyError:
            raise HTTPError(404, "Model with name %s does not exist." % name)
        return _ok(json.dumps({"name": name, "unload": True}))


class _BodyTooLarge(Exception):
    pass


async def _read_request(reader: asyncio.StreamReader, max_body: int):
    line = await reader.readline()
    if not line:
        return None
    parts = line.decode("latin-1").rstrip("\r\n").split(" ")
    if len(parts) != 3:
        raise ValueError("bad request line")
    method, target, version = parts
    headers: Dict[str, str] = {}
    while True:
        h = await reader.readline()
        if h in (b"\r\n", b"\n", b""):
            break
        k, _, v = h.decode("latin-1").partition(":")
        headers[k.strip().lower()] = v.strip()
    if headers.get("transfer-encoding", "").lower() == "chunked":
        chunks = []
        total = 0
        while True:
            size = int((await reader.readline()).split(b";")[0].strip() or b"0", 16)
            if size == 0:
                await reader.readline()
                break
            total += size
            if total > max_body:
                raise _BodyTooLarge()
            chunks.append(await reader.readexactly(size))
            await reader.readline()
        body = b"".join(chunks)
    else:
        n = int(headers.get("content-length", "0") or 0)
        if n > max_body:
            raise _BodyTooLarge()
        body = await reader.readexactly(n) if n else b""
    return method, target, version, headers, body


def _serialize(resp: Response, keep_alive: bool) -> bytes:
    code, reason, hdrs, body = resp
    out = [f"HTTP/1.1 {code} {status_reason(reason)}\r\n"]
    hdrs = dict(hdrs)
    hdrs["Content-Length"] = str(len(body))
    hdrs.setdefault("Server", "kfserving-amd")
    if not keep_alive:
        hdrs["Connection"] = "close"
    for k, v in hdrs.items():
        out.append(f"{k}: {status_reason(str(v))}\r\n")
    out.append("\r\n")
    return "".join(out).encode("latin-1", errors="replace") + body


class KFServer:
    def __init__(self, http_port: int = args.http_port,
                 grpc_port: int = args.grpc_port,
                 max_buffer_size: int = args.max_buffer_size,
                 workers: int = args.workers,
                 registered_models: KFModelRepository = None,
                 max_batchsize: int = args.max_batchsize,
                 max_latency_ms: int = args.max_latency_ms,
                 fast_json: bool = not args.no_fast_json,
                 http_io_threads: int = args.http_io_threads):
        self.registered_models = registered_models if registered_models is not None \
            else KFModelRepository()
        self.http_port = http_port
        self.grpc_port = grpc_port
        self.max_buffer_size = max_buffer_size
        self.workers = workers
        self.max_batchsize = max_batchsize
        self.max_latency_ms = max_latency_ms
        self.fast_json = fast_json
        self.http_io_threads = max(1, int(http_io_threads))
        self.front_end = None
        self.native_http: Optional[bool] = None   # None: KF_NATIVE_HTTP (default on)
        self._server = None
        self._sock: Optional[socket.socket] = None

    def create_application(self) -> Application:
        factory = None
        if self.max_batchsize and self.max_batchsize > 0:
            from ..batcher.batcher import ModelBatcher
            from ..batcher.native import NativeModelBatcher, native_batching_enabled
            size, lat = self.max_batchsize, self.max_latency_ms

            def factory(model, call, kind="instances"):
                # the GPU tree plugins batch in native code (kfbatch.h); any
                # other KFModel keeps the asyncio batcher
                if native_batching_enabled(model):
                    return NativeModelBatcher(model, kind=kind, max_batch_size=size,
                                              max_latency_ms=lat)
                return ModelBatcher(model, call, kind=kind, max_batch_size=size,
                                    max_latency_ms=lat)
        return Application(self.registered_models, batcher_factory=factory,
                           fast_json=self.fast_json)

    def register_model(self, model) -> None:
        if not model.name:
            raise Exception("Failed to register model, model.name must be provided.")
        self.registered_models.update(model)
        logging.info("Registering model: %s", model.name)

    async def _serve_conn(self, app: Application, reader, writer):
        try:
            while True:
                try:
                    req = await _read_request(reader, self.max_buffer_size)
                except _BodyTooLarge:
                    writer.write(_serialize(error_response(413, "Request Entity Too Large"), False))
                    await writer.drain()
                    break
                except (ValueError, asyncio.IncompleteReadError):
                    writer.write(_serialize(error_response(400, "Bad Request"), False))
                    await writer.drain()
                    break
                if req is None:
                    break
                method, target, version, headers, body = req
                keep = headers.get("connection", "").lower() != "close" and version == "HTTP/1.1"
                resp = await app.handle(method, target, headers, body)
                writer.write(_serialize(resp, keep))
                await writer.drain()
                if not keep:
                    break
        except (ConnectionResetError, BrokenPipeError):
            pass
        finally:
            try:
                writer.close()
            except Exception:
                pass

    def bind(self, host: str = "0.0.0.0") -> socket.socket:
        sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        sock.bind((host, self.http_port))
        sock.listen(4096)
        sock.setblocking(False)
        self.http_port = sock.getsockname()[1]
        self._sock = sock
        return sock

    async def serve(self, sock: Optional[socket.socket] = None) -> None:
        """Serve on an already-bound socket until cancelled (used by tests).

        With batching on and a model the native HTTP front end can answer
        (kfserving.native_http: xgbserver models), the socket is served by
        native IO threads -- batched v1 :predict requests never enter the
        interpreter, every other request is handed to the same Application --
        unless KF_NATIVE_HTTP=0."""
        app = self.create_application()
        sock = sock or self._sock or self.bind()
        from . import native_http
        use = self.native_http if self.native_http is not None else native_http.native_http_enabled()
        if use and any(
                native_http.route_spec_static(app, m) for m in app.models.get_models()):
            fe = native_http.NativeFrontEnd(app, sock, io_threads=self.http_io_threads,
                                            max_body=self.max_buffer_size)
            fe.add_routes()
            if fe.routes:
                self.front_end = fe
                await fe.serve_forever()
                return
            fe.close()
        self._server = await asyncio.start_server(
            lambda r, w: self._serve_conn(app, r, w), sock=sock, limit=2 ** 20)
        async with self._server:
            await self._server.serve_forever()

    def start(self, models: List, nest_asyncio: bool = False) -> None:
        for model in models:
            self.register_model(model)
        sock = self.bind()
        tune_gc()
        logging.info("Listening on port %s", self.http_port)
        logging.info("Will fork %d workers", self.workers)
        index = 0
        for i in range(1, max(1, self.workers)):
            if os.fork() == 0:    # child: serve on the shared socket (GPU is lazily initialised)
                index = i
                break
        pin_worker_device(index, self.workers)
        asyncio.run(self.serve(sock))
