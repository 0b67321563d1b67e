"""ctypes binding of the native HTTP front end (include/kfhttp.h, in
libkfserve.so) and its bridge to the Python application.

The native IO threads read and parse every request on the server's socket.
Batched ``POST /v1/models/<name>:predict`` requests of the plugins that
declare a native route (``native_v1_transform``) are answered entirely in
native code through the model's native batcher; every other request is
handed to :class:`Application.handle` on this process's event loop, and the
bytes ``_serialize`` makes of its answer are written back by the IO thread
that owns the connection.  Responses are the same bytes the Python server
writes (status line, headers, JSON body), so this is a transport change, not
an API change (reference: python/kfserving/kfserving/kfserver.py:61-99,
handlers/http.py:53-95).
"""
from __future__ import annotations

import asyncio
import ctypes
import logging
import os
from typing import Dict, Optional

from . import fastjson
from .kfmodel import KFModel

KH_ABI_VERSION = 1

EXPORTED_SYMBOLS = ("kh_create", "kh_add_v1_predict", "kh_add_v1_inputs_predict",
                    "kh_add_v2_tensor_predict", "kh_remove_route", "kh_start",
                    "kh_fallback_fd", "kh_next_fallback", "kh_respond", "kh_get_stats",
                    "kh_destroy", "kh_repr_double", "kh_abi_version")


class KhConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("listen_fd", ctypes.c_int32),
                ("io_threads", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("max_body_bytes", ctypes.c_int64)]


class KhRequest(ctypes.Structure):
    _fields_ = [("id", ctypes.c_uint64), ("method", ctypes.c_void_p),
                ("target", ctypes.c_void_p), ("version", ctypes.c_void_p),
                ("headers", ctypes.c_void_p), ("headers_len", ctypes.c_int64),
                ("body", ctypes.c_void_p), ("body_len", ctypes.c_int64),
                ("keep_alive", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class KhStats(ctypes.Structure):
    _fields_ = [("connections", ctypes.c_int64), ("native_requests", ctypes.c_int64),
                ("python_requests", ctypes.c_int64), ("bad_requests", ctypes.c_int64)]


_bound = None


def load_library() -> ctypes.CDLL:
    global _bound
    lib = fastjson.load_library()
    if _bound is lib:
        return lib
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    lib.kh_abi_version.restype = i32
    lib.kh_abi_version.argtypes = []
    if lib.kh_abi_version() != KH_ABI_VERSION:
        raise RuntimeError(f"kfhttp ABI mismatch: library {lib.kh_abi_version()}, "
                           f"binding {KH_ABI_VERSION}")
    lib.kh_create.restype = ctypes.c_int
    lib.kh_create.argtypes = [ctypes.POINTER(KhConfig), ctypes.POINTER(vp)]
    lib.kh_add_v1_predict.restype = ctypes.c_int
    lib.kh_add_v1_predict.argtypes = [vp, ctypes.c_char_p, vp, i32, i32, i32, i32,
                                      ctypes.c_char_p, ctypes.POINTER(i32), i32]
    lib.kh_add_v1_inputs_predict.restype = ctypes.c_int
    lib.kh_add_v1_inputs_predict.argtypes = [vp, ctypes.c_char_p, vp, i32, i32, i32,
                                             ctypes.c_char_p, ctypes.POINTER(i32)]
    lib.kh_add_v2_tensor_predict.restype = ctypes.c_int
    lib.kh_add_v2_tensor_predict.argtypes = [vp, ctypes.c_char_p, vp, i32, i32, i32, i32]
    lib.kh_remove_route.restype = ctypes.c_int
    lib.kh_remove_route.argtypes = [vp, ctypes.c_char_p]
    lib.kh_start.restype = ctypes.c_int
    lib.kh_start.argtypes = [vp]
    lib.kh_fallback_fd.restype = ctypes.c_int
    lib.kh_fallback_fd.argtypes = [vp]
    lib.kh_next_fallback.restype = ctypes.c_int
    lib.kh_next_fallback.argtypes = [vp, ctypes.POINTER(KhRequest)]
    lib.kh_respond.restype = ctypes.c_int
    lib.kh_respond.argtypes = [vp, u64, ctypes.c_char_p, i64, i32]
    lib.kh_get_stats.restype = ctypes.c_int
    lib.kh_get_stats.argtypes = [vp, ctypes.POINTER(KhStats)]
    lib.kh_destroy.restype = ctypes.c_int
    lib.kh_destroy.argtypes = [vp]
    lib.kh_repr_double.restype = ctypes.c_int
    lib.kh_repr_double.argtypes = [ctypes.c_double, ctypes.c_char_p, i32]
    _bound = lib
    return lib


def repr_double(v: float) -> str:
    """kh_repr_double: the native formatter of prediction floats."""
    b = ctypes.create_string_buffer(64)
    n = load_library().kh_repr_double(v, b, len(b))
    return b.raw[:n].decode()


def native_http_enabled() -> bool:
    return os.environ.get("KF_NATIVE_HTTP", "1") != "0"


def route_spec(app, model, name: str):
    """(batcher, n_cols, out_width, out_elem_bytes, transform) when ``model``
    can be answered natively on ``/v1/models/<name>:predict``: the server
    batches (--max_batchsize) with the native batcher, decodes v1 bodies
    natively (not --no_fast_json), the plugin declares its element rule
    (``native_v1_transform``: xgbserver's DMatrix(list)), keeps the base
    preprocess / postprocess and is ready; else None."""
    from ..batcher.native import NativeModelBatcher
    transform = getattr(model, "native_v1_transform", None)
    if transform is None or app._batcher_factory is None or not app.fast_json:
        return None
    if not getattr(model, "ready", False) or not getattr(model, "accepts_array_instances", False):
        return None
    if type(model).preprocess is not KFModel.preprocess or \
            type(model).postprocess is not KFModel.postprocess:
        return None
    try:
        batcher = app._batcher_for(model, name, route_kind(model))
    except Exception as e:   # no device here: the application's path serves it
        logging.warning("no native route for %s: %s", name, e)
        return None
    return _spec_of(batcher, model)


def route_kind(model) -> str:
    """The batcher kind the route's requests take in the application:
    lgbserver's ``inputs`` bodies, everyone else's ``instances``."""
    return "inputs" if getattr(model, "native_v1_names", None) is not None else "instances"


def _blob(strings):
    offs = [0]
    for x in strings:
        offs.append(offs[-1] + len(x.encode()))
    return "".join(strings).encode(), (ctypes.c_int32 * len(offs))(*offs)


def _spec_of(batcher, model):
    from ..batcher.native import NativeModelBatcher
    from ..forest import OUT_PREDICT
    if not isinstance(batcher, NativeModelBatcher) or batcher._nb._h is None:
        return None
    f = model._forest
    import numpy as np
    labels = getattr(model, "native_v1_labels", None)
    names = getattr(model, "native_v1_names", None)
    return (batcher._nb._h, f.n_features, f.output_width(OUT_PREDICT),
            np.dtype(f.output_dtype(OUT_PREDICT)).itemsize, int(model.native_v1_transform),
            labels() if callable(labels) else None, names() if callable(names) else None)


class NativeFrontEnd:
    """The native HTTP server on ``sock`` in front of ``app``."""

    def __init__(self, app, sock, io_threads: int = 2, max_body: int = 104857600):
        self.app = app
        self._lib = load_library()
        self._sock = sock
        cfg = KhConfig(abi_version=KH_ABI_VERSION, listen_fd=sock.fileno(),
                       io_threads=int(io_threads), max_body_bytes=int(max_body))
        h = ctypes.c_void_p()
        rc = self._lib.kh_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"kh_create failed ({rc})")
        self._h = h
        self._fd = self._lib.kh_fallback_fd(h)
        self._req = KhRequest()
        self.routes: Dict[str, int] = {}
        app.batcher_listeners.append(self._on_batcher)

    def add_routes(self) -> None:
        for model in self.app.models.get_models():
            self._add(model, model.name)

    def _add(self, model, name: str) -> None:
        spec = route_spec(self.app, model, name)
        if spec is None:
            return
        self._register(name, spec)

    def _register(self, name, spec) -> None:
        h, F, w, e, tr, labels, names = spec
        if name in self.routes:
            self._remove_route(name)
        if names is not None:
            blob, offs = _blob(names)
            rc = self._lib.kh_add_v1_inputs_predict(self._h, name.encode(), h, F, w, e, blob, offs)
        else:
            blob, offs, n = None, None, 0
            if labels is not None:
                blob, offs = _blob(labels)
                n = len(labels)
            rc = self._lib.kh_add_v1_predict(self._h, name.encode(), h, F, w, e, tr, blob, offs, n)
        if rc == 0:
            self.routes[name] = h

    def _remove_route(self, key: str) -> None:
        rc = self._lib.kh_remove_route(self._h, key.encode())
        if rc == -2:   # requests still on the batcher after 20 s: it stays attached
            logging.warning("native route %s retired with requests still in flight; "
                            "their answers follow when the batcher drains", key)
        del self.routes[key]

    def _on_batcher(self, event: str, name: str, kind: str, batcher) -> None:
        if self._h is None:
            return
        if kind == "tensor":
            self._on_tensor_batcher(event, name, batcher)
            return
        if kind not in ("instances", "inputs"):
            return
        model = batcher.model
        if kind != route_kind(model):
            return
        if event == "retire" and name in self.routes:
            # detach before the batcher stops: kh_remove_route returns once the
            # requests already on it are answered
            self._remove_route(name)
        elif event == "create":
            if route_spec_static(self.app, model) and not self.routes.get(name):
                spec = _spec_of(batcher, model)
                if spec is not None:
                    self._register(name, spec)

    def _on_tensor_batcher(self, event: str, name: str, batcher) -> None:
        """V2 tensor requests (/v2/models/<name>/infer with "datatype") of a
        plugin that declares ``native_v2_transform`` (its tensor conversion
        as kb_submit_convert's plain cast plus KH_CHECK_* flags) go natively
        through the model's tensor batcher, which the application makes on
        the first such request (route key "v2:<name>")."""
        key = "v2:" + name
        if event == "retire" and key in self.routes:
            self._remove_route(key)
        elif event == "create" and key not in self.routes:
            model = batcher.model
            tr = getattr(model, "native_v2_transform", None)
            if tr is None or not route_spec_static(self.app, model):
                return
            spec = _spec_of(batcher, model)
            if spec is None:
                return
            h, F, w, e = spec[:4]
            if self._lib.kh_add_v2_tensor_predict(self._h, name.encode(), h, F, w, e,
                                                  int(tr)) == 0:
                self.routes[key] = h

    def stats(self) -> dict:
        st = KhStats()
        self._lib.kh_get_stats(self._h, ctypes.byref(st))
        return {k: getattr(st, k) for k, _ in KhStats._fields_}

    def _drain(self) -> None:
        try:
            os.read(self._fd, 8)
        except (BlockingIOError, InterruptedError):
            pass
        lib, h, r = self._lib, self._h, self._req
        while h is not None and lib.kh_next_fallback(h, ctypes.byref(r)) == 1:
            req = (r.id, ctypes.string_at(r.method).decode("latin-1"),
                   ctypes.string_at(r.target).decode("latin-1"),
                   ctypes.string_at(r.version).decode("latin-1"),
                   ctypes.string_at(r.headers, r.headers_len).decode("latin-1"),
                   ctypes.string_at(r.body, r.body_len) if r.body_len else b"",
                   bool(r.keep_alive))
            asyncio.ensure_future(self._answer(*req))

    async def _answer(self, rid, method, target, version, headers, body, keep) -> None:
        from .kfserver import _serialize, error_response
        hd = {}
        for line in headers.split("\n"):
            if line:
                k, _, v = line.partition(": ")
                hd[k] = v
        try:
            resp = await self.app.handle(method, target, hd, body)
        except Exception as e:   # handle() answers every handler error itself
            logging.exception("request failed: %s", e)
            resp = error_response(500, "Internal Server Error")
        data = _serialize(resp, keep)
        if self._h is not None:
            self._lib.kh_respond(self._h, rid, data, len(data), 0 if keep else 1)

    async def serve_forever(self) -> None:
        loop = asyncio.get_running_loop()
        loop.add_reader(self._fd, self._drain)
        self._lib.kh_start(self._h)
        try:
            await asyncio.Future()
        finally:
            try:
                loop.remove_reader(self._fd)
            except Exception:
                pass
            self.close()

    def close(self) -> None:
        if self._h is None:
            return
        try:
            self.app.batcher_listeners.remove(self._on_batcher)
        except ValueError:
            pass
        h, self._h = self._h, None
        self._lib.kh_destroy(h)   # joins the IO threads after the routes' requests
        self.routes.clear()


def route_spec_static(app, model) -> bool:
    """route_spec's conditions that do not need the batcher."""
    return (getattr(model, "native_v1_transform", None) is not None and app.fast_json and
            app._batcher_factory is not None and getattr(model, "ready", False) and
            getattr(model, "accepts_array_instances", False) and
            type(model).preprocess is KFModel.preprocess and
            type(model).postprocess is KFModel.postprocess)


__all__ = ["NativeFrontEnd", "native_http_enabled", "route_spec", "repr_double",
           "load_library", "EXPORTED_SYMBOLS", "KhConfig", "KhRequest", "KhStats"]
