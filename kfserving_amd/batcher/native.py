"""ctypes binding of the native request batcher (include/kfbatch.h, in
libkfserve.so) and its asyncio front.

The batcher itself -- pkg/batcher's rows-counted flush, the MaxLatency
deadline from the first request, fan-out by index and one batchId per batch
(pkg/batcher/handler.go:98-263) -- runs in C++ threads and calls the model
through a function pointer with ti_predict's signature, so a batch goes from
the requests' rows to libtreeinfer without the interpreter.  Python converts
each request the way its plugin converts a request (``native_rows``), submits
the matrix, and gets the request's rows of the output back through an eventfd
that the event loop watches.

:class:`NativeModelBatcher` is the drop-in for :class:`ModelBatcher` in front
of the GPU tree plugins (``KFServer --max_batchsize``): same ``submit`` and
the same response dict (``message``, ``batchId``, ``predictions``).
"""
from __future__ import annotations

import asyncio
import ctypes
import itertools
import os
import threading
from typing import Any, Callable, Dict, Optional

import numpy as np

from ..forest import OUT_PREDICT, TI_F32, TI_F64, TI_I32
from ..kfserving import fastjson
from ..kfserving.errors import HTTPError

KB_ABI_VERSION = 1
KB_OK, KB_ERR_INVALID, KB_ERR_CLOSED, KB_ERR_SYSTEM, KB_ERR_MODEL = 0, -1, -2, -3, -4
KB_IN_PLAIN, KB_IN_XGB_LIST = 0, 1   # kb_submit_convert transforms

EXPORTED_SYMBOLS = ("kb_create", "kb_destroy", "kb_flush", "kb_notify_fd", "kb_submit",
                    "kb_submit_convert", "kb_set_done_callback", "kb_poll",
                    "kb_batch_message", "kb_get_stats", "kb_now_ns", "kb_loadgen",
                    "kb_abi_version")


class KbConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("x_dtype", ctypes.c_int32),
                ("n_cols", ctypes.c_int32), ("output_kind", ctypes.c_int32),
                ("out_width", ctypes.c_int32), ("out_elem_bytes", ctypes.c_int32),
                ("max_batch_rows", ctypes.c_int64), ("max_latency_us", ctypes.c_int64),
                ("max_inflight", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class KbCompletion(ctypes.Structure):
    _fields_ = [("tag", ctypes.c_uint64), ("status", ctypes.c_int32),
                ("batch_rows", ctypes.c_int32), ("t_done_ns", ctypes.c_int64),
                ("batch_seq", ctypes.c_uint64), ("batch_id", ctypes.c_char * 40)]


class KbStats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_int64), ("rows", ctypes.c_int64),
                ("max_batch_rows", ctypes.c_int64), ("full_flushes", ctypes.c_int64),
                ("timer_flushes", ctypes.c_int64), ("failed_batches", ctypes.c_int64),
                ("model_ms_total", ctypes.c_double)]


# the model call: ti_predict's signature (include/treeinfer.h)
PREDICT_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                              ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                              ctypes.c_void_p, ctypes.c_int64)
ERROR_FN = ctypes.CFUNCTYPE(ctypes.c_void_p)   # returns a const char*

_bound = None


def load_library() -> ctypes.CDLL:
    """libkfserve.so (the v1 body parser's library) with the kb_* prototypes."""
    global _bound
    lib = fastjson.load_library()
    if _bound is lib:
        return lib
    vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
    lib.kb_abi_version.restype = i32
    lib.kb_abi_version.argtypes = []
    if lib.kb_abi_version() != KB_ABI_VERSION:
        raise RuntimeError(f"kfbatch ABI mismatch: library {lib.kb_abi_version()}, "
                           f"binding {KB_ABI_VERSION}")
    lib.kb_create.restype = ctypes.c_int
    lib.kb_create.argtypes = [ctypes.POINTER(KbConfig), vp, vp, vp, ctypes.POINTER(vp)]
    lib.kb_destroy.restype = ctypes.c_int
    lib.kb_destroy.argtypes = [vp]
    lib.kb_flush.restype = ctypes.c_int
    lib.kb_flush.argtypes = [vp]
    lib.kb_notify_fd.restype = ctypes.c_int
    lib.kb_notify_fd.argtypes = [vp]
    lib.kb_submit.restype = ctypes.c_int
    lib.kb_submit.argtypes = [vp, vp, i64, i64, vp, u64]
    lib.kb_submit_convert.restype = ctypes.c_int
    lib.kb_submit_convert.argtypes = [vp, vp, i32, i64, i64, i32, vp, u64]
    lib.kb_set_done_callback.restype = ctypes.c_int
    lib.kb_set_done_callback.argtypes = [vp, vp, vp]
    lib.kb_poll.restype = ctypes.c_int
    lib.kb_poll.argtypes = [vp, ctypes.POINTER(KbCompletion), i32]
    lib.kb_batch_message.restype = ctypes.c_int
    lib.kb_batch_message.argtypes = [vp, u64, ctypes.c_char_p, i32]
    lib.kb_get_stats.restype = ctypes.c_int
    lib.kb_get_stats.argtypes = [vp, ctypes.POINTER(KbStats)]
    lib.kb_now_ns.restype = i64
    lib.kb_now_ns.argtypes = []
    lib.kb_loadgen.restype = ctypes.c_int
    lib.kb_loadgen.argtypes = [vp, vp, vp, i64, vp, i64, vp, vp, vp, ctypes.POINTER(i64)]
    _bound = lib
    return lib


_NP_OF = {TI_F32: np.float32, TI_F64: np.float64, TI_I32: np.int32}


class BatchError(Exception):
    """The model call of the request's batch failed (the batch's message)."""


class NativeBatcher:
    """One kb_* batcher: requests of `n_cols` columns in, `out_width` output
    elements per row back.

    ``predict`` is either a C function pointer with ti_predict's signature
    (``model`` its first argument, ``error`` its ti_last_error) or a Python
    callable ``predict(X, out) -> int`` (tests: any model, no GPU)."""

    def __init__(self, predict, n_cols: int, x_dtype: int, out_width: int, out_dtype: int,
                 max_batch_size: int, max_latency_ms: float, kind: int = OUT_PREDICT,
                 max_inflight: int = 2, model: Optional[int] = None, error: Optional[int] = None,
                 keepalive: Any = None):
        self._lib = load_library()
        self.n_cols, self.x_dtype, self.kind = int(n_cols), int(x_dtype), int(kind)
        self.out_width = int(out_width)
        # out_dtype: a TI_* code or a numpy type (Forest.output_dtype)
        self._o_np = _NP_OF[out_dtype] if isinstance(out_dtype, int) else np.dtype(out_dtype).type
        self._x_np = _NP_OF[self.x_dtype]
        self.max_batch_size, self.max_latency_ms = max_batch_size, max_latency_ms
        self._keep = keepalive
        if callable(predict):
            x_np, o_np, w = self._x_np, self._o_np, self.out_width

            def trampoline(_model, xp, _xdt, rows, cols, stride, _kind, op, out_len):
                try:
                    X = np.ctypeslib.as_array(ctypes.cast(xp, ctypes.POINTER(
                        np.ctypeslib.as_ctypes_type(x_np))), shape=(rows, stride))[:, :cols]
                    out = np.ctypeslib.as_array(ctypes.cast(op, ctypes.POINTER(
                        np.ctypeslib.as_ctypes_type(o_np))), shape=(out_len,))
                    return int(predict(X, out.reshape(rows, w) if w > 1 else out))
                except Exception as e:   # a raising model is a failed call
                    # by OS thread: a foreign thread's callback state (and any
                    # threading.local) does not outlive one callback
                    errs[threading.get_ident()] = ctypes.create_string_buffer(
                        str(e).encode("utf-8", "replace"))
                    return -1

            def last_error():   # called on the model thread right after the call
                buf = errs.get(threading.get_ident())
                return ctypes.addressof(buf) if buf is not None else None
            errs: Dict[int, Any] = {}
            self._errs = errs
            self._cb = PREDICT_FN(trampoline)
            self._ecb = ERROR_FN(last_error)
            fn_ptr, model = ctypes.cast(self._cb, ctypes.c_void_p).value, None
            error = ctypes.cast(self._ecb, ctypes.c_void_p).value
        else:
            fn_ptr = int(predict)
        cfg = KbConfig(abi_version=KB_ABI_VERSION, x_dtype=self.x_dtype, n_cols=self.n_cols,
                       output_kind=self.kind, out_width=self.out_width,
                       out_elem_bytes=np.dtype(self._o_np).itemsize,
                       max_batch_rows=int(max_batch_size),
                       max_latency_us=int(round(max_latency_ms * 1000)),
                       max_inflight=int(max_inflight))
        h = ctypes.c_void_p()
        rc = self._lib.kb_create(ctypes.byref(cfg), fn_ptr, model, error, ctypes.byref(h))
        if rc != KB_OK:
            raise RuntimeError(f"kb_create failed ({rc})")
        self._h = h
        self._fd = self._lib.kb_notify_fd(h)
        self._tags = itertools.count(1)
        self._pending: Dict[int, tuple] = {}
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._buf = (KbCompletion * 256)()

    @classmethod
    def for_device_forest(cls, dev, max_batch_size: int, max_latency_ms: float,
                          kind: int = OUT_PREDICT, max_inflight: int = 2) -> "NativeBatcher":
        """A batcher whose model call is libtreeinfer's ti_predict on `dev`."""
        f = dev.forest
        lib = dev._lib
        return cls(ctypes.cast(lib.ti_predict, ctypes.c_void_p).value, f.n_features,
                   f.input_dtype, f.output_width(kind), f.output_dtype(kind), max_batch_size,
                   max_latency_ms, kind=kind, max_inflight=max_inflight,
                   model=dev._handle.value,
                   error=ctypes.cast(lib.ti_last_error, ctypes.c_void_p).value, keepalive=dev)

    # ----------------------------------------------------------------- submit
    def _attach(self, loop: asyncio.AbstractEventLoop) -> None:
        if self._loop is loop:
            return
        if self._loop is not None:
            raise RuntimeError("a NativeBatcher serves one event loop")
        loop.add_reader(self._fd, self._drain)
        self._loop = loop

    def submit_nowait(self, X: np.ndarray, transform: int = KB_IN_PLAIN) -> "asyncio.Future":
        """Queue the rows of X; the future resolves to ``(out, batch_id)`` or
        raises :class:`BatchError`.  float32 / float64 rows are converted to
        the batcher's input type while they are copied (kb_submit_convert),
        after ``transform`` (KB_IN_XGB_LIST: xgboost's DMatrix(list) rule)."""
        if self._h is None:
            raise RuntimeError("batcher is closed")
        loop = asyncio.get_running_loop()
        self._attach(loop)
        X = np.asarray(X)
        # rows at a non-negative whole-element stride past their columns go as
        # they are (kb_submit_convert reads the stride); anything else is copied
        if X.dtype not in (np.float32, np.float64) or X.ndim != 2 or X.strides[1] != X.itemsize \
                or X.strides[0] % X.itemsize or X.strides[0] < X.shape[1] * X.itemsize:
            X = np.ascontiguousarray(X, dtype=self._x_np)
        if X.ndim != 2 or X.shape[0] == 0:
            raise HTTPError(400, "no instances in the request")
        if X.shape[1] != self.n_cols:
            raise ValueError(f"expected {self.n_cols} columns, got {X.shape[1]}")
        rows = X.shape[0]
        out = np.empty((rows, self.out_width) if self.out_width > 1 else rows, dtype=self._o_np)
        tag = next(self._tags)
        fut = loop.create_future()
        self._pending[tag] = (fut, out)
        rc = self._lib.kb_submit_convert(self._h, X.ctypes.data, 0 if X.dtype == np.float32 else 1,
                                         rows, X.strides[0] // X.itemsize, int(transform),
                                         out.ctypes.data, tag)
        if rc != KB_OK:
            del self._pending[tag]
            raise RuntimeError(f"kb_submit failed ({rc})")
        return fut

    async def submit(self, X: np.ndarray, transform: int = KB_IN_PLAIN):
        return await self.submit_nowait(X, transform)

    def _drain(self) -> None:
        try:
            os.read(self._fd, 8)
        except (BlockingIOError, InterruptedError):
            pass
        lib, h, buf = self._lib, self._h, self._buf
        while True:
            n = lib.kb_poll(h, buf, len(buf))
            if n <= 0:
                break
            for i in range(n):
                c = buf[i]
                fut, out = self._pending.pop(c.tag, (None, None))
                if fut is None or fut.done():
                    continue
                if c.status == KB_OK:
                    fut.set_result((out, c.batch_id.decode()))
                else:
                    fut.set_exception(BatchError(self.message(c.batch_seq)))

    def flush(self) -> None:
        """Send the forming batch to the model now (kb_flush)."""
        if self._h is not None:
            self._lib.kb_flush(self._h)

    async def drain(self) -> None:
        """Flush, then wait until every submitted request is answered."""
        self.flush()
        futs = [f for f, _ in self._pending.values()]
        if futs:
            await asyncio.gather(*futs, return_exceptions=True)

    def message(self, seq: int) -> str:
        b = ctypes.create_string_buffer(4096)
        n = self._lib.kb_batch_message(self._h, seq, b, len(b))
        return b.value.decode("utf-8", "replace") if n >= 0 else "model call failed"

    def stats(self) -> dict:
        s = KbStats()
        self._lib.kb_get_stats(self._h, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in KbStats._fields_}

    # ------------------------------------------------------------ measurement
    def loadgen(self, arrival_s: np.ndarray, rows: np.ndarray, pool: np.ndarray):
        """kb_loadgen: open-loop arrivals submitted from a native thread at
        their scheduled times; returns (latency_ms, status, out, t0_ns)."""
        n = len(arrival_s)
        arr = np.ascontiguousarray(arrival_s, dtype=np.float64)
        rws = np.ascontiguousarray(rows, dtype=np.int32)
        pool = np.ascontiguousarray(pool, dtype=self._x_np)
        out = np.zeros(n * 64 * self.out_width, dtype=self._o_np)
        lat = np.zeros(n, dtype=np.float64)
        st = np.zeros(n, dtype=np.int32)
        t0 = ctypes.c_int64()
        rc = self._lib.kb_loadgen(self._h, arr.ctypes.data, rws.ctypes.data, n, pool.ctypes.data,
                                  pool.shape[0], out.ctypes.data, lat.ctypes.data, st.ctypes.data,
                                  ctypes.byref(t0))
        if rc != KB_OK:
            raise RuntimeError(f"kb_loadgen failed ({rc})")
        return lat, st, out, int(t0.value)

    def close(self) -> None:
        if getattr(self, "_h", None) is None:
            return
        if self._loop is not None and not self._loop.is_closed():
            try:
                self._loop.remove_reader(self._fd)
            except Exception:
                pass
        self._lib.kb_destroy(self._h)   # in-flight batches finish first
        self._h = None
        for fut, _ in self._pending.values():
            if not fut.done():
                fut.set_exception(RuntimeError("batcher closed"))
        self._pending.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def now_ns() -> int:
    return int(load_library().kb_now_ns())


class NativeModelBatcher:
    """ModelBatcher's contract (``submit(chunk) -> {"message", "batchId",
    "predictions"}``) over a :class:`NativeBatcher` in front of a GPU tree
    plugin.  Each request is converted by the plugin (``native_rows``: the
    same conversion its ``predict`` applies) and its rows of the batch's
    output are turned into its predictions (``native_predictions``); a
    request the conversion rejects fails alone with the plugin's message."""

    def __init__(self, model, kind: str = "instances", max_batch_size: int = 32,
                 max_latency_ms: float = 5000, max_inflight: int = 2):
        self.model = model
        self.kind = kind
        self.max_batch_size, self.max_latency_ms = max_batch_size, max_latency_ms
        from ..tree_model import GPUForestMixin
        if "predict_matrix" not in vars(model) and \
                getattr(type(model), "predict_matrix", None) is GPUForestMixin.predict_matrix:
            # the plugin predicts on the GPU: batches go straight to ti_predict
            self._nb = NativeBatcher.for_device_forest(model.device_forest(), max_batch_size,
                                                       max_latency_ms, max_inflight=max_inflight)
        else:
            # the plugin's predict_matrix was replaced (the CPU tests' stand-in
            # model): the same native batching, with that function as the call
            f = model._forest

            def call(X, out):
                out[...] = np.asarray(model.predict_matrix(X, OUT_PREDICT)).reshape(out.shape)
                return 0
            self._nb = NativeBatcher(call, f.n_features, f.input_dtype,
                                     f.output_width(OUT_PREDICT), f.output_dtype(OUT_PREDICT),
                                     max_batch_size, max_latency_ms, max_inflight=max_inflight)

    async def submit(self, chunk) -> Dict[str, Any]:
        try:
            X, transform = self.model.native_request(chunk, self.kind)
        except HTTPError:
            raise
        except Exception as e:
            return {"message": "Failed to predict %s" % e, "batchId": "", "predictions": None}
        if X.shape[0] == 0:
            raise HTTPError(400, "no instances in the request")
        try:
            out, batch_id = await self._nb.submit(X, transform)
        except BatchError as e:
            return {"message": "Failed to predict %s" % e, "batchId": "", "predictions": None}
        return {"message": "", "batchId": batch_id,
                "predictions": self.model.native_predictions(out, self.kind)}

    def stats(self) -> dict:
        return self._nb.stats()

    def close(self) -> None:
        self._nb.close()

    async def aclose(self) -> None:
        """Answer every request already submitted, then stop the threads."""
        await self._nb.drain()
        self._nb.close()


def native_batching_enabled(model) -> bool:
    """The native batcher fronts models that declare it (the GPU tree
    plugins); KF_NATIVE_BATCHER=0 keeps the asyncio batcher for every model."""
    return os.environ.get("KF_NATIVE_BATCHER", "1") != "0" and \
        bool(getattr(model, "native_batching", False))


__all__ = ["NativeBatcher", "NativeModelBatcher", "BatchError", "load_library", "now_ns",
           "KB_IN_PLAIN", "KB_IN_XGB_LIST",
           "native_batching_enabled", "EXPORTED_SYMBOLS", "PREDICT_FN", "ERROR_FN"]
