"""Request coalescing with pkg/batcher semantics (pkg/batcher/handler.go:98-263).

Kept from the Go batcher:
* a batch is flushed when its *row* count reaches max_batch_size (whole
  requests are appended first, so a batch may overshoot, handler.go:165-180)
  or when max_latency_ms have elapsed since its first request arrived
  (``Now.Sub(Start).Milliseconds() >= MaxLatency``, handler.go:179-182);
* every request gets back only its own rows, by index, and one ``batchId``
  (UUIDv4) shared by the batch (handler.go:118, 138-149);
* failures fan out to every waiter as ``message`` with ``predictions`` null:
  the model's error text (batchId ""), or "size of prediction is not equal to
  the size of instances" (batchId set) (handler.go:107-136);
* empty ``instances`` is rejected with 400 "no instances in the request"
  (handler.go:238-241).

Deliberately different: the Go loop runs
``batchPredict`` synchronously, so no request is accepted while a batch is
on the model (head-of-line blocking).  Here a flushed batch runs as its own
task and the next batch keeps forming (``pipeline=True``; at most
``max_inflight`` batches on the model).  ``pipeline=False`` restores the
blocking behaviour.  Timers replace the 100 us polling loop.
"""
from __future__ import annotations

import asyncio
import time
import uuid
from typing import Any, Awaitable, Callable, Dict, List, Optional, Tuple

import numpy as np

from ..kfserving.errors import HTTPError
from ..kfserving.fastjson import JsonInstances

MAX_BATCH_SIZE = 32       # handler.go:34
MAX_LATENCY_MS = 5000     # handler.go:35

SIZE_MISMATCH = "size of prediction is not equal to the size of instances"

PredictBatch = Callable[[List[Any]], Awaitable[Dict[str, Any]]]


class Batcher:
    def __init__(self, predict_batch: PredictBatch, max_batch_size: int = MAX_BATCH_SIZE,
                 max_latency_ms: int = MAX_LATENCY_MS, pipeline: bool = True,
                 max_inflight: int = 2):
        # Consume(): non-positive settings fall back to the defaults (handler.go:187-195)
        self.max_batch_size = max_batch_size if max_batch_size > 0 else MAX_BATCH_SIZE
        self.max_latency_ms = max_latency_ms if max_latency_ms > 0 else MAX_LATENCY_MS
        self.predict_batch = predict_batch
        self.pipeline = pipeline
        self._sem = asyncio.Semaphore(max_inflight if pipeline else 1)
        self._instances: List[Any] = []   # one chunk (list or matrix) per request
        self._rows = 0
        self._waiters: List[Tuple[asyncio.Future, int, int]] = []
        self._start = 0.0
        self._timer: Optional[asyncio.TimerHandle] = None
        self._tasks = set()
        self.stats = {"batches": 0, "rows": 0, "max_batch_rows": 0}

    async def submit(self, instances: List[Any]) -> Dict[str, Any]:
        """Queue one request's rows: a list, or a 2-D matrix decoded natively
        from the body (kfserving.fastjson.JsonInstances)."""
        return await self.enqueue(instances)

    def enqueue(self, instances: List[Any]) -> "asyncio.Future":
        """submit() without the coroutine: queue the rows and return the future
        their response resolves (for callers that attach a callback instead of
        awaiting, such as bench.py's open-loop load)."""
        if isinstance(instances, np.ndarray):
            if instances.ndim != 2 or instances.shape[0] == 0:
                raise HTTPError(400, "no instances in the request")
        elif not isinstance(instances, list) or len(instances) == 0:
            raise HTTPError(400, "no instances in the request")
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        if not self._instances:
            self._start = time.monotonic()
        lo = self._rows
        self._instances.append(instances)
        self._rows += len(instances)
        self._waiters.append((fut, lo, self._rows))
        if self._rows >= self.max_batch_size:
            self._flush()
        elif self._timer is None:
            delay = self.max_latency_ms / 1000.0 - (time.monotonic() - self._start)
            self._timer = loop.call_later(max(delay, 0.0), self._flush)
        return fut

    def _flush(self) -> None:
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        if not self._instances:
            return
        batch, waiters = _combine(self._instances), self._waiters
        self._instances, self._waiters, self._rows = [], [], 0
        self.stats["batches"] += 1
        self.stats["rows"] += len(batch)
        self.stats["max_batch_rows"] = max(self.stats["max_batch_rows"], len(batch))
        task = asyncio.ensure_future(self._run(batch, waiters))
        self._tasks.add(task)
        task.add_done_callback(self._tasks.discard)

    async def _run(self, batch: List[Any], waiters) -> None:
        async with self._sem:
            try:
                response = await self.predict_batch(batch)
            except Exception as e:   # non-200 from the model: body fanned out as message
                msg = getattr(e, "reason", None) or str(e)
                for fut, _, _ in waiters:
                    if not fut.done():
                        fut.set_result({"message": msg, "batchId": "", "predictions": None})
                return
        batch_id = str(uuid.uuid4())
        preds = response.get("predictions") if isinstance(response, dict) else None
        if preds is None or not hasattr(preds, "__len__") or len(preds) != len(batch):
            for fut, _, _ in waiters:
                if not fut.done():
                    fut.set_result({"message": SIZE_MISMATCH, "batchId": batch_id,
                                    "predictions": None})
            return
        for fut, lo, hi in waiters:
            if not fut.done():
                fut.set_result({"message": "", "batchId": batch_id, "predictions": preds[lo:hi]})

    async def drain(self) -> None:
        self._flush()
        while self._tasks:
            await asyncio.gather(*list(self._tasks))


def _combine(chunks: List[Any]):
    """One batch from the queued requests: matrices of equal width are
    concatenated (keeping the JsonInstances marker when every chunk has it);
    anything else becomes one list of rows, as the Go batcher appends them."""
    if all(isinstance(c, np.ndarray) for c in chunks) and \
            len({c.shape[1] for c in chunks}) == 1:
        out = np.concatenate(chunks, axis=0) if len(chunks) > 1 else chunks[0]
        if all(isinstance(c, JsonInstances) for c in chunks):
            return out.view(JsonInstances)
        return np.asarray(out)
    rows: List[Any] = []
    for c in chunks:
        rows.extend(c.tolist() if isinstance(c, np.ndarray) else c)
    return rows


class ModelBatcher(Batcher):
    """In-process batcher in front of a KFModel's ``predict`` (KFServer
    --max_batchsize): coalesced instances go straight to the model, with no
    second HTTP hop and no second JSON round trip.

    ``kind="inputs"`` batches lgbserver requests, which the Go batcher rejects
    with 400 because it only reads ``instances`` (§8(f1) asks
    for this): each request's ``inputs`` are first turned into the float64
    matrix its columns select by feature name (``model.batch_inputs``, the
    same conversion ``predict`` does), the batch is their row concatenation,
    and ``model.predict_batched`` predicts it."""

    def __init__(self, model, call, kind: str = "instances", **kw):
        self.model = model
        self.kind = kind

        if kind == "inputs":
            async def predict_batch(X):
                return await call(model.predict_batched, X)
        elif kind == "tensor":   # V2 tensors (kfserving.v2): matrices, numpy semantics
            async def predict_batch(X):
                return await call(model.predict_tensor_batched, X)
        else:
            async def predict_batch(instances):
                return await call(model.predict, {"instances": instances})

        super().__init__(predict_batch, **kw)
