"""Agent-mode batcher: an HTTP front end that coalesces ``:predict`` requests
and forwards each batch to the model server, the role of the Go sidecar
(cmd/agent/main.go:206-223 startBatcher, :289-323 buildServer) with
pkg/batcher in its handler chain.  Other paths are proxied unchanged.

  python -m kfserving_amd.batcher --port 9081 --component-port 8080 \\
      --enable-batcher --max-batchsize 32 --max-latency 5000

Flag names follow cmd/agent/main.go:47-50 ("--enable-batcher" is a plain
switch here; the Go flag-parsing quirk of SURVEY.md 3.3 is not reproduced).
"""
from __future__ import annotations

import argparse
import asyncio
import http.client
import json
import logging
import re
from concurrent.futures import ThreadPoolExecutor

from ..kfserving.errors import HTTPError
from ..kfserving.kfserver import JSON_CT, _BodyTooLarge, _read_request, _serialize, error_response
from .batcher import MAX_BATCH_SIZE, MAX_LATENCY_MS, Batcher

_PREDICT = re.compile(r":predict$")


class Agent:
    def __init__(self, component_host: str = "127.0.0.1", component_port: int = 8080,
                 enable_batcher: bool = True, max_batch_size: int = MAX_BATCH_SIZE,
                 max_latency_ms: int = MAX_LATENCY_MS, pipeline: bool = True):
        self.host = component_host
        self.port = component_port
        self.enable_batcher = enable_batcher
        self.max_batch_size = max_batch_size
        self.max_latency_ms = max_latency_ms
        self.pipeline = pipeline
        self.pool = ThreadPoolExecutor(max_workers=16)
        self._batchers = {}

    def _forward_sync(self, method, path, headers, body):
        conn = http.client.HTTPConnection(self.host, self.port, timeout=600)
        try:
            hdrs = {k: v for k, v in headers.items()
                    if k not in ("host", "content-length", "connection", "transfer-encoding")}
            conn.request(method, path, body=body, headers=hdrs)
            r = conn.getresponse()
            return r.status, r.reason, {"Content-Type": r.getheader("Content-Type", JSON_CT)}, \
                r.read()
        finally:
            conn.close()

    async def forward(self, method, path, headers, body):
        return await asyncio.get_running_loop().run_in_executor(
            self.pool, self._forward_sync, method, path, headers, body)

    def _batcher(self, path: str) -> Batcher:
        b = self._batchers.get(path)
        if b is None:
            async def predict_batch(instances, path=path):
                code, reason, _, payload = await self.forward(
                    "POST", path, {"content-type": "application/json"},
                    json.dumps({"instances": instances}).encode())
                if code != 200:
                    raise RuntimeError(payload.decode("utf-8", "replace"))
                return json.loads(payload)
            b = Batcher(predict_batch, self.max_batch_size, self.max_latency_ms, self.pipeline)
            self._batchers[path] = b
        return b

    async def handle(self, method, path, headers, body):
        if not (self.enable_batcher and method == "POST" and _PREDICT.search(path.split("?")[0])):
            return await self.forward(method, path, headers, body)
        try:
            req = json.loads(body)
        except (json.JSONDecodeError, UnicodeDecodeError):
            return error_response(400, "can't Unmarshal body")
        instances = req.get("instances") if isinstance(req, dict) else None
        if instances is not None and not isinstance(instances, list):
            # a body that does not unmarshal into Request{Instances []interface{}}
            # (handler.go:234-241)
            return error_response(400, "can't Unmarshal body")
        if not instances:
            return error_response(400, "no instances in the request")
        # the Go batcher keys one loop per handler; the last request's path wins
        # for a mixed batch (handler.go:164) -- here each path gets its own loop
        res = await self._batcher(path.split("?")[0]).submit(instances)
        return 200, "OK", {"Content-Type": "application/json"}, \
            json.dumps(res, separators=(",", ":")).encode()

    async def _conn(self, reader, writer):
        try:
            while True:
                try:
                    req = await _read_request(reader, 1 << 30)
                except _BodyTooLarge:
                    writer.write(_serialize(error_response(413, "Request Entity Too Large"), False))
                    await writer.drain()
                    break
                if req is None:
                    break
                method, target, version, headers, body = req
                try:
                    resp = await self.handle(method, target, headers, body)
                except HTTPError as e:
                    resp = error_response(e.status_code, e.reason)
                keep = headers.get("connection", "").lower() != "close"
                writer.write(_serialize(resp, keep))
                await writer.drain()
                if not keep:
                    break
        except (ConnectionResetError, BrokenPipeError, asyncio.IncompleteReadError, ValueError):
            pass
        finally:
            writer.close()

    async def serve(self, port: int):
        server = await asyncio.start_server(self._conn, "0.0.0.0", port, limit=2 ** 20)
        async with server:
            await server.serve_forever()


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--port", type=int, default=9081)
    p.add_argument("--component-port", type=int, default=8080)
    p.add_argument("--enable-batcher", action="store_true")
    p.add_argument("--max-batchsize", type=int, default=MAX_BATCH_SIZE)
    p.add_argument("--max-latency", type=int, default=MAX_LATENCY_MS)
    p.add_argument("--no-pipeline", action="store_true")
    a = p.parse_args(argv)
    if a.max_batchsize <= 0 or a.max_latency <= 0:   # startBatcher validation (main.go:206-223)
        raise SystemExit("max-batchsize and max-latency must be > 0")
    logging.basicConfig(level=logging.INFO)
    agent = Agent("127.0.0.1", a.component_port, a.enable_batcher, a.max_batchsize,
                  a.max_latency, pipeline=not a.no_pipeline)
    asyncio.run(agent.serve(a.port))


if __name__ == "__main__":
    main()
