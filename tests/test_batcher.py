"""Batcher semantics (pkg/batcher/handler.go), CPU only.

The reference's own test (pkg/batcher/handler_test.go:50-88) fires 10
concurrent 1-row requests through New(32, 50, proxy) and only checks that
they all complete; the e2e test (test/e2e/batcher/test_batcher.py:71-78)
checks concurrent requests share one batchId.  These tests pin those and the
flush / fan-out / error rules stated in kfserving_amd/batcher/batcher.py.
"""
import asyncio
import json
import threading
import time

import pytest

from kfserving_amd.batcher import Batcher
from kfserving_amd.batcher.batcher import SIZE_MISMATCH
from kfserving_amd.kfserving import HTTPError


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def echo_batcher(**kw):
    calls = []

    async def predict(instances):
        calls.append(list(instances))
        return {"predictions": instances}
    return Batcher(predict, **kw), calls


def test_ten_concurrent_requests_complete():          # handler_test.go:50-88
    async def main():
        b, calls = echo_batcher(max_batch_size=32, max_latency_ms=50)
        res = await asyncio.gather(*[b.submit([[i, i, i]]) for i in range(10)])
        return res, calls
    res, calls = run(main())
    assert len(calls) == 1 and len(calls[0]) == 10
    assert len({r["batchId"] for r in res}) == 1           # test_batcher.py:71-78
    assert [r["predictions"] for r in res] == [[[i, i, i]] for i in range(10)]


def test_flush_on_rows_counts_rows_not_requests():
    async def main():
        b, calls = echo_batcher(max_batch_size=4, max_latency_ms=10_000)
        t0 = time.monotonic()
        res = await asyncio.gather(b.submit([[1], [2], [3]]), b.submit([[4], [5]]))
        return res, calls, time.monotonic() - t0
    res, calls, dt = run(main())
    assert dt < 1.0                                   # size flush, not latency
    assert calls == [[[1], [2], [3], [4], [5]]]       # overshoot: whole requests appended
    assert res[0]["predictions"] == [[1], [2], [3]] and res[1]["predictions"] == [[4], [5]]


def test_flush_on_latency():
    async def main():
        b, calls = echo_batcher(max_batch_size=1000, max_latency_ms=30)
        t0 = time.monotonic()
        r = await b.submit([[7]])
        return r, time.monotonic() - t0
    r, dt = run(main())
    assert r["predictions"] == [[7]] and 0.025 <= dt < 1.0


def test_empty_instances_rejected():
    b, _ = echo_batcher()
    with pytest.raises(HTTPError) as e:
        run(b.submit([]))
    assert e.value.status_code == 400


def test_error_fanout_and_size_mismatch():
    async def failing(instances):
        raise RuntimeError("model exploded")

    async def short(instances):
        return {"predictions": instances[:-1]}

    async def main():
        b1 = Batcher(failing, max_batch_size=2, max_latency_ms=1000)
        r1 = await asyncio.gather(b1.submit([[1]]), b1.submit([[2]]))
        b2 = Batcher(short, max_batch_size=2, max_latency_ms=1000)
        r2 = await asyncio.gather(b2.submit([[1]]), b2.submit([[2]]))
        return r1, r2
    r1, r2 = run(main())
    assert all(r == {"message": "model exploded", "batchId": "", "predictions": None} for r in r1)
    assert all(r["message"] == SIZE_MISMATCH and r["batchId"] and r["predictions"] is None
               for r in r2)


def test_pipelined_batches_overlap():
    """Batch n+1 forms while batch n is still on the model (no HOL blocking)."""
    async def main(pipeline):
        started = []

        async def slow(instances):
            started.append(time.monotonic())
            await asyncio.sleep(0.2)
            return {"predictions": instances}
        b = Batcher(slow, max_batch_size=2, max_latency_ms=1000, pipeline=pipeline)
        t0 = time.monotonic()
        await asyncio.gather(*[b.submit([[i]]) for i in range(4)])
        return time.monotonic() - t0
    assert run(main(True)) < 0.35
    assert run(main(False)) >= 0.39


def test_agent_proxy_end_to_end():
    """Agent (cmd/agent + pkg/batcher) in front of a KFServer model server."""
    from tests.test_server import SyncModel, _Running
    from kfserving_amd.batcher.agent import Agent
    from kfserving_amd.kfserving import KFModelRepository, KFServer

    server = KFServer(registered_models=KFModelRepository())
    server.register_model(SyncModel("m"))
    backend = _Running(server)
    agent = Agent("127.0.0.1", backend.port, True, max_batch_size=4, max_latency_ms=50)

    class _AgentServer:
        def __init__(self):
            import socket
            self.sock = socket.socket()
            self.sock.bind(("127.0.0.1", 0))
            self.port = self.sock.getsockname()[1]
            self.sock.close()
            self.loop = asyncio.new_event_loop()
            self.t = threading.Thread(target=lambda: self.loop.run_until_complete(
                agent.serve(self.port)), daemon=True)
            self.t.start()
            time.sleep(0.3)

    a = _AgentServer()
    import http.client
    out = []

    def one(i):
        c = http.client.HTTPConnection("127.0.0.1", a.port, timeout=30)
        c.request("POST", "/v1/models/m:predict", body=json.dumps({"instances": [[i]]}))
        r = c.getresponse()
        out.append((r.status, json.loads(r.read())))
    th = [threading.Thread(target=one, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(s == 200 for s, _ in out)
    assert len({b["batchId"] for _, b in out}) == 1
    assert sorted(b["predictions"][0][0] for _, b in out) == [0, 2, 4, 6]
    c = http.client.HTTPConnection("127.0.0.1", a.port, timeout=30)
    c.request("GET", "/v1/models/m")
    r = c.getresponse()
    r.read()
    assert r.status == 200                               # non-predict paths proxied
    # instances that do not unmarshal into []interface{}: 400 (handler.go:234-241),
    # and the connection stays usable
    for bad in (b'{"instances": {"a": 1}}', b'{"instances": "x"}', b'{"instances": 3}'):
        c.request("POST", "/v1/models/m:predict", body=bad)
        r = c.getresponse()
        assert r.status == 400 and b"can't Unmarshal body" in r.read()
    c.request("POST", "/v1/models/m:predict", body=b'{"instances": []}')
    r = c.getresponse()
    assert r.status == 400 and b"no instances in the request" in r.read()
    backend.stop()


def test_bench_batched_latency_leg_on_cpu():
    """bench.py's C5-style leg with a CPU stand-in for the device forest."""
    import numpy as np
    import bench

    class FakeDev:
        def predict(self, X):
            return X.sum(axis=1)

    r = bench.batched_latency(FakeDev(), 28, qps=2000, seconds=0.5, max_latency_ms=5)
    assert r["requests"] == 1000 and r["batches"] >= 1
    assert 1.0 <= r["p50_ms"] < 100 and r["p99_ms"] >= r["p50_ms"]
    assert r["mean_batch_rows"] > 32


def test_matrix_chunks_concatenate_and_fan_out():
    import numpy as np
    from kfserving_amd.kfserving.fastjson import JsonInstances
    seen = []

    async def predict_batch(instances):
        seen.append(instances)
        X = np.asarray(instances, dtype=np.float64)
        return {"predictions": X.sum(axis=1).tolist()}

    async def go():
        b = Batcher(predict_batch, max_batch_size=6, max_latency_ms=1000)
        m1 = np.array([[1.0, 2.0], [3.0, 4.0]]).view(JsonInstances)
        m2 = np.array([[5.0, 6.0]]).view(JsonInstances)
        m3 = np.array([[7.0, 8.0], [9.0, 10.0], [11.0, 12.0]]).view(JsonInstances)
        r = await asyncio.gather(b.submit(m1), b.submit(m2), b.submit(m3))
        mixed = await asyncio.gather(b.submit([[1, 1]]), b.submit(m2), b.submit([[2, 2]] * 4))
        return r, mixed
    r, mixed = run(go())
    assert isinstance(seen[0], JsonInstances) and seen[0].shape == (6, 2)
    assert [x["predictions"] for x in r] == [[3.0, 7.0], [11.0], [15.0, 19.0, 23.0]]
    assert len({x["batchId"] for x in r}) == 1
    assert isinstance(seen[1], list) and len(seen[1]) == 6          # mixed -> rows list
    assert [x["predictions"] for x in mixed] == [[2.0], [11.0], [4.0] * 4]
    with pytest.raises(Exception):
        run(Batcher(predict_batch).submit(np.zeros((0, 3))))


def test_enqueue_futures_resolve_like_submit():
    """Batcher.enqueue (submit without the coroutine, bench.py's load): the
    futures resolve with the same per-request slices and one batchId, and an
    empty request raises at once."""
    import numpy as np

    async def main():
        b, calls = echo_batcher(max_batch_size=7, max_latency_ms=50)
        got = {}
        futs = []
        for i, n in enumerate([3, 2, 2]):
            f = b.enqueue(np.full((n, 2), float(i), dtype=np.float32))
            f.add_done_callback(lambda fut, i=i: got.__setitem__(i, fut.result()))
            futs.append(f)
        await asyncio.gather(*futs)
        with pytest.raises(HTTPError):
            b.enqueue(np.zeros((0, 2), dtype=np.float32))
        return got, calls
    got, calls = run(main())
    assert len(calls) == 1 and len(calls[0]) == 7            # one batch of 7 rows
    assert len({r["batchId"] for r in got.values()}) == 1
    for i, n in enumerate([3, 2, 2]):
        assert np.asarray(got[i]["predictions"]).shape == (n, 2)
        assert np.all(np.asarray(got[i]["predictions"]) == float(i))
