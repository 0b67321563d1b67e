"""BASELINE config C5 on one GPU: 4,096 concurrent HTTP
clients of 1-64-row v1 :predict requests against xgbserver with the C2 forest,
batcher maxBatchSize 65,536 rows / maxLatency 5 ms.

Two parts, one server:
  * correctness under concurrency: 256 requests of known rows in flight at
    once; every response equals the oracle's sigmoid(margin) of its own rows
    (1e-5 relative, north_star) -- rows are coalesced across requests and
    fanned back out, so a mis-sliced batch shows up here;
  * the load itself: scripts/loadgen (C, epoll, open-loop Poisson) over 4,096
    keep-alive connections for a short window; no request may be lost, fail
    or see a non-200, and latency stays bounded.

The 8-GPU C5 figure is the driver's to measure; this is the same path on
the one GPU a test box has (the server pins worker i to GPU i mod n)."""
import http.client
import json
import os
import resource
import signal
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

pytestmark = pytest.mark.gpu

PORT = 18431
CONNS = 4096


def _post(body):
    c = http.client.HTTPConnection("127.0.0.1", PORT, timeout=60)
    c.request("POST", "/v1/models/model:predict", body=body,
              headers={"Content-Type": "application/json"})
    r = c.getresponse()
    out = r.read()
    c.close()
    return r.status, out


def test_c5_concurrent_http_serving():
    import bench_serving as bs
    from oracle import xgb_ref
    if not os.path.exists(bs.LOADGEN):
        pytest.fail("kfserving_amd/lib/loadgen missing: run __graft_entry__.build()")
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if hard < 2 * CONNS + 256:
        pytest.skip(f"RLIMIT_NOFILE hard limit {hard} < {2 * CONNS + 256}")
    resource.setrlimit(resource.RLIMIT_NOFILE, (hard, hard))
    tmp = tempfile.mkdtemp()
    bs.write_c2_model(tmp)
    bodies = os.path.join(tmp, "bodies.bin")
    bs.write_bodies(bodies, 28, 4, seed=5)
    cmd = [sys.executable, "-m", "kfserving_amd.xgbserver", "--model_dir", tmp,
           "--model_name", "model", "--http_port", str(PORT), "--workers", "2",
           "--max_batchsize", "65536", "--max_latency_ms", "5"]
    log = open(os.path.join(tmp, "server.log"), "w")
    server = subprocess.Popen(cmd, cwd=ROOT, start_new_session=True, stdout=subprocess.DEVNULL,
                              stderr=log)
    try:
        assert bs.wait_ready(PORT), open(os.path.join(tmp, "server.log")).read()[-2000:]
        # ---- correctness: 256 concurrent requests of 1..64 known rows
        rng = np.random.default_rng(9)
        reqs = [rng.standard_normal((int(rng.integers(1, 65)), 28), dtype=np.float32)
                for _ in range(256)]
        with ThreadPoolExecutor(max_workers=64) as ex:
            res = list(ex.map(lambda X: _post(json.dumps({"instances": X.tolist()}).encode()),
                              reqs))
        # the JSON rows are float64 text of float32 values: the server's
        # DMatrix(list) path reads them back exactly (0 would be missing there;
        # standard normal rows hold no exact 0).  The checker reads the same
        # model file (0.82 legacy binary: base_score in margin space).
        m = xgb_ref.read_xgb_binary(os.path.join(tmp, "model.bst"))
        want = xgb_ref.predict(m, np.concatenate(reqs))
        lo = 0
        for X, (code, out) in zip(reqs, res):
            assert code == 200, out[:200]
            got = np.asarray(json.loads(out)["predictions"], dtype=np.float64)
            np.testing.assert_allclose(got, want[lo:lo + len(X)], rtol=1e-5)
            lo += len(X)
        # ---- the load: 4,096 connections, open-loop 5,000 req/s
        out = subprocess.run([bs.LOADGEN, "--port", str(PORT), "--conns", str(CONNS),
                              "--qps", "5000", "--duration", "3", "--warmup", "1",
                              "--bodies", bodies, "--path", "/v1/models/model:predict"],
                             capture_output=True, text=True, timeout=90)
        assert out.returncode == 0, out.stderr[-2000:]
        r = json.loads(out.stdout)
        print(json.dumps(r))
        assert r["conns"] == CONNS
        assert r["completed"] > 10000 and r["lost"] == 0
        assert r["non200"] == 0 and r["conn_errors"] == 0
        assert r["p50_ms"] >= 5.0 * 0.5          # requests do wait for their batch window
        # a request waits at most one window (5 ms) plus its batch's predict and
        # the HTTP/JSON round trip (measured p50 ~5.3, p99 6.6 ms on one idle
        # MI355X, profiles/r3f_c5_serving.txt).  The pass/fail gate leaves room
        # for host noise (the load generator shares the box): the median
        # within 1.6 windows and p99 within 5; the tight figures are reported
        # by bench.py's batched_latency and the serving profiles
        assert r["p50_ms"] <= 1.6 * 5.0, r
        assert r["p99_ms"] <= 5 * 5.0, r
    finally:
        try:
            os.killpg(server.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            server.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(server.pid, signal.SIGKILL)
        log.close()
