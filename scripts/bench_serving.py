"""C5 serving benchmark: many concurrent HTTP clients of
1-64-row v1 :predict requests, open-loop at fixed aggregate QPS, through
KFServer's in-process batcher (maxBatchSize 65,536 rows, maxLatency 5 ms)
into the GPU engine.  Model: the C2 forest (500 depth-8 trees, 28 features,
XGBoost legacy binary, binary:logistic).

  python scripts/bench_serving.py [--qps 5000,10000,20000] [--conns 4096]
        [--workers 4] [--duration 10] [--model c2|dummy]

Starts `python -m kfserving_amd.xgbserver` as a child process (its own
process group, ended by PID), drives it with the C load generator
(kfserving_amd/lib/loadgen, built by __graft_entry__.build), prints one JSON
line per QPS point.  --model dummy serves a CPU echo model (no GPU) for
testing the harness itself.
"""
import argparse
import http.client
import json
import os
import resource
import signal
import struct
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LOADGEN = os.path.join(ROOT, "kfserving_amd", "lib", "loadgen")

DUMMY_SERVER = r'''
import sys
sys.path.insert(0, %(root)r)
from kfserving_amd.kfserving import KFModel, KFServer, KFModelRepository
class Echo(KFModel):
    accepts_array_instances = True
    def __init__(self):
        super().__init__("model"); self.ready = True
    def predict(self, request):
        return {"predictions": [0.5] * len(request["instances"])}
KFServer(http_port=%(port)d, workers=%(workers)d, max_batchsize=%(mbs)d,
         max_latency_ms=%(lat)d, registered_models=KFModelRepository()).start([Echo()])
'''


def body_of(X, protocol="v1"):
    """A request of rows X: v1 {"instances": rows}, or a V2 inference request
    with one FP32 tensor of JSON data (docs/predict-api/v2/required_api.md)."""
    if protocol == "v2":
        return json.dumps({"inputs": [{"name": "input-0", "shape": list(X.shape),
                                       "datatype": "FP32",
                                       "data": X.reshape(-1).tolist()}]}).encode()
    if protocol == "v2bin":   # u32 head length, JSON head, raw little-endian FP32 rows
        raw = np.ascontiguousarray(X, dtype="<f4").tobytes()
        head = json.dumps({"inputs": [{"name": "input-0", "shape": list(X.shape),
                                       "datatype": "FP32",
                                       "parameters": {"binary_data_size": len(raw)}}]}).encode()
        return struct.pack("<I", len(head)) + head + raw
    return json.dumps({"instances": X.tolist()}).encode()


def predict_path(protocol="v1", model="model"):
    return f"/v2/models/{model}/infer" if protocol != "v1" else f"/v1/models/{model}:predict"


def write_bodies(path, n_feat, variants, seed, protocol="v1"):
    rng = np.random.default_rng(seed)
    with open(path, "wb") as fh:
        fh.write(struct.pack("<I", variants))
        for r in range(1, 65):
            for _ in range(variants):
                X = rng.standard_normal((r, n_feat), dtype=np.float32)
                b = body_of(X, protocol)
                fh.write(struct.pack("<I", len(b)))
                fh.write(b)


def write_c2_model(d):
    from kfserving_amd.formats.xgboost_format import (synthetic_complete_trees,
                                                      write_legacy_binary)
    trees, ti = synthetic_complete_trees(500, 8, 28, seed=0)
    write_legacy_binary(os.path.join(d, "model.bst"), trees, ti, 28, 0, 0.5,
                        "binary:logistic")


def wait_ready(port, timeout=180):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=2)
            c.request("GET", "/v1/models/model")
            r = c.getresponse()
            r.read()
            c.close()
            if r.status == 200:
                return True
        except OSError:
            pass
        time.sleep(0.5)
    return False


def warm(port, n_feat, n=20, protocol="v1"):
    body = body_of(np.zeros((64, n_feat), dtype=np.float32), protocol)
    hdrs = {"Content-Type": "application/json"}
    if protocol == "v2bin":
        head = struct.unpack("<I", body[:4])[0]
        body = body[4:]
        hdrs = {"Content-Type": "application/octet-stream",
                "Inference-Header-Content-Length": str(head)}
    for _ in range(n):
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
        c.request("POST", predict_path(protocol), body=body, headers=hdrs)
        r = c.getresponse()
        r.read()
        c.close()
        if r.status != 200:
            raise RuntimeError(f"warm-up predict returned {r.status}")


def point_passes(res, p99_bound_ms):
    """A capacity-search point holds when its p99 is within the bound and no
    request was lost, failed or answered non-200."""
    return (res.get("p99_ms") is not None and res["p99_ms"] <= p99_bound_ms
            and not res.get("lost") and not res.get("non200") and not res.get("conn_errors"))


def capacity_search(measure, done, p99_bound_ms, points, grow=1.5, resolution=1.1):
    """The highest offered rate whose point passes (`point_passes`), searched
    after the fixed points `done` [(qps, result)]: from the best passing rate,
    grow by `grow` until a point fails, then bisect (geometric midpoint)
    between the best pass and the lowest fail until they are within
    `resolution` or `points` more runs are spent.  `measure(qps)` runs one
    point.  Returns {capacity_req_per_s, first_fail_req_per_s, searched}."""
    ok = [q for q, r in done if point_passes(r, p99_bound_ms)]
    bad = [q for q, r in done if not point_passes(r, p99_bound_ms)]
    lo = max(ok) if ok else None
    hi = min([q for q in bad if lo is None or q > lo], default=None)
    searched = []
    for _ in range(max(0, points)):
        if lo is None:                       # even the lowest fixed point failed
            if hi is None:
                break
            q = hi / 2.0
        elif hi is None:
            q = lo * grow
        else:
            if hi / lo <= resolution:
                break
            q = (lo * hi) ** 0.5
        q = float(round(q, -2)) if q >= 1000 else float(round(q))
        try:
            r = measure(q)
        except Exception as e:              # a point the load generator could not finish
            r = {"error": str(e)[-300:]}
        passed = point_passes(r, p99_bound_ms)
        searched.append({"offered_qps": q, "p99_ms": r.get("p99_ms"), "lost": r.get("lost"),
                         "non200": r.get("non200"), "req_per_s": r.get("req_per_s"),
                         "passed": passed, **({"error": r["error"]} if "error" in r else {})})
        if passed:
            lo = q if lo is None else max(lo, q)
        else:
            hi = q if hi is None else min(hi, q)
    return {"capacity_req_per_s": lo, "first_fail_req_per_s": hi,
            "criterion": f"p99 <= {p99_bound_ms:g} ms (2 x maxLatency), 0 lost, 0 non-200",
            "searched": searched}


def serve_and_measure(qps_list, workers=4, io_threads=2, duration=8.0, warmup=2.0, conns=4096,
                      port=18080, model="c2", max_batch=65536, max_latency_ms=5, env=None,
                      ready_timeout=180, loadgen_threads=1, echo=True, protocol="v1",
                      capacity_points=0, capacity_out=None):
    """Start the server, drive it with the C load generator at each offered
    rate in turn, stop it; one result dict per rate.  With capacity_points > 0
    the same server then runs `capacity_search` (p99 <= 2 x maxLatency, no
    loss) for up to that many more points and fills `capacity_out`."""
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    resource.setrlimit(resource.RLIMIT_NOFILE, (hard, hard))
    n_feat = 28
    tmp = tempfile.mkdtemp()
    bodies = os.path.join(tmp, "bodies.bin")
    write_bodies(bodies, n_feat, 8, seed=3, protocol=protocol)
    env = dict(os.environ if env is None else env)
    if model == "c2":
        write_c2_model(tmp)
        cmd = [sys.executable, "-m", "kfserving_amd.xgbserver", "--model_dir", tmp,
               "--model_name", "model", "--http_port", str(port),
               "--workers", str(workers), "--max_batchsize", str(max_batch),
               "--max_latency_ms", str(max_latency_ms), "--http_io_threads", str(io_threads)]
    else:
        code = DUMMY_SERVER % {"root": ROOT, "port": port, "workers": workers,
                               "mbs": max_batch, "lat": max_latency_ms}
        cmd = [sys.executable, "-c", code]
    server = subprocess.Popen(cmd, cwd=ROOT, env=env, start_new_session=True,
                              stdout=subprocess.DEVNULL, stderr=open(os.path.join(tmp, "server.log"), "w"))
    results = []
    try:
        if not wait_ready(port, ready_timeout):
            raise RuntimeError("server did not become ready: " +
                               open(os.path.join(tmp, "server.log")).read()[-2000:])
        warm(port, n_feat, protocol=protocol)

        def measure(q):
            out = subprocess.run([LOADGEN, "--port", str(port), "--conns", str(conns),
                                  "--qps", str(q), "--duration", str(duration),
                                  "--warmup", str(warmup), "--bodies", bodies,
                                  "--threads", str(loadgen_threads),
                                  "--path", predict_path(protocol),
                                  "--v2-binary", "1" if protocol == "v2bin" else "0"],
                                 capture_output=True, text=True,
                                 timeout=duration + warmup + 60)   # loadgen drains by +30 s
            if out.returncode != 0:
                raise RuntimeError(f"loadgen failed: {out.stderr[-2000:]}")
            res = json.loads(out.stdout)
            res.update({"config": {"v2": "C5 dynamic batching: V2 /infer FP32 JSON tensors",
                                   "v2bin": "C5 dynamic batching: V2 /infer FP32 binary tensors"}
                        .get(protocol, "C5 dynamic batching: v1 :predict") +
                                  " over HTTP, KFServer in-process batcher", "model": model,
                        "protocol": protocol,
                        "workers": workers, "max_batch_size": max_batch,
                        "max_latency_ms": max_latency_ms,
                        "native_http": env.get("KF_NATIVE_HTTP", "1") != "0",
                        "native_batcher": env.get("KF_NATIVE_BATCHER", "1") != "0",
                        "io_threads": io_threads, "loadgen_threads": loadgen_threads,
                        "gpus_visible": env.get("TREEINFER_DEVICES", "all")})
            if echo:   # bench.py's leg prints nothing of its own (one JSON line)
                print(json.dumps(res), flush=True)
            return res

        for q in qps_list:
            results.append(measure(q))
        if capacity_points > 0:
            cap = capacity_search(measure, list(zip(qps_list, results)), 2.0 * max_latency_ms,
                                  capacity_points)
            if capacity_out is not None:
                capacity_out.update(cap)
            if echo:
                print(json.dumps({"capacity": cap}), flush=True)
    finally:
        try:
            os.killpg(server.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            server.wait(timeout=20)
        except subprocess.TimeoutExpired:
            os.killpg(server.pid, signal.SIGKILL)
    return results


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--qps", default="5000,10000,20000")
    p.add_argument("--conns", type=int, default=4096)
    p.add_argument("--workers", type=int, default=4)
    p.add_argument("--duration", type=float, default=8.0)
    p.add_argument("--warmup", type=float, default=2.0)
    p.add_argument("--port", type=int, default=18080)
    p.add_argument("--model", default="c2", choices=["c2", "dummy"])
    p.add_argument("--max-batch", type=int, default=65536)
    p.add_argument("--max-latency-ms", type=int, default=5)
    p.add_argument("--loadgen-threads", type=int, default=1,
                   help="load generator threads (each its own epoll loop and share of the "
                        "connections and rate)")
    p.add_argument("--io-threads", type=int, default=2,
                   help="native HTTP front end IO threads per worker (KF_NATIVE_HTTP=0: "
                        "the asyncio server)")
    p.add_argument("--protocol", default="v1", choices=["v1", "v2", "v2bin"],
                   help="v1 :predict instances, V2 /infer FP32 JSON tensors, or V2 binary tensors")
    p.add_argument("--capacity-points", type=int, default=0,
                   help="after the fixed points, search this many more for the highest rate "
                        "with p99 <= 2 x maxLatency and no loss")
    args = p.parse_args()
    serve_and_measure([float(x) for x in args.qps.split(",")], args.workers, args.io_threads,
                      args.duration, args.warmup, args.conns, args.port, args.model,
                      args.max_batch, args.max_latency_ms, loadgen_threads=args.loadgen_threads,
                      protocol=args.protocol, capacity_points=args.capacity_points)


if __name__ == "__main__":
    main()
