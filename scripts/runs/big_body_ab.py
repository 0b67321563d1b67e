"""Latency of large v1 :predict requests (one client, keep-alive, one at a
time) against xgbserver with the C2 model, with the native HTTP front end and
with the asyncio server (KF_NATIVE_HTTP=0), on the same bodies.

  python scripts/big_body_ab.py [--rows 4096,65536] [--repeats 10]

One JSON line per (server, rows): median / min request time and rows/s."""
import argparse
import http.client
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import bench_serving as bs  # noqa: E402


def run_server(native: bool, port: int, tmp: str, rows_list, repeats: int):
    env = dict(os.environ, KF_NATIVE_HTTP="1" if native else "0")
    cmd = [sys.executable, "-m", "kfserving_amd.xgbserver", "--model_dir", tmp,
           "--model_name", "model", "--http_port", str(port), "--workers", "1",
           "--max_batchsize", "65536", "--max_latency_ms", "5", "--http_io_threads", "4"]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    log_path = os.path.join(ROOT, "gpurun_out", f"big_body_server_{int(native)}_{port}.log")
    log = open(log_path, "w")
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, start_new_session=True,
                           stdout=subprocess.DEVNULL, stderr=log)
    out = []
    try:
        if not bs.wait_ready(port, 120):
            raise RuntimeError("server not ready")
        bs.warm(port, 28)
        rng = np.random.default_rng(7)
        for rows in rows_list:
            X = rng.standard_normal((rows, 28)).astype(np.float32)
            body = json.dumps({"instances": X.tolist()}).encode()
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
            ts = []
            first = None
            for i in range(repeats + 2):
                t0 = time.perf_counter()
                c.request("POST", "/v1/models/model:predict", body=body,
                          headers={"Content-Type": "application/json"})
                r = c.getresponse()
                data = r.read()
                dt = time.perf_counter() - t0
                if r.status != 200:
                    raise RuntimeError(f"status {r.status}: {data[:200]!r}")
                if first is None:
                    first = json.loads(data)["predictions"]
                if i >= 2:
                    ts.append(dt)
            c.close()
            med = float(np.median(ts))
            out.append({"server": "native front end" if native else "asyncio",
                        "rows": rows, "body_MB": len(body) / 1e6, "median_ms": med * 1e3,
                        "min_ms": min(ts) * 1e3, "rows_per_s": rows / med,
                        "checksum": float(np.sum(np.asarray(first, dtype=np.float64)))})
    except Exception:
        print(f"[{'native' if native else 'asyncio'}] server exit code {srv.poll()}, log "
              f"{log_path}", file=sys.stderr, flush=True)
        raise
    finally:
        if srv.poll() is None:
            os.killpg(srv.pid, 15)
        srv.wait(timeout=30)
    return out


def concurrent(native: bool, port: int, tmp: str, rows: int, clients: int, seconds: float,
               native_workers: int = 1):
    """`clients` keep-alive connections, each sending `rows`-row requests back
    to back for `seconds`: whole-server rows/s and request latency."""
    import threading
    env = dict(os.environ, KF_NATIVE_HTTP="1" if native else "0")
    cmd = [sys.executable, "-m", "kfserving_amd.xgbserver", "--model_dir", tmp,
           "--model_name", "model", "--http_port", str(port),
           "--workers", str(native_workers) if native else "8",
           "--max_batchsize", "65536", "--max_latency_ms", "5",
           "--http_io_threads", str(max(2, 16 // native_workers))]
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, start_new_session=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        if not bs.wait_ready(port, 120):
            raise RuntimeError("server not ready")
        bs.warm(port, 28)
        X = np.random.default_rng(3).standard_normal((rows, 28)).astype(np.float32)
        body = json.dumps({"instances": X.tolist()}).encode()
        lat, stop = [], time.perf_counter() + seconds
        lock = threading.Lock()

        def client():
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
            mine = []
            while time.perf_counter() < stop:
                t0 = time.perf_counter()
                c.request("POST", "/v1/models/model:predict", body=body,
                          headers={"Content-Type": "application/json"})
                r = c.getresponse()
                r.read()
                if r.status != 200:
                    raise RuntimeError(f"status {r.status}")
                mine.append(time.perf_counter() - t0)
            c.close()
            with lock:
                lat.extend(mine)
        t0 = time.perf_counter()
        th = [threading.Thread(target=client) for _ in range(clients)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        lat_ms = np.asarray(lat) * 1e3
        return {"server": f"native front end ({native_workers} workers)" if native
                else "asyncio (8 workers)",
                "rows": rows, "clients": clients, "requests": len(lat),
                "rows_per_s": len(lat) * rows / wall, "p50_ms": float(np.percentile(lat_ms, 50)),
                "p99_ms": float(np.percentile(lat_ms, 99))}
    finally:
        os.killpg(srv.pid, 15)
        srv.wait(timeout=30)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="4096,65536")
    p.add_argument("--repeats", type=int, default=10)
    p.add_argument("--port", type=int, default=18300)
    p.add_argument("--clients", type=int, default=0,
                   help="> 0: that many concurrent clients of --rows rows each (one size)")
    p.add_argument("--seconds", type=float, default=8.0)
    p.add_argument("--native-workers", type=int, default=1)
    a = p.parse_args()
    if a.clients > 0:
        tmp = tempfile.mkdtemp()
        bs.write_c2_model(tmp)
        for rep in range(2):
            for native in (True, False):
                r = concurrent(native, a.port + 2 * rep + int(native), tmp, int(a.rows),
                               a.clients, a.seconds, a.native_workers)
                r["round"] = rep
                print(json.dumps(r), flush=True)
        return
    rows_list = [int(r) for r in a.rows.split(",")]
    tmp = tempfile.mkdtemp()
    bs.write_c2_model(tmp)
    res = {}
    for rep in range(2):
        for native in (True, False):
            for r in run_server(native, a.port + 2 * rep + int(native), tmp, rows_list, a.repeats):
                r["round"] = rep
                print(json.dumps(r), flush=True)
                res.setdefault(r["rows"], set()).add(round(r["checksum"], 6))
    for rows, sums in res.items():   # both servers answered the same predictions
        if len(sums) != 1:
            raise SystemExit(f"predictions differ at {rows} rows: {sums}")


if __name__ == "__main__":
    main()
