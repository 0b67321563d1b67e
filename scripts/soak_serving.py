"""Soak of the native HTTP front end + native batcher on the GPU: one
xgbserver worker (C2 forest, 16 IO threads), the 4-thread load generator at a
fixed rate for several rounds; the server's resident memory and the latency of
every round are printed, so a leak or a drift shows as growth across rounds.
Usage: python scripts/soak_serving.py [--qps 150000] [--rounds 4] [--seconds 15]"""
import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_serving as bs   # noqa: E402


def rss_mb(pid: int) -> float:
    with open(f"/proc/{pid}/status") as fh:
        for line in fh:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return -1.0


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--qps", type=float, default=150000)
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--seconds", type=float, default=15)
    p.add_argument("--port", type=int, default=18555)
    a = p.parse_args()
    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    resource.setrlimit(resource.RLIMIT_NOFILE, (hard, hard))
    tmp = tempfile.mkdtemp()
    bs.write_c2_model(tmp)
    bodies = os.path.join(tmp, "bodies.bin")
    bs.write_bodies(bodies, 28, 8, seed=3)
    cmd = [sys.executable, "-m", "kfserving_amd.xgbserver", "--model_dir", tmp, "--model_name",
           "model", "--http_port", str(a.port), "--workers", "1", "--max_batchsize", "65536",
           "--max_latency_ms", "5", "--http_io_threads", "16"]
    srv = subprocess.Popen(cmd, cwd=bs.ROOT, start_new_session=True, stdout=subprocess.DEVNULL,
                           stderr=open(os.path.join(tmp, "server.log"), "w"))
    try:
        if not bs.wait_ready(a.port, 120):
            raise RuntimeError(open(os.path.join(tmp, "server.log")).read()[-2000:])
        bs.warm(a.port, 28)
        print(json.dumps({"round": 0, "server_rss_mb": rss_mb(srv.pid)}), flush=True)
        for r in range(1, a.rounds + 1):
            out = subprocess.run([bs.LOADGEN, "--port", str(a.port), "--conns", "4096", "--qps",
                                  str(a.qps), "--duration", str(a.seconds), "--warmup", "1",
                                  "--bodies", bodies, "--threads", "4",
                                  "--path", "/v1/models/model:predict"],
                                 capture_output=True, text=True, timeout=a.seconds + 90)
            res = json.loads(out.stdout)
            keep = {k: res[k] for k in ("req_per_s", "p50_ms", "p99_ms", "max_ms", "lost",
                                        "non200", "conn_errors")}
            print(json.dumps({"round": r, "server_rss_mb": rss_mb(srv.pid), **keep}), flush=True)
    finally:
        os.killpg(srv.pid, signal.SIGTERM)
        srv.wait(timeout=30)


if __name__ == "__main__":
    main()
