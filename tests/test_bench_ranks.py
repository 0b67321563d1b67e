"""bench.py's rank path end to end on CPU (gloo, world size 2) with a stub
engine: weak-scaling headline (every rank its own batch), max-over-ranks wall
time, strong-scaling C3 shard, and the JSON line rank 0 assembles."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class StubEngine:
    """Stands in for DeviceForest: records the calls, sleeps per call so the
    slower rank's wall time is known (rank 1: 20 ms per predict)."""

    def __init__(self, forest, rank):
        self.forest = forest
        self.rank = rank
        self.calls = []

    def predict_device(self, x_ptr, x_dtype, n_rows, n_cols, row_stride, kind, out_ptr,
                       out_len, slot=0, stream=0):
        self.calls.append((n_rows, n_cols))
        time.sleep(0.02 if self.rank == 1 else 0.001)

    def transform_device(self, margin_ptr, n_rows, out_ptr, out_len, slot=0, stream=0):
        pass

    def predict(self, X, kind=0):
        """Host-buffer predict (the host_pipeline legs): zeros."""
        import numpy as np
        return np.zeros(np.asarray(X).shape[0], dtype=np.float32)

    def info(self):
        return {"layout": 3}

    def close(self):
        pass


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import bench
    args = bench.parse_args(["--steps", "5", "--warmup", "1", "--rows", "4096",
                             "--configs", "c3", "--rows3", "1000", "--config-steps", "2",
                             "--no-cpu-baseline", "--latency-qps", "0",
                             "--host-rows-configs", "1000"])
    engines = []

    def make(forest):
        e = StubEngine(forest, rank)
        engines.append(e)
        return e

    line = bench.run(args, device="cpu", backend="gloo", make_engine=make)
    q.put((rank, line, [e.calls for e in engines]))


def test_bench_rank_path_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, line, calls0), (_, none, calls1) = res
    assert none is None                                   # only rank 0 prints
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["rows_per_gpu"] == 4096
    # headline: warmup 1 + 5 timed steps of a full 4096-row batch on every rank
    assert calls0[0] == [(4096, 28)] * 6 and calls1[0] == [(4096, 28)] * 6
    # the max over ranks: rank 1's 5 x 20 ms dominates
    assert line["ms_per_step"] >= 20.0
    assert abs(line["value"] - 4096 * 2 * 5 / (line["ms_per_step"] * 5e-3)) < 1e-6 * line["value"]
    # no GPU: one stream, and the one-stream region is the headline's; the
    # stand-in engine writes no outputs, so there is nothing to compare
    assert line["config"]["streams"] == 1 and line["streams_outputs_identical"] is None
    assert line["single_stream"]["value"] == line["value"]
    # the tree-sharded leg: every rank predicts all 4096 rows over its slice
    # (1 untimed + 5 timed steps), the partial margins reduced to rank 0
    assert calls0[1] == [(4096, 28)] * 6 and calls1[1] == [(4096, 28)] * 6
    ts = line["tree_shard"]
    assert ts["ranks"] == 2 and ts["rows"] == 4096 and ts["ms_per_step"] >= 20.0
    # C3: strong scaling, 500 rows per rank, 1 untimed + 2 timed steps
    assert calls0[2] == [(500, 100)] * 3 and calls1[2] == [(500, 100)] * 3
    c3 = line["c3"]
    assert c3["rows"] == 1000 and c3["rows_per_gpu"] == 500 and c3["scaling"] == "strong"
    assert c3["ms_per_step"] >= 20.0
    # the plugins' host-buffer path for the config
    # workloads, on rank 0 (the stand-in's host predict)
    hp = line["host_pipeline_c3"]
    assert hp["rows"] == 1000 and hp["input_GBps"] > 0 and hp["dtype"] == "float32"
    assert hp["bytes_per_row_in"] == 400
    rf = line["roofline"]
    assert rf["bound"] == "valu_issue" and rf["unit"] == "Ginst/s"
    assert 0 < rf["hbm_compulsory_frac"] < 1


def test_bench_cli_gpus_n_starts_n_ranks():
    """`python bench.py --gpus 2` as the driver runs it (no launcher, no
    WORLD_SIZE): bench.py starts the two ranks itself, only rank 0 prints,
    n_gpus is 2 and value = both ranks' rows / the slowest rank's wall."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "4"                           # the job's host share
    env.pop("BENCH_HOST_THREADS", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--engine", "tests.bench_stub:make", "--steps", "5", "--warmup", "1",
           "--rows", "2048", "--configs", "c3", "--rows3", "2000", "--config-steps", "1",
           "--cpu-seconds", "0.2", "--latency-qps", "200", "--latency-seconds", "0.5",
           "--nan-variant", "0", "--host-rows", "0", "--host-rows-configs", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                      # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["parallelism"] == "rows sharded x2"
    assert line["ms_per_step"] >= 20.0                    # rank 1's 20 ms steps dominate
    want = 2048 * 2 * 5 / (line["ms_per_step"] * 5e-3)
    assert abs(line["value"] - want) < 1e-6 * want
    # the CPU baselines at N > 1, timed on rank 0 with the
    # whole host share (not OMP_NUM_THREADS / N), the thread count stated
    cb = line["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["cores"] == 4 and cb["kind"] == "port"
    c3 = line["c3"]
    assert c3["rows"] == 2000 and c3["rows_per_gpu"] == 1000
    assert c3["cpu_baseline"]["value"] > 0 and c3["cpu_baseline"]["cores"] == 4
    assert "_cpu" not in c3
    # the C5 leg drives every rank's device, pooled on rank 0
    bl = line["batched_latency"]
    assert bl["devices"] == 2 and len(bl["p99_ms_per_rank"]) == 2
    assert bl["qps_offered"] == 2 * bl["qps_offered_per_gpu"] == 400
    assert bl["p50_ms"] <= bl["p99_ms"] <= bl["max_ms"] and bl["requests"] > 0
    assert "_lat_ms" not in bl
    # the leg runs through the native batcher, every request's rows checked
    # against a direct predict; the asyncio batcher's run is beside it
    assert "native batcher" in bl["path"] and bl["outputs_match_direct_predict"] is True
    ba = line["batched_latency_asyncio"]
    assert ba["devices"] == 2 and ba["requests"] == bl["requests"] and "_lat_ms" not in ba
    # the tree-sharded leg (a reduce over the ranks) is in the line
    ts = line["tree_shard"]
    assert ts["ranks"] == 2 and ts["reduce_bytes"] == 2048 * 4 and ts["rows_per_s"] > 0
    assert 0 < ts["trees_rank0"] < 500


def test_bench_cli_world2_c5_scales_and_tree_shard_checks():
    """VERDICT r5 items 1 and 8 through the CLI at world 2 (gloo, CPU): the
    C5-over-HTTP leg offers per-GPU rates x N with connections and load
    generator threads per GPU and the one-GPU IO thread count, and searches
    the capacity; the tree-sharded leg's reduced predictions are checked
    against the replicated forest (an engine that computes on CPU)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_serving as bs
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "4"
    http = os.path.exists(bs.LOADGEN)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--engine", "tests.bench_stub:make_canon", "--steps", "2", "--warmup", "1",
           "--rows", "1024", "--configs", "", "--no-cpu-baseline", "--latency-qps", "0",
           "--nan-variant", "0", "--host-rows", "0", "--c5-http-v2-qps", "",
           "--c5-http-qps", "100,200" if http else "", "--c5-http-cpu",
           "--c5-conns-per-gpu", "16", "--c5-loadgen-threads-per-gpu", "1",
           "--c5-io-threads", "2", "--c5-capacity-points", "1", "--c5-http-seconds", "0.5"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    ts = line["tree_shard"]
    assert ts["ranks"] == 2 and ts["within_1e-5"] is True, ts
    assert ts["max_rel_diff_vs_replicated"] <= 1e-5
    if not http:
        pytest.skip("loadgen not built: the C5 HTTP half is not exercised")
    c5 = line["c5_http"]
    assert "error" not in c5, c5
    assert c5["devices"] == 2 and c5["workers"] == 2
    assert c5["offered_qps_per_gpu"] == [100.0, 200.0]
    assert c5["offered_qps_node"] == [200.0, 400.0]                # doubled at world 2
    assert [p["offered_qps"] for p in c5["points"]] == [200.0, 400.0]
    assert c5["conns"] == 32 and c5["loadgen_threads"] == 2
    assert c5["io_threads_per_worker"] == 2                       # not divided by N
    cap = c5["capacity"]
    assert len(cap["searched"]) <= 1 and "criterion" in cap
    assert c5["capacity_req_per_s"] == cap["capacity_req_per_s"]


def test_capacity_search_grows_then_bisects():
    """bench_serving.capacity_search on a synthetic server whose p99 crosses
    10 ms at 250k req/s: grows from the best fixed point, then bisects."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_serving as bs

    def fake(q):
        return {"p99_ms": 5.3 if q <= 250_000 else 40.0, "lost": 0, "non200": 0,
                "conn_errors": 0, "req_per_s": q}
    done = [(q, fake(q)) for q in (20_000, 100_000, 200_000)]
    cap = bs.capacity_search(fake, done, 10.0, points=6)
    assert 200_000 <= cap["capacity_req_per_s"] <= 250_000
    assert cap["first_fail_req_per_s"] > 250_000
    assert cap["searched"][0]["offered_qps"] == 300_000 and not cap["searched"][0]["passed"]
    assert cap["first_fail_req_per_s"] / cap["capacity_req_per_s"] <= 1.25
    # a lost request fails a point whatever its p99
    assert not bs.point_passes({"p99_ms": 1.0, "lost": 3, "non200": 0}, 10.0)
    # nothing passes: halve from the lowest failure
    cap = bs.capacity_search(lambda q: {"p99_ms": 99.0}, [(1000.0, {"p99_ms": 99.0})], 10.0, 2)
    assert cap["capacity_req_per_s"] is None and [s["offered_qps"] for s in cap["searched"]] == [500.0, 250.0]


def test_headline_defaults_two_streams():
    """The headline keeps two batches in flight by default (DESIGN.md section
    4); without a GPU there is one stream and the two timings coincide."""
    import bench
    assert bench.parse_args([]).streams == 2
    assert bench.parse_args(["--streams", "1"]).streams == 1


def test_http_leg_prints_nothing_of_its_own(capsys):
    """bench.py's c5_http leg calls bench_serving.serve_and_measure with
    echo=False: rank 0's stdout must stay the one JSON line (here with the
    CPU echo model and a short load)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_serving as bs
    if not os.path.exists(bs.LOADGEN):
        pytest.skip("loadgen not built")
    pts = bs.serve_and_measure([500.0], workers=1, io_threads=1, duration=0.5, warmup=0.2,
                               conns=16, port=18000 + os.getpid() % 900, model="dummy",
                               ready_timeout=60, loadgen_threads=2, echo=False)
    assert len(pts) == 1 and pts[0]["completed"] > 0 and pts[0]["non200"] == 0
    assert capsys.readouterr().out == ""
