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
                             "--no-cpu-baseline", "--latency-qps", "0"])
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
           "--nan-variant", "0", "--host-rows", "0"]
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
