"""bench.py's rank path end to end on CPU (gloo, world size 2) with a stub
engine: weak-scaling headline (every rank its own batch), max-over-ranks wall
time, strong-scaling C3 shard, and the JSON line rank 0 assembles."""
import os
import socket
import time

import torch.multiprocessing as mp


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
    # C3: strong scaling, 500 rows per rank, 1 untimed + 2 timed steps
    assert calls0[1] == [(500, 100)] * 3 and calls1[1] == [(500, 100)] * 3
    c3 = line["c3"]
    assert c3["rows"] == 1000 and c3["rows_per_gpu"] == 500 and c3["scaling"] == "strong"
    assert c3["ms_per_step"] >= 20.0
    rf = line["roofline"]
    assert rf["bound"] == "valu_issue" and rf["unit"] == "Ginst/s"
    assert 0 < rf["hbm_compulsory_frac"] < 1
