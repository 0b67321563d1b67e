"""Benchmark: predicted rows/sec of the BASELINE.json headline workload.

Workload (BASELINE.json configs[1]): synthetic HIGGS-shaped
XGBoost binary:logistic model, 500 complete depth-8 trees, 28 features,
base_score 0.5; a 1M-row float32 batch per GPU, resident in HBM when the timed
region starts.  One step = one fused predict (traversal + sigmoid) over the
batch.  Multi-GPU: one process per GPU (torchrun), rows sharded with no
collective ("weak": every rank predicts its own 1M rows); value = all ranks'
rows / max-over-ranks wall time.

Also reported (rank 0):
  roofline     -- SURVEY.md 8(d) byte model per launch: B_visit = 8 B x V + 4 B x F
                  + 4 B out, V = node visits per row (500 x 8 = 4000), divided by
                  the kernel's average duration measured with HIP events on the
                  launch stream; traffic = HBM bytes from a committed rocprofv3 PMC
                  pass (profiles/), or null.
  cpu_baseline -- the C/OpenMP restatement of xgboost 0.82's predict loop
                  (oracle/c/tree_port.c, kind "port": xgboost is not installed)
                  timed on this host on a bounded sample of the same rows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_TREES, DEPTH, N_FEAT, ROWS = 500, 8, 28, 1_000_000
HBM_PEAK = 8.0e12          # MI355X HBM3E, bytes/s (MI355X_MICROARCH.md)
LAYOUT_NAMES = {0: "heap", 1: "explicit", 2: "compact", 3: "bheap", 4: "bexplicit",
                5: "sexplicit", 6: "rexplicit"}


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rows", type=int, default=ROWS)
    p.add_argument("--nan-variant", type=float, default=0.01,
                   help="also time the same batch with this fraction of NaN features "
                        "(SURVEY.md 8(d) C2 1%%-NaN variant; 0 = skip)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="target CPU work for the cpu_baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--latency-qps", type=float, default=10000.0,
                   help="offered requests/s for the batched-latency leg (0 = skip)")
    p.add_argument("--latency-seconds", type=float, default=3.0)
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_c2.json"))
    return p.parse_args()


def build_model():
    from kfserving_amd.formats.xgboost_format import (forest_from_raw_trees,
                                                      synthetic_complete_trees)
    trees, ti = synthetic_complete_trees(N_TREES, DEPTH, N_FEAT, seed=0)
    # xgboost 0.82 stores base_score in margin space: ProbToMargin(0.5) = 0
    forest = forest_from_raw_trees(trees, ti, N_FEAT, 0, 0.0, "binary:logistic")
    return trees, ti, forest


def shard_rows(total_rows: int, rank: int, world: int):
    """Weak scaling: every rank owns a full batch of `total_rows` rows with its own seed
    (rows are independent: no data-path collective)."""
    return total_rows, 1000 + rank


def max_over_ranks(value: float, device) -> float:
    """The slowest rank's wall time (the only collective, outside the timed region)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(trees, ti, X_host, target_s):
    from oracle import port
    n_thr = port.num_threads()
    probe = min(20_000, X_host.shape[0])
    t0 = time.perf_counter()
    port.xgb_predict(trees, ti, 1, 0.0, N_FEAT, X_host[:probe], sigmoid=True)
    rate = probe / max(time.perf_counter() - t0, 1e-9)
    n = int(min(X_host.shape[0], max(probe, rate * target_s)))
    t0 = time.perf_counter()
    port.xgb_predict(trees, ti, 1, 0.0, N_FEAT, X_host[:n], sigmoid=True)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "rows/s", "cores": n_thr, "kind": "port",
            "sample": f"{n} rows of the same 1M x 28 batch, oracle/c/tree_port.c "
                      f"(xgboost 0.82 predict loop restated, OpenMP {n_thr} threads), "
                      f"{dt:.1f} s"}


def batched_latency(dev, n_feat, qps, seconds, max_batch=65536, max_latency_ms=5, seed=7,
                    freeze_gc=True):
    """C5-style leg: open-loop Poisson arrivals of requests of
    U{1..64} rows into the pipelined in-process batcher (pkg/batcher semantics,
    maxBatchSize rows, maxLatency ms) in front of the GPU engine (host buffers:
    H2D + kernel + D2H per batch).  Latency = result time - scheduled arrival."""
    import asyncio
    from concurrent.futures import ThreadPoolExecutor
    from kfserving_amd.batcher import Batcher
    rng = np.random.default_rng(seed)
    warm = int(qps * 0.5)                 # first 0.5 s of load is warmup, not reported
    n_req = int(qps * seconds) + warm
    gaps = rng.exponential(1.0 / qps, n_req)
    sizes = rng.integers(1, 65, n_req)
    pool = np.random.default_rng(seed + 1).standard_normal((64 * 1024, n_feat), dtype=np.float32)
    pool_rows = list(pool)
    pool_ex = ThreadPoolExecutor(max_workers=2)
    lat = np.zeros(n_req)
    batch_rows = []
    batch_ms = []

    async def predict_batch(instances):
        X = np.stack(instances)
        batch_rows.append(X.shape[0])
        t = time.perf_counter()
        out = await asyncio.get_running_loop().run_in_executor(pool_ex, dev.predict, X)
        batch_ms.append((time.perf_counter() - t) * 1e3)
        return {"predictions": out}

    async def run():
        b = Batcher(predict_batch, max_batch_size=max_batch, max_latency_ms=max_latency_ms)
        loop = asyncio.get_running_loop()
        t0 = loop.time() + 0.05
        arrivals = t0 + np.cumsum(gaps)
        tasks = []

        async def one(i):
            off = (i * 64) % (len(pool_rows) - 64)
            await b.submit(pool_rows[off:off + int(sizes[i])])
            lat[i] = loop.time() - arrivals[i]

        for i in range(n_req):
            delay = arrivals[i] - loop.time()
            if delay > 0:
                await asyncio.sleep(delay)
            tasks.append(asyncio.ensure_future(one(i)))
        await asyncio.gather(*tasks)
        return loop.time() - t0

    import gc
    old = gc.get_threshold()
    if freeze_gc:          # what KFServer.start does after load (kfserver.tune_gc)
        from kfserving_amd.kfserving.kfserver import tune_gc
        tune_gc()
    try:
        wall = asyncio.run(run())
    finally:
        if freeze_gc:
            gc.unfreeze()
            gc.set_threshold(*old)
    pool_ex.shutdown()
    lat_ms = lat[warm:] * 1e3
    return {"qps_offered": qps, "requests": n_req - warm, "rows_per_request": "U{1..64}",
            "max_batch_size": max_batch, "max_latency_ms": max_latency_ms,
            "p50_ms": float(np.percentile(lat_ms, 50)), "p99_ms": float(np.percentile(lat_ms, 99)),
            "max_ms": float(lat_ms.max()), "rows_per_s": float(sizes.sum() / wall),
            "p90_ms": float(np.percentile(lat_ms, 90)),
            "batches": len(batch_rows), "mean_batch_rows": float(np.mean(batch_rows)),
            "predict_ms_p50": float(np.percentile(batch_ms, 50)),
            "predict_ms_p99": float(np.percentile(batch_ms, 99)), "gc_frozen": freeze_gc,
            "path": "in-process batcher -> ti_predict (host buffers), 1 GPU, no HTTP/JSON"}


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local_rank)

    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_PREDICT, TI_F32

    trees, ti, forest = build_model()
    dev = DeviceForest(forest, devices=[local_rank])
    info = dev.info()
    rows, seed = shard_rows(args.rows, rank, world)
    X_host = np.random.default_rng(seed).standard_normal((rows, N_FEAT), dtype=np.float32)
    X = torch.from_numpy(X_host).to(f"cuda:{local_rank}")
    out = torch.empty(rows, dtype=torch.float32, device=f"cuda:{local_rank}")
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def step():
        dev.predict_device(X.data_ptr(), TI_F32, rows, N_FEAT, N_FEAT, OUT_PREDICT,
                           out.data_ptr(), rows, slot=0, stream=sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    wall = max_over_ranks(wall, f"cuda:{local_rank}")
    total_rows = rows * world * args.steps
    value = total_rows / wall

    nan_variant = None
    if args.nan_variant > 0 and rank == 0:
        # same shape, seed 1, NaN at random positions: every tile takes the
        # kernel's NaN-checking path (not part of the headline value)
        Xn_host = np.random.default_rng(1).standard_normal((rows, N_FEAT), dtype=np.float32)
        Xn_host[np.random.default_rng(2).random(Xn_host.shape) < args.nan_variant] = np.nan
        Xn = torch.from_numpy(Xn_host).to(f"cuda:{local_rank}")
        for _ in range(2):
            dev.predict_device(Xn.data_ptr(), TI_F32, rows, N_FEAT, N_FEAT, OUT_PREDICT,
                               out.data_ptr(), rows, slot=0, stream=sh)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            dev.predict_device(Xn.data_ptr(), TI_F32, rows, N_FEAT, N_FEAT, OUT_PREDICT,
                               out.data_ptr(), rows, slot=0, stream=sh)
        e1.record(stream)
        torch.cuda.synchronize()
        nms = e0.elapsed_time(e1) / args.steps
        nan_variant = {"nan_fraction": args.nan_variant, "kernel_ms": nms,
                       "rows_per_s": rows / (nms * 1e-3)}
        del Xn

    if rank == 0:
        visits = N_TREES * DEPTH                     # complete trees: every row visits D nodes
        b_visit = 8 * visits + 4 * N_FEAT + 4        # SURVEY.md 8(d) B_visit
        achieved = b_visit * rows / (kernel_ms * 1e-3)
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as fh:
                    pmc = json.load(fh)
                if (pmc.get("rows") == rows and pmc.get("workload") == "c2"
                        and pmc.get("layout", "heap") == LAYOUT_NAMES.get(info["layout"])):
                    traffic = pmc.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        roofline = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                    "unit": "GB/s", "frac": achieved / HBM_PEAK, "traffic": traffic,
                    "bytes_per_row_visit_model": b_visit,
                    "compulsory_GBps": (4 * N_FEAT + 4) * rows / (kernel_ms * 1e-3) / 1e9,
                    "kernel_ms": kernel_ms}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(trees, ti, X_host, args.cpu_seconds)
        latency = None
        if args.latency_qps > 0:
            latency = batched_latency(dev, N_FEAT, args.latency_qps, args.latency_seconds)
        line = {
            "metric": "predicted rows/sec (500-tree XGB, 28 feat)",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: X ~ N(0,1) float32, seeded; random 500 x depth-8 XGBoost "
                    "binary:logistic trees (SURVEY.md 8(d) C2)",
            "config": {"workload": "C2 synthetic HIGGS-shaped XGBoost binary: 28 features, "
                                   "500 trees depth 8, 1M-row batch per GPU",
                       "rows_per_gpu": rows, "trees": N_TREES, "depth": DEPTH,
                       "features": N_FEAT, "layout": LAYOUT_NAMES.get(info["layout"]),
                       "parallelism": f"rows sharded x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "batched_latency": latency,
            "nan_variant": nan_variant,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
