"""Device-resident throughput of the non-headline BASELINE.json configs at
their named sizes (the headline C2 is bench.py).  One JSON line per config:

  C3  LightGBM leaf-wise, 1000 trees x 255 leaves, 100 features, float32
      input; 100M rows (BASELINE configs[2]) generated on the device, row-
      sharded over the ranks of a torchrun launch (strong scaling: the 100M
      rows are split).  CPU baseline: oracle/c/tree_port.c, the lightgbm
      predict loop restated in C/OpenMP (lightgbm is not installed).
  C4  sklearn RandomForestRegressor(200, max_depth=16, max_features=1/3),
      64 features, fitted here on N(0,1) [--fit-rows x 64] with a nonlinear
      target; predict 10M rows (BASELINE configs[3]).  CPU baseline: sklearn's
      own predict (n_jobs = the host threads) on a bounded sample.

Each line carries a roofline block in the SURVEY.md 8(d) byte model for the
explicit layouts: B_visit = 16 B x V + 4 B x F + out bytes per row (V = node
visits per row, measured from the leaves reached on a sample), divided by the
kernel time, against 8 TB/s HBM; and a parity spot check of the first rows of
the device batch against the oracle (C3) / sklearn itself (C4).

Usage: python scripts/bench_configs.py [--configs c3,c4] [--rows3 N] [--rows4 N]
       python -m torch.distributed.run --nproc-per-node G scripts/bench_configs.py ...
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK = 8.0e12


def dist_info():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def max_over_ranks(v):
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return v
    t = torch.tensor([v], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard(total, world, rank):
    per = (total + world - 1) // world
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


def time_device(dev, X_t, out_t, rows, cols, kind, xdt, steps, warmup):
    import torch
    import torch.distributed as dist
    stream = torch.cuda.current_stream()
    for _ in range(warmup):
        dev.predict_device(X_t.data_ptr(), xdt, rows, cols, cols, kind, out_t.data_ptr(),
                           out_t.numel(), stream=stream.cuda_stream)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        dev.predict_device(X_t.data_ptr(), xdt, rows, cols, cols, kind, out_t.data_ptr(),
                           out_t.numel(), stream=stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    wall = max_over_ranks(time.perf_counter() - t0)
    return wall / steps, e0.elapsed_time(e1) / steps


def device_normal(rows, cols, seed):
    """X ~ N(0,1) float32 generated on the device in 8M-row chunks (seed, chunk)."""
    import torch
    X = torch.empty((rows, cols), dtype=torch.float32, device="cuda")
    chunk = 8 << 20
    for i, lo in enumerate(range(0, rows, chunk)):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed * 1000003 + i)
        hi = min(rows, lo + chunk)
        X[lo:hi] = torch.randn((hi - lo, cols), generator=g, device="cuda", dtype=torch.float32)
    return X


def _node_depths(f):
    d = np.zeros(f.n_nodes, dtype=np.int64)
    for t in range(f.n_trees):
        b = int(f.tree_offset[t])
        n = int(f.tree_offset[t + 1]) - b
        for v in range(n):
            g = b + v
            if f.feature[g] >= 0:
                d[b + f.left[g]] = d[g] + 1
                d[b + f.right[g]] = d[g] + 1
    return d


def visits_per_row(f, X_sample):
    from tests import canon_eval
    lv = canon_eval.leaves(f, X_sample)
    node_depth = _node_depths(f)
    return float(np.mean(np.sum(node_depth[f.tree_offset[:-1][None, :] + lv], axis=1)))


def roofline(visits, n_feat, out_bytes, rows, kernel_ms):
    b = 16 * visits + 4 * n_feat + out_bytes
    achieved = b * rows / (kernel_ms * 1e-3)
    return {"bound": "hbm", "bytes_per_row_visit_model": b, "achieved": achieved / 1e9,
            "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
            "compulsory_GBps": (4 * n_feat + out_bytes) * rows / (kernel_ms * 1e-3) / 1e9}


def c3(args, world, rank):
    import torch
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.formats import lightgbm_format as lf
    from kfserving_amd.forest import OUT_MARGIN, TI_F32
    from oracle import port
    F = args.f3
    trees = lf.synthetic_leafwise_trees(1000, 255, F, seed=1)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, F, "binary sigmoid:1")
        f = lf.load_lightgbm_model(p)
    depths = f.depths()
    dev = DeviceForest(f, [torch.cuda.current_device()])
    lo, hi = shard(args.rows3, world, rank)
    rows = hi - lo
    X = device_normal(rows, F, seed=3 + rank)
    out = torch.empty(rows, dtype=torch.float64, device="cuda")
    step_s, kms = time_device(dev, X, out, rows, F, OUT_MARGIN, TI_F32, args.steps, 1)
    if rank != 0:
        return None
    n_chk = min(rows, 20_000)
    Xs = X[:n_chk].cpu().numpy()
    exact = bool(np.array_equal(out[:n_chk].cpu().numpy(),
                                port.lgb_predict_raw(trees, 1, F, Xs.astype(np.float64))[:, 0]))
    visits = visits_per_row(f, Xs[:2000])
    n = min(n_chk, 50_000)
    t0 = time.perf_counter()
    port.lgb_predict_raw(trees, 1, F, Xs[:n].astype(np.float64))
    cpu = n / (time.perf_counter() - t0)
    return {"config": f"C3 LightGBM leaf-wise 1000x255 leaves, {F} feat, f32 input",
            "rows": args.rows3, "n_gpus": world, "rows_per_gpu": rows, "scaling": "strong",
            "rows_per_s": args.rows3 / step_s, "step_ms": step_s * 1e3, "kernel_ms": kms,
            "layout": dev.info()["layout"], "max_depth": int(depths.max()),
            "mean_tree_depth": float(depths.mean()), "node_visits_per_row": visits,
            "roofline": roofline(visits, F, 8, rows, kms),
            "bit_exact_vs_port_first_rows": exact, "parity_rows": n_chk,
            "cpu_baseline": {"rows_per_s": cpu, "kind": "port", "threads": port.num_threads(),
                             "sample_rows": n}}


def c4(args, world, rank):
    import torch
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn
    from kfserving_amd.forest import OUT_PREDICT, TI_F32
    n_thr = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count()))
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import make_c4_model as mk
    est = None
    fit_s = 0.0
    if args.fit_rows == 200_000 and os.path.exists(mk.MODEL):
        from kfserving_amd.formats.sklearn_format import load_tree_arrays
        f = load_tree_arrays(mk.MODEL)     # the cached C4 fit (scripts/make_c4_model.py)
    else:
        t0 = time.perf_counter()
        est = mk.fit(args.fit_rows, n_thr)
        fit_s = time.perf_counter() - t0
        f = forest_from_sklearn(est)
    dev = DeviceForest(f, [torch.cuda.current_device()])
    lo, hi = shard(args.rows4, world, rank)
    rows = hi - lo
    X = device_normal(rows, 64, seed=2 + rank)
    out = torch.empty(rows, dtype=torch.float64, device="cuda")
    step_s, kms = time_device(dev, X, out, rows, 64, OUT_PREDICT, TI_F32, args.steps, 1)
    if rank != 0:
        return None
    Xs = X[:4096].cpu().numpy()
    visits = visits_per_row(f, Xs[:1000])
    if est is not None:
        est.set_params(n_jobs=1)
        exact = bool(np.array_equal(out[:4096].cpu().numpy(), est.predict(Xs)))
        est.set_params(n_jobs=n_thr)
        Xc = X[:min(rows, 200_000)].cpu().numpy()
        t0 = time.perf_counter()
        est.predict(Xc)
        cpu = Xc.shape[0] / (time.perf_counter() - t0)
        cpu_kind = "reference (sklearn 1.7.2 predict)"
    else:   # cached arrays: sklearn's own outputs are in the check file (tests/)
        from tests import canon_eval
        exact = bool(np.array_equal(out[:4096].cpu().numpy(), canon_eval.predict(f, Xs)))
        Xc = Xs
        cpu, cpu_kind = None, "see bench.py (oracle port)"
    return {"config": "C4 sklearn RandomForestRegressor 200 x depth16, 64 feat",
            "rows": args.rows4, "n_gpus": world, "rows_per_gpu": rows, "scaling": "strong",
            "rows_per_s": args.rows4 / step_s, "step_ms": step_s * 1e3, "kernel_ms": kms,
            "layout": dev.info()["layout"], "nodes_per_tree": f.n_nodes / f.n_trees,
            "node_visits_per_row": visits, "roofline": roofline(visits, 64, 8, rows, kms),
            "fit_s": fit_s, "bit_exact_vs_sklearn_4096": exact,
            "cpu_baseline": {"rows_per_s": cpu, "kind": cpu_kind,
                             "threads": n_thr, "sample_rows": Xc.shape[0]}}


def shap(args, world, rank):
    """TreeSHAP contributions (TI_OUTPUT_CONTRIB) of the C2 model: 500 trees
    depth 8, 28 features; work per row = sum over the 128k root-to-leaf paths
    of O(len^2) path-weight updates (len <= 8 unique features)."""
    import torch
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.formats import xgboost_format as xf
    from kfserving_amd.forest import OUT_CONTRIB, TI_F32
    from oracle import port
    trees, ti = xf.synthetic_complete_trees(500, 8, 28, seed=0)
    f = xf.forest_from_raw_trees(trees, ti, 28, 0, 0.5, "binary:logistic")
    dev = DeviceForest(f, [torch.cuda.current_device()])
    lo, hi = shard(args.rows_shap, world, rank)
    rows = hi - lo
    X = device_normal(rows, 28, seed=5 + rank)
    W = 29
    out = torch.empty(rows * W, dtype=torch.float32, device="cuda")
    step_s, kms = time_device(dev, X, out, rows, 28, OUT_CONTRIB, TI_F32, args.steps, 1)
    if rank != 0:
        return None
    n = min(rows, 2000)
    Xs = X[:n].cpu().numpy()
    t0 = time.perf_counter()
    want = port.tree_shap(f, Xs.astype(np.float64))
    cpu = n / (time.perf_counter() - t0)
    got = out[:n * W].cpu().numpy().reshape(n, W).astype(np.float64)
    scale = np.maximum(np.abs(want).max(axis=1, keepdims=True), 1.0)
    return {"config": "TreeSHAP contributions of the C2 model (500 x depth 8, 28 feat)",
            "rows": args.rows_shap, "n_gpus": world, "rows_per_gpu": rows, "scaling": "strong",
            "rows_per_s": args.rows_shap / step_s, "step_ms": step_s * 1e3, "kernel_ms": kms,
            "max_scaled_err_vs_port": float((np.abs(got - want) / scale).max()),
            "parity_rows": n,
            "cpu_baseline": {"rows_per_s": cpu, "kind": "port (oracle/c/shap_port.c)",
                             "threads": port.num_threads(), "sample_rows": n}}


def ts(args, world, rank):
    """Tree-sharded C2 (kfserving_amd/tree_shard.py): every rank predicts the
    same 1M rows over its 500/world trees, partial margins summed by one
    RCCL reduce to rank 0, transform there.  Strong scaling in trees."""
    import torch
    import torch.distributed as dist
    from kfserving_amd.formats import xgboost_format as xf
    from kfserving_amd.forest import OUT_PREDICT
    from kfserving_amd.tree_shard import TreeShardedForest
    trees, ti = xf.synthetic_complete_trees(500, 8, 28, seed=0)
    f = xf.forest_from_raw_trees(trees, ti, 28, 0, 0.5, "binary:logistic")
    sh = TreeShardedForest(f, device=torch.cuda.current_device())
    X = device_normal(args.rows_ts, 28, seed=0)
    for _ in range(2):
        sh.predict(X, OUT_PREDICT)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = sh.predict(X, OUT_PREDICT)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    wall = max_over_ranks(time.perf_counter() - t0) / args.steps
    if rank != 0:
        return None
    from kfserving_amd.engine import DeviceForest
    ref = torch.empty_like(out)
    DeviceForest(f, [torch.cuda.current_device()]).predict_device(
        X.data_ptr(), 0, args.rows_ts, 28, 28, OUT_PREDICT, ref.data_ptr(), ref.numel(),
        stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    err = float(((out - ref).abs() / ref.abs().clamp_min(1e-30)).max())
    return {"config": "C2 tree-sharded (trees split over ranks, RCCL reduce of margins)",
            "rows": args.rows_ts, "n_gpus": world, "trees_per_rank": [b - a for a, b in sh.ranges],
            "scaling": "strong", "rows_per_s": args.rows_ts / wall, "step_ms": wall * 1e3,
            "max_rel_err_vs_one_device": err}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="c3,c4")
    p.add_argument("--rows3", type=int, default=100_000_000)
    p.add_argument("--f3", type=int, default=100, help="C3 feature count (BASELINE: 100)")
    p.add_argument("--rows4", type=int, default=10_000_000)
    p.add_argument("--fit-rows", type=int, default=200_000)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--rows-shap", type=int, default=100_000)
    p.add_argument("--rows-ts", type=int, default=1_000_000)
    args = p.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's, loaded first)
    import torch.distributed as dist
    world, rank, local = dist_info()
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    for c in args.configs.split(","):
        res = {"c3": c3, "c4": c4, "shap": shap, "ts": ts}[c.strip()](args, world, rank)
        if res is not None:
            print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
