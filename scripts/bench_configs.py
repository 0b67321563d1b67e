"""Device-resident throughput of the non-headline BASELINE.json configs on one
GPU (the headline C2 is bench.py).  One JSON line per config:

  C3  LightGBM leaf-wise, 1000 trees x 255 leaves, 100 features (f32 input;
      BASELINE: 100M rows sharded over 1-8 GPUs -- measured per GPU on a
      --rows3 batch), CPU baseline = oracle/c/tree_port.c lightgbm restatement.
  C4  sklearn RandomForestRegressor(200, max_depth=16, max_features=1/3),
      64 features, fitted here on N(0,1) [--fit-rows x 64] with a nonlinear
      target; predict on a --rows4 batch (BASELINE: 10M rows).  CPU baseline =
      sklearn's own predict(n_jobs=all threads) on a bounded sample.

Usage: python scripts/bench_configs.py [--configs c3,c4] [--rows3 N] [--rows4 N]
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


def time_device(dev, X_t, out_t, rows, cols, kind, xdt, steps, warmup):
    import torch
    stream = torch.cuda.current_stream()
    for _ in range(warmup):
        dev.predict_device(X_t.data_ptr(), xdt, rows, cols, cols, kind, out_t.data_ptr(),
                           out_t.numel(), stream=stream.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        dev.predict_device(X_t.data_ptr(), xdt, rows, cols, cols, kind, out_t.data_ptr(),
                           out_t.numel(), stream=stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return rows * steps / wall, e0.elapsed_time(e1) / steps


def c3(args):
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
    dev = DeviceForest(f, [0])
    rows = args.rows3
    X = np.random.default_rng(3).standard_normal((rows, F), dtype=np.float32)
    Xt = torch.from_numpy(X).cuda()
    out = torch.empty(rows, dtype=torch.float64, device="cuda")
    rate, kms = time_device(dev, Xt, out, rows, F, OUT_MARGIN, TI_F32, args.steps, 2)
    # node visits per row, measured from the leaves reached on a sample
    from tests import canon_eval
    lv = canon_eval.leaves(f, X[:2000])
    node_depth = _node_depths(f)
    visits = float(np.mean(np.sum(node_depth[f.tree_offset[:-1][None, :] + lv], axis=1)))
    n = min(rows, 50_000)
    t0 = time.perf_counter()
    port.lgb_predict_raw(trees, 1, F, X[:n].astype(np.float64))
    cpu = n / (time.perf_counter() - t0)
    return {"config": f"C3 LightGBM leaf-wise 1000x255 leaves, {F} feat, f32 input",
            "rows": rows, "rows_per_s": rate, "kernel_ms": kms, "layout": dev.info()["layout"],
            "max_depth": int(depths.max()), "mean_tree_depth": float(depths.mean()),
            "node_visits_per_row": visits,
            "cpu_baseline": {"rows_per_s": cpu, "kind": "port", "threads": port.num_threads(),
                             "sample_rows": n}}


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


def c4(args):
    import torch
    from sklearn.ensemble import RandomForestRegressor
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn
    from kfserving_amd.forest import OUT_PREDICT, TI_F32
    rng = np.random.default_rng(0)
    n_thr = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count()))
    Xtr = rng.standard_normal((args.fit_rows, 64)).astype(np.float32)
    ytr = np.sin(2 * Xtr[:, 0]) + Xtr[:, 1] * Xtr[:, 2] + Xtr[:, 3] ** 2 + \
        0.1 * rng.standard_normal(args.fit_rows)
    t0 = time.perf_counter()
    est = RandomForestRegressor(n_estimators=200, max_depth=16, max_features=1 / 3,
                                random_state=0, n_jobs=n_thr).fit(Xtr, ytr)
    fit_s = time.perf_counter() - t0
    f = forest_from_sklearn(est)
    dev = DeviceForest(f, [0])
    rows = args.rows4
    X = np.random.default_rng(2).standard_normal((rows, 64), dtype=np.float32)
    Xt = torch.from_numpy(X).cuda()
    out = torch.empty(rows, dtype=torch.float64, device="cuda")
    rate, kms = time_device(dev, Xt, out, rows, 64, OUT_PREDICT, TI_F32, args.steps, 2)
    got = out[:4096].cpu().numpy()
    est.set_params(n_jobs=1)
    exact = bool(np.array_equal(got, est.predict(X[:4096])))
    est.set_params(n_jobs=n_thr)
    n = min(rows, 200_000)
    t0 = time.perf_counter()
    est.predict(X[:n])
    cpu = n / (time.perf_counter() - t0)
    return {"config": "C4 sklearn RandomForestRegressor 200 x depth16, 64 feat",
            "rows": rows, "rows_per_s": rate, "kernel_ms": kms, "layout": dev.info()["layout"],
            "nodes_per_tree": f.n_nodes / f.n_trees, "fit_s": fit_s,
            "bit_exact_vs_sklearn_4096": exact,
            "cpu_baseline": {"rows_per_s": cpu, "kind": "reference (sklearn 1.7.2 predict)",
                             "threads": n_thr, "sample_rows": n}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="c3,c4")
    p.add_argument("--rows3", type=int, default=1_000_000)
    p.add_argument("--f3", type=int, default=100, help="C3 feature count (BASELINE: 100)")
    p.add_argument("--rows4", type=int, default=1_000_000)
    p.add_argument("--fit-rows", type=int, default=200_000)
    p.add_argument("--steps", type=int, default=5)
    args = p.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's, loaded first)
    for c in args.configs.split(","):
        res = {"c3": c3, "c4": c4}[c.strip()](args)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
