"""One named workload's predict kernel on one GPU, for rocprofv3 passes
(scripts/kernel_pmc.sh) and quick timings: the forest and device-resident
N(0,1) batch of bench.py's config, --steps launches of OUT_PREDICT on the
launch stream, one JSON line with the event time per launch.

  c2         500 x depth-8 XGBoost binary, 28 features, float32 (bench headline)
  c2_hist    the same trees with hist-style thresholds (253 quantile bounds: u8 bins)
  c3 / c3_f64  LightGBM leaf-wise 1000 x 255 leaves, 100 features, float32 /
             float64 input (lgbserver's DataFrame dtype)
  c3_maxbin  the LightGBM-shaped variant (thresholds on 255 quantile bin edges,
             nested along each path; lightgbm_format.synthetic_maxbin_trees)
  c4         the cached sklearn RandomForestRegressor 200 x depth 16, 64 features

Usage: python scripts/kernel_workload.py --workload c3 [--rows 1000000] [--steps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def forest_of(workload):
    import bench
    if workload == "c2":
        return bench.build_model()[2], bench.N_FEAT, "float32"
    if workload == "c2_hist":
        return bench.c2_hist_forest()[0], bench.N_FEAT, "float32"
    if workload in ("c3", "c3_f64"):
        return bench.c3_forest()[0], 100, "float64" if workload == "c3_f64" else "float32"
    if workload == "c3_maxbin":
        return bench.c3_maxbin_forest()[0], 100, "float32"
    if workload == "c4":
        return bench.c4_forest()[0], 64, "float32"
    raise ValueError(workload)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", required=True)
    p.add_argument("--rows", type=int, default=1_000_000)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--trees", type=int, default=0,
                   help="c2 / c2_hist / c3*: the first N trees (fixed cost vs per-tree cost; "
                        "C3's image against one XCD's 4 MB L2)")
    p.add_argument("--tree-start", type=int, default=0,
                   help="c4: the slice starts at this tree (with --trees: trees [start, start + N))")
    p.add_argument("--x-buffers", type=int, default=1,
                   help="copies of the batch the launches rotate through (bench.py uses 3 for C2)")
    p.add_argument("--streams", type=int, default=1,
                   help="launch streams the steps rotate over (batches in flight, as bench.py --streams)")
    a = p.parse_args()
    import torch
    import bench
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_PREDICT, TI_F32, TI_F64
    forest, F, dtype = forest_of(a.workload)
    if a.trees and a.workload in ("c2", "c2_hist"):
        from kfserving_amd.formats.xgboost_format import (forest_from_raw_trees,
                                                          synthetic_complete_trees)
        trees, ti = synthetic_complete_trees(bench.N_TREES, bench.DEPTH, F, seed=0,
                                             max_bin=254 if a.workload == "c2_hist" else 0)
        forest = forest_from_raw_trees(trees[:a.trees], ti[:a.trees], F, 0, 0.0, "binary:logistic")
    elif a.trees and a.workload in ("c3", "c3_f64", "c3_maxbin"):
        from kfserving_amd.formats import lightgbm_format as lf
        gen = lf.synthetic_maxbin_trees if a.workload == "c3_maxbin" else lf.synthetic_leafwise_trees
        forest = bench._lgb_forest(gen(1000, 255, 100, seed=1)[:a.trees], "first trees")[0]
    elif (a.trees or a.tree_start) and a.workload == "c4":
        t1 = a.tree_start + a.trees if a.trees else forest.n_trees
        forest = forest.tree_subset(a.tree_start, t1, keep_base=True)
    dev = DeviceForest(forest, [0])
    Xs = [bench.device_normal(a.rows, F, 3, "cuda:0", dtype)]
    Xs += [Xs[0].clone() for _ in range(max(0, a.x_buffers - 1))]
    it = [0]
    xdt = TI_F64 if dtype == "float64" else TI_F32
    S = max(1, a.streams)
    outs = [torch.empty(a.rows * forest.output_width(OUT_PREDICT),
                        dtype=torch.float64 if forest.accum_dtype else torch.float32, device="cuda")
            for _ in range(S)]
    cur = torch.cuda.current_stream()
    strs = [cur] + [torch.cuda.Stream() for _ in range(S - 1)]

    def step():
        X = Xs[it[0] % len(Xs)]
        k = it[0] % S
        it[0] += 1
        dev.predict_device(X.data_ptr(), xdt, a.rows, F, F, OUT_PREDICT, outs[k].data_ptr(),
                           outs[k].numel(), stream=strs[k].cuda_stream)
    for _ in range(S):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for st in strs[1:]:
        st.wait_stream(cur)
    for _ in range(a.steps):
        step()
    for st in strs[1:]:
        cur.wait_stream(st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    info = dev.info()
    print(json.dumps({"workload": a.workload, "rows": a.rows, "dtype": dtype, "trees": forest.n_trees,
                      "layout": bench.LAYOUT_NAMES.get(info["layout"]), "walk": info["walk"],
                      "bin_bits": info["bin_bits"], "tree_ilp": info["tree_ilp"],
                      "n_stages": info["n_stages"], "top_depth": info["top_depth"],
                      "bottom": info["bottom"], "streams": S, "kernel_ms": ms,
                      "rows_per_s": a.rows / (ms * 1e-3)}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
