"""Explicit-layout sweep on one GPU: C3 (LightGBM leaf-wise 1000 x 255 leaves,
F = 100) and C4 (the cached sklearn RandomForest, scripts/make_c4_model.py)
on 1M-row device batches, for several (layout, ILP) settings.  Every setting
is checked bit for bit against the first one's output.  One JSON line each.

Usage: python scripts/explicit_sweep.py [--configs c3,c4] [--rows N]
       [--settings "rexplicit:16,lexplicit:8,lexplicit:4,rexplicit:8"]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def c3_forest(n_trees=1000):
    from kfserving_amd.formats import lightgbm_format as lf
    trees = lf.synthetic_leafwise_trees(1000, 255, 100, seed=1)[:n_trees]
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 100, "binary sigmoid:1")
        return lf.load_lightgbm_model(p), 100


def c4_forest():
    import make_c4_model as mk
    from kfserving_amd.formats.sklearn_format import load_tree_arrays
    return load_tree_arrays(mk.MODEL), 64


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="c3,c4")
    p.add_argument("--rows", type=int, default=1_000_000)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--nan", type=float, default=0.0)
    p.add_argument("--trees", type=int, default=0, help="C3: the first N trees only (0 = all)")
    p.add_argument("--settings", default="rexplicit:16,lexplicit:8,lexplicit:4,rexplicit:8")
    a = p.parse_args()
    import torch
    from bench_configs import device_normal, time_device
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_MARGIN, TI_F32
    for c in a.configs.split(","):
        f, F = (c3_forest(a.trees) if c == "c3" and a.trees else
                {"c3": c3_forest, "c4": c4_forest}[c]())
        X = device_normal(a.rows, F, seed=3)
        if a.nan > 0:
            g = torch.Generator(device="cuda")
            g.manual_seed(11)
            X[torch.rand(X.shape, generator=g, device="cuda") < a.nan] = float("nan")
        ref = None
        for s in a.settings.split(","):
            lay, ilp, *extra = s.split(":")
            for kv in extra:   # per-setting env knobs, e.g. lexplicit:8:TI_LX_WGS=3
                k, v = kv.split("=")
                os.environ[k] = v
            os.environ["TI_FORCE_LAYOUT"] = lay
            os.environ["TI_RX_ILP"] = ilp
            os.environ["TI_BEXP_ILP"] = ilp
            os.environ["TI_LX_ILP"] = ilp
            dev = DeviceForest(f, [0])
            out = torch.empty(a.rows, dtype=torch.float64, device="cuda")
            step_s, kms = time_device(dev, X, out, a.rows, F, OUT_MARGIN, TI_F32, a.steps, 1)
            o = out.cpu().numpy()
            if ref is None:
                ref = o
            print(json.dumps({"config": c, "layout": lay, "got_layout": dev.info()["layout"],
                              "ilp": int(ilp), "env": extra, "rows": a.rows, "nan": a.nan,
                              "trees": a.trees or None, "kernel_ms": kms,
                              "rows_per_s": a.rows / (kms * 1e-3),
                              "same_as_first": bool(np.array_equal(o, ref))}), flush=True)
            dev.close()
            for kv in extra:
                del os.environ[kv.split("=")[0]]
        del X


if __name__ == "__main__":
    main()
