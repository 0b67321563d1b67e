"""Layout 9 plan sweep on one workload in one process: the forest and the
device batch are built once, then for every setting of the TI_* knobs read
at ti_forest_create (TI_TX8, TI_TX_TOP, TI_LX_ILP, TI_RX_ROWS8 ...) a new
DeviceForest is created and its kernel timed with HIP events on the launch
stream.  One JSON line per setting.

Usage: python scripts/tx_sweep.py --workload c3_maxbin --grid 'TI_TX8=0,1;TI_TX_TOP=5,6,7,8'
"""
import argparse
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="c3_maxbin")
    p.add_argument("--rows", type=int, default=1_000_000)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--grid", required=True)
    a = p.parse_args()
    import torch
    import bench
    import kernel_workload as kw
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_PREDICT, TI_F32, TI_F64
    forest, F, dtype = kw.forest_of(a.workload)
    X = bench.device_normal(a.rows, F, 3, "cuda:0", dtype)
    xdt = TI_F64 if dtype == "float64" else TI_F32
    out = torch.empty(a.rows * forest.output_width(OUT_PREDICT),
                      dtype=torch.float64 if forest.accum_dtype else torch.float32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    axes = []
    for part in a.grid.split(";"):
        k, vs = part.split("=")
        axes.append([(k.strip(), v.strip()) for v in vs.split(",")])
    ref = None
    for combo in itertools.product(*axes):
        for k, v in combo:
            os.environ[k] = v
        dev = DeviceForest(forest, [0])

        def step():
            dev.predict_device(X.data_ptr(), xdt, a.rows, F, F, OUT_PREDICT, out.data_ptr(),
                               out.numel(), stream=sh)
        step()
        torch.cuda.synchronize()
        same = None
        if ref is None:
            ref = out.clone()
        else:
            same = bool(torch.equal(out, ref))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        info = dev.info()
        print(json.dumps({"workload": a.workload, **dict(combo), "layout": info["layout"],
                          "bin_bits": info["bin_bits"], "tree_ilp": info["tree_ilp"],
                          "n_stages": info["n_stages"], "top_depth": info["top_depth"],
                          "bottom": info["bottom"], "kernel_ms": ms,
                          "rows_per_s": a.rows / (ms * 1e-3), "same_as_first": same}),
              flush=True)
        dev.close()
        for k, _ in combo:
            del os.environ[k]


if __name__ == "__main__":
    main()
