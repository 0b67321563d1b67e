"""TreeSHAP contributions (TI_OUTPUT_CONTRIB) on the C2 model: rows/s of
ti_predict_device at a few batch sizes with each kernel -- the coefficient
table and the per-row extend / unwind arithmetic, chosen per forest with
ti_forest_set_option(TI_OPT_SHAP_TABLE_ROWS) -- one JSON line each, with the
table's bytes and build time (ti_forest_info) and whether the
two kernels' contributions are bit-identical.

Usage: python scripts/shap_bench.py [--rows 4096,16384,100000] [--reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="4096,16384,100000")
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    import torch
    import bench
    from kfserving_amd.engine import OPT_SHAP_TABLE_ROWS, DeviceForest
    from kfserving_amd.forest import OUT_CONTRIB, TI_F32
    _, _, forest = bench.build_model()
    dev = DeviceForest(forest, [0])
    W = forest.output_width(OUT_CONTRIB)
    sh = torch.cuda.current_stream().cuda_stream
    for n in [int(x) for x in a.rows.split(",")]:
        X = bench.device_normal(n, bench.N_FEAT, 5, "cuda:0")
        outs = {}
        for kernel in ("table", "arith"):
            dev.set_option(OPT_SHAP_TABLE_ROWS, 1 << 40 if kernel == "table" else 0)
            out = torch.empty(n * W, dtype=torch.float32, device="cuda")

            def run():
                dev.predict_device(X.data_ptr(), TI_F32, n, bench.N_FEAT, bench.N_FEAT,
                                   OUT_CONTRIB, out.data_ptr(), out.numel(), stream=sh)
            run()                      # the first table use builds it
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            info = dev.info()
            outs[kernel] = out
            print(json.dumps({"rows": n, "kernel": kernel, "ms": ms, "rows_per_s": n / (ms * 1e-3),
                              "shap_table": info["shap_table"],
                              "table_MiB": info["shap_table_bytes"] / 2**20,
                              "table_build_ms": info["shap_table_build_ms"]}), flush=True)
        print(json.dumps({"rows": n, "bit_identical": bool(torch.equal(outs["table"], outs["arith"]))}),
              flush=True)
    dev.close()


if __name__ == "__main__":
    main()
