"""TreeSHAP contributions (TI_OUTPUT_CONTRIB) on the C2 model: rows/s of
ti_predict_device at a few batch sizes, one JSON line each.  TI_SHAP_TABLE_MB
(read when the forest first computes contributions) selects the coefficient
table (default) or the per-row extend / unwind (0); --dump saves the first
batch's contributions (.npy), so two runs can be compared bit for bit.

Usage: python scripts/shap_bench.py [--rows 4096,100000,1000000] [--dump out.npy]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="4096,100000,1000000")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--dump", default=None)
    a = p.parse_args()
    import torch
    import bench
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_CONTRIB, TI_F32
    _, _, forest = bench.build_model()
    dev = DeviceForest(forest, [0])
    W = forest.output_width(OUT_CONTRIB)
    sh = torch.cuda.current_stream().cuda_stream
    for n in [int(x) for x in a.rows.split(",")]:
        X = bench.device_normal(n, bench.N_FEAT, 5, "cuda:0")
        out = torch.empty(n * W, dtype=torch.float32, device="cuda")
        dev.predict_device(X.data_ptr(), TI_F32, n, bench.N_FEAT, bench.N_FEAT, OUT_CONTRIB,
                           out.data_ptr(), out.numel(), stream=sh)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            dev.predict_device(X.data_ptr(), TI_F32, n, bench.N_FEAT, bench.N_FEAT, OUT_CONTRIB,
                               out.data_ptr(), out.numel(), stream=sh)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        line = {"rows": n, "ms": ms, "rows_per_s": n / (ms * 1e-3),
                "table_mb_env": os.environ.get("TI_SHAP_TABLE_MB", "2048 (default)"),
                "checksum": float(out.double().sum().item())}
        print(json.dumps(line), flush=True)
        if a.dump:
            import numpy as np
            np.save(a.dump, out.cpu().numpy())
            a.dump = None
    dev.close()


if __name__ == "__main__":
    main()
