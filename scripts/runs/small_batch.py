"""Latency of one ti_predict call on host buffers (the serving path: pinned
copy, H2D, kernel, D2H) for C2 at serving batch sizes, one JSON line per
size: median / p99 over --reps calls, plus the kernel alone on a device
buffer (HIP events).  TI_BHEAP_ROWS (the binned heap's rows per tile, fixed
when the forest is created) is read from the environment, so running this
under several values compares tile sizes for small batches.

Usage: TI_BHEAP_ROWS=64 python scripts/small_batch.py [--reps 300]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=300)
    p.add_argument("--sizes", default="64,512,1024,2048,4096,8192,16384,65536")
    a = p.parse_args()
    import torch
    import bench
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_PREDICT, TI_F32
    _, _, forest = bench.build_model()
    dev = DeviceForest(forest, [0])
    info = dev.info()
    X = np.random.default_rng(0).standard_normal((65536, bench.N_FEAT), dtype=np.float32)
    Xd = torch.from_numpy(X).cuda()
    out = torch.empty(65536, dtype=torch.float32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    for n in [int(s) for s in a.sizes.split(",")]:
        Xn = np.ascontiguousarray(X[:n])
        for _ in range(10):
            dev.predict(Xn, OUT_PREDICT)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            dev.predict(Xn, OUT_PREDICT)
            ts.append((time.perf_counter() - t0) * 1e3)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dev.predict_device(Xd.data_ptr(), TI_F32, n, bench.N_FEAT, bench.N_FEAT, OUT_PREDICT,
                           out.data_ptr(), n, stream=sh)
        e0.record()
        for _ in range(20):
            dev.predict_device(Xd.data_ptr(), TI_F32, n, bench.N_FEAT, bench.N_FEAT, OUT_PREDICT,
                               out.data_ptr(), n, stream=sh)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"rows": n, "tile_rows_env": os.environ.get("TI_BHEAP_ROWS"),
                          "walk": info.get("walk"), "call_ms_p50": float(np.percentile(ts, 50)),
                          "call_ms_p99": float(np.percentile(ts, 99)),
                          "kernel_ms": e0.elapsed_time(e1) / 20}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
