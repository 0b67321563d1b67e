"""Batched-latency leg of bench.py at several offered loads, GC frozen or not."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402  (torch's HIP runtime first)
import bench  # noqa: E402
from kfserving_amd.engine import DeviceForest  # noqa: E402

_, _, forest = bench.build_model()
dev = DeviceForest(forest, [0])
for qps in (2000, 10000, 20000):
    for fz in (False, True):
        r = bench.batched_latency(dev, bench.N_FEAT, qps, 3.0, freeze_gc=fz)
        print(json.dumps({k: r[k] for k in ("qps_offered", "gc_frozen", "p50_ms", "p90_ms",
                                           "p99_ms", "max_ms", "rows_per_s", "mean_batch_rows",
                                           "predict_ms_p50", "predict_ms_p99")}), flush=True)
