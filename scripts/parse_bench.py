"""Host-side v1 body decode rates (libkfserve.so): json.loads + numpy vs the
one-thread native parser vs kf_parse_instances_mt, on 28-feature float32 rows
serialised by json.dumps.  One JSON line per (rows, threads)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kfserving_amd.kfserving.fastjson import parse_instances  # noqa: E402


def main():
    for rows in (64, 4096, 65536, 1_000_000):
        X = np.random.default_rng(rows).standard_normal((rows, 28)).astype(np.float32)
        body = json.dumps({"instances": X.tolist()}).encode()
        want = np.asarray(X, dtype=np.float64)
        if rows <= 65536:
            t0 = time.perf_counter()
            np.asarray(json.loads(body)["instances"], dtype=np.float64)
            ref_s = time.perf_counter() - t0
        else:
            ref_s = None
        for t in (1, 2, 4, 8, 16):
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                got = parse_instances(body, threads=t)
                best = min(best, time.perf_counter() - t0)
            assert got is not None and np.array_equal(np.asarray(got), want)
            print(json.dumps({"rows": rows, "body_MB": len(body) / 1e6, "threads": t,
                              "ms": best * 1e3, "rows_per_s": rows / best,
                              "GB_per_s": len(body) / best / 1e9,
                              "json_loads_ms": ref_s * 1e3 if ref_s else None}), flush=True)


if __name__ == "__main__":
    main()
