"""the host-buffer predict path of C2 (ti_predict from
pageable numpy to numpy, PCIe-inclusive) with the caller's buffers
page-locked for the call (TI_HOST_REGISTER=1: H2D / D2H straight from / into
them, predict_registered) against the pinned-chunk pipeline (0: every byte
copied once on the host into 64 MB pinned chunks), interleaved, on 8M and
32M rows.  One JSON line per timing."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import bench
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_PREDICT
    _, _, forest = bench.build_model()
    dev = DeviceForest(forest, [0])
    base = np.random.default_rng(0).standard_normal((1_000_000, bench.N_FEAT), dtype=np.float32)
    for rows in (8_000_000, 32_000_000):
        X = np.tile(base, (rows // base.shape[0], 1))
        ref = None
        for rep in range(3):
            for v in ("0", "1"):
                os.environ["TI_HOST_REGISTER"] = v
                dev.predict(X[:4096], OUT_PREDICT)
                t0 = time.perf_counter()
                out = dev.predict(X, OUT_PREDICT)
                dt = time.perf_counter() - t0
                same = True if ref is None else bool(np.array_equal(out, ref))
                ref = out if ref is None else ref
                print(json.dumps({"rows": rows, "host_register": int(v), "rep": rep, "ms": dt * 1e3,
                                  "rows_per_s": rows / dt, "input_GBps": X.nbytes / dt / 1e9,
                                  "same_as_first": same}), flush=True)
        del X


if __name__ == "__main__":
    main()
