"""Round 6: host-buffer predict (pageable numpy -> pinned chunks -> H2D ->
kernel -> D2H -> numpy) for the bench's configs at several chunk sizes, with
and without the chunks aligned to whole launch rounds (TI_CHUNK_ROUNDS, a
developer knob), interleaved.  One JSON line per measurement."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
os.environ["TI_DEV_KNOBS"] = "1"

import numpy as np  # noqa: E402


def main():
    import kernel_workload as kw
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_PREDICT
    rows = 8_000_000
    for wl in ("c3", "c3_f64", "c2", "c4"):
        forest, F, dtype = kw.forest_of(wl)
        base = np.random.default_rng(3).standard_normal((500_000, F)).astype(dtype)
        X = np.tile(base, (rows // base.shape[0], 1))
        for rnd in range(2):
            for mb in (64, 128):
                for aligned in (1, 0):
                    os.environ["TI_CHUNK_MB"] = str(mb)
                    os.environ["TI_CHUNK_ROUNDS"] = str(aligned)
                    dev = DeviceForest(forest, [0])
                    dev.predict(X[:4096], OUT_PREDICT)
                    ts = []
                    for _ in range(3):
                        t0 = time.perf_counter()
                        dev.predict(X, OUT_PREDICT)
                        ts.append(time.perf_counter() - t0)
                    t = min(ts)
                    print(json.dumps({"workload": wl, "round": rnd, "chunk_mb": mb, "aligned": aligned,
                                      "rows": rows, "rows_per_s": rows / t,
                                      "input_GBps": X.nbytes / t / 1e9}), flush=True)
                    dev.close()
        del X


if __name__ == "__main__":
    main()
