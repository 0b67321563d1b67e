"""Interleaved A/B of C2 kernel variants in one process (cdna_hip_programming.md
7: "interleaved A/B in one process").  The engine reads TI_BHEAP_FIX and
TI_BHEAP_NG at every launch, so those variants share one forest replica and the same three 1M-row device batches (KARY=0 selects a second replica built
with Eytzinger instead of 5-ary rank tables: TI_KARY is read at create time);
each round times
every setting for --steps launches with HIP events on the launch stream, and
the medians over rounds are printed, one JSON line per setting, with a check
that every setting's margins equal the first's.

Usage: python scripts/c2_ab.py [--settings "FIX=1,NG=1;FIX=0"] [--nan 0.0]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

KNOBS = {"FIX": "TI_BHEAP_FIX", "NG": "TI_BHEAP_NG"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--settings", default="FIX=1,NG=1;FIX=1,NG=2;FIX=0")
    p.add_argument("--rows", type=int, default=1_000_000)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--nan", type=float, default=0.0)
    a = p.parse_args()
    import torch
    import bench
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_MARGIN, TI_F32
    _, _, forest = bench.build_model()
    dev = DeviceForest(forest, [0])
    os.environ["TI_KARY"] = "0"
    dev_eyt = DeviceForest(forest, [0])
    del os.environ["TI_KARY"]
    rng = np.random.default_rng(1000)
    Xh = rng.standard_normal((a.rows, bench.N_FEAT), dtype=np.float32)
    if a.nan > 0:
        Xh[np.random.default_rng(2).random(Xh.shape) < a.nan] = np.nan
    Xs = [torch.from_numpy(Xh).cuda()]
    Xs += [Xs[0].clone() for _ in range(2)]
    out = torch.empty(a.rows, dtype=torch.float32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    settings = [dict(kv.split("=") for kv in s.split(",")) for s in a.settings.split(";")]

    def apply(st):
        for k, env in KNOBS.items():
            if k in st:
                os.environ[env] = st[k]
            else:
                os.environ.pop(env, None)

    times = [[] for _ in settings]
    ref = None
    same = [True] * len(settings)
    for r in range(a.rounds):
        for i, st in enumerate(settings):
            apply(st)
            d = dev_eyt if st.get("KARY") == "0" else dev
            for j in range(2):
                d.predict_device(Xs[j % 3].data_ptr(), TI_F32, a.rows, bench.N_FEAT,
                                   bench.N_FEAT, OUT_MARGIN, out.data_ptr(), a.rows, stream=sh)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for j in range(a.steps):
                d.predict_device(Xs[j % 3].data_ptr(), TI_F32, a.rows, bench.N_FEAT,
                                   bench.N_FEAT, OUT_MARGIN, out.data_ptr(), a.rows, stream=sh)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.steps)
            if r == 0:
                d.predict_device(Xs[0].data_ptr(), TI_F32, a.rows, bench.N_FEAT, bench.N_FEAT,
                                   OUT_MARGIN, out.data_ptr(), a.rows, stream=sh)
                torch.cuda.synchronize()
                o = out.cpu().numpy().copy()
                if ref is None:
                    ref = o
                same[i] = bool(np.array_equal(o, ref))
    for i, st in enumerate(settings):
        ms = float(np.median(times[i]))
        print(json.dumps({"setting": st, "kernel_ms_median": ms, "kernel_ms_all": times[i],
                          "rows_per_s": a.rows / (ms * 1e-3), "nan": a.nan,
                          "same_as_first": same[i]}), flush=True)
    dev.close()
    dev_eyt.close()


if __name__ == "__main__":
    main()
