"""On the GPU: the kernels the engine picks for the bench's forests are the
ones the committed PMC passes were taken on (bench.pmc_mismatch), so the
driver's bench line carries a roofline and not an `error`."""
import os

import pytest

import bench

pytestmark = pytest.mark.gpu


def _info(forest):
    from kfserving_amd.engine import DeviceForest
    dev = DeviceForest(forest, devices=[0])
    try:
        return dev.info()
    finally:
        dev.close()


def test_c2_launch_matches_pmc_pass():
    _, _, forest = bench.build_model()
    info = _info(forest)
    pmc = bench.load_pmc(bench.pmc_path("c2"))
    assert bench.pmc_mismatch(pmc, "c2", bench.ROWS, info) is None, info
    rf = bench.roofline(0.72, bench.ROWS, info, bench.pmc_path("c2"))
    assert rf["frac"] and rf["traffic"] and rf["lds_bank_conflict_frac"] is not None


@pytest.mark.parametrize("key", ["c3", "c3_maxbin", "c4"])
def test_config_launch_matches_pmc_pass(key):
    forest = {"c3": bench.c3_forest, "c3_maxbin": bench.c3_maxbin_forest,
              "c4": bench.c4_forest}[key]()[0]
    info = _info(forest)
    pmc = bench.load_pmc(bench.pmc_path(key))
    assert bench.pmc_mismatch(pmc, key, None, info) is None, info


def test_headline_two_streams_same_outputs():
    """The headline's batches in flight (--streams 2) compute every row: each
    stream's output equals the others' bit for bit, the one-stream kernel time
    is reported beside, and value = rows x steps / the multi-stream wall."""
    args = bench.parse_args(["--steps", "6", "--warmup", "2", "--rows", "262144", "--configs", "",
                             "--no-cpu-baseline", "--latency-qps", "0", "--host-rows", "0",
                             "--nan-variant", "0", "--streams", "2"])
    line = bench.run(args)
    assert line["config"]["streams"] == 2
    assert line["streams_outputs_identical"] is True
    ss = line["single_stream"]
    assert ss["kernel_ms"] > 0 and ss["ms_per_step"] > 0
    assert abs(line["value"] - 262144 * 6 / (line["ms_per_step"] * 6e-3)) < 1e-6 * line["value"]
    assert line["roofline"]["kernel_ms"] == ss["kernel_ms"]


@pytest.mark.parametrize("key", ["c2", "c2_hist", "c3", "c3_f64", "c3_maxbin", "c4"])
def test_pmc_pass_duration_matches_this_box(key):
    """a committed PMC pass prices the launch bench.py
    times only if its profiled kernel duration (the pass's own
    --kernel-trace) is within 10 % of the same kernel timed here with HIP
    events on its launch stream, on the same 1M-row workload as
    scripts/kernel_workload.py (its forest, dtype and seed)."""
    import sys
    import torch
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "scripts"))
    import kernel_workload as kw
    from kfserving_amd.engine import DeviceForest
    from kfserving_amd.forest import OUT_PREDICT, TI_F32, TI_F64
    forest, F, dtype = kw.forest_of(key)
    pmc = bench.load_pmc(bench.pmc_path(key))
    rows = int(pmc["rows"])
    dev = DeviceForest(forest, [0])
    try:
        assert bench.pmc_mismatch(pmc, key, rows, dev.info()) is None
        X = bench.device_normal(rows, F, 3, "cuda:0", dtype)
        out = torch.empty(rows * forest.output_width(OUT_PREDICT),
                          dtype=torch.float64 if forest.accum_dtype else torch.float32,
                          device="cuda")
        xdt = TI_F64 if dtype == "float64" else TI_F32
        st = torch.cuda.current_stream()

        def step():
            dev.predict_device(X.data_ptr(), xdt, rows, F, F, OUT_PREDICT, out.data_ptr(),
                               out.numel(), stream=st.cuda_stream)
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
    finally:
        dev.close()
    prof_ms = pmc["profiled_kernel_ns"] / 1e6
    assert abs(ms - prof_ms) <= 0.10 * prof_ms, (key, ms, prof_ms)
