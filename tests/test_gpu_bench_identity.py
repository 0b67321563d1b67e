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
