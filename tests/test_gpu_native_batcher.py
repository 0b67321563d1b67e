"""The native batcher (include/kfbatch.h) in front of libtreeinfer on the GPU:
batches of many requests go to ti_predict through the function pointer, and
every request's rows come back bit-identical to a direct predict of them --
under the open-loop native load (kb_loadgen) and from asyncio submissions of
the three plugins' request kinds.  The CPU twin is tests/test_native_batcher.py."""
import asyncio
import os

import numpy as np
import pytest

from kfserving_amd.batcher.native import NativeBatcher, NativeModelBatcher
from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_MARGIN, OUT_PREDICT

pytestmark = pytest.mark.gpu


def _c2_like(trees=64, seed=5):
    from kfserving_amd.formats.xgboost_format import forest_from_raw_trees, synthetic_complete_trees
    t, ti = synthetic_complete_trees(trees, 8, 28, seed=seed)
    return forest_from_raw_trees(t, ti, 28, 0, 0.0, "binary:logistic")


@pytest.mark.parametrize("kind", [OUT_PREDICT, OUT_MARGIN])
def test_loadgen_outputs_equal_direct_predict(kind):
    dev = DeviceForest(_c2_like(), devices=[0])
    nb = NativeBatcher.for_device_forest(dev, 65536, 2, kind=kind)
    rng = np.random.default_rng(11)
    n = 3000
    arr = np.cumsum(rng.exponential(1 / 5000.0, n))
    sz = rng.integers(1, 65, n).astype(np.int32)
    pool = rng.standard_normal((8192, 28)).astype(np.float32)
    pool[rng.random(pool.shape) < 0.01] = np.nan
    lat, st, out, _ = nb.loadgen(arr, sz, pool)
    stats = nb.stats()
    nb.close()
    want = dev.predict(pool, kind).reshape(-1)
    assert (st == 0).all() and (lat > 0).all()
    assert stats["batches"] > 1 and stats["rows"] == int(sz.sum()) and stats["failed_batches"] == 0
    for i in range(n):
        off = (i * 64) % (8192 - 64)
        assert np.array_equal(out[i * 64:i * 64 + sz[i]], want[off:off + sz[i]]), i
    dev.close()


def test_full_batches_flush_at_max_rows():
    """MaxBatchSize flushes (handler.go:179): at 512 rows a batch, a burst of
    requests is answered by several full batches, each request exactly."""
    dev = DeviceForest(_c2_like(), devices=[0])
    nb = NativeBatcher.for_device_forest(dev, 512, 10_000)
    rng = np.random.default_rng(2)
    xs = [rng.standard_normal((int(r), 28)).astype(np.float32) for r in rng.integers(1, 65, 100)]

    async def go():   # the last, partial batch is flushed by drain
        futs = [nb.submit_nowait(x) for x in xs]
        await nb.drain()
        return [f.result() for f in futs]
    res = asyncio.run(go())
    stats = nb.stats()
    nb.close()
    assert stats["full_flushes"] >= 3
    for x, (out, bid) in zip(xs, res):
        assert np.array_equal(out, dev.predict(x, OUT_PREDICT)) and bid
    dev.close()


def test_plugins_through_native_model_batcher(golden, tmp_path):
    """NativeModelBatcher answers each plugin request kind with what the
    plugin's own predict answers for that request alone."""
    import shutil
    from kfserving_amd.kfserving.fastjson import JsonInstances
    from kfserving_amd.sklearnserver import SKLearnModel
    from kfserving_amd.xgbserver import XGBoostModel
    from tests.test_lgb_batching import _lgb_model, _requests

    d = tmp_path / "x"
    d.mkdir()
    shutil.copy(os.path.join(golden, "xgb_iris_legacy_082.bst"), str(d / "model.bst"))
    xgb = XGBoostModel("x", str(d), 1)
    xgb.load()
    d = tmp_path / "s"
    d.mkdir()
    shutil.copy(os.path.join(golden, "sk_rf_reg_model.npz"), str(d / "model.npz"))
    sk = SKLearnModel("s", str(d))
    sk.load()
    lgb = _lgb_model(golden, tmp_path, stub=False)
    rng = np.random.default_rng(4)

    async def go():
        out = {}
        bx = NativeModelBatcher(xgb, "instances", max_batch_size=64, max_latency_ms=5)
        reqs = [rng.uniform(0, 7, (int(r), 4)).round(1) for r in rng.integers(1, 9, 20)]
        for r in reqs:
            r[r < 1.0] = 0.0                      # DMatrix(list): 0 is missing
        res = await asyncio.gather(*[bx.submit(r.view(JsonInstances)) for r in reqs])
        out["xgb"] = [(xgb.predict({"instances": r.tolist()})["predictions"], b) for r, b in
                      zip(reqs, res)]
        bx.close()
        bs = NativeModelBatcher(sk, "instances", max_batch_size=64, max_latency_ms=5)
        g = np.load(os.path.join(golden, "sk_rf_reg.npz"))
        Xs = np.nan_to_num(g["X"][:40]).astype(np.float64)
        reqs = [Xs[i:i + 4] for i in range(0, 40, 4)]
        res = await asyncio.gather(*[bs.submit(r.tolist()) for r in reqs])
        out["sk"] = [(sk.predict({"instances": r.tolist()})["predictions"], b) for r, b in
                     zip(reqs, res)]
        bs.close()
        bl = NativeModelBatcher(lgb, "inputs", max_batch_size=64, max_latency_ms=5)
        reqs = _requests(12)
        res = await asyncio.gather(*[bl.submit(lgb.batch_inputs(r)) for r in reqs])
        out["lgb"] = [(lgb.predict(r)["predictions"], b) for r, b in zip(reqs, res)]
        bl.close()
        return out
    out = asyncio.run(go())
    for name, pairs in out.items():
        ids = {b["batchId"] for _, b in pairs}
        assert len(ids) < len(pairs), name                       # requests shared batches
        for want, b in pairs:
            assert b["message"] == "" and b["predictions"] == want, name
