"""Forests with more than 16 outputs per row (the kernels' register budget):
the library splits them into parts of at most 16 groups (treeinfer.hip,
create_chunked) and runs the output transform over the assembled margins.
Margins and leaf ids bit-exact, probabilities within 1e-5 (north_star), class
labels exact -- for scalar leaves (XGBoost / LightGBM multiclass: a part holds
its groups' trees in order) and vector leaves (sklearn classifier: every part
holds every tree, with a slice of each leaf vector)."""
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN, OUT_PREDICT
from kfserving_amd.formats import load_lightgbm_model
from kfserving_amd.formats import lightgbm_format as lf
from kfserving_amd.formats import xgboost_format as xf
from oracle import lgb_ref, xgb_ref

pytestmark = pytest.mark.gpu
RTOL = 1e-5


@pytest.mark.parametrize("objective", ["multi:softprob", "multi:softmax"])
def test_xgboost_20_classes(objective):
    K = 20
    trees, ti = xf.synthetic_complete_trees(K * 6, 5, 16, seed=4, num_class=K)
    forest = xf.forest_from_raw_trees(trees, ti, 16, K, 0.5, objective)
    ref = xgb_ref.from_raw_trees(trees, ti, 16, K, 0.5, objective)
    dev = DeviceForest(forest, [0])
    assert dev.info()["n_groups"] == K
    rng = np.random.default_rng(5)
    X = rng.standard_normal((3001, 16)).astype(np.float32)
    X[rng.random(X.shape) < 0.02] = np.nan
    margin = dev.predict(X, OUT_MARGIN)
    assert margin.shape == (3001, K)
    assert np.array_equal(margin, xgb_ref.predict(ref, X, output_margin=True))
    assert np.array_equal(dev.predict(X, OUT_LEAF), xgb_ref.leaf_index(ref, X))
    pred = dev.predict(X, OUT_PREDICT)
    want = xgb_ref.predict(ref, X)
    if objective == "multi:softmax":
        assert np.array_equal(pred, want)                  # labels exact
    else:
        np.testing.assert_allclose(pred, want, rtol=RTOL)


def test_lightgbm_18_classes_explicit():
    K = 18
    trees = lf.synthetic_leafwise_trees(K * 4, 31, 12, seed=9)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 12, f"multiclass num_class:{K}", num_class=K)
        f = load_lightgbm_model(p)
        m = lgb_ref.read_lgb_text(p)
    dev = DeviceForest(f, [0])
    X = np.random.default_rng(6).standard_normal((2000, 12))
    X[::7, 3] = 0.0
    X[::11, 5] = np.nan
    assert np.array_equal(dev.predict(X, OUT_MARGIN), lgb_ref.predict(m, X, raw_score=True))
    assert np.array_equal(dev.predict(X, OUT_LEAF), lgb_ref.leaf_index(m, X))
    np.testing.assert_allclose(dev.predict(X, OUT_PREDICT), lgb_ref.predict(m, X), rtol=RTOL)


def test_sklearn_classifier_20_classes_vector_leaves():
    from sklearn.ensemble import RandomForestClassifier
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn
    rng = np.random.default_rng(7)
    Xtr = rng.standard_normal((3000, 10)).astype(np.float32)
    ytr = (np.floor((Xtr[:, 0] + 3) * 3.3).astype(int) % 20)
    est = RandomForestClassifier(n_estimators=12, max_depth=10, random_state=0).fit(Xtr, ytr)
    assert len(est.classes_) == 20
    f = forest_from_sklearn(est)
    assert f.leaf_width == 20
    dev = DeviceForest(f, [0])
    X = rng.standard_normal((2500, 10)).astype(np.float32)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), est.predict_proba(X))
    lab = f.meta["classes"].take(dev.predict(X, OUT_PREDICT).astype(np.int64))
    assert np.array_equal(lab, est.predict(X))
    assert np.array_equal(dev.predict(X, OUT_LEAF), est.apply(X))


def test_many_groups_device_path_and_sharding():
    K = 33
    trees, ti = xf.synthetic_complete_trees(K * 2, 4, 8, seed=11, num_class=K)
    forest = xf.forest_from_raw_trees(trees, ti, 8, K, 0.5, "multi:softprob")
    ref = xgb_ref.from_raw_trees(trees, ti, 8, K, 0.5, "multi:softprob")
    X = np.random.default_rng(8).standard_normal((1001, 8)).astype(np.float32)
    dev2 = DeviceForest(forest, [0, 0])          # two slots: rows sharded
    assert np.array_equal(dev2.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))
    import torch
    Xt = torch.from_numpy(X).cuda()
    out = torch.empty((1001, K), dtype=torch.float32, device="cuda")
    dev = DeviceForest(forest, [0])
    s = torch.cuda.current_stream()
    dev.predict_device(Xt.data_ptr(), 0, 1001, 8, 8, OUT_PREDICT, out.data_ptr(), out.numel(),
                       stream=s.cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_allclose(out.cpu().numpy(), xgb_ref.predict(ref, X), rtol=RTOL)
