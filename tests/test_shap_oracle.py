"""Pin the TreeSHAP restatement (oracle/shap_ref.py) without xgboost: on small
forests its contributions equal the Shapley values of the path-dependent value
function computed by brute-force subset enumeration, and on every forest they
satisfy efficiency (sum of contributions + bias == margin)."""
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.forest import OUT_MARGIN
from kfserving_amd.formats import load_lightgbm_model
from kfserving_amd.formats import lightgbm_format as lf
from kfserving_amd.formats import xgboost_format as xf
from kfserving_amd.formats.sklearn_format import forest_from_sklearn
from oracle import shap_ref
from tests import canon_eval


def _xgb(n_trees, depth, F, seed, K=0):
    trees, ti = xf.synthetic_complete_trees(n_trees, depth, F, seed=seed, num_class=K)
    obj = "multi:softprob" if K else "binary:logistic"
    return xf.forest_from_raw_trees(trees, ti, F, K, 0.5, obj)


def _lgb(n_trees, leaves, F, seed, K=1):
    trees = lf.synthetic_leafwise_trees(n_trees, leaves, F, seed=seed)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "m.txt")
        obj = f"multiclass num_class:{K}" if K > 1 else "binary sigmoid:1"
        lf.write_lightgbm_text(p, trees, F, obj, num_class=K)
        return load_lightgbm_model(p)


def _rows(F, n, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, F))
    X[rng.random(X.shape) < 0.1] = np.nan
    X[rng.random(X.shape) < 0.1] = 0.0
    return X.astype(np.float32).astype(np.float64)


def _sk_forest():
    from sklearn.ensemble import RandomForestClassifier
    rng = np.random.default_rng(3)
    X = rng.standard_normal((200, 4)).astype(np.float32)
    y = (X[:, 0] > 0).astype(int) + (X[:, 1] > 0.5).astype(int)
    est = RandomForestClassifier(n_estimators=3, max_depth=4, random_state=0).fit(X, y)
    return forest_from_sklearn(est)


@pytest.mark.parametrize("make", [
    lambda: _xgb(3, 3, 4, seed=1),
    lambda: _xgb(4, 2, 3, seed=2, K=2),
    lambda: _lgb(3, 7, 4, seed=3),
    lambda: _sk_forest(),
], ids=["xgb", "xgb-multiclass", "lgb-zero-missing", "sklearn-vector-leaves"])
def test_restatement_equals_brute_force_shapley(make):
    f = make()
    X = _rows(f.n_features, 12, seed=5)
    got = shap_ref.contributions(f, X)
    for r in range(X.shape[0]):
        np.testing.assert_allclose(got[r], shap_ref.brute_force(f, X[r]), rtol=1e-10,
                                   atol=1e-12)


@pytest.mark.parametrize("make", [
    lambda: _xgb(20, 5, 8, seed=4),
    lambda: _lgb(10, 31, 8, seed=6, K=3),
    lambda: _sk_forest(),
], ids=["xgb", "lgb-multiclass", "sklearn"])
def test_efficiency(make):
    f = make()
    X = _rows(f.n_features, 40, seed=7)
    c = shap_ref.contributions(f, X).reshape(X.shape[0], f.n_groups, f.n_features + 1)
    margin = canon_eval.predict(f, X, OUT_MARGIN).reshape(X.shape[0], f.n_groups)
    np.testing.assert_allclose(c.sum(axis=2), margin, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("make", [
    lambda: _xgb(20, 6, 8, seed=4),
    lambda: _xgb(6, 4, 5, seed=8, K=3),
    lambda: _lgb(10, 63, 12, seed=6, K=3),
    lambda: _sk_forest(),
], ids=["xgb", "xgb-multiclass", "lgb-multiclass", "sklearn"])
def test_c_port_matches_restatement(make):
    """oracle/c/shap_port.c (the CPU baseline) == the numpy restatement."""
    from oracle import port
    f = make()
    X = _rows(f.n_features, 50, seed=9)
    np.testing.assert_allclose(port.tree_shap(f, X, nthread=2), shap_ref.contributions(f, X),
                               rtol=1e-12, atol=1e-12)
