"""Randomised parity on the GPU (round 6): seeded forests of every shape the
engine's layouts branch on -- LightGBM leaf-wise trees with i.i.d. (u16 bins)
or max_bin-style (u8 bins) thresholds, 1 to 40 trees (fewer than a group of
the two-lanes-a-row walk, one group plus one, several stages), stumps to 255
leaves, 1 to 120 features, 1 or 3 classes, every missing type, float32 and
float64 rows with NaN / +-0 / +-inf / 1e-36, row counts that end inside a
tile; and XGBoost complete trees of depth 1 to 8 -- against the C
restatement of each library's predict loop (oracle/c/tree_port.c): raw
scores bit-exact, leaf ids equal to the canonical evaluator's
(tests/canon_eval.py)."""
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN
from kfserving_amd.formats import load_lightgbm_model
from kfserving_amd.formats import lightgbm_format as lf
from oracle import port
from tests import canon_eval

pytestmark = pytest.mark.gpu

SPECIALS = np.array([np.nan, 0.0, -0.0, 1e-36, -1e-40, np.inf, -np.inf])


def _rows(rng, n, F, dtype, frac):
    X = rng.standard_normal((n, F))
    m = rng.random(X.shape) < frac
    X[m] = SPECIALS[rng.integers(0, len(SPECIALS), m.sum())]
    return X.astype(dtype)


def _env(seed):
    """Every other case forces a layout or a walk (developer knobs; the
    conftest sets TI_DEV_KNOBS), so each kernel family meets random shapes."""
    return FORCED[(seed // 2) % len(FORCED)] if seed % 2 == 1 else {}


def _lgb_case(seed):
    rng = np.random.default_rng([seed, 61])
    T = int(rng.choice([1, 2, 3, 7, 9, 17, 40]))
    leaves = int(rng.choice([2, 3, 17, 128, 255]))
    F = int(rng.choice([1, 3, 28, 100, 120]))
    K = int(rng.choice([1, 1, 3]))
    maxbin = bool(rng.integers(0, 2))
    if "TI_TX16_SPLIT" in _env(seed):   # the one-lane u16 walk: i.i.d. thresholds
        maxbin, leaves = False, 255
    mts = [(lf.MISSING_NONE,), (lf.MISSING_ZERO,), (lf.MISSING_NAN,),
           (lf.MISSING_NONE, lf.MISSING_ZERO, lf.MISSING_NAN)][int(rng.integers(0, 4))]
    if maxbin:
        trees = lf.synthetic_maxbin_trees(T * K, leaves, F, seed=seed,
                                          max_bin=125 if lf.MISSING_ZERO in mts else 255,
                                          missing_types=mts)
    else:
        trees = lf.synthetic_leafwise_trees(T * K, leaves, F, seed=seed, missing_types=mts)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, F, "binary sigmoid:1" if K == 1 else
                               f"multiclass num_class:{K}", num_class=K)
        f = load_lightgbm_model(p)
    return rng, trees, f, F, K, dict(T=T * K, leaves=leaves, F=F, K=K, maxbin=maxbin, mts=mts)


FORCED = [{}, {"TI_TX16_SPLIT": "0"}, {"TI_FORCE_LAYOUT": "lexplicit"},
          {"TI_FORCE_LAYOUT": "rexplicit"}, {"TI_FORCE_LAYOUT": "hexplicit"},
          {"TI_FORCE_LAYOUT": "explicit"}, {"TI_TX8": "0"}, {"TI_TX16": "0"}]


@pytest.mark.parametrize("seed", range(64))
def test_fuzz_lightgbm_forests(seed, monkeypatch):
    rng, trees, f, F, K, desc = _lgb_case(seed)
    env = _env(seed)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    desc["env"] = env
    dev = DeviceForest(f, [0])
    info = dev.info()
    try:
        for n in (1, int(rng.integers(2, 300)), int(rng.integers(300, 3000))):
            for dt in (np.float64, np.float32):
                X = _rows(rng, n, F, dt, float(rng.choice([0.0, 0.02, 0.2])))
                want = port.lgb_predict_raw(trees, K, F, X.astype(np.float64))
                got = dev.predict(X, OUT_MARGIN).reshape(n, K)
                assert np.array_equal(got, want), (desc, info, n, dt)
                leaf = dev.predict(X, OUT_LEAF)
                assert np.array_equal(leaf, canon_eval.predict(f, X, OUT_LEAF)), (desc, info, n, dt)
    finally:
        dev.close()


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_xgboost_complete_trees(seed):
    from kfserving_amd.formats.xgboost_format import forest_from_raw_trees, synthetic_complete_trees
    from oracle import xgb_ref
    rng = np.random.default_rng([seed, 62])
    T = int(rng.choice([1, 3, 5, 33, 64]))
    depth = int(rng.integers(1, 9))
    F = int(rng.choice([1, 4, 28, 60]))
    trees, ti = synthetic_complete_trees(T, depth, F, seed=seed)
    f = forest_from_raw_trees(trees, ti, F, 0, 0.5, "binary:logistic")
    ref = xgb_ref.from_raw_trees(trees, ti, F, 0, 0.5, "binary:logistic")
    dev = DeviceForest(f, [0])
    try:
        for n in (1, int(rng.integers(2, 600)), int(rng.integers(600, 5000))):
            X = _rows(rng, n, F, np.float32, float(rng.choice([0.0, 0.05])))
            assert np.array_equal(dev.predict(X, OUT_MARGIN),
                                  xgb_ref.predict(ref, X, output_margin=True)), (T, depth, F, n)
            assert np.array_equal(dev.predict(X, OUT_LEAF), xgb_ref.leaf_index(ref, X)), (T, depth, F, n)
    finally:
        dev.close()


def test_fuzz_cases_reach_every_walk(monkeypatch):
    """The seeds above land on the walks they are meant to cover: layout 9
    with the u16 bottom two lanes a row (3) and one lane a row (2), the u8
    compact bottom (1) and records (0), and the record layouts 6, 7, 8 and
    the float explicit layout 1."""
    seen = set()
    for seed in range(64):
        _, _, f, _, _, _ = _lgb_case(seed)
        env = _env(seed)
        with monkeypatch.context() as m:
            for k, v in env.items():
                m.setenv(k, v)
            dev = DeviceForest(f, [0])
            info = dev.info()
            dev.close()
        seen.add((info["layout"], info["bottom"] if info["layout"] == 9 else -1))
    want = {(9, 3), (9, 2), (9, 1), (9, 0), (7, -1), (6, -1), (8, -1), (1, -1)}
    assert want <= seen, sorted(seen)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_sklearn_forests_vs_sklearn(seed, monkeypatch):
    """Random sklearn forests fitted here (RandomForest / ExtraTrees,
    regressor / classifier, depth 1 to unlimited, 1 to 20 estimators, 1 to 40
    features), every other one on a forced layout, checked against sklearn
    1.7.2's own predict / predict_proba / apply on rows with NaN (the trees'
    missing_go_to_left)."""
    from sklearn.ensemble import (ExtraTreesClassifier, ExtraTreesRegressor,
                                  RandomForestClassifier, RandomForestRegressor)
    from kfserving_amd.forest import OUT_PREDICT
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn
    rng = np.random.default_rng([seed, 63])
    F = int(rng.choice([1, 7, 40]))
    n_est = int(rng.choice([1, 5, 20]))
    depth = [1, 4, 12, None][int(rng.integers(0, 4))]
    kind = int(rng.integers(0, 4))
    Xt = rng.standard_normal((1500, F)).astype(np.float32)
    if kind < 2:
        y = Xt[:, 0] * 2 + np.sin(Xt[:, -1] * 3) + rng.normal(0, 0.3, 1500)
        Est = RandomForestRegressor if kind == 0 else ExtraTreesRegressor
    else:
        y = (Xt[:, 0] + rng.normal(0, 0.5, 1500) > 0).astype(int) + (Xt[:, -1] > 1).astype(int)
        Est = RandomForestClassifier if kind == 2 else ExtraTreesClassifier
    est = Est(n_estimators=n_est, max_depth=depth, max_leaf_nodes=None if depth else 300,
              random_state=seed, n_jobs=1).fit(Xt, y)
    if seed % 2 == 1:
        monkeypatch.setenv("TI_FORCE_LAYOUT", ["rexplicit", "lexplicit", "texplicit",
                                               "explicit"][(seed // 2) % 4])
    f = forest_from_sklearn(est)
    dev = DeviceForest(f, [0])
    try:
        for n in (1, 257, 3001):
            X = rng.standard_normal((n, F)).astype(np.float32)
            X[rng.random(X.shape) < 0.02] = np.nan
            if kind < 2:
                assert np.array_equal(dev.predict(X, OUT_PREDICT), est.predict(X)), (seed, n)
            else:
                got = dev.predict(X, OUT_MARGIN).reshape(n, -1)
                assert np.array_equal(got, est.predict_proba(X)), (seed, n)
            assert np.array_equal(dev.predict(X, OUT_LEAF), est.apply(X)), (seed, n)
    finally:
        dev.close()
