"""Layout 9's compact u16 bottom (t16explicit_predict_kernel, round 5) and
its two-lanes-a-row walk (t16split_predict_kernel, round 6, the default;
TI_TX16_SPLIT=0 keeps the one-lane walk) against the C port of LightGBM's predict loop: zero-missing leaf-wise trees
of 255 leaves with NaN, +-0, the 1e-35 zero map, denormals and +-inf
(exercising the slow step's zero-flip table), ragged tiles, float32 and
float64 X, several top depths; raw scores bit-exact, leaf ids equal to the
record bottom's."""
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN
from kfserving_amd.formats import load_lightgbm_model
from kfserving_amd.formats import lightgbm_format as lf
from oracle import port

pytestmark = pytest.mark.gpu

SPECIALS = np.array([np.nan, 0.0, -0.0, 1e-40, -1e-36, 1e-35, 2e-35, np.inf, -np.inf])


def _forest(n_trees=41, leaves=255, F=40, seed=7, K=1):
    trees = lf.synthetic_leafwise_trees(n_trees, leaves, F, seed=seed)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, F, "binary sigmoid:1" if K == 1 else
                               f"multiclass num_class:{K}", num_class=K)
        return trees, load_lightgbm_model(p)


def _rows(n, F, seed, frac=0.15):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, F))
    m = rng.random(X.shape) < frac
    X[m] = SPECIALS[rng.integers(0, len(SPECIALS), m.sum())]
    return X


def _dev(f, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return DeviceForest(f, [0])
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("env,bottom", [({}, 3), ({"TI_TX_TOP": 0}, 3), ({"TI_TX_TOP": 4}, 3),
                                        ({"TI_TX16_SPLIT": 0}, 2),
                                        ({"TI_TX16_SPLIT": 0, "TI_TX_TOP": 0}, 2),
                                        ({"TI_TX16_SPLIT": 0, "TI_TX16_ILP": 4, "TI_TX_TOP": 6}, 2)],
                         ids=["split", "split-top0", "split-top4", "onelane", "onelane-top0",
                              "onelane-ilp4top6"])
def test_t16_bottoms_bit_exact(env, bottom):
    trees, f = _forest()
    dev = _dev(f, **env)
    rec = _dev(f, TI_TX16=0)
    assert dev.info()["layout"] == 9 and dev.info()["bottom"] == bottom
    assert rec.info()["bottom"] == 0
    for rows, seed in ((1, 1), (255, 256), (257, 3), (3000, 4)):
        X = _rows(rows, 40, seed)
        want = port.lgb_predict_raw(trees, 1, 40, X)[:, 0]
        assert np.array_equal(dev.predict(X, OUT_MARGIN), want), rows
        assert np.array_equal(dev.predict(X, OUT_LEAF), rec.predict(X, OUT_LEAF)), rows
        X32 = X.astype(np.float32)
        want32 = port.lgb_predict_raw(trees, 1, 40, X32.astype(np.float64))[:, 0]
        assert np.array_equal(dev.predict(X32, OUT_MARGIN), want32), rows
    # fast tiles only (no NaN, no exact zero)
    X = np.random.default_rng(9).standard_normal((2048, 40))
    assert np.array_equal(dev.predict(X, OUT_MARGIN), port.lgb_predict_raw(trees, 1, 40, X)[:, 0])


def test_t16_c3_shape_full_model():
    """C3's named model (1,000 x 255 leaves, 100 features) on 100k rows with 1 %
    specials, both u16 compact walks (two lanes a row, one lane a row)
    against the C port (the per-lane-progress walk measured 2.9x slower in
    round 5 was removed in round 6)."""
    import bench
    f, trees, _ = bench.c3_forest()
    rng = np.random.default_rng(11)
    X = rng.standard_normal((100_000, 100))
    m = rng.random(X.shape) < 0.01
    X[m] = SPECIALS[rng.integers(0, len(SPECIALS), m.sum())]
    want = port.lgb_predict_raw(trees, 1, 100, X)[:, 0]
    for env, bottom in (({}, 3), ({"TI_TX16_SPLIT": 0}, 2)):
        dev = _dev(f, **env)
        assert dev.info()["bottom"] == bottom
        assert np.array_equal(dev.predict(X, OUT_MARGIN), want), env
        dev.close()


@pytest.mark.parametrize("n_trees", [24, 37])
def test_t16_split_multiclass_tree_order(n_trees):
    """Three classes (tree t adds to class t mod 3): the split walk's lower
    lane adds its own four trees then its partner's, so every class's float64
    sum keeps LightGBM's tree order; a tree count that leaves a ragged last
    group (37) checks the padding trees add nothing."""
    trees, f = _forest(n_trees=n_trees, leaves=255, F=40, seed=11, K=3)
    dev = _dev(f)
    one = _dev(f, TI_TX16_SPLIT=0)
    assert dev.info()["bottom"] == 3 and one.info()["bottom"] == 2
    for rows, seed in ((1, 1), (300, 2), (2049, 3)):
        X = _rows(rows, 40, seed)
        want = port.lgb_predict_raw(trees, 3, 40, X)
        got = dev.predict(X, OUT_MARGIN).reshape(rows, 3)
        assert np.array_equal(got, want), rows
        assert np.array_equal(dev.predict(X, OUT_LEAF), one.predict(X, OUT_LEAF)), rows
