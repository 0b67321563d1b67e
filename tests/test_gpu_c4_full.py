"""C4 at its named model size on the GPU (BASELINE.json configs[3]): a
200-tree, max_depth-16 sklearn RandomForestRegressor on 64 features, checked
bit for bit against sklearn's own predict() and apply() on 4,096 rows with
1 % NaN.  The model and sklearn's outputs come from
scripts/make_c4_model.py (bench_data/, git-ignored, travels with the tree);
without that cache the test fits the same estimator on 5,000 rows here."""
import os
import sys

import numpy as np
import pytest

from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_LEAF, OUT_PREDICT

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def _c4():
    import make_c4_model as mk
    from kfserving_amd.formats.sklearn_format import forest_from_sklearn, load_tree_arrays
    if os.path.exists(mk.MODEL) and os.path.exists(mk.CHECK):
        z = np.load(mk.CHECK, allow_pickle=False)
        return load_tree_arrays(mk.MODEL), z["X"], z["predict"], z["apply"], "cached"
    est = mk.fit(5_000, os.cpu_count() or 1)
    est.set_params(n_jobs=1)
    X = mk.check_rows()
    return forest_from_sklearn(est), X, est.predict(X), est.apply(X), "fitted"


@pytest.mark.parametrize("layout", [None, "rexplicit"])
def test_c4_full_model_bit_exact_vs_sklearn(layout, monkeypatch):
    """The default layout (8: heap tops in LDS, gathered bottoms) and layout 6."""
    f, X, want, leaves, src = _c4()
    assert f.n_trees == 200 and f.n_features == 64 and f.depths().max() == 16
    assert np.isnan(X).any() and X.shape[0] >= 4096
    if layout:
        monkeypatch.setenv("TI_FORCE_LAYOUT", layout)
    dev = DeviceForest(f, [0])
    assert dev.info()["layout"] == (6 if layout else 8)
    assert np.array_equal(dev.predict(X, OUT_PREDICT), want), src
    assert np.array_equal(dev.predict(X, OUT_LEAF), leaves), src
    dev.close()


def test_c4_row_shards_cut_mid_tile():
    """ti_predict with three device slots (all on GPU 0): the row blocks
    (1,366 rows each) end inside a 256-row tile; the result equals one slot."""
    f, X, want, _, _ = _c4()
    X = X[:4097]
    one = DeviceForest(f, [0])
    three = DeviceForest(f, [0, 0, 0])
    assert three.info()["n_devices"] == 3
    assert np.array_equal(three.predict(X, OUT_PREDICT), one.predict(X, OUT_PREDICT))
    assert np.array_equal(three.predict(X, OUT_PREDICT), want[:4097])
    assert np.array_equal(three.predict(X, OUT_LEAF), one.predict(X, OUT_LEAF))
