"""GPU parity of the binned heap layout (rank-binned features, 4-byte nodes).

The binned kernel replaces every float compare ``x <= t`` by an integer
compare of ranks, so these tests aim at the places where that could go
wrong: values exactly at a threshold and one ulp either side, ±0, ±inf,
NaN, denormals, thresholds of -inf (xgboost's NaN canonical threshold), both
bin widths (u8 when every feature has <= 253 distinct thresholds, u16
otherwise), wide rows (smaller tiles), float64 inputs (their own ranks), and
float64 accumulation.  Oracle: the numpy / C restatements (oracle/).
"""
import os
import tempfile

import numpy as np
import pytest

from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN, OUT_PREDICT
from kfserving_amd.formats import load_lightgbm_model
from kfserving_amd.formats import lightgbm_format as lf
from kfserving_amd.formats import xgboost_format as xf
from oracle import port, xgb_ref

pytestmark = pytest.mark.gpu

BHEAP = 3


def _xgb(n_trees, depth, F, seed, quantize=None, num_class=0, neg_inf=0.0):
    trees, ti = xf.synthetic_complete_trees(n_trees, depth, F, seed=seed, num_class=num_class)
    n_int = (1 << depth) - 1
    rng = np.random.default_rng(seed + 100)
    for t in trees:
        v = t["value"][:n_int]
        if quantize:
            v[:] = np.round(v * quantize) / quantize
        if neg_inf:
            v[rng.random(n_int) < neg_inf] = -np.inf
    obj = "multi:softprob" if num_class else "binary:logistic"
    forest = xf.forest_from_raw_trees(trees, ti, F, num_class, 0.5, obj)
    ref = xgb_ref.from_raw_trees(trees, ti, F, num_class, 0.5, obj)
    return trees, ti, forest, ref


def _edge_rows(trees, depth, F, n, seed):
    """Rows mixing N(0,1) values, exact thresholds, their float32 neighbours and
    specials."""
    rng = np.random.default_rng(seed)
    n_int = (1 << depth) - 1
    thr = np.concatenate([t["value"][:n_int] for t in trees]).astype(np.float32)
    thr = thr[np.isfinite(thr)]
    X = rng.standard_normal((n, F)).astype(np.float32)
    pick = rng.random(X.shape)
    at = thr[rng.integers(0, len(thr), X.shape)]
    X = np.where(pick < 0.25, at, X)
    X = np.where((pick >= 0.25) & (pick < 0.35), np.nextafter(at, np.float32(np.inf)), X)
    X = np.where((pick >= 0.35) & (pick < 0.45), np.nextafter(at, np.float32(-np.inf)), X)
    sp = np.array([np.nan, 0.0, -0.0, 1e-40, -1e-40, np.inf, -np.inf], dtype=np.float32)
    m = rng.random(X.shape) < 0.05
    X[m] = sp[rng.integers(0, len(sp), m.sum())]
    return X.astype(np.float32)


@pytest.mark.parametrize("quantize", [16, None], ids=["u8", "u16"])
def test_bheap_edges_both_widths(quantize):
    trees, ti, forest, ref = _xgb(64, 8, 28, seed=31, quantize=quantize, neg_inf=0.02)
    dev = DeviceForest(forest, [0])
    assert dev.info()["layout"] == BHEAP
    for rows in (1, 255, 256, 257, 5000):
        X = _edge_rows(trees, 8, 28, rows, seed=rows)
        assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))
        assert np.array_equal(dev.predict(X, OUT_LEAF), xgb_ref.leaf_index(ref, X))
    # NaN-free tiles take the fast path: check it separately
    X = _edge_rows(trees, 8, 28, 3000, seed=9)
    X[~np.isfinite(X)] = 0.5
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))


def test_bheap_float64_input_has_own_ranks():
    # float64 inputs compare in float64 (their own rank tables): values between
    # two float32 neighbours of a threshold separate only in that view.  The
    # float-compare heap kernel is the reference for the float64 semantics.
    trees, ti, forest, ref = _xgb(32, 6, 12, seed=7)
    dev = DeviceForest(forest, [0])
    assert dev.info()["layout"] == BHEAP
    old = os.environ.get("TI_FORCE_LAYOUT")
    os.environ["TI_FORCE_LAYOUT"] = "heap"
    try:
        heap = DeviceForest(forest, [0])
    finally:
        if old is None:
            del os.environ["TI_FORCE_LAYOUT"]
        else:
            os.environ["TI_FORCE_LAYOUT"] = old
    assert heap.info()["layout"] == 0
    X = _edge_rows(trees, 6, 12, 2000, seed=3).astype(np.float64)
    X[::3] -= 1e-12
    X[1::3] += 1e-12
    assert np.array_equal(dev.predict(X, OUT_MARGIN), heap.predict(X, OUT_MARGIN))
    assert np.array_equal(dev.predict(X, OUT_LEAF), heap.predict(X, OUT_LEAF))
    # on float32-exact values the float64 path agrees with xgboost's float32 one
    X32 = X.astype(np.float32)
    assert np.array_equal(dev.predict(X32.astype(np.float64), OUT_MARGIN),
                          xgb_ref.predict(ref, X32, output_margin=True))


def test_bheap_wide_rows_small_tiles():
    # F = 100 with u16 bins -> 50 words/row: 128-row tiles keep node offsets in 15 bits
    trees, ti, forest, ref = _xgb(40, 7, 100, seed=11)
    dev = DeviceForest(forest, [0])
    assert dev.info()["layout"] == BHEAP
    X = _edge_rows(trees, 7, 100, 3001, seed=4)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))


def test_bheap_stumps_and_multiclass():
    trees, ti, forest, ref = _xgb(30, 1, 5, seed=2)
    dev = DeviceForest(forest, [0])
    assert dev.info()["layout"] == BHEAP and dev.info()["depth"] == 1
    X = _edge_rows(trees, 1, 5, 999, seed=5)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))
    trees, ti, forest, ref = _xgb(45, 5, 16, seed=3, num_class=3)
    dev = DeviceForest(forest, [0])
    assert dev.info()["layout"] == BHEAP
    X = _edge_rows(trees, 5, 16, 1500, seed=6)
    assert np.array_equal(dev.predict(X, OUT_MARGIN), xgb_ref.predict(ref, X, output_margin=True))
    np.testing.assert_allclose(dev.predict(X, OUT_PREDICT), xgb_ref.predict(ref, X), rtol=1e-5)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_bheap_lightgbm_float64_accumulation(dtype):
    # shallow leaf-wise trees without Zero-missing nodes qualify for the
    # binned heap; float64 leaves, float64 sums in tree order
    trees = lf.synthetic_leafwise_trees(50, 12, 20, seed=8,
                                        missing_types=(lf.MISSING_NONE, lf.MISSING_NAN))
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 20, "binary sigmoid:1")
        f = load_lightgbm_model(p)
    dev = DeviceForest(f, [0])
    if f.depths().max() > 8:
        pytest.skip("generator drew a tree deeper than 8")
    assert dev.info()["layout"] == BHEAP
    rng = np.random.default_rng(12)
    X = rng.standard_normal((4000, 20))
    sp = np.array([np.nan, 0.0, -0.0, 1e-40, 1e-36, np.inf, -np.inf])
    m = rng.random(X.shape) < 0.08
    X[m] = sp[rng.integers(0, len(sp), m.sum())]
    X = X.astype(dtype)
    want = port.lgb_predict_raw(trees, 1, 20, X.astype(np.float64))[:, 0]
    assert np.array_equal(dev.predict(X, OUT_MARGIN), want)


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("ng", ["1", "2"])
@pytest.mark.parametrize("quantize", [16, None], ids=["u8", "u16"])
def test_bheap_fixed_walk(quantize, ng):
    """The fixed-layout walk (bheap_fix_kernel: compile-time LDS addresses, the
    pair address from the node word's heap index) against the oracle and the
    indexed walk: a partial last stage (37 trees), shallow trees padded to
    depth 8, NaN and NaN-free tiles, ragged tiles of the 512-row layout, one
    and four stage groups, u8 and u16 bins, and a multiclass forest (tree
    groups, KMAX 4)."""
    deep, ti_d = xf.synthetic_complete_trees(30, 8, 28, seed=41)
    shallow, ti_s = xf.synthetic_complete_trees(7, 3, 28, seed=42)
    trees = deep[:20] + shallow + deep[20:]
    ti = np.concatenate([ti_d[:20], ti_s, ti_d[20:]])
    if quantize:                                    # <= 253 thresholds per feature: u8 bins
        for t in trees:
            v = t["value"][:int((t["cleft"] >= 0).sum())]
            v[:] = np.round(v * quantize) / quantize
    forest = xf.forest_from_raw_trees(trees, ti, 28, 0, 0.5, "binary:logistic")
    ref = xgb_ref.from_raw_trees(trees, ti, 28, 0, 0.5, "binary:logistic")
    env = {"TI_BHEAP_NG": ng}
    dev = _with_env(env, lambda: DeviceForest(forest, [0]))
    inf = dev.info()
    assert inf["layout"] == BHEAP and inf["walk"] == 2 and inf["depth"] == 8
    assert inf["bin_bits"] == (8 if quantize else 16)
    for rows in (1, 511, 512, 513, 4097):
        X = _edge_rows(deep, 8, 28, rows, seed=rows + 3)
        got = _with_env(env, lambda: dev.predict(X, OUT_MARGIN))
        assert np.array_equal(got, xgb_ref.predict(ref, X, output_margin=True)), rows
        np.testing.assert_allclose(_with_env(env, lambda: dev.predict(X, OUT_PREDICT)),
                                   xgb_ref.predict(ref, X), rtol=1e-5, atol=0)
        idx = _with_env({"TI_BHEAP_FIX": "0"}, lambda: dev.predict(X, OUT_MARGIN))
        assert np.array_equal(got, idx)
    X = _edge_rows(deep, 8, 28, 3000, seed=9)
    X[~np.isfinite(X)] = 0.25                       # every tile on the fast step
    assert np.array_equal(_with_env(env, lambda: dev.predict(X, OUT_MARGIN)),
                          xgb_ref.predict(ref, X, output_margin=True))
    # multiclass: 3 groups of depth-8 trees, LW = 1 (tree_group per tree)
    trees3, ti3 = xf.synthetic_complete_trees(27, 8, 28, seed=43, num_class=3)
    f3 = xf.forest_from_raw_trees(trees3, ti3, 28, 3, 0.5, "multi:softprob")
    r3 = xgb_ref.from_raw_trees(trees3, ti3, 28, 3, 0.5, "multi:softprob")
    d3 = _with_env(env, lambda: DeviceForest(f3, [0]))
    assert d3.info()["walk"] == 2
    X = _edge_rows(trees3, 8, 28, 2049, seed=11)
    assert np.array_equal(_with_env(env, lambda: d3.predict(X, OUT_MARGIN)),
                          xgb_ref.predict(r3, X, output_margin=True))
    np.testing.assert_allclose(_with_env(env, lambda: d3.predict(X, OUT_PREDICT)),
                               xgb_ref.predict(r3, X), rtol=1e-5, atol=0)
    # leaf ids keep the indexed walk
    assert np.array_equal(dev.predict(X[:, :28], OUT_LEAF), xgb_ref.leaf_index(ref, X[:, :28]))


def test_fix_image_uploaded_once_and_freed():
    # the fixed walk's permuted image was uploaded inside the
    # per-view loop, so each replica held (and leaked) a second copy.  With
    # the permutation on, a replica holds exactly one more tree image than
    # without it, and create/predict/destroy cycles give the memory back.
    import torch
    trees, ti, forest, ref = _xgb(500, 8, 28, seed=5)
    X = _edge_rows(trees, 8, 28, 1024, seed=2)

    def make(perm):
        d = _with_env({"TI_FIX_PERM": perm}, lambda: DeviceForest(forest, [0]))
        d.predict(X, OUT_MARGIN)              # the replica is created on first use
        return d

    on, off = make("1"), make("0")
    ion, ioff = on.info(), off.info()
    assert ion["walk"] == 2 and ion["tree_stride_bytes"] > 0
    assert ion["device_bytes"] - ioff["device_bytes"] == 500 * ion["tree_stride_bytes"]
    on.close()
    off.close()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    for _ in range(8):
        make("1").close()
    torch.cuda.synchronize()
    # 8 leaked 1 MB images would show; allow the allocator's own slack
    assert free0 - torch.cuda.mem_get_info(0)[0] < 4 * 500 * ion["tree_stride_bytes"]
