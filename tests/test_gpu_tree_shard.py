"""Tree-sharded predict on the GPU (one device here; the reduce itself is
covered with gloo in tests/test_tree_shard.py): the shards' partial margins,
summed, equal the one-device margins within 1e-5 (north_star), the library
transform (ti_transform_device) over the summed margins equals the one-device
predict within 1e-5 and labels exactly, shard leaf ids concatenate to the
full leaf ids, and shard TreeSHAP contributions sum to the full ones."""
import numpy as np
import pytest
import torch

from kfserving_amd.engine import DeviceForest
from kfserving_amd.forest import OUT_CONTRIB, OUT_LEAF, OUT_MARGIN, OUT_PREDICT
from kfserving_amd.formats import xgboost_format as xf
from kfserving_amd.tree_shard import TreeShardedForest, partition_trees

pytestmark = pytest.mark.gpu


def _forest(K, obj):
    trees, ti = xf.synthetic_complete_trees(120, 6, 16, seed=7, num_class=K)
    return xf.forest_from_raw_trees(trees, ti, 16, K, 0.5, obj)


@pytest.mark.parametrize("K,obj", [(0, "binary:logistic"), (5, "multi:softprob"),
                                   (5, "multi:softmax")])
@pytest.mark.parametrize("world", [2, 3])
def test_shards_sum_to_full(K, obj, world):
    f = _forest(K, obj)
    full = DeviceForest(f, [0])
    X = torch.randn(5000, 16, device="cuda")
    X[torch.rand_like(X) < 0.02] = float("nan")
    rows = X.shape[0]
    Kg = f.n_groups
    ref_m = torch.empty(rows * Kg, device="cuda")
    full.predict_device(X.data_ptr(), 0, rows, 16, 16, OUT_MARGIN, ref_m.data_ptr(), ref_m.numel())
    ref_p = torch.empty(rows * f.output_width(OUT_PREDICT), device="cuda")
    full.predict_device(X.data_ptr(), 0, rows, 16, 16, OUT_PREDICT, ref_p.data_ptr(),
                        ref_p.numel())
    acc = torch.zeros(rows * Kg, device="cuda")
    leaves = []
    engines = []
    for r, (a, b) in enumerate(partition_trees(f, world)):
        e = DeviceForest(f.tree_subset(a, b, keep_base=r == 0), [0])
        engines.append(e)
        part = torch.empty(rows * Kg, device="cuda")
        e.predict_device(X.data_ptr(), 0, rows, 16, 16, OUT_MARGIN, part.data_ptr(), part.numel())
        acc += part
        lv = torch.empty(rows * (b - a), dtype=torch.int32, device="cuda")
        e.predict_device(X.data_ptr(), 0, rows, 16, 16, OUT_LEAF, lv.data_ptr(), lv.numel())
        leaves.append(lv.reshape(rows, b - a))
    torch.testing.assert_close(acc, ref_m, rtol=1e-5, atol=1e-5)
    out = torch.empty_like(ref_p)
    engines[0].transform_device(acc.data_ptr(), rows, out.data_ptr(), out.numel())
    torch.cuda.synchronize()
    if obj == "multi:softmax":
        # labels exact wherever the top two margins are not within rounding
        top2 = ref_m.reshape(rows, Kg).topk(2, dim=1).values
        clear = (top2[:, 0] - top2[:, 1]) > 1e-4
        assert torch.equal(out[clear], ref_p[clear])
    else:
        torch.testing.assert_close(out, ref_p, rtol=1e-5, atol=1e-6)
    full_leaf = torch.empty(rows * f.n_trees, dtype=torch.int32, device="cuda")
    full.predict_device(X.data_ptr(), 0, rows, 16, 16, OUT_LEAF, full_leaf.data_ptr(),
                        full_leaf.numel())
    assert torch.equal(torch.cat(leaves, dim=1).reshape(-1), full_leaf)


def test_contributions_are_additive_over_shards():
    f = _forest(3, "multi:softprob")
    X = torch.randn(700, 16, device="cuda")
    W = f.output_width(OUT_CONTRIB)
    ref = torch.empty(700 * W, device="cuda")
    DeviceForest(f, [0]).predict_device(X.data_ptr(), 0, 700, 16, 16, OUT_CONTRIB,
                                        ref.data_ptr(), ref.numel())
    acc = torch.zeros_like(ref)
    for r, (a, b) in enumerate(partition_trees(f, 3)):
        part = torch.empty_like(ref)
        DeviceForest(f.tree_subset(a, b, keep_base=r == 0), [0]).predict_device(
            X.data_ptr(), 0, 700, 16, 16, OUT_CONTRIB, part.data_ptr(), part.numel())
        acc += part
    torch.testing.assert_close(acc, ref, rtol=1e-5, atol=1e-5)


def test_single_rank_sharded_forest_is_the_full_forest():
    f = _forest(0, "binary:logistic")
    ts = TreeShardedForest(f, device=0)
    X = torch.randn(1000, 16, device="cuda")
    p = ts.predict(X, OUT_PREDICT)
    want = DeviceForest(f, [0]).predict(X.cpu().numpy(), OUT_PREDICT)
    torch.testing.assert_close(p.cpu(), torch.from_numpy(want), rtol=1e-6, atol=1e-7)
    assert torch.equal(ts.predict(X, OUT_LEAF).cpu(),
                       torch.from_numpy(DeviceForest(f, [0]).predict(X.cpu().numpy(), OUT_LEAF)))


def test_transform_rejects_aliasing():
    from kfserving_amd.engine import TreeInferError
    f = _forest(0, "binary:logistic")
    e = DeviceForest(f, [0])
    m = torch.zeros(10, device="cuda")
    with pytest.raises(TreeInferError, match="alias"):
        e.transform_device(m.data_ptr(), 10, m.data_ptr(), 10)
