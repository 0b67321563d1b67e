"""Tree-sharded predict (kfserving_amd/tree_shard.py) on CPU: gloo, world
size 2 and 3, with a stand-in engine that evaluates each rank's slice of the
trees with the canonical restatement (tests/canon_eval.py).  Checks the tree
partition, base margin on the root only, the sum-reduce of partial margins
(within 1e-5 of the one-device margins, north_star), the gathered leaf ids
(exact) and the transform on the root."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN, OUT_PREDICT
from kfserving_amd.formats import xgboost_format as xf
from kfserving_amd.tree_shard import partition_trees
from tests import canon_eval


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _view(ptr, n, dtype):
    ct = {np.float32: ctypes.c_float, np.float64: ctypes.c_double, np.int32: ctypes.c_int32}[dtype]
    return np.ctypeslib.as_array((ct * n).from_address(ptr))


class CanonEngine:
    """Stands in for DeviceForest on CPU tensors (same predict_device /
    transform_device signatures)."""

    def __init__(self, forest, device):
        self.f = forest

    def predict_device(self, x_ptr, xdt, rows, cols, stride, kind, out_ptr, out_len, slot=0,
                       stream=0):
        X = _view(x_ptr, rows * stride, np.float32 if xdt == 0 else np.float64)
        X = X.reshape(rows, stride)[:, :cols].astype(np.float64)
        res = canon_eval.predict(self.f, X, kind)
        dt = np.int32 if kind == OUT_LEAF else np.float32
        _view(out_ptr, out_len, dt)[:] = np.asarray(res, dtype=dt).reshape(-1)

    def transform_device(self, m_ptr, rows, out_ptr, out_len, slot=0, stream=0):
        m = _view(m_ptr, rows * self.f.n_groups, np.float32)
        _view(out_ptr, out_len, np.float32)[:] = np.asarray(
            canon_eval.transform(self.f, m), np.float32).reshape(-1)


def _forest(K):
    trees, ti = xf.synthetic_complete_trees(24 if K else 17, 4, 6, seed=3, num_class=K)
    return xf.forest_from_raw_trees(trees, ti, 6, K, 0.5,
                                    "multi:softprob" if K else "binary:logistic")


def _worker(rank, world, port, K, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def no_all_gather(*a, **k):   # leaf ids go to the root alone
        raise AssertionError("tree_shard must gather to the root, not all_gather")
    dist.all_gather = no_all_gather
    from kfserving_amd.tree_shard import TreeShardedForest
    f = _forest(K)
    ts = TreeShardedForest(f, engine_factory=CanonEngine)
    X = torch.from_numpy(np.random.default_rng(0).standard_normal((300, 6)).astype(np.float32))
    res = {k: ts.predict(X, k) for k in (OUT_MARGIN, OUT_PREDICT, OUT_LEAF)}
    out = {k: (None if v is None else v.numpy()) for k, v in res.items()}
    q.put((rank, ts.ranges, float(ts.local_forest.base_margin.sum()), out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,K", [(2, 0), (3, 4)])
def test_tree_sharded_predict(world, K):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    f = _forest(K)
    X = np.random.default_rng(0).standard_normal((300, 6)).astype(np.float32).astype(np.float64)
    ranges = res[0][1]
    assert ranges[0][0] == 0 and ranges[-1][1] == f.n_trees
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert res[0][2] == float(f.base_margin.sum()) and all(r[2] == 0.0 for r in res[1:])
    root = res[0][3]
    assert all(v is None for r in res[1:] for v in r[3].values())
    m_full = canon_eval.predict(f, X, OUT_MARGIN).reshape(300, -1)
    np.testing.assert_allclose(root[OUT_MARGIN].reshape(300, -1), m_full, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(root[OUT_PREDICT].reshape(300, -1),
                               canon_eval.predict(f, X, OUT_PREDICT).reshape(300, -1),
                               rtol=1e-5, atol=1e-6)
    assert np.array_equal(root[OUT_LEAF], canon_eval.predict(f, X, OUT_LEAF))


def test_partition_balances_nodes_and_covers_every_tree():
    f = _forest(0)
    for world in (1, 2, 5, 17):
        r = partition_trees(f, world)
        assert len(r) == world and r[0][0] == 0 and r[-1][1] == f.n_trees
        assert all(b > a for a, b in r)
    with pytest.raises(ValueError):
        partition_trees(f, f.n_trees + 1)


def test_tree_subset_keeps_groups_and_zeroes_base():
    f = _forest(4)
    s = f.tree_subset(5, 13, keep_base=False)
    assert s.n_trees == 8 and np.all(s.base_margin == 0)
    assert np.array_equal(s.tree_group, f.tree_group[5:13])
    X = np.random.default_rng(1).standard_normal((50, 6))
    assert np.array_equal(canon_eval.predict(s, X, OUT_LEAF),
                          canon_eval.predict(f, X, OUT_LEAF)[:, 5:13])
