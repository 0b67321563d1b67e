"""The host-buffer predict path (ti_predict) on batches larger than one chunk:
chunks alternate between two streams with bounded pinned buffers
(treeinfer.hip predict_pipelined).  TI_CHUNK_MB=1 makes a 50,003-row C2-shaped
batch six chunks, the last one ragged; results are bit-exact against the C
port and against one device-resident launch."""
import os

import numpy as np
import pytest
import torch

from kfserving_amd.engine import OPT_HOST_REGISTER, DeviceForest
from kfserving_amd.formats.xgboost_format import forest_from_raw_trees, synthetic_complete_trees
from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN, OUT_PREDICT, TI_F32
from oracle import port

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_chunks():
    old = os.environ.get("TI_CHUNK_MB")
    os.environ["TI_CHUNK_MB"] = "1"
    yield
    if old is None:
        del os.environ["TI_CHUNK_MB"]
    else:
        os.environ["TI_CHUNK_MB"] = old


def test_chunked_host_predict_bit_exact(small_chunks):
    trees, ti = synthetic_complete_trees(100, 8, 28, seed=4)
    f = forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    dev = DeviceForest(f, [0])
    rows = 50_003                            # > 5 chunks of 9,216 rows
    X = np.random.default_rng(5).standard_normal((rows, 28)).astype(np.float32)
    X[np.random.default_rng(6).random(X.shape) < 0.01] = np.nan
    got = dev.predict(X, OUT_MARGIN)
    assert np.array_equal(got, port.xgb_predict(trees, ti, 1, 0.0, 28, X)[:, 0])
    # one device-resident launch over the whole batch
    Xd = torch.from_numpy(X).cuda()
    out = torch.empty(rows, dtype=torch.float32, device="cuda")
    dev.predict_device(Xd.data_ptr(), TI_F32, rows, 28, 28, OUT_MARGIN, out.data_ptr(), rows,
                       stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(got, out.cpu().numpy())
    # leaf ids (int32, 100 per row) and the transformed output through the same path
    leaf = dev.predict(X, OUT_LEAF)
    assert leaf.shape == (rows, 100)
    assert np.array_equal(leaf[-9000:], DeviceForest(f, [0]).predict(X[-9000:], OUT_LEAF))
    prob = dev.predict(X, OUT_PREDICT)
    np.testing.assert_allclose(prob, 1 / (1 + np.exp(-got.astype(np.float64))), rtol=1e-5)
    # twice: the lanes' buffers are reused
    assert np.array_equal(dev.predict(X, OUT_MARGIN), got)


@pytest.mark.parametrize("strided", [False, True])
def test_registered_host_predict_bit_exact(small_chunks, strided):
    """TI_OPT_HOST_REGISTER=1: the caller's X and out page-locked for the
    call, chunks copied straight from / into them (predict_registered), the
    same bits as the pinned-chunk pipeline; a row stride and a ragged last
    chunk."""
    trees, ti = synthetic_complete_trees(100, 8, 28, seed=4)
    f = forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    dev = DeviceForest(f, [0])
    rows = 40_001
    W = np.random.default_rng(7).standard_normal((rows, 32 if strided else 28)).astype(np.float32)
    X = W[:, :28]
    want = port.xgb_predict(trees, ti, 1, 0.0, 28, np.ascontiguousarray(X))[:, 0]
    dev.set_option(OPT_HOST_REGISTER, 1)
    lib, ptr = dev._lib, lambda a: a.ctypes.data
    out = np.empty(rows, dtype=np.float32)
    rc = lib.ti_predict(dev._handle, ptr(W), TI_F32, rows, 28, W.shape[1], OUT_MARGIN, ptr(out), rows)
    assert rc == 0
    assert np.array_equal(out, want)
    assert np.array_equal(dev.predict(np.ascontiguousarray(X), OUT_MARGIN), want)   # reused lanes
    leaf = dev.predict(np.ascontiguousarray(X), OUT_LEAF)
    dev.set_option(OPT_HOST_REGISTER, 0)
    assert np.array_equal(leaf, dev.predict(np.ascontiguousarray(X), OUT_LEAF))


def test_registered_host_predict_multi_device_and_already_registered(small_chunks):
    """with several device slots the whole batch is page-locked
    once before the shard threads start (slices sharing boundary pages used
    to register and unregister them per thread); a buffer whose pages are
    already registered by someone else is not used for direct DMA (the
    pinned staging chunks take it).  Bit-exact against the C port both ways."""
    trees, ti = synthetic_complete_trees(60, 8, 28, seed=8)
    f = forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
    dev = DeviceForest(f, [0, 0, 0])           # three slots: 3 shard threads
    dev.set_option(OPT_HOST_REGISTER, 1)
    rows = 61_111                              # 20,371 a slot: > 2 chunks each, ragged
    X = np.random.default_rng(9).standard_normal((rows, 28)).astype(np.float32)
    want = port.xgb_predict(trees, ti, 1, 0.0, 28, X)[:, 0]
    for _ in range(2):
        assert np.array_equal(dev.predict(X, OUT_MARGIN), want)
    # X registered by another owner for the duration: the call must not rely
    # on (or unregister) those pages
    cudart = torch.cuda.cudart()
    assert int(cudart.cudaHostRegister(X.ctypes.data, X.nbytes, 0)) == 0
    try:
        assert np.array_equal(dev.predict(X, OUT_MARGIN), want)
        one = DeviceForest(f, [0])
        one.set_option(OPT_HOST_REGISTER, 1)
        assert np.array_equal(one.predict(X, OUT_MARGIN), want)
        one.close()
    finally:
        assert int(cudart.cudaHostUnregister(X.ctypes.data)) == 0
    dev.close()
