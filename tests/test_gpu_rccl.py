"""The RCCL collectives of the multi-GPU path on the box's one GPU: a world-1
process group over the nccl backend (RCCL on ROCm, as bench.py and
tree_shard.py open it at N > 1: init_process_group("nccl", device_id=...)),
then every collective those paths issue, on device tensors of the shapes and
dtypes they pass:
  * bench.max_over_ranks: all_reduce(MAX) of a float64 wall time;
  * bench.barrier_sync: barrier;
  * TreeShardedForest.predict: reduce(SUM) of the [rows, K] float32 partial
    margins to the root, after the engine wrote them on torch's stream;
  * TreeShardedForest._gather_leaves: gather of [rows, tmax] int32 leaf ids.
At world 1 each is an identity, which the test checks; world > 1 needs the
driver's node.  Runs in a spawned process so the group does not
outlive the test."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1",
                          RANK="0", LOCAL_RANK="0")
        import torch
        import torch.distributed as dist
        import bench
        from kfserving_amd.engine import DeviceForest
        from kfserving_amd.forest import OUT_LEAF, OUT_MARGIN, TI_F32
        from kfserving_amd.formats.xgboost_format import (forest_from_raw_trees,
                                                          synthetic_complete_trees)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda:0"))
        out = {"backend": dist.get_backend()}
        # bench.max_over_ranks / barrier_sync
        out["max_over_ranks"] = bench.max_over_ranks(1.25, "cuda:0")
        t = torch.tensor([1.25], dtype=torch.float64, device="cuda:0")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out["all_reduce_max"] = float(t.item())
        dist.barrier()
        # the tree-shard reduce and gather on engine outputs
        trees, ti = synthetic_complete_trees(40, 6, 28, seed=3)
        forest = forest_from_raw_trees(trees, ti, 28, 0, 0.0, "binary:logistic")
        dev = DeviceForest(forest, [0])
        rows = 4096
        X = bench.device_normal(rows, 28, 9, "cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        part = torch.empty((rows, 1), dtype=torch.float32, device="cuda:0")
        dev.predict_device(X.data_ptr(), TI_F32, rows, 28, 28, OUT_MARGIN, part.data_ptr(),
                           part.numel(), stream=st)
        want = part.clone()
        dist.reduce(part, dst=0, op=dist.ReduceOp.SUM)
        out["reduce_identity"] = bool(torch.equal(part, want))
        leaves = torch.empty((rows, 40), dtype=torch.int32, device="cuda:0")
        dev.predict_device(X.data_ptr(), TI_F32, rows, 28, 28, OUT_LEAF, leaves.data_ptr(),
                           leaves.numel(), stream=st)
        bufs = [torch.empty_like(leaves)]
        dist.gather(leaves, gather_list=bufs, dst=0)
        out["gather_identity"] = bool(torch.equal(bufs[0], leaves))
        out["leaves_in_range"] = bool((leaves >= 0).all().item())
        torch.cuda.synchronize()
        dev.close()
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as e:   # surfaced in the parent
        q.put((None, repr(e)))


def test_rccl_world1_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    out, err = q.get(timeout=110)
    p.join(timeout=30)
    assert err is None, err
    assert out["backend"] == "nccl"
    assert out["max_over_ranks"] == 1.25 and out["all_reduce_max"] == 1.25
    assert out["reduce_identity"] and out["gather_identity"] and out["leaves_in_range"], out
