"""Tree-sharded predict for ensembles too large for one GPU (SURVEY.md §8(e),
the north_star's "very large ensembles may instead shard trees and sum
margins with an RCCL reduce over xGMI").

Rows are the natural shard (bench.py, DeviceForest with several devices): the
forest is replicated and no collective runs.  When the forest itself should be
split -- more trees than one device should hold, or one batch served by every
GPU of the node at once -- each rank instead keeps a contiguous slice of the
trees (balanced by node count, so every rank streams about the same node
bytes) and predicts partial margins of every row; one reduce (sum) over the
process group -- RCCL over xGMI for ``backend="nccl"``, ``[rows, K]`` fp32 or
fp64, 4 MB for C2's 1M rows -- gives the root the full margins, and the
library's own output transform (``ti_transform_device``) runs there.

Numerics: each rank sums its trees in order and the reduce adds the partial
sums, so margins differ from the one-device order by rounding only
(north_star: within 1e-5 relative); leaf ids are gathered to the root (a
``gather``, so each rank sends its block once and only the root receives), not
summed, and stay exact.  TreeSHAP contributions are additive over trees too (each shard's bias
holds its trees' expected values; the base margin lives on the root's shard)
and are reduced the same way.

The reference has no counterpart (its predict is single-process per model,
python/xgbserver/xgbserver/model.py:43-50); the API follows DeviceForest's.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import numpy as np

from .forest import OUT_CONTRIB, OUT_LEAF, OUT_MARGIN, OUT_PREDICT, TI_F32, Forest


def partition_trees(forest: Forest, world: int) -> List[Tuple[int, int]]:
    """Contiguous tree ranges, one per rank, with about equal node counts
    (every range non-empty)."""
    T = forest.n_trees
    if world < 1:
        raise ValueError("world size must be >= 1")
    if world > T:
        raise ValueError(f"{world} ranks for {T} trees: every rank needs a tree")
    nodes = np.diff(forest.tree_offset).astype(np.float64)
    cum = np.concatenate([[0.0], np.cumsum(nodes)])
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(cum, cum[-1] * r / world, side="left"))
        c = max(c, cuts[-1] + 1)               # non-empty
        c = min(c, T - (world - r))            # leave a tree for every later rank
        cuts.append(c)
    cuts.append(T)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


class TreeShardedForest:
    """One rank's slice of a tree-sharded forest.

    ``engine_factory(sub_forest, device)`` builds the local engine (default:
    :class:`kfserving_amd.engine.DeviceForest` on ``device``); every rank of
    ``group`` must construct the same forest and call :meth:`predict` together.
    """

    def __init__(self, forest: Forest, group=None, device: Optional[int] = None, root: int = 0,
                 engine_factory: Optional[Callable] = None):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.root = root
        self.forest = forest
        self.ranges = partition_trees(forest, self.world)
        t0, t1 = self.ranges[self.rank]
        self.local_forest = forest.tree_subset(t0, t1, keep_base=self.rank == root)
        if engine_factory is None:
            from .engine import DeviceForest
            engine_factory = lambda f, dev: DeviceForest(f, [dev])   # noqa: E731
        self.device = device
        self.engine = engine_factory(self.local_forest, device)

    # ------------------------------------------------------------------
    def _gloo(self) -> bool:
        import torch.distributed as dist
        return dist.get_backend(self.group) == "gloo"

    def _dtype(self, kind: int):
        import torch
        if kind == OUT_LEAF:
            return torch.int32
        return torch.float32 if self.forest.accum_dtype == TI_F32 else torch.float64

    def predict(self, X, kind: int = OUT_PREDICT, stream: int = 0):
        """X: [rows, cols] tensor on this rank's device (every rank passes the
        same rows).  Returns the full output on the root (PREDICT and LEAF
        shaped as DeviceForest.predict returns them, MARGIN [rows, K], CONTRIB
        [rows, K * (F + 1)]) and None elsewhere."""
        import torch
        import torch.distributed as dist
        rows, cols = int(X.shape[0]), int(X.shape[1])
        xdt = 0 if X.dtype == torch.float32 else 1
        if not stream and X.is_cuda:   # torch's stream, which the collectives order against
            stream = torch.cuda.current_stream(X.device).cuda_stream
        f = self.forest
        dev = X.device
        if kind == OUT_LEAF:
            return self._gather_leaves(X, rows, cols, xdt, stream)
        part_kind = OUT_CONTRIB if kind == OUT_CONTRIB else OUT_MARGIN
        width = f.output_width(part_kind)
        part = torch.empty((rows, width), dtype=self._dtype(kind), device=dev)
        self.engine.predict_device(X.data_ptr(), xdt, rows, cols, cols, part_kind,
                                   part.data_ptr(), part.numel(), stream=stream)
        if self.world > 1:
            if part.is_cuda and self._gloo():
                # gloo reduces host tensors only (a CPU test rig of the RCCL path)
                host = part.cpu()
                dist.reduce(host, dst=self.root, op=dist.ReduceOp.SUM, group=self.group)
                if self.rank == self.root:
                    part.copy_(host)
            else:
                dist.reduce(part, dst=self.root, op=dist.ReduceOp.SUM, group=self.group)
        if self.rank != self.root:
            return None
        if kind != OUT_PREDICT:
            return part
        out_w = f.output_width(OUT_PREDICT)
        out = torch.empty(rows * out_w, dtype=part.dtype, device=dev)
        self.engine.transform_device(part.data_ptr(), rows, out.data_ptr(), out.numel(),
                                     stream=stream)
        return out if out_w == 1 else out.reshape(rows, out_w)

    def _gather_leaves(self, X, rows, cols, xdt, stream):
        import torch
        import torch.distributed as dist
        t0, t1 = self.ranges[self.rank]
        tmax = max(b - a for a, b in self.ranges)
        local = torch.full((rows, tmax), -1, dtype=torch.int32, device=X.device)
        mine = torch.empty((rows, t1 - t0), dtype=torch.int32, device=X.device)
        self.engine.predict_device(X.data_ptr(), xdt, rows, cols, cols, OUT_LEAF,
                                   mine.data_ptr(), mine.numel(), stream=stream)
        local[:, :t1 - t0] = mine
        if self.world == 1:
            return mine
        # a gather to the root, not an all_gather: only the root uses the ids,
        # so each rank sends its [rows, tmax] block once and receives nothing
        is_root = self.rank == self.root
        if local.is_cuda and self._gloo():   # gloo gathers host tensors only
            bufs = ([torch.empty_like(local, device="cpu") for _ in range(self.world)]
                    if is_root else None)
            dist.gather(local.cpu(), gather_list=bufs, dst=self.root, group=self.group)
            if is_root:
                bufs = [b.to(X.device) for b in bufs]
        else:
            bufs = [torch.empty_like(local) for _ in range(self.world)] if is_root else None
            dist.gather(local, gather_list=bufs, dst=self.root, group=self.group)
        if not is_root:
            return None
        return torch.cat([bufs[r][:, :b - a] for r, (a, b) in enumerate(self.ranges)], dim=1)
