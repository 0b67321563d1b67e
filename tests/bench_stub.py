"""A CPU stand-in for DeviceForest that bench.py loads with
`--engine tests.bench_stub:make` (tests/test_bench_ranks.py): it records
nothing on a device, sleeps per call so the slower rank's wall time is known
(local rank 1: 20 ms a predict, others 1 ms)."""
import time

import numpy as np


class StubEngine:
    def __init__(self, forest, rank):
        self.forest = forest
        self.rank = rank
        self.calls = []

    def predict_device(self, x_ptr, x_dtype, n_rows, n_cols, row_stride, kind, out_ptr,
                       out_len, slot=0, stream=0):
        self.calls.append((n_rows, n_cols))
        time.sleep(0.02 if self.rank == 1 else 0.001)

    def predict(self, X, kind=0):
        """Host-buffer predict (bench.py's C5 leg): 1 ms a batch, zeros."""
        time.sleep(0.001)
        return np.zeros(np.asarray(X).shape[0], dtype=np.float32)

    def transform_device(self, margin_ptr, n_rows, out_ptr, out_len, slot=0, stream=0):
        pass

    def info(self):
        return {"layout": 3}

    def close(self):
        pass


def make(forest, local_rank):
    return StubEngine(forest, local_rank)


class CanonStubEngine(StubEngine):
    """The stand-in that also computes: predict_device on CPU tensors through
    the canonical numpy evaluator (tests/canon_eval.py), so bench.py's
    tree-sharded leg can check its reduced margins at --device cpu
    (`--engine tests.bench_stub:make_canon`)."""
    computes = True

    def predict_device(self, x_ptr, x_dtype, n_rows, n_cols, row_stride, kind, out_ptr,
                       out_len, slot=0, stream=0):
        from tests.test_tree_shard import CanonEngine
        super().predict_device(x_ptr, x_dtype, n_rows, n_cols, row_stride, kind, out_ptr,
                               out_len)
        CanonEngine(self.forest, None).predict_device(x_ptr, x_dtype, n_rows, n_cols,
                                                      row_stride, kind, out_ptr, out_len)

    def transform_device(self, margin_ptr, n_rows, out_ptr, out_len, slot=0, stream=0):
        from tests.test_tree_shard import CanonEngine
        CanonEngine(self.forest, None).transform_device(margin_ptr, n_rows, out_ptr, out_len)


def make_canon(forest, local_rank):
    return CanonStubEngine(forest, local_rank)
