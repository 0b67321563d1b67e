"""A CPU stand-in for DeviceForest that bench.py loads with
`--engine tests.bench_stub:make` (tests/test_bench_ranks.py): it records
nothing on a device, sleeps per call so the slower rank's wall time is known
(local rank 1: 20 ms a predict, others 1 ms)."""
import time


class StubEngine:
    def __init__(self, forest, rank):
        self.forest = forest
        self.rank = rank
        self.calls = []

    def predict_device(self, x_ptr, x_dtype, n_rows, n_cols, row_stride, kind, out_ptr,
                       out_len, slot=0, stream=0):
        self.calls.append((n_rows, n_cols))
        time.sleep(0.02 if self.rank == 1 else 0.001)

    def info(self):
        return {"layout": 3}

    def close(self):
        pass


def make(forest, local_rank):
    return StubEngine(forest, local_rank)
