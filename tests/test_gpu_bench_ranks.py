"""bench.py's rank path with the real engine on the GPU: two ranks (both on
cuda:0 -- the box has one GPU -- over gloo instead of RCCL, which refuses two
ranks on one device) run the headline and a strong-sharded C3 leg: the
forest is created per rank, each rank predicts its own batch, rank 0 alone
prints, value = both ranks' rows / the slowest rank's wall, C3's rows split
in contiguous halves; the C5-over-HTTP leg with two server workers."""
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


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
                      RANK=str(rank), LOCAL_RANK="0")
    try:
        import bench
        args = bench.parse_args(["--steps", "4", "--warmup", "1", "--rows", "65536",
                                 "--configs", "c3", "--rows3", "200000", "--config-steps", "1",
                                 "--no-cpu-baseline", "--latency-qps", "0", "--host-rows", "0",
                                 "--nan-variant", "0", "--c5-http-qps", "5000",
                                 "--c5-http-v2-qps", "5000", "--c5-http-seconds", "2"])
        q.put((rank, bench.run(args, device="cuda", backend="gloo"), None))
    except Exception as e:          # surface the failure in the parent
        q.put((rank, None, repr(e)))


def test_two_ranks_one_gpu_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=140) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=30)
    assert res[0][2] is None and res[1][2] is None, res
    line, other = res[0][1], res[1][1]
    assert other is None
    assert line["n_gpus"] == 2 and line["config"]["rows_per_gpu"] == 65536
    want = 65536 * 2 * 4 / (line["ms_per_step"] * 4e-3)
    assert abs(line["value"] - want) < 1e-6 * want
    assert line["roofline"]["kernel"] == "bheap_fix_kernel"
    c3 = line["c3"]
    assert c3["rows"] == 200000 and c3["rows_per_gpu"] == 100000 and c3["scaling"] == "strong"
    assert c3["layout"] == "texplicit"
    # the tree-sharded leg with the real engine: each rank half the trees, the
    # partial margins reduced to rank 0 (over the host with gloo here; RCCL on
    # a node), within north_star's 1e-5 of the replicated forest's predict
    ts = line["tree_shard"]
    assert ts["ranks"] == 2 and ts["rows"] == 65536 and 0 < ts["trees_rank0"] < 500
    assert ts["within_1e-5"], ts
    # C5 over HTTP at world 2: one xgbserver worker per rank (both on this
    # GPU here), the native front end in each, every request answered
    c5 = line["c5_http"]
    assert c5 is not None and "error" not in c5, c5
    assert c5["workers"] == 2 and c5["devices"] == 2
    assert all(p["lost"] == 0 and p["non200"] == 0 and p["requests"] > 0 for p in c5["points"])
    c5v2 = line["c5_http_v2"]
    assert c5v2 is not None and "error" not in c5v2 and c5v2["workers"] == 2, c5v2
    assert all(p["lost"] == 0 and p["non200"] == 0 and p["requests"] > 0 for p in c5v2["points"])
