"""Benchmark: predicted rows/sec of the BASELINE.json headline workload.

Workload (BASELINE.json configs[1]): synthetic HIGGS-shaped
XGBoost binary:logistic model, 500 complete depth-8 trees, 28 features,
base_score 0.5; a 1M-row float32 batch per GPU, resident in HBM when the timed
region starts.  One step = one fused predict (traversal + sigmoid) over the
batch.  Multi-GPU: one process per GPU (torchrun), rows sharded with no
collective ("weak": every rank predicts its own 1M rows); value = all ranks'
rows / max-over-ranks wall time.

Also reported (rank 0):
  roofline     -- the resource that binds the C2 kernel:
                  the busiest of VALU issue, the LDS array and the TD in the
                  committed rocprofv3 PMC pass of the same kernel
                  (profiles/r6c_c2_pmc.json), priced on that pass's own cycles
                  (GRBM_GUI_ACTIVE per XCD): the LDS array, ~0.67.  `valu`
                  keeps the VALU view: achieved = VALU wave-instructions per
                  launch / the kernel's average duration from HIP events on
                  the launch stream; peak = 1,024 SIMDs x 2.4 GHz / 2 cycles
                  per wave64 instruction (MI355X_MICROARCH.md); `peak_mix`,
                  the ceiling of the walk's own instruction mix measured by
                  scripts/micro/valu_rate.hip (profiles/r3_valu_rate.jsonl).
                  The HBM view is kept beside it: compulsory bytes (X + out)
                  and counter bytes (FETCH_SIZE x 2 + WRITE_SIZE) per launch
                  as fractions of 8 TB/s.
  cpu_baseline -- the C/OpenMP restatement of xgboost 0.82's predict loop
                  (oracle/c/tree_port.c, kind "port": xgboost is not installed)
                  timed on this host on a bounded sample of the same rows.
  c3, c3_f64, c3_maxbin, c4 -- the other named GPU configs at their BASELINE
                  sizes, row-sharded over the ranks (strong scaling, max-over-
                  ranks wall): C3 LightGBM leaf-wise 1000 x 255 leaves, F = 100,
                  100M rows, float32 X (c3) and float64 X (c3_f64: what
                  lgbserver's DataFrame path feeds, lgbserver/model.py:46-51);
                  c3_maxbin the same shape as a max_bin-255 LightGBM model
                  (quantile-edge thresholds: u8 bins); C4 sklearn
                  RandomForestRegressor 200 x depth 16, F = 64, 10M rows (the
                  cached fit of scripts/make_c4_model.py).  Each carries a
                  `roofline` (config_roofline): the busiest of VALU issue, LDS
                  array and TD cycles of a committed PMC pass, priced on that
                  pass's own cycles.  C4's cpu_baseline is sklearn's own
                  RandomForestRegressor.predict (kind "library").
  batched_latency (native batcher), batched_latency_asyncio, nan_variant --
  see the functions below.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_TREES, DEPTH, N_FEAT, ROWS = 500, 8, 28, 1_000_000
HBM_PEAK = 8.0e12          # MI355X HBM3E, bytes/s (MI355X_MICROARCH.md)
SIMDS, CLOCK_HZ, VALU_CYCLES = 1024, 2.4e9, 2.0   # MI355X_MICROARCH.md: wave64 over 2 cycles
VALU_PEAK = SIMDS * CLOCK_HZ / VALU_CYCLES     # wave64 VALU instructions / s (1,228.8 G)
VALU_RATE_JSONL = os.path.join(ROOT, "profiles", "r3_valu_rate.jsonl")
# the binned-heap walk (ti_forest_info.walk) -> its step's row in VALU_RATE_JSONL
# (level 0 from the scalar-loaded root, walk 2, leaves the step itself unchanged)
WALK_STEPS = {0: "step r2", 1: "step fixed (and_or, and, cmp_sdwa, cndmask)",
              2: "step fixed (and_or, and, cmp_sdwa, cndmask)"}
LAYOUT_NAMES = {0: "heap", 1: "explicit", 3: "bheap", 6: "rexplicit", 7: "lexplicit",
                8: "hexplicit", 9: "texplicit"}
# the kernel a layout launches (its name in rocprofv3's kernel trace and in the
# committed PMC passes' "kernel"): a pass describes a launch only if they agree
LAYOUT_KERNELS = {0: "heap_predict_kernel", 1: "explicit_predict_kernel",
                  6: "rexplicit_predict_kernel", 7: "lexplicit_predict_kernel",
                  8: "hexplicit_predict_kernel"}
WALK_KERNELS = {0: "bheap_predict_kernel", 1: "bheap_fix_kernel", 2: "bheap_fix_kernel"}
# the committed PMC pass each workload's roofline is priced on
# (scripts/kernel_pmc.sh -> scripts/make_pmc_json.py)
PMC_PASSES = {"c2": "profiles/r6c_c2_pmc.json", "c3": "profiles/r6g_c3_pmc.json",
              "c3_f64": "profiles/r6g_c3_f64_pmc.json", "c3_maxbin": "profiles/r6c_c3_maxbin_pmc.json",
              "c4": "profiles/r6c_c4_pmc.json", "c2_hist": "profiles/r6c_c2_hist_pmc.json"}


def pmc_path(key: str) -> str:
    return os.path.join(ROOT, PMC_PASSES[key])


def launched_kernel(info: dict) -> str:
    """The predict kernel the engine launches for a forest (ti_forest_info)."""
    layout = info.get("layout")
    if layout == 3:
        return WALK_KERNELS.get(info.get("walk"), "bheap_predict_kernel")
    if layout == 9:
        return {1: "t8explicit_predict_kernel", 2: "t16explicit_predict_kernel",
                3: "t16split_predict_kernel"}.get(
            info.get("bottom"), "texplicit_predict_kernel")
    return LAYOUT_KERNELS.get(layout, f"layout{layout}")


def pmc_mismatch(pmc, workload: str, rows: int, info: dict):
    """Why a committed PMC pass does not describe this launch (None: it does).
    The identity is the workload, the row count, the layout, the launched
    kernel's name and, for the binned-heap walk, the integer walk id."""
    if pmc is None:
        return "no PMC pass file"
    layout = LAYOUT_NAMES.get(info.get("layout"))
    want = launched_kernel(info)
    if pmc.get("workload") != workload:
        return f"PMC pass is of workload {pmc.get('workload')!r}, not {workload!r}"
    if pmc.get("layout") != layout:
        return f"PMC pass is of layout {pmc.get('layout')!r}, this launch is {layout!r}"
    if f"::{want}<" not in str(pmc.get("kernel", "")):
        return f"PMC pass kernel {pmc.get('kernel')!r} is not the launched {want}"
    if info.get("layout") == 3 and pmc.get("walk_id") != info.get("walk"):
        return f"PMC pass walk id {pmc.get('walk_id')} != the launched walk {info.get('walk')}"
    if rows is not None and pmc.get("rows") != rows:
        return f"PMC pass rows {pmc.get('rows')} != {rows}"
    if "valu_insts_per_launch" not in pmc:
        return "PMC pass lacks SQ_INSTS_VALU"
    return None


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rows", type=int, default=ROWS)
    p.add_argument("--nan-variant", type=float, default=0.01,
                   help="also time the same batch with this fraction of NaN features "
                        "(SURVEY.md 8(d) C2 1%%-NaN variant; 0 = skip)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="target CPU work for the cpu_baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--latency-qps", type=float, default=10000.0,
                   help="offered requests/s for the batched-latency leg (0 = skip)")
    p.add_argument("--latency-seconds", type=float, default=3.0)
    p.add_argument("--configs", default="c3,c3_f64,c3_maxbin,c4,c2_hist",
                   help="other named configs to time after the headline ('' = none)")
    p.add_argument("--rows3", type=int, default=100_000_000)
    p.add_argument("--rows4", type=int, default=10_000_000)
    p.add_argument("--config-steps", type=int, default=2)
    p.add_argument("--pmc-json", default=os.path.join(ROOT, PMC_PASSES["c2"]))
    p.add_argument("--streams", type=int, default=2,
                   help="launch streams the headline's steps rotate over (batches in flight); "
                        "the roofline prices the one-stream launch duration")
    p.add_argument("--x-buffers", type=int, default=3,
                   help="copies of the batch the timed steps rotate through (3 x 112 MB "
                        "exceeds the 256 MB Infinity Cache)")
    p.add_argument("--host-rows", type=int, default=8_000_000,
                   help="rows of the host-to-host (PCIe-inclusive) C2 leg (0 = skip)")
    p.add_argument("--host-rows-configs", type=int, default=8_000_000,
                   help="rows of the host-to-host (PCIe-inclusive) legs of the config "
                        "workloads c3 / c3_f64 / c3_maxbin / c4 (rank 0; 0 = skip)")
    p.add_argument("--c5-http-qps", default="20000,100000,200000",
                   help="C5 over HTTP: offered req/s PER GPU of the points (x N for the node; "
                        "empty: skip); rank 0, after the GPU legs, a server of one worker per GPU")
    p.add_argument("--c5-conns-per-gpu", type=int, default=4096,
                   help="C5 over HTTP: keep-alive client connections per GPU")
    p.add_argument("--c5-loadgen-threads-per-gpu", type=int, default=4)
    p.add_argument("--c5-io-threads", type=int, default=16,
                   help="native HTTP IO threads per worker (the one-GPU value at every N)")
    p.add_argument("--c5-capacity-points", type=int, default=3,
                   help="C5 over HTTP: extra points searching the highest offered rate with "
                        "p99 <= 2 x maxLatency and no loss (0 = no search)")
    p.add_argument("--c5-http-cpu", action="store_true",
                   help="--device cpu: run the C5 HTTP leg against the CPU echo model (tests)")
    p.add_argument("--c5-http-seconds", type=float, default=4.0)
    p.add_argument("--c5-http-v2-qps", default="100000",
                   help="the same with V2 FP32 JSON tensor bodies on /v2/models/<name>/infer "
                        "(empty: skip)")
    p.add_argument("--no-tree-shard", action="store_true",
                   help="skip the tree-sharded C2 leg (every rank a slice of the trees, "
                        "partial margins summed by one reduce: RCCL over xGMI at N > 1)")
    p.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                   help="cpu: the rank logic only, over gloo, with --engine's stand-in "
                        "(tests/test_bench_ranks.py)")
    p.add_argument("--engine", default="",
                   help="MODULE:FACTORY returning the engine for (forest, local_rank) "
                        "('' = kfserving_amd.engine.DeviceForest on the rank's GPU)")
    return p.parse_args(argv)


def build_model():
    from kfserving_amd.formats.xgboost_format import (forest_from_raw_trees,
                                                      synthetic_complete_trees)
    trees, ti = synthetic_complete_trees(N_TREES, DEPTH, N_FEAT, seed=0)
    # xgboost 0.82 stores base_score in margin space: ProbToMargin(0.5) = 0
    forest = forest_from_raw_trees(trees, ti, N_FEAT, 0, 0.0, "binary:logistic")
    return trees, ti, forest


def shard_rows(total_rows: int, rank: int, world: int):
    """Weak scaling: every rank owns a full batch of `total_rows` rows with its own seed
    (rows are independent: no data-path collective)."""
    return total_rows, 1000 + rank


def strong_shard(total: int, rank: int, world: int):
    """Strong scaling (C3 / C4): contiguous row blocks of one batch."""
    per = (total + world - 1) // world
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


def max_over_ranks(value: float, device) -> float:
    """The slowest rank's wall time (the only collective, outside the timed region)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier_sync(dev_sync):
    import torch.distributed as dist
    dev_sync()
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
    dev_sync()


def timed_steps(step, steps, dev_sync, events=None, fork=None, join=None):
    """K steps bracketed by barrier + device sync on both sides; returns the
    wall time and (with `events` = (start, end) timing events recorded on the
    launch stream) the event time per step in ms.  fork / join (--streams > 1)
    make the other launch streams wait for the start event and the launch
    stream wait for them before the end event."""
    barrier_sync(dev_sync)
    t0 = time.perf_counter()
    if events:
        events[0].record()
    if fork:
        fork()
    for _ in range(steps):
        step()
    if join:
        join()
    if events:
        events[1].record()
    barrier_sync(dev_sync)
    wall = time.perf_counter() - t0
    ev_ms = events[0].elapsed_time(events[1]) / steps if events else None
    return wall, ev_ms


def streams_match(dev, Xs, outs, last_x, rows, sh, dev_sync, on_device=True):
    """Each stream's last output equals a one-stream predict of the batch
    that launch read (bit for bit).  None without a device (the CPU stand-in
    engine writes no outputs)."""
    import torch
    from kfserving_amd.forest import OUT_PREDICT, TI_F32
    if not on_device:
        return None
    dev_sync()
    ok = True
    for k, o in enumerate(outs):
        if last_x[k] is None:
            continue
        ref = torch.empty_like(o)
        Xi = Xs[last_x[k]]
        dev.predict_device(Xi.data_ptr(), TI_F32, rows, N_FEAT, N_FEAT, OUT_PREDICT,
                           ref.data_ptr(), rows, slot=0, stream=sh)
        dev_sync()
        ok = ok and bool(torch.equal(ref, o))
    return ok


def batch_latency_events(launch, n_str, strs, steps, dev_sync):
    """Untimed pass after the headline: the same round-robin launches with a
    start and an end event around each on its own stream, so a batch's
    launch-to-completion time beside the other stream's batch is measured
    (the headline's own region carries no per-launch events)."""
    import torch
    cur = torch.cuda.current_stream()
    dev_sync()
    for st in strs[1:]:
        st.wait_stream(cur)
    evs = []
    for i in range(steps):
        k = i % n_str
        s = cur if k == 0 else strs[k]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch(k)
        e1.record(s)
        evs.append((e0, e1))
    dev_sync()
    per = [a.elapsed_time(b) for a, b in evs]
    return {"batch_ms_mean": float(np.mean(per)), "batch_ms_max": float(np.max(per)),
            "batches": len(per),
            "basis": "start/end HIP events around each launch on its own stream, "
                     "round-robin over the streams as in the headline (untimed pass)"}


def cpu_baseline(trees, ti, X_host, target_s):
    """C2 on the host: the port timed on about target_s seconds of rows (the
    batch tiled when that is more than its 1M rows)."""
    from oracle import port
    n_thr = baseline_threads()
    n, dt = _scaled_sample(
        lambda Xs: port.xgb_predict(trees, ti, 1, 0.0, N_FEAT, Xs, sigmoid=True, nthread=n_thr),
        sample_taker(X_host), target_s)
    return {"value": n / dt, "unit": "rows/s", "cores": n_thr, "kind": "port",
            "sample": f"{n} rows of the same 1M x 28 batch (tiled past 1M), oracle/c/tree_port.c "
                      f"(xgboost 0.82 predict loop restated, OpenMP {n_thr} threads), "
                      f"{dt:.1f} s"}


def valu_step_rate(op_prefix: str, waves_per_simd: int = 8, path: str = VALU_RATE_JSONL):
    """The measured issue cost of one walk step (scripts/micro/valu_rate.hip
    rows "step ..."): (VALU per step, cycles per step per SIMD, clock GHz)."""
    try:
        with open(path) as fh:
            rows = [json.loads(l) for l in fh if l.strip().startswith("{")]
    except (OSError, ValueError):
        return None
    for r in rows:
        if r["op"].startswith(op_prefix) and r["waves_per_simd"] == waves_per_simd:
            return r
    return None


def load_pmc(path: str):
    try:
        with open(path) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return None


def roofline(kernel_ms: float, rows: int, info: dict, pmc_path: str):
    """Roofline of the C2 kernel (see the module docstring): the busiest of
    the issue resources the committed PMC pass of the same kernel counts --
    VALU issue, the LDS array, the TD -- each priced on that pass's own
    cycles, as config_roofline does for C3 / C4.  `bound` / `frac` are the
    busiest; `achieved` / `peak` are in that resource's unit (LDS-array and TD
    cycles per second per CU against the 2.4 GHz clock; VALU wave64
    instructions per second against the 2-cycle issue peak).  The VALU view,
    the step-mix ceiling and the HBM view stay beside it.  A pass that does
    not describe this launch (pmc_mismatch) leaves `frac` unset and says why
    in `error`: the line never carries bare nulls."""
    layout = LAYOUT_NAMES.get(info.get("layout"))
    step_op = WALK_STEPS.get(info.get("walk")) if info.get("layout") == 3 else None
    pmc = load_pmc(pmc_path)
    why = pmc_mismatch(pmc, "c2", rows, info)
    t = kernel_ms * 1e-3
    compulsory = (4 * N_FEAT + 4) * rows
    out = {"bound": "valu_issue", "unit": "Ginst/s", "peak": VALU_PEAK / 1e9,
           "kernel": launched_kernel(info), "kernel_ms": kernel_ms,
           "peak_basis": f"{SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz / {VALU_CYCLES:g} cycles per "
                         "wave64 VALU instruction (MI355X_MICROARCH.md)",
           "hbm_compulsory_bytes": compulsory,
           "hbm_compulsory_GBps": compulsory / t / 1e9,
           "hbm_compulsory_frac": compulsory / t / HBM_PEAK}
    if why:
        out.update(achieved=None, frac=None, traffic=None,
                   error=f"{os.path.relpath(pmc_path, ROOT)}: {why}")
        return out
    valu = pmc["valu_insts_per_launch"]
    cfg = config_roofline(kernel_ms, rows, info, "c2", pmc_path) or {}
    fr = cfg.get("fracs") or {}
    valu_view = {"achieved": valu / t / 1e9, "peak": VALU_PEAK / 1e9, "unit": "Ginst/s",
                 "frac": valu / t / VALU_PEAK, "valu_insts_per_launch": valu,
                 "peak_basis": out["peak_basis"]}
    cyc = pmc.get("gui_active_cycles_per_xcd")
    if cyc:
        valu_view["profiled"] = {
            "frac": valu * VALU_CYCLES / (SIMDS * cyc),
            "kernel_ms": (pmc.get("profiled_kernel_ns") or 0) * 1e-6 or None,
            "clock_GHz": pmc.get("profiled_clock_GHz"),
            "basis": "VALU x 2 cycles / (1,024 SIMDs x GRBM_GUI_ACTIVE/8 of the PMC pass)"}
    if step_op:
        st = valu_step_rate(step_op)
        if st:
            mix = st["valu_per_step"] / st["cycles_per_step_per_simd"] * SIMDS * CLOCK_HZ
            valu_view["peak_mix"] = mix / 1e9
            valu_view["frac_mix"] = valu / t / mix
            valu_view["peak_mix_basis"] = (
                f"walk step '{st['op']}': {st['valu_per_step']} VALU in "
                f"{st['cycles_per_step_per_simd']:.2f} cycles per SIMD at 8 waves/SIMD "
                f"(profiles/r3_valu_rate.jsonl), x {SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz")
    out["valu"] = valu_view
    out["fracs"] = fr
    out["fracs_bench"] = cfg.get("fracs_bench")
    bound = cfg.get("bound", "valu_issue")
    out["bound"] = bound
    out["frac"] = fr.get(bound, valu_view["frac"])
    if bound == "valu_issue":
        out.update(achieved=valu_view["achieved"], peak=valu_view["peak"], unit="Ginst/s")
    else:
        # busy cycles per CU per second of the profiled run (achieved / peak =
        # the busy fraction of the PMC pass's own cycles)
        out.update(achieved=out["frac"] * CLOCK_HZ / 1e9, peak=CLOCK_HZ / 1e9,
                   unit=f"G {bound} cycles/s per CU",
                   peak_basis=f"one {bound} cycle per clock per CU at {CLOCK_HZ / 1e9} GHz; frac "
                              "priced on the PMC pass's own cycles (GRBM_GUI_ACTIVE per XCD)")
    for k in ("lds_bank_conflict_frac", "wait_frac", "l2_hit_rate", "waves_per_simd"):
        if pmc.get(k) is not None:
            out[k] = pmc[k]
    out["traffic"] = pmc.get("hbm_bytes_per_launch")
    if out["traffic"]:
        out["hbm_counter_GBps"] = out["traffic"] / t / 1e9
        out["hbm_counter_frac"] = out["traffic"] / t / HBM_PEAK
        out["traffic_over_compulsory"] = out["traffic"] / (compulsory + pmc.get("model_bytes", 0))
    out["pmc_source"] = pmc.get("source")
    out["pmc_kernel"] = pmc.get("kernel")
    return out


CUS = 256
B_VISIT = 8 * N_TREES * DEPTH + 4 * N_FEAT + 4   # SURVEY.md 8(d)'s per-row visit bytes


def headline_roofline(kernel_ms, rows, info, pmc_path, step_s, two_stream, n_str):
    """roofline() of the one-stream launch, plus what the headline's own
    region did: `two_stream` prices the PMC pass's LDS-array cycles per batch
    on the two-stream step time (256 CUs x 2.4 GHz x ms_per_step) and carries
    the per-batch launch-to-completion time measured with events; `b_visit_*`
    is SURVEY.md 8(d)'s visit-byte model, whose nodes are LDS-resident, so
    its fraction of HBM peak is not a bound (it exceeds 1)."""
    out = roofline(kernel_ms, rows, info, pmc_path)
    bv = B_VISIT * rows / (kernel_ms * 1e-3)
    out["b_visit_bytes_per_row"] = B_VISIT
    out["b_visit_GBps"] = bv / 1e9
    out["b_visit_frac"] = bv / HBM_PEAK
    out["b_visit_note"] = ("8 B x 500 trees x 8 levels + X + out per row: the node bytes are "
                           "read from LDS (the stage), not HBM, so this 'HBM' fraction exceeds 1 "
                           "and bounds nothing; the binding resource is `bound` (LDS array)")
    if n_str > 1:
        pmc = load_pmc(pmc_path)
        ts = {"streams": n_str, "ms_per_step": step_s * 1e3,
              "batch_ms_one_stream": kernel_ms}
        if pmc and pmc.get("lds_idx_active_per_launch") and not out.get("error"):
            lds = pmc["lds_idx_active_per_launch"] * rows / pmc["rows"]
            ts["lds_array_frac"] = lds / (CUS * CLOCK_HZ * step_s)
            ts["lds_array_frac_one_stream"] = lds / (CUS * CLOCK_HZ * kernel_ms * 1e-3)
            ts["basis"] = ("PMC pass LDS-array cycles per batch / (256 CUs x 2.4 GHz x the "
                           "step time of each mode)")
        if two_stream:
            ts["batch_ms_two_streams"] = two_stream["batch_ms_mean"]
            ts["batch_ms_two_streams_max"] = two_stream["batch_ms_max"]
            ts["batch_latency_basis"] = two_stream["basis"]
        out["two_stream"] = ts
    return out


def config_roofline(kernel_ms: float, rows: int, info: dict, workload: str, pmc_path: str):
    """Binding-resource roofline of a C3 / C4 launch from a committed PMC pass
    of the same kernel at 1M rows (scripts/kernel_pmc.sh ->
    scripts/make_pmc_json.py).  Three issue-type resources are priced, each
    against its own peak per cycle: VALU issue (wave64 instructions at 2
    cycles on 1,024 SIMDs), the LDS array (cycles, one array per CU) and the
    TD (vector-memory data path, busy cycles per CU: what a node gather
    occupies).  `frac` is priced on the PMC run's own cycles
    (GRBM_GUI_ACTIVE per XCD: its duration at its clock), never on another
    run's time; `fracs_bench` re-prices the per-row counts on this run's
    kernel time at the nominal 2.4 GHz.  `bound` is the busiest resource."""
    pmc = load_pmc(pmc_path)
    why = pmc_mismatch(pmc, workload, None, info)
    if why:               # a pass of another kernel does not describe this one
        return {"bound": None, "frac": None, "error": f"{os.path.relpath(pmc_path, ROOT)}: {why}"}
    cyc = pmc.get("gui_active_cycles_per_xcd")
    # (count, units, the cycles of the pass that counted it)
    counts = {"valu_issue": (pmc["valu_insts_per_launch"] * VALU_CYCLES, SIMDS,
                             pmc.get("valu_pass_cycles_per_xcd") or cyc)}
    if pmc.get("lds_idx_active_per_launch"):
        counts["lds_array"] = (pmc["lds_idx_active_per_launch"], CUS,
                               pmc.get("lds_pass_cycles_per_xcd") or cyc)
    if pmc.get("td_busy_per_launch"):
        counts["td_busy"] = (pmc["td_busy_per_launch"], CUS, pmc.get("td_pass_cycles_per_xcd") or cyc)
    fr = {k: c / (u * cy) for k, (c, u, cy) in counts.items() if cy}
    t = kernel_ms * 1e-3
    scale = rows / pmc["rows"]
    fb = {k: c * scale / (u * CLOCK_HZ * t) for k, (c, u, _) in counts.items()}
    src = fr or fb
    bound = max(src, key=src.get)
    out = {"bound": bound, "frac": src[bound], "fracs": src, "fracs_bench": fb,
           "basis": ("counts of the PMC pass / (units x that pass's GRBM_GUI_ACTIVE per XCD); "
                     "VALU at 2 cycles per wave64 instruction"),
           "profiled_kernel_ms": (pmc.get("profiled_kernel_ns") or 0) * 1e-6 or None,
           "profiled_clock_GHz": pmc.get("profiled_clock_GHz"),
           "pmc_source": pmc.get("source"), "pmc_rows": pmc["rows"]}
    for k in ("lds_bank_conflict_frac", "wait_frac", "l2_hit_rate", "waves_per_simd"):
        if pmc.get(k) is not None:
            out[k] = pmc[k]
    if pmc.get("hbm_bytes_per_launch"):
        out["traffic"] = pmc["hbm_bytes_per_launch"] * scale
    return out


def batched_latency(dev, n_feat, qps, seconds, max_batch=65536, max_latency_ms=5, seed=7,
                    freeze_gc=True):
    """C5-style leg: open-loop Poisson arrivals of requests of
    U{1..64} rows into the pipelined in-process batcher (pkg/batcher semantics,
    maxBatchSize rows, maxLatency ms) in front of the GPU engine (host buffers:
    H2D + kernel + D2H per batch).  Each request is a float32 matrix, as
    KFServer's native body parser hands it to the batcher.  Latency = result
    time - scheduled arrival."""
    import asyncio
    import functools
    from concurrent.futures import ThreadPoolExecutor
    from kfserving_amd.batcher import Batcher
    rng = np.random.default_rng(seed)
    warm = int(qps * 0.5)                 # first 0.5 s of load is warmup, not reported
    n_req = int(qps * seconds) + warm
    gaps = rng.exponential(1.0 / qps, n_req)
    sizes = rng.integers(1, 65, n_req)
    pool = np.random.default_rng(seed + 1).standard_normal((64 * 1024, n_feat), dtype=np.float32)
    pool_ex = ThreadPoolExecutor(max_workers=2)
    lat = np.zeros(n_req)
    done_at = np.zeros(n_req)
    batch_rows = []
    batch_ms = []
    batch_span = []          # (loop time the batch was flushed, loop time its result was back)
    lag = []                 # the load generator's wake-up lateness (event-loop stalls)

    async def predict_batch(instances):
        # the batcher concatenates the requests' matrices (as KFServer's
        # natively decoded bodies reach it); a list of rows is stacked
        X = instances if isinstance(instances, np.ndarray) else np.stack(instances)
        batch_rows.append(X.shape[0])
        loop = asyncio.get_running_loop()
        t0l = loop.time()
        t = time.perf_counter()
        out = await loop.run_in_executor(pool_ex, dev.predict, X)
        batch_ms.append((time.perf_counter() - t) * 1e3)
        batch_span.append((t0l, loop.time()))
        return {"predictions": out}

    async def run_load():
        # open-loop arrivals: every request due by now is enqueued at once
        # (the generator wakes at most every `tick` s, not once per request,
        # so its own event-loop load stays small); latency runs from the
        # scheduled arrival, so the tick's lateness is counted, not hidden
        b = Batcher(predict_batch, max_batch_size=max_batch, max_latency_ms=max_latency_ms)
        loop = asyncio.get_running_loop()
        t0 = loop.time() + 0.05
        arrivals = t0 + np.cumsum(gaps)
        tick = 2e-4
        all_done = asyncio.Event()
        n_done = [0]

        # completion is counted in the callbacks: an asyncio.gather over the
        # ~35k futures at the end blocked the loop thread for ~35-45 ms
        # (attaching a callback to each), which held back the last batch's
        # flush timer and was round 3's unexplained 50 ms max_ms
        def done(i, _fut):
            done_at[i] = loop.time()
            lat[i] = done_at[i] - arrivals[i]
            n_done[0] += 1
            if n_done[0] == n_req:
                all_done.set()

        i = 0
        while i < n_req:
            now = loop.time()
            while i < n_req and arrivals[i] <= now:
                off = (i * 64) % (len(pool) - 64)
                f = b.enqueue(pool[off:off + int(sizes[i])])
                f.add_done_callback(functools.partial(done, i))
                i += 1
            if i < n_req:
                want = max(tick, arrivals[i] - loop.time())
                t_s = loop.time()
                await asyncio.sleep(want)
                lag.append(loop.time() - t_s - want)
        await all_done.wait()
        return loop.time() - t0, t0

    import gc
    old = gc.get_threshold()
    old_si = sys.getswitchinterval()
    if freeze_gc:          # what KFServer.start does after load (kfserver.tune_gc: GC, GIL interval)
        from kfserving_amd.kfserving.kfserver import tune_gc
        tune_gc()
    try:
        wall, t_start = asyncio.run(run_load())
    finally:
        if freeze_gc:
            gc.unfreeze()
            gc.set_threshold(*old)
            sys.setswitchinterval(old_si)
    pool_ex.shutdown()
    lat_ms = lat[warm:] * 1e3
    # where the worst request's time went: the batch that answered it (its
    # flush time and predict), the event loop's largest stall around it
    iw = warm + int(np.argmax(lat_ms))
    spans = np.asarray(batch_span)
    bi = int(np.argmin(np.abs(spans[:, 1] - done_at[iw])))
    arr_w = done_at[iw] - lat[iw]
    worst = {"at_s": float(arr_w - t_start), "latency_ms": float(lat[iw] * 1e3),
             "wait_to_flush_ms": float((spans[bi, 0] - arr_w) * 1e3),
             "batch_predict_ms": float(batch_ms[bi]), "batch_rows": int(batch_rows[bi]),
             "batch_index": bi, "max_loop_lag_ms": float(max(lag) * 1e3) if lag else None,
             "requests_over_20ms": int((lat_ms > 20).sum())}
    return {"qps_offered": qps, "requests": n_req - warm, "rows_per_request": "U{1..64}",
            "max_batch_size": max_batch, "max_latency_ms": max_latency_ms,
            "p50_ms": float(np.percentile(lat_ms, 50)), "p99_ms": float(np.percentile(lat_ms, 99)),
            "max_ms": float(lat_ms.max()), "rows_per_s": float(sizes.sum() / wall),
            "p90_ms": float(np.percentile(lat_ms, 90)),
            "batches": len(batch_rows), "mean_batch_rows": float(np.mean(batch_rows)),
            "predict_ms_p50": float(np.percentile(batch_ms, 50)),
            "predict_ms_p99": float(np.percentile(batch_ms, 99)), "gc_frozen": freeze_gc,
            "p999_ms": float(np.percentile(lat_ms, 99.9)), "worst": worst,
            "path": "in-process batcher -> ti_predict (host buffers), 1 GPU, no HTTP/JSON",
            "_lat_ms": lat_ms}


def native_batched_latency(dev, n_feat, qps, seconds, max_batch=65536, max_latency_ms=5,
                           seed=7):
    """The C5 leg through the native batcher (include/kfbatch.h): the same
    open-loop Poisson arrivals of U{1..64}-row float32 requests as
    batched_latency, submitted at their scheduled times by a native thread
    (kb_loadgen: a timed sleep, then a spin), batched in C++ with pkg/batcher
    semantics and handed straight to ti_predict on host buffers.  Latency =
    completion (CLOCK_MONOTONIC, stamped when the request's rows are written)
    - scheduled arrival.  Every request's outputs are then compared with one
    direct predict of the rows it sent."""
    from kfserving_amd.batcher.native import NativeBatcher
    from kfserving_amd.forest import OUT_PREDICT
    rng = np.random.default_rng(seed)
    warm = int(qps * 0.5)                 # first 0.5 s of load is warmup, not reported
    n_req = int(qps * seconds) + warm
    gaps = rng.exponential(1.0 / qps, n_req)
    sizes = rng.integers(1, 65, n_req).astype(np.int32)
    pool = np.random.default_rng(seed + 1).standard_normal((64 * 1024, n_feat), dtype=np.float32)
    if hasattr(dev, "_handle") and hasattr(dev, "_lib"):
        nb = NativeBatcher.for_device_forest(dev, max_batch, max_latency_ms, kind=OUT_PREDICT)
    else:   # a stand-in engine (tests/bench_stub.py): its predict behind the same batcher
        def call(X, out):
            out[...] = np.asarray(dev.predict(X, OUT_PREDICT)).reshape(out.shape)
            return 0
        nb = NativeBatcher(call, n_feat, 0, 1, np.float32, max_batch, max_latency_ms)
    dev.predict(pool[:4096], OUT_PREDICT)
    arrivals = np.cumsum(gaps)
    lat, st, out, t0 = nb.loadgen(arrivals, sizes, pool)
    stats = nb.stats()
    nb.close()
    want = np.asarray(dev.predict(pool, OUT_PREDICT)).reshape(-1)
    ok = bool((st == 0).all())
    for i in range(n_req):
        off = (i * 64) % (pool.shape[0] - 64)
        s = int(sizes[i])
        if not np.array_equal(out[i * 64:i * 64 + s], want[off:off + s]):
            ok = False
            break
    lat_ms = lat[warm:]
    wall = (arrivals[-1] + lat[-1] * 1e-3)   # first arrival at t0 .. last completion
    nb_ = max(1, stats["batches"])
    return {"qps_offered": qps, "requests": n_req - warm, "rows_per_request": "U{1..64}",
            "max_batch_size": max_batch, "max_latency_ms": max_latency_ms,
            "p50_ms": float(np.percentile(lat_ms, 50)), "p99_ms": float(np.percentile(lat_ms, 99)),
            "max_ms": float(lat_ms.max()), "rows_per_s": float(sizes.sum() / wall),
            "p90_ms": float(np.percentile(lat_ms, 90)),
            "p999_ms": float(np.percentile(lat_ms, 99.9)),
            "batches": int(stats["batches"]), "mean_batch_rows": stats["rows"] / nb_,
            "timer_flushes": int(stats["timer_flushes"]), "full_flushes": int(stats["full_flushes"]),
            "model_ms_mean": stats["model_ms_total"] / nb_,
            "outputs_match_direct_predict": ok,
            "path": "native batcher (libkfserve kb_*, pkg/batcher semantics) -> ti_predict "
                    "(host buffers), arrivals submitted by a native thread (kb_loadgen), 1 GPU, "
                    "no HTTP/JSON",
            "_lat_ms": lat_ms}


def c5_http_leg(args, world, protocol="v1", device="cuda"):
    """BASELINE config C5 as named, over HTTP: xgbserver with the C2 forest
    (`python -m kfserving_amd.xgbserver`, --max_batchsize 65536
    --max_latency_ms 5) behind the native HTTP front end and native batcher,
    one worker process per GPU of the job (worker i drives GPU i), keep-alive
    connections from the C load generator (scripts/loadgen.c: open-loop
    Poisson arrivals of U{1..64}-row v1 :predict bodies, latency from the
    scheduled arrival; each thread its own epoll loop).  Run on rank 0 after
    every rank's GPU legs.

    Sized with N: the points are per-GPU rates x N (the
    node offered 1.6M req/s at N = 8 for the 200k per-GPU point), 4,096
    connections and 4 load-generator threads per GPU, and every worker keeps
    the one-GPU worker's 16 IO threads.  After the fixed points the same
    server searches the node's capacity: the highest offered rate with p99 <=
    2 x maxLatency and no request lost (scripts/bench_serving.capacity_search;
    reference pkg/batcher/handler.go:156-185, kfserver.py:99 start(workers)).
    `--device cpu` (tests) serves bench_serving's CPU echo model instead."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_serving as bs
    env = dict(os.environ)
    if world == 1 and device != "cpu":
        import torch
        env["TREEINFER_DEVICES"] = str(torch.cuda.current_device())
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
              "MASTER_PORT", "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    spec = args.c5_http_v2_qps if protocol == "v2" else args.c5_http_qps
    per_gpu = [float(q) for q in spec.split(",") if q.strip()]
    qps = [q * world for q in per_gpu]
    io = args.c5_io_threads
    conns = args.c5_conns_per_gpu * world
    lg_threads = args.c5_loadgen_threads_per_gpu * world
    cap = {}
    try:
        pts = bs.serve_and_measure(qps, workers=world, io_threads=io,
                                   duration=args.c5_http_seconds, warmup=1.5, conns=conns,
                                   port=18090 + (os.getpid() % 500) + (600 if protocol == "v2" else 0),
                                   env=env, ready_timeout=90, loadgen_threads=lg_threads,
                                   echo=False, protocol=protocol,
                                   model="dummy" if device == "cpu" else "c2",
                                   capacity_points=(args.c5_capacity_points
                                                    if protocol == "v1" else 0),
                                   capacity_out=cap)
    except Exception as e:   # reported, not fatal: the headline stands without it
        return {"error": str(e)[-500:]}
    keep = ("offered_qps", "req_per_s", "rows_per_s", "p50_ms", "p90_ms", "p99_ms", "max_ms",
            "requests", "lost", "non200", "conn_errors", "conns")
    res = {"devices": world, "workers": world, "io_threads_per_worker": io,
           "conns": conns, "conns_per_gpu": args.c5_conns_per_gpu,
           "loadgen_threads": lg_threads, "rows_per_request": "U{1..64}",
           "offered_qps_per_gpu": per_gpu, "offered_qps_node": qps,
           "max_batch_size": 65536,
           "max_latency_ms": 5, "model": ("C2 (500 x depth 8, 28 features), xgbserver"
                                          if device != "cpu" else "CPU echo model (tests)"),
           "path": "HTTP/1.1 keep-alive -> native front end (kfhttp.h) -> native batcher "
                   "(kfbatch.h) -> ti_predict (host buffers)",
           "protocol": ("V2 /infer, one FP32 tensor of JSON data" if protocol == "v2"
                        else "v1 :predict instances"),
           "points": [{k: p.get(k) for k in keep} for p in pts]}
    if cap:
        c = cap.get("capacity_req_per_s")
        res["capacity_req_per_s"] = c
        res["capacity_req_per_s_per_gpu"] = None if c is None else c / world
        res["capacity"] = cap
    return res


def tree_shard_leg(forest, dev, rows, args, world, rank, local_rank, device, dev_sync,
                   make_engine=None):
    """SURVEY 8(e)'s alternative sharding on C2: every rank holds a contiguous
    slice of the 500 trees (kfserving_amd.tree_shard), all ranks predict the
    same 1M rows, the partial margins meet in one dist.reduce(SUM) on rank 0
    (RCCL over xGMI with the nccl backend: rows x 4 B) and rank 0 applies the
    sigmoid on the device.  K steps, barrier-bracketed, max over ranks;
    rank 0 checks the result against the replicated forest's predict of the
    same rows (north_star: 1e-5 relative; bit-identical at N = 1)."""
    import torch
    from kfserving_amd.forest import OUT_PREDICT, TI_F32
    from kfserving_amd.tree_shard import TreeShardedForest
    factory = None
    if make_engine is not None:
        factory = lambda f, d: make_engine(f)            # noqa: E731
    ts = TreeShardedForest(forest, device=local_rank if device != "cpu" else None,
                           engine_factory=factory)
    X = device_normal(rows, N_FEAT, 5, device)           # the same batch on every rank
    out = [None]

    def step():
        out[0] = ts.predict(X, OUT_PREDICT)

    step()
    ev = ((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          if device != "cpu" else None)
    wall, _ = timed_steps(step, args.steps, dev_sync, ev)
    wall = max_over_ranks(wall, device)
    res = None
    if rank == 0:
        t0, t1 = ts.ranges[0]
        res = {"rows": rows, "ranks": world, "trees_rank0": t1 - t0, "steps": args.steps,
               "ms_per_step": wall / args.steps * 1e3, "rows_per_s": rows * args.steps / wall,
               "reduce_bytes": rows * 4 * forest.n_groups if world > 1 else 0,
               "collective": "dist.reduce(SUM) of [rows, K] float32 partial margins to rank 0"
                             if world > 1 else "none (one rank)",
               "path": "kfserving_amd.tree_shard.TreeShardedForest"}
        # the check runs on the GPU, and on CPU with an engine that computes
        # (tests/bench_stub.py:make_canon), not with the sleeping stand-in
        if device != "cpu" or getattr(dev, "computes", False):
            ref = torch.empty(rows, dtype=torch.float32, device=device)
            dev.predict_device(X.data_ptr(), TI_F32, rows, N_FEAT, N_FEAT, OUT_PREDICT,
                               ref.data_ptr(), rows, slot=0,
                               stream=(torch.cuda.current_stream().cuda_stream
                                       if device != "cpu" else 0))
            dev_sync()
            got = out[0].reshape(-1).double()
            want = ref.double()
            rel = ((got - want).abs() / want.abs().clamp_min(1e-30)).max().item()
            res["max_rel_diff_vs_replicated"] = rel
            res["bit_identical"] = bool(torch.equal(out[0].reshape(-1), ref))
            res["within_1e-5"] = rel <= 1e-5
    ts.engine.close()
    del X
    return res


def pool_latency(mine: dict, world: int, rank: int, device):
    """The C5 leg over all ranks: every rank's request latencies gathered to
    rank 0 (all_gather_object, outside any timed region) and the percentiles
    taken over the pooled requests; rows/s is the sum over ranks, the offered
    rate the sum of the ranks' rates."""
    import torch.distributed as dist
    lat = mine.pop("_lat_ms")
    if world == 1 or not dist.is_initialized():
        mine.update(devices=1, qps_offered_per_gpu=mine["qps_offered"])
        return mine
    got = [None] * world
    dist.all_gather_object(got, (lat, mine["rows_per_s"], mine["p99_ms"], mine["batches"],
                                 mine.get("outputs_match_direct_predict")))
    if rank != 0:
        return None
    allm = np.concatenate([g[0] for g in got])
    out = dict(mine)
    out.update(devices=world, qps_offered_per_gpu=mine["qps_offered"],
               qps_offered=mine["qps_offered"] * world, requests=int(allm.size),
               p50_ms=float(np.percentile(allm, 50)), p90_ms=float(np.percentile(allm, 90)),
               p99_ms=float(np.percentile(allm, 99)), p999_ms=float(np.percentile(allm, 99.9)),
               max_ms=float(allm.max()), rows_per_s=float(sum(g[1] for g in got)),
               p99_ms_per_rank=[float(g[2]) for g in got],
               batches=int(sum(g[3] for g in got)),
               **({"outputs_match_direct_predict": all(g[4] for g in got)}
                  if "outputs_match_direct_predict" in mine else {}),
               path=f"{world} ranks, each on its own GPU: {mine['path']}; percentiles over "
                    "all ranks' requests (rank 0's batch statistics)")
    return out


_H2D = {}


def pinned_h2d_GBps(device) -> float:
    """Pinned host -> device copy rate of this box (1 GiB, best of 3), the
    bound a host-buffer predict's input stream meets; measured once."""
    if device in _H2D:
        return _H2D[device]
    import torch
    n = 1 << 30
    src = torch.empty(n, dtype=torch.uint8).pin_memory()
    dst = torch.empty(n, dtype=torch.uint8, device=device)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(3):
        t0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, n / (time.perf_counter() - t0) / 1e9)
    del src, dst
    _H2D[device] = best
    return best


def host_to_host(dev, X_host, rows, reps=3, device="cuda"):
    """A workload through ti_predict from pageable host memory to host memory
    (the path the plugins take): chunks of TI_CHUNK_MB (64) MB alternate
    between two streams, so H2D, kernel and D2H of neighbouring chunks overlap
    (DESIGN.md 5).  PCIe-inclusive; never the headline value.  Beside the rate:
    the input bytes a row, the box's pinned H2D rate and the rate that alone
    would allow (`pcie_bound_rows_per_s`), and the fraction reached."""
    from kfserving_amd.forest import OUT_PREDICT
    Xb = np.tile(X_host, (max(1, -(-rows // X_host.shape[0])), 1))[:max(rows, 1)]
    dev.predict(Xb[:4096], OUT_PREDICT)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dev.predict(Xb, OUT_PREDICT)
        times.append(time.perf_counter() - t0)
    t = min(times)
    row_b = Xb.nbytes / Xb.shape[0]
    res = {"rows": Xb.shape[0], "dtype": str(Xb.dtype), "bytes_per_row_in": row_b,
           "chunk_mb": int(os.environ.get("TI_CHUNK_MB", "64")),
           "rows_per_s": Xb.shape[0] / t, "ms": t * 1e3, "input_GBps": Xb.nbytes / t / 1e9,
           "reps": reps, "path": "pageable numpy -> pinned chunks -> H2D -> kernel -> D2H -> "
                                 "numpy, two streams"}
    if device != "cpu":
        h2d = pinned_h2d_GBps(device)
        res.update(h2d_pinned_GBps=h2d, pcie_bound_rows_per_s=h2d * 1e9 / row_b,
                   frac_of_pcie_bound=res["input_GBps"] / h2d)
    del Xb
    return res


# ------------------------------------------------------------ other configs
def device_normal(rows, cols, seed, device, dtype="float32"):
    """X ~ N(0,1) generated on the device in 8M-row chunks (seed, chunk), as
    float32 or float64 (the float64 draws are not the float32 ones widened)."""
    import torch
    dt = torch.float64 if dtype == "float64" else torch.float32
    X = torch.empty((rows, cols), dtype=dt, device=device)
    chunk = 8 << 20
    for i, lo in enumerate(range(0, rows, chunk)):
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1000003 + i)
        hi = min(rows, lo + chunk)
        X[lo:hi] = torch.randn((hi - lo, cols), generator=g, device=device, dtype=dt)
    return X


def _lgb_forest(trees, what):
    import tempfile
    from kfserving_amd.formats import lightgbm_format as lf
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "model.txt")
        lf.write_lightgbm_text(p, trees, 100, "binary sigmoid:1")
        return lf.load_lightgbm_model(p), trees, what


def c2_hist_forest():
    """C2's shape as xgboost's hist / approx tree methods train it: the same
    draws with every threshold on the nearest of 253 N(0,1) quantile bin
    bounds (max_bin 254), so at most 253 thresholds a feature and u8 bins."""
    from kfserving_amd.formats.xgboost_format import (forest_from_raw_trees,
                                                      synthetic_complete_trees)
    trees, ti = synthetic_complete_trees(N_TREES, DEPTH, N_FEAT, seed=0, max_bin=254)
    return (forest_from_raw_trees(trees, ti, N_FEAT, 0, 0.0, "binary:logistic"), (trees, ti),
            "XGBoost binary:logistic, 500 x depth 8, thresholds on 253 quantile bin bounds")


_C3_CACHE = []


def c3_forest():
    """The C3 forest (built once: c3 and c3_f64 share it)."""
    if not _C3_CACHE:
        from kfserving_amd.formats import lightgbm_format as lf
        _C3_CACHE.append(_lgb_forest(lf.synthetic_leafwise_trees(1000, 255, 100, seed=1),
                                     "LightGBM text v3, seeded leaf-wise generator "
                                     "(i.i.d. N(0,1) thresholds)"))
    return _C3_CACHE[0]


def c3_maxbin_forest():
    """C3 shaped like a LightGBM model trained at max_bin = 255 on N(0,1)
    features (lightgbm_format.synthetic_maxbin_trees): thresholds on the 254
    quantile bin edges, intervals nested along each path, missing type None.
    At most 254 thresholds a feature, so layout 9 bins to u8."""
    from kfserving_amd.formats import lightgbm_format as lf
    return _lgb_forest(lf.synthetic_maxbin_trees(1000, 255, 100, seed=1),
                       "LightGBM text v3, seeded max_bin-255 leaf-wise generator "
                       "(quantile-edge thresholds, nested intervals, missing type None)")


def c4_forest():
    """The C4 forest and its raw sklearn tree arrays (for the CPU baseline)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import make_c4_model as mk
    from kfserving_amd.formats.sklearn_format import (forest_from_sklearn, load_tree_arrays,
                                                      tree_arrays_from_sklearn)
    if os.path.exists(mk.MODEL):
        z = np.load(mk.MODEL, allow_pickle=False)
        keys = ("children_left", "children_right", "feature", "threshold",
                "missing_go_to_left", "value")
        raw = [{k: z[f"t{i}_{k}"] for k in keys} for i in range(int(z["n_trees"]))]
        return load_tree_arrays(mk.MODEL), raw, ("cached fit on 200k rows "
                                                 f"({os.path.relpath(mk.MODEL, ROOT)})")
    rows = 20_000      # the full fit takes minutes: a smaller training set, said so in the output
    est = mk.fit(rows, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())))
    raw = [tree_arrays_from_sklearn(e.tree_) for e in est.estimators_]
    return forest_from_sklearn(est), raw, f"fitted here on {rows} rows (cache absent)"


def run_config(forest, n_feat, total_rows, seed, args, world, rank, device, dev_sync,
               make_engine, cpu_fn=None, pmc_workload=None, pmc_path=None, dtype="float32",
               cpu_cap=2_000_000, host_leg=False):
    """Strong scaling: this rank's block of the batch, K steps, max-over-ranks wall.
    The CPU baseline is not timed here: rank 0 keeps a host sample of its
    block (at most cpu_cap rows) and run() times it at the end."""
    import torch
    from kfserving_amd.forest import OUT_PREDICT, TI_F32, TI_F64
    lo, hi = strong_shard(total_rows, rank, world)
    rows = hi - lo
    eng = make_engine(forest)
    X = device_normal(rows, n_feat, seed + rank, device, dtype)
    xdt = TI_F64 if dtype == "float64" else TI_F32
    out = torch.empty(rows * forest.output_width(OUT_PREDICT),
                      dtype=torch.float64 if forest.accum_dtype else torch.float32, device=device)
    sh = torch.cuda.current_stream().cuda_stream if device != "cpu" else 0

    def step():
        eng.predict_device(X.data_ptr(), xdt, rows, n_feat, n_feat, OUT_PREDICT,
                           out.data_ptr(), out.numel(), slot=0, stream=sh)

    step()
    ev = ((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          if device != "cpu" else None)
    wall, kms = timed_steps(step, args.config_steps, dev_sync, ev)
    wall = max_over_ranks(wall, device)
    res = None
    if rank == 0:
        res = {"rows": total_rows, "rows_per_gpu": rows, "scaling": "strong", "dtype": dtype,
               "steps": args.config_steps, "rows_per_s": total_rows * args.config_steps / wall,
               "ms_per_step": wall / args.config_steps * 1e3, "kernel_ms_rank0": kms,
               "layout": LAYOUT_NAMES.get(eng.info()["layout"]),
               "bin_bits": eng.info().get("bin_bits"),
               "compulsory_GBps": ((X.element_size() * n_feat + out.element_size()) * rows
                                   / (kms * 1e-3) / 1e9 if kms else None)}
        if pmc_path and kms:
            res["roofline"] = config_roofline(kms, rows, eng.info(), pmc_workload, pmc_path)
        if cpu_fn is not None and not args.no_cpu_baseline:
            # timed later (run: after every rank's GPU legs, on the full host):
            # keep a host copy of this rank's block, up to the sample cap
            res["_cpu"] = (cpu_fn, X[:min(rows, cpu_cap)].cpu().numpy())
        if host_leg and args.host_rows_configs > 0 and hasattr(eng, "predict"):
            # the plugins' real path: pageable numpy of
            # the config's dtype -> ti_predict's pinned chunks -> H2D ->
            # kernel -> D2H -> numpy (lgbserver hands float64 DataFrames,
            # lgbserver/model.py:46-51; sklearnserver float32 after
            # check_array, sklearnserver/model.py:46-51)
            Xh = X[:min(rows, 1_000_000)].cpu().numpy()
            res["_host_pipeline"] = host_to_host(eng, Xh, args.host_rows_configs, device=device)
    del X, out
    eng.close()
    if device != "cpu":
        torch.cuda.empty_cache()
    return res


def sample_taker(Xh: np.ndarray):
    """take(n): the first n rows of a host sample, tiled when the sample (a
    rank's block at large N) is shorter than n."""
    def take(n):
        n = int(n)
        if n <= Xh.shape[0]:
            return Xh[:n]
        reps = -(-n // Xh.shape[0])
        return np.concatenate([Xh] * reps)[:n]
    return take


def baseline_threads() -> int:
    """Host threads for the CPU baselines: the whole host share of the job.
    launch_ranks records it in BENCH_HOST_THREADS before it splits
    OMP_NUM_THREADS over the ranks; under an outside launcher it is
    OMP_NUM_THREADS (the box's share, which torchrun leaves alone when set)
    or the affinity mask."""
    env = os.environ.get("BENCH_HOST_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return host_threads()


def _scaled_sample(fn, take, target_s, probe=20_000, cap=10_000_000):
    """Time fn on a probe, then on a sample sized for about target_s seconds;
    a sample that ran under half the target (a probe too small to show the
    steady rate: thread-pool start-up) is re-sized from its own rate once."""
    Xp = take(probe)
    t0 = time.perf_counter()
    fn(Xp)
    rate = Xp.shape[0] / max(time.perf_counter() - t0, 1e-9)
    n, dt = 0, 0.0
    for _ in range(2):
        Xs = take(int(min(cap, max(probe, rate * target_s))))
        t0 = time.perf_counter()
        fn(Xs)
        n, dt = Xs.shape[0], time.perf_counter() - t0
        if dt >= 0.5 * target_s or n >= cap:
            break
        rate = n / max(dt, 1e-9)
    return n, dt


def c3_cpu(trees, target_s, dtype="float32"):
    def fn(take):
        from oracle import port
        thr = baseline_threads()
        n, dt = _scaled_sample(
            lambda Xs: port.lgb_predict_raw(trees, 1, 100, Xs.astype(np.float64), nthread=thr),
            take, target_s)
        return {"value": n / dt, "unit": "rows/s", "cores": thr,
                "kind": "port", "sample": f"{n} rows of the same {dtype} batch, "
                                          "oracle/c/tree_port.c (lightgbm predict loop restated, "
                                          f"OpenMP {thr} threads), {dt:.1f} s"}
    return fn


def host_threads() -> int:
    """The host threads this process may use: OMP_NUM_THREADS when set (the
    GPU box sets it to the box's CPU share, 16), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def c4_cpu(raw_trees, target_s):
    """C4's CPU baseline is the library: sklearn's own RandomForestRegressor
    .predict (sklearnserver/model.py:46-51) on the fitted forest rebuilt from
    its cached arrays (scripts/make_c4_model.sklearn_estimator, checked bit for
    bit against the fitted estimator's answers), n_jobs = the host threads.
    The C restatement is timed beside it as `cpu_baseline_port`."""
    def fn(take):
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import make_c4_model as mk
        res = {}
        if os.path.exists(mk.MODEL) and os.path.exists(mk.CHECK):
            est = mk.sklearn_estimator()
            same = mk.check(est)
            thr = baseline_threads()
            est.set_params(n_jobs=thr)
            n, dt = _scaled_sample(est.predict, take, target_s, probe=4096)
            import sklearn
            res["cpu_baseline"] = {
                "value": n / dt, "unit": "rows/s", "cores": thr, "kind": "library",
                "sample": f"{n} rows of the same float32 batch, sklearn {sklearn.__version__} "
                          f"RandomForestRegressor.predict(n_jobs={thr}) on the cached fit "
                          f"(rebuilt from its arrays; equal to the fitted estimator on the "
                          f"check rows: {same}), {dt:.1f} s"}
        from oracle import port
        pthr = baseline_threads()
        n, dt = _scaled_sample(lambda Xs: port.sk_predict(raw_trees, 1, 64, Xs, nthread=pthr),
                               take, min(target_s, 5.0), probe=4096)
        res["cpu_baseline_port"] = {
            "value": n / dt, "unit": "rows/s", "cores": pthr, "kind": "port",
            "sample": f"{n} rows, oracle/c/tree_port.c (sklearn forest predict restated), "
                      f"{dt:.1f} s"}
        return res
    return fn


# ------------------------------------------------------------------- main
def run(args, device="cuda", backend="nccl", make_engine=None):
    """The rank logic of bench.py.  `make_engine(forest)` returns an object with
    predict_device / predict / info / close (DeviceForest on the GPU; the CPU
    tests pass a stub).  Returns the JSON line rank 0 prints (None elsewhere)."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if device == "cuda":
        torch.cuda.set_device(local_rank)          # before the process group
        device = f"cuda:{local_rank}"
        dev_sync = torch.cuda.synchronize
    else:
        dev_sync = lambda: None                    # noqa: E731
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": torch.device(device)} if backend == "nccl" else {}
        dist.init_process_group(backend, init_method="env://", **kw)
    if make_engine is None:
        from kfserving_amd.engine import DeviceForest
        make_engine = lambda f: DeviceForest(f, devices=[local_rank])   # noqa: E731

    from kfserving_amd.forest import OUT_PREDICT, TI_F32

    trees, ti, forest = build_model()
    dev = make_engine(forest)
    info = dev.info()
    rows, seed = shard_rows(args.rows, rank, world)
    X_host = np.random.default_rng(seed).standard_normal((rows, N_FEAT), dtype=np.float32)
    X = torch.from_numpy(X_host).to(device)
    # consecutive steps read different batches: 3 x 112 MB is more than the
    # 256 MB Infinity Cache, so a step's X comes from HBM, not from the
    # previous step's cache lines.  Each buffer is its own batch (seeded), so
    # the check after the timed region can tell the batches in flight apart
    Xs = [X] + [device_normal(rows, N_FEAT, seed * 7919 + i, device)
                for i in range(1, max(1, args.x_buffers))]
    out = torch.empty(rows, dtype=torch.float32, device=device)
    sh = torch.cuda.current_stream().cuda_stream if device != "cpu" else 0
    it = [0]
    # --streams S > 1: consecutive steps (independent batches) go round-robin
    # over S streams, each with its own output, as batches in flight do
    n_str = max(1, args.streams) if device != "cpu" else 1
    strs = [None] + [torch.cuda.Stream(device=device) for _ in range(n_str - 1)]
    outs = [out] + [torch.empty_like(out) for _ in range(n_str - 1)]

    last_x = [None] * n_str     # the X buffer each stream's last launch read

    def launch(k):
        last_x[k] = it[0] % len(Xs)
        Xi = Xs[last_x[k]]
        it[0] += 1
        dev.predict_device(Xi.data_ptr(), TI_F32, rows, N_FEAT, N_FEAT, OUT_PREDICT,
                           outs[k].data_ptr(), rows, slot=0,
                           stream=sh if k == 0 else strs[k].cuda_stream)

    def step1():   # one stream: each launch alone on the chip
        launch(0)

    def step():    # --streams S: batch i on stream i mod S
        launch(it[0] % n_str)

    def fork():
        for st in strs[1:]:
            st.wait_stream(torch.cuda.current_stream())

    def join():
        for st in strs[1:]:
            torch.cuda.current_stream().wait_stream(st)

    def events():
        return ((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                if device != "cpu" else None)

    # K steps on one stream: the kernel's own launch duration (events on the
    # stream it runs on), which the roofline and the rocprof summary price
    for _ in range(args.warmup):
        step1()
    wall1, kernel_ms = timed_steps(step1, args.steps, dev_sync, events())
    if kernel_ms is None:
        kernel_ms = wall1 / args.steps * 1e3
    wall1 = max_over_ranks(wall1, device)
    wall = wall1
    if n_str > 1:
        # the headline: the same K steps with S batches in flight, so one
        # batch's binning and tail overlap the previous batch's walk
        for _ in range(args.warmup):
            step()
        wall, _ = timed_steps(step, args.steps, dev_sync, events(), fork, join)
        wall = max_over_ranks(wall, device)
    # each stream's last output against a one-stream predict of the batch it
    # read (every X buffer is a distinct batch): no batch in flight was
    # skipped, cut short or written by the other stream
    outputs_identical = streams_match(dev, Xs, outs, last_x, rows, sh, dev_sync, device != "cpu")
    value = rows * world * args.steps / wall
    two_stream = None
    if n_str > 1:
        two_stream = batch_latency_events(launch, n_str, strs, args.steps, dev_sync)

    # the serving-latency leg runs right after the headline, before the legs
    # that load the host (CPU baselines' thread pools, the 8M-row host
    # pipeline) or hold tens of GB on the device (C3 / C4): its p99 then
    # measures the batcher and the engine, not what ran before it
    latency = latency_asyncio = None
    if args.latency_qps > 0:
        # C5 on every GPU at once: each rank is one serving worker with its own
        # batcher in front of its own GPU (KFServer's pre-forked workers, one
        # GPU each), offered latency_qps; the latencies of all ranks are
        # pooled on rank 0
        barrier_sync(dev_sync)
        mine = native_batched_latency(dev, N_FEAT, args.latency_qps, args.latency_seconds,
                                      seed=7 + 1000 * rank)
        latency = pool_latency(mine, world, rank, device)
        # the same load through the asyncio batcher (kfserving_amd.batcher.Batcher,
        # KF_NATIVE_BATCHER=0), for comparison
        barrier_sync(dev_sync)
        mine = batched_latency(dev, N_FEAT, args.latency_qps, args.latency_seconds,
                               seed=7 + 1000 * rank)
        latency_asyncio = pool_latency(mine, world, rank, device)

    nan_variant = None
    if args.nan_variant > 0 and rank == 0 and device != "cpu":
        # same shape, seed 1, NaN at random positions: every tile takes the
        # kernel's NaN-checking path (not part of the headline value)
        Xn_host = np.random.default_rng(1).standard_normal((rows, N_FEAT), dtype=np.float32)
        Xn_host[np.random.default_rng(2).random(Xn_host.shape) < args.nan_variant] = np.nan
        Xn = torch.from_numpy(Xn_host).to(device)

        def nstep():
            dev.predict_device(Xn.data_ptr(), TI_F32, rows, N_FEAT, N_FEAT, OUT_PREDICT,
                               out.data_ptr(), rows, slot=0, stream=sh)
        nstep()
        nstep()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            nstep()
        e1.record()
        torch.cuda.synchronize()
        nms = e0.elapsed_time(e1) / args.steps
        nan_variant = {"nan_fraction": args.nan_variant, "kernel_ms": nms,
                       "rows_per_s": rows / (nms * 1e-3)}
        del Xn

    tree_shard = None
    if not args.no_tree_shard:
        tree_shard = tree_shard_leg(forest, dev, rows, args, world, rank, local_rank, device,
                                    dev_sync, make_engine if device == "cpu" else None)

    host_pipeline = None
    if args.host_rows > 0 and rank == 0 and device != "cpu":
        host_pipeline = host_to_host(dev, X_host, args.host_rows, device=device)

    configs = {}
    for name in [c.strip() for c in args.configs.split(",") if c.strip()]:
        if name in ("c3", "c3_f64", "c3_maxbin"):
            f3, t3, src = c3_maxbin_forest() if name == "c3_maxbin" else c3_forest()
            dt = "float64" if name == "c3_f64" else "float32"
            r = run_config(f3, 100, args.rows3, 3, args, world, rank, device, dev_sync,
                           make_engine, c3_cpu(t3, args.cpu_seconds / 2, dt), name,
                           pmc_path(name), dt, host_leg=name != "c3_maxbin")
            if r is not None:
                r.update(config=f"C3 LightGBM leaf-wise 1000 trees x 255 leaves, 100 features, "
                                f"{dt} input, float64 sigmoid of the raw score", model=src)
        elif name == "c2_hist":
            f2, _, src = c2_hist_forest()
            r = run_config(f2, N_FEAT, args.rows, 4, args, world, rank, device, dev_sync,
                           make_engine, None, "c2_hist", pmc_path("c2_hist"))
            if r is not None:
                r.update(config="C2 shape, hist-trained thresholds (u8 bins): 500 trees depth 8, "
                                "28 features, float32 input, float32 sums", model=src)
        elif name == "c4":
            f4, raw4, src = c4_forest()
            r = run_config(f4, 64, args.rows4, 2, args, world, rank, device, dev_sync,
                           make_engine, c4_cpu(raw4, args.cpu_seconds / 2), "c4",
                           pmc_path("c4"), cpu_cap=10_000_000, host_leg=True)
            if r is not None:
                r.update(config="C4 sklearn RandomForestRegressor 200 trees max_depth 16, "
                                "64 features, float32 input, float64 mean", model=src)
        else:
            raise ValueError(f"unknown config {name!r}")
        configs[name] = r

    # the CPU baselines, at every world size: after the last rank's GPU legs,
    # on rank 0 alone with the whole host share (the other ranks have left
    # the process group and exit; none of them spins on a device sync)
    barrier_sync(dev_sync)
    dev.close()
    if world > 1:
        dist.destroy_process_group()
    if rank != 0:
        return None
    c5_http = c5_http_v2 = None
    http_ok = device != "cpu" or args.c5_http_cpu
    if args.c5_http_qps and http_ok:
        c5_http = c5_http_leg(args, world, device=device)
    if args.c5_http_v2_qps and http_ok:
        c5_http_v2 = c5_http_leg(args, world, "v2", device=device)
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline(trees, ti, X_host, args.cpu_seconds)
        for name, r in configs.items():
            if r is not None and "_cpu" in r:
                fn, Xh = r.pop("_cpu")
                got = fn(sample_taker(Xh))
                if "cpu_baseline" in got or "cpu_baseline_port" in got:
                    r.update(got)               # C4: the library and the port
                else:
                    r["cpu_baseline"] = got
    host_configs = {}
    for name, r in configs.items():
        if r is not None:
            r.pop("_cpu", None)
            if "_host_pipeline" in r:
                host_configs["host_pipeline_" + name] = r.pop("_host_pipeline")
    line = None
    if rank == 0:
        line = {
            "metric": "predicted rows/sec (500-tree XGB, 28 feat)",
            "value": value,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: X ~ N(0,1) float32, seeded; random 500 x depth-8 XGBoost "
                    "binary:logistic trees (SURVEY.md 8(d) C2)",
            "config": {"workload": "C2 synthetic HIGGS-shaped XGBoost binary: 28 features, "
                                   "500 trees depth 8, 1M-row batch per GPU",
                       "rows_per_gpu": rows, "trees": N_TREES, "depth": DEPTH,
                       "features": N_FEAT, "layout": LAYOUT_NAMES.get(info["layout"]),
                       "parallelism": f"rows sharded x{world}", "x_buffers": len(Xs),
                       "streams": n_str},
            "single_stream": {"ms_per_step": wall1 / args.steps * 1e3,
                              "value": rows * world * args.steps / wall1,
                              "kernel_ms": kernel_ms},
            "streams_outputs_identical": outputs_identical,
            "roofline": headline_roofline(kernel_ms, rows, info, args.pmc_json, wall / args.steps,
                                          two_stream, n_str),
            "cpu_baseline": cpu,
            "batched_latency": latency,
            "batched_latency_asyncio": latency_asyncio,
            "nan_variant": nan_variant,
            "host_pipeline": host_pipeline,
            "tree_shard": tree_shard,
            "c5_http": c5_http,
            "c5_http_v2": c5_http_v2,
        }
        line.update(configs)
        line.update(host_configs)
    return line


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started without a launcher: start N ranks, one
    process per GPU, under torch.distributed.run (a child process, never an
    exec: nothing here has touched the GPU) and return its exit code.  Rank 0
    prints the JSON line; value = all ranks' rows / the slowest rank's wall
    (the reference's parallelism this stands for: KFServer's pre-forked
    workers, python/kfserving/kfserving/kfserver.py:99)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # the CPU baselines run on rank 0 after the GPU legs with the whole host
    # share; the ranks' own host work gets an equal part of it
    env.setdefault("BENCH_HOST_THREADS", str(host_threads()))
    env["OMP_NUM_THREADS"] = str(max(1, host_threads() // n))
    return subprocess.run(cmd, env=env).returncode


def resolve_engine(spec: str):
    """--engine MODULE:FACTORY -> make_engine(forest) for this rank (None: the GPU engine)."""
    if not spec:
        return None
    import importlib
    mod, _, attr = spec.partition(":")
    factory = getattr(importlib.import_module(mod), attr)
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    return lambda forest: factory(forest, local_rank)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; timing {world} rank(s)",
              file=sys.stderr, flush=True)
    backend = "gloo" if args.device == "cpu" else "nccl"
    line = run(args, device=args.device, backend=backend, make_engine=resolve_engine(args.engine))
    if line is not None:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
