"""Replays tests/golden/kfhttp_corpus.jsonl through libkfserve.so (the native
HTTP front end kh_* and the body parsers kf_parse_*) in this process.  Run by
tests/test_asan_fuzz.py as a child process with KFSERVE_LIB pointing at the
AddressSanitizer + UBSan build (__graft_entry__.build_host(asan=True)) and
LD_PRELOAD=libasan, so any out-of-bounds access, use-after-free or undefined
behaviour in the native code aborts the child with the sanitizer's report.

Checks, beside the sanitizer: every HTTP case's first status is one the case
allows (the reference's 400 / 413 contract, handlers/http.py:68-74,
kfserver.py:39, or the application's answer), the server still answers after
the corpus, and every parser call returns a documented code with its rows
inside the output buffer.  Bodies handed to the parsers are exact-size
malloc blocks, so a read one byte past the body is caught.  Prints one JSON
summary line; exits 1 on a failed expectation.
"""
import base64
import ctypes
import json
import os
import shutil
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

CORPUS = os.path.join(ROOT, "tests", "golden", "kfhttp_corpus.jsonl")
MODEL = "xgboost-iris"
GOOD = b'{"instances": [[6.8, 2.8, 4.8, 1.4], [6.0, 3.4, 4.5, 1.6]]}'
LGB_NAMES = ["sepal_length_(cm)", "sepal_width_(cm)", "petal_length_(cm)", "petal_width_(cm)"]

_libc = ctypes.CDLL(None)
_libc.malloc.restype = ctypes.c_void_p
_libc.malloc.argtypes = [ctypes.c_size_t]
_libc.free.argtypes = [ctypes.c_void_p]
failures = []


def fail(msg):
    failures.append(msg)
    print("FAIL", msg, file=sys.stderr, flush=True)


def req(body, path=f"/v1/models/{MODEL}:predict".encode(), extra=b""):
    return (b"POST " + path + b" HTTP/1.1\r\nHost: x\r\n" + extra +
            b"Content-Length: %d\r\n\r\n" % len(body) + body)


# ---------------------------------------------------------------- HTTP
def send(port, data, shut=True, timeout=10.0, read=True):
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    out = []
    try:
        try:
            s.sendall(data)
            if shut:
                s.shutdown(socket.SHUT_WR)
        except (BrokenPipeError, ConnectionResetError):
            pass
        while read:
            try:
                b = s.recv(65536)
            except (socket.timeout, ConnectionResetError):
                break
            if not b:
                break
            out.append(b)
    finally:
        s.close()
    return b"".join(out)


def first_status(resp):
    if not resp.startswith(b"HTTP/1."):
        return None
    try:
        return int(resp[9:12])
    except ValueError:
        return None


def recipe(name, port, model):
    if name == "header_line_over_limit":
        return send(port, req(GOOD, extra=b"X-Long: " + b"a" * ((1 << 20) + 100) + b"\r\n"))
    if name == "request_line_over_limit":
        return send(port, b"GET /" + b"a" * ((1 << 20) + 100) + b" HTTP/1.1\r\n\r\n")
    if name == "many_headers":
        return send(port, req(GOOD, extra=b"".join(b"X-H%d: v\r\n" % i for i in range(5000))))
    if name == "body_cut_at_every_offset":
        full = req(GOOD)
        first = None
        for cut in range(1, len(full)):
            r = send(port, full[:cut], timeout=5)
            st = first_status(r)
            if st not in (None, 200, 400):
                fail(f"cut at {cut}: status {st}")
            first = first if first is not None else r
        return send(port, full)
    if name == "slow_request_pipelined_megabytes":
        fast = model.predict_matrix

        def slow(X, kind=1):
            time.sleep(0.5)
            return fast(X, kind)
        model.predict_matrix = slow
        try:
            return send(port, req(GOOD) + b"x" * (8 << 20), timeout=20)
        finally:
            model.predict_matrix = fast
    raise ValueError(name)


# ---------------------------------------------------------------- parsers
def bind_parsers(lib):
    i64p = ctypes.POINTER(ctypes.c_int64)
    vp = ctypes.c_void_p
    lib.kf_parse_instances.restype = ctypes.c_int
    lib.kf_parse_instances.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int64, i64p, i64p]
    lib.kf_parse_instances_mt.restype = ctypes.c_int
    lib.kf_parse_instances_mt.argtypes = lib.kf_parse_instances.argtypes + [ctypes.c_int32]
    lib.kf_parse_inputs.restype = ctypes.c_int
    lib.kf_parse_inputs.argtypes = [vp, ctypes.c_int64, vp, vp, ctypes.c_int32, vp,
                                    ctypes.c_int64, i64p]
    lib.kf_parse_v2_tensor.restype = ctypes.c_int
    lib.kf_parse_v2_tensor.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_int64,
                                       i64p, i64p, ctypes.POINTER(ctypes.c_int32), i64p, i64p,
                                       ctypes.POINTER(ctypes.c_int32)]


class Exact:
    """An exact-size malloc block holding `data` (ASan red zones either side)."""

    def __init__(self, data: bytes):
        self.n = len(data)
        self.p = _libc.malloc(max(1, self.n) if self.n == 0 else self.n)
        ctypes.memmove(self.p, data, self.n)

    def __del__(self):
        _libc.free(self.p)


def run_parser(lib, parser, body, head_len=-1, cap=None, names=None):
    b = Exact(body)
    cap = (len(body) + 1) // 2 if cap is None else cap
    out = _libc.malloc(max(1, cap) * 8)
    rows, cols = ctypes.c_int64(-7), ctypes.c_int64(-7)
    try:
        if parser == "instances":
            rc = lib.kf_parse_instances(b.p, b.n, out, cap, ctypes.byref(rows), ctypes.byref(cols))
        elif parser == "instances_mt":
            rc = lib.kf_parse_instances_mt(b.p, b.n, out, cap, ctypes.byref(rows),
                                           ctypes.byref(cols), 4)
        elif parser == "inputs":
            blob, offs = names
            rc = lib.kf_parse_inputs(b.p, b.n, blob.p, offs.ctypes.data, len(offs) - 1, out, cap,
                                     ctypes.byref(rows))
            cols.value = len(offs) - 1
        else:
            dt, io, il, bo = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
            rc = lib.kf_parse_v2_tensor(b.p, b.n, head_len, out, cap, ctypes.byref(rows),
                                        ctypes.byref(cols), ctypes.byref(dt), ctypes.byref(io),
                                        ctypes.byref(il), ctypes.byref(bo))
            if rc == 1 and not (0 <= io.value and io.value + il.value <= b.n):
                fail(f"{parser}: id span {io.value}+{il.value} outside {b.n}")
    finally:
        _libc.free(out)
    if rc not in (1, 0, -1):
        fail(f"{parser}: return code {rc}")
    if rc == 1 and not (0 < rows.value and 0 <= cols.value and rows.value * cols.value <= cap):
        fail(f"{parser}: {rows.value} x {cols.value} rows outside cap {cap}")
    return rc


def mutations(body, rng, n):
    for _ in range(n):
        if not body:
            return
        i = int(rng.integers(0, len(body)))
        v = int(rng.integers(0, 256))
        yield body[:i] + bytes([v]) + body[i + 1:]
        yield body[:i] + body[i + 1:]                    # a byte dropped
        yield body[:i] + body[i:i + 1] * 2 + body[i + 1:]   # a byte doubled


def canary(lib):
    """A deliberate read past an exact-size body (the length says 16 bytes
    more than the block holds): the sanitizer must stop the process here,
    which shows the recipe really runs instrumented code."""
    b = Exact(GOOD)
    out = _libc.malloc(1 << 12)
    rows, cols = ctypes.c_int64(), ctypes.c_int64()
    lib.kf_parse_instances(b.p, b.n + 16, out, 512, ctypes.byref(rows), ctypes.byref(cols))
    print("canary: no sanitizer report", flush=True)
    sys.exit(3)


def main():
    from kfserving_amd.kfserving import fastjson
    lib = fastjson.load_library()
    bind_parsers(lib)
    if "--canary" in sys.argv:
        canary(lib)
    cases = [json.loads(l) for l in open(CORPUS)]
    rng = np.random.default_rng(0)
    blob_bytes = b"".join(n.encode() for n in LGB_NAMES)
    offs = np.cumsum([0] + [len(n) for n in LGB_NAMES]).astype(np.int32)
    names = (Exact(blob_bytes), offs)
    n_calls = 0
    for c in cases:
        if c["kind"] != "parse":
            continue
        body = base64.b64decode(c["data"])
        variants = [body[:k] for k in range(len(body) + 1)] if c["cuts"] else [body]
        variants += list(mutations(body, rng, 60))
        for v in variants:
            run_parser(lib, c["parser"], v, c["head_len"], names=names)
            run_parser(lib, c["parser"], v, c["head_len"], cap=1, names=names)   # KF_ERR_SPACE
            n_calls += 2
    # the threaded parser engages at >= 1 MB: a big body, cut and mutated
    rows = ", ".join("[%r, %r, %r, %r]" % tuple(float(v) for v in np.round(rng.standard_normal(4), 6))
                     for _ in range(26000))
    big = ('{"instances": [' + rows + ']}').encode()
    assert len(big) > (1 << 20)
    cuts = sorted(set(int(x) for x in np.linspace(0, len(big), 120)) | {len(big) - 1, len(big) - 2})
    for v in [big[:k] for k in cuts] + list(mutations(big, rng, 40)):
        run_parser(lib, "instances_mt", v)
        n_calls += 1
    if run_parser(lib, "instances_mt", big) != 1:
        fail("the 1 MB body did not parse")

    # ---- the HTTP front end, in this process -----------------------------
    from kfserving_amd.forest import OUT_PREDICT
    from kfserving_amd.kfserving import KFServer
    from kfserving_amd.xgbserver import XGBoostModel
    from tests import canon_eval
    from tests.test_server import _Running
    tmp = tempfile.mkdtemp()
    d = os.path.join(tmp, MODEL)
    os.makedirs(d)
    shutil.copy(os.path.join(ROOT, "tests", "golden", "xgb_iris_legacy_082.bst"),
                os.path.join(d, "model.bst"))
    model = XGBoostModel(MODEL, d, 1)
    model.load()
    model.predict_matrix = lambda X, kind=OUT_PREDICT: canon_eval.predict(model._forest, X, kind)
    srv = KFServer(max_batchsize=64, max_latency_ms=2)
    srv.native_http = True
    srv.register_model(model)
    run = _Running(srv)
    t0 = time.time()
    while srv.front_end is None and time.time() - t0 < 30:
        time.sleep(0.02)
    if srv.front_end is None:
        fail("native front end did not start")
    n_http = 0
    try:
        for c in cases:
            if c["kind"] == "http":
                resp = send(run.port, base64.b64decode(c["data"]), shut=c["shut"])
            elif c["kind"] == "http_gen":
                resp = recipe(c["recipe"], run.port, model)
            else:
                continue
            n_http += 1
            st = first_status(resp)
            if c["expect"] and st not in c["expect"]:
                fail(f"{c['name']}: status {st}, expected {c['expect']}: {resp[:120]!r}")
        # the corpus again from 16 client threads at once (the IO threads,
        # the batcher's completions and the application's answers interleave:
        # a race that frees or reuses a connection's buffers early shows here)
        import threading
        small = [base64.b64decode(c["data"]) for c in cases if c["kind"] == "http"]
        errs = []

        def hammer(k):
            rng_k = np.random.default_rng(1000 + k)
            for _ in range(40):
                data = small[int(rng_k.integers(0, len(small)))]
                try:
                    send(run.port, data, shut=True, timeout=10)
                except OSError as e:   # a refused or reset connection is an answer too
                    errs.append(str(e))
        th = [threading.Thread(target=hammer, args=(k,)) for k in range(16)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        n_http += 16 * 40
        alive = send(run.port, b"GET /v1/models/%s HTTP/1.1\r\nHost: x\r\n\r\n" % MODEL.encode())
        if first_status(alive) != 200:
            fail(f"server not answering after the corpus: {alive[:120]!r}")
        ok = send(run.port, req(GOOD))
        if first_status(ok) != 200 or b'"predictions": [1.0, 1.0]' not in ok:
            fail(f"a good request after the corpus: {ok[-200:]!r}")
        stats = srv.front_end.stats()
    finally:
        run.stop()
        shutil.rmtree(tmp, ignore_errors=True)
    print(json.dumps({"parser_calls": n_calls, "http_cases": n_http, "front_end": stats,
                      "failures": failures,
                      "lib": os.environ.get("KFSERVE_LIB", "default")}), flush=True)
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
