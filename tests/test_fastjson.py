"""The native v1 body parser (libkfserve.so) against json.loads + numpy: bit
for bit on every body of its subset, and a fallback (None) on everything else."""
import json
import math
import random
import struct

import numpy as np
import pytest

from kfserving_amd.kfserving.fastjson import JsonInstances, parse_instances


def _ref(body: bytes):
    return np.asarray(json.loads(body)["instances"], dtype=np.float64)


def _same(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def _rand_number(rng: random.Random) -> str:
    k = rng.randrange(12)
    if k == 0:
        return repr(struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]) \
            .replace("nan", "NaN").replace("inf", "Infinity")
    if k == 1:
        return str(rng.randrange(-10 ** 18 + 1, 10 ** 18))
    if k == 2:
        return str(rng.randrange(-1000, 1000))
    if k == 3:
        return f"{rng.uniform(-1, 1):.{rng.randrange(1, 25)}f}"
    if k == 4:
        return f"{rng.randrange(1, 10 ** rng.randrange(1, 21))}e{rng.randrange(-340, 320)}"
    if k == 5:
        return f"{rng.uniform(-1e6, 1e6):.{rng.randrange(1, 17)}e}".replace("e+", "E+")
    if k == 6:
        return rng.choice(["0", "-0", "0.0", "-0.0", "NaN", "Infinity", "-Infinity", "1e308",
                           "1e309", "-1e-400", "4.9e-324", "2.2250738585072014e-308",
                           "9007199254740993", "9007199254740993.0", "0.1", "1E22", "1e23",
                           "123456789012345678", "0.30000000000000004"])
    if k == 7:
        digits = "".join(rng.choice("0123456789") for _ in range(rng.randrange(1, 40)))
        return f"{rng.randrange(10)}.{digits}"
    if k == 8:
        return "0." + "0" * rng.randrange(0, 30) + str(rng.randrange(1, 10 ** 6))
    return repr(rng.gauss(0, 1) * 10 ** rng.randrange(-30, 30))


def _body(rng, rows, cols):
    ws = [" ", "", "\n", "\t", "\r\n  "]
    w = lambda: rng.choice(ws)   # noqa: E731
    rs = []
    for _ in range(rows):
        rs.append("[" + w() + ("," + w()).join(_rand_number(rng) + w() for _ in range(cols)) + "]")
    return ("{" + w() + '"instances"' + w() + ":" + w() + "[" + w() +
            ("," + w()).join(r + w() for r in rs) + "]" + w() + "}" + w()).encode()


def test_fuzz_bit_exact():
    rng = random.Random(1234)
    for _ in range(3000):
        body = _body(rng, rng.randrange(1, 6), rng.randrange(1, 9))
        got = parse_instances(body)
        assert got is not None, body
        assert isinstance(got, JsonInstances)
        assert _same(np.asarray(got), _ref(body)), body


def test_typical_float_rows():
    X = np.random.default_rng(0).standard_normal((64, 28))
    body = json.dumps({"instances": X.tolist()}).encode()
    got = parse_instances(body)
    assert _same(np.asarray(got), X)
    body = json.dumps({"instances": X.astype(np.float32).tolist()}).encode()
    assert _same(np.asarray(parse_instances(body)), _ref(body))


@pytest.mark.parametrize("body", [
    b'{"instances": []}', b'{"instances": [[]]}', b'{"instances": [[1, 2], [3]]}',
    b'{"instances": [1, 2]}', b'{"instances": [[1, "2"]]}', b'{"instances": [[true]]}',
    b'{"instances": [[null]]}', b'{"instances": [[1]], "x": 1}', b'{"x": 1, "instances": [[1]]}',
    b'{"instances": [[01]]}', b'{"instances": [[1.]]}', b'{"instances": [[.5]]}',
    b'{"instances": [[+1]]}', b'{"instances": [[1e]]}', b'{"instances": [[-NaN]]}',
    b'{"instances": [[1]]} x', b'{"instances": [[1]]', b'{"instances": [[1,]]}',
    b'{"instances": [[[1]]]}', b'{"inst\\u0061nces": [[1]]}', b'\xef\xbb\xbf{"instances": [[1]]}',
    b'{"instances": [[1234567890123456789]]}', b'', b'[]', b'{"instances": [[1], ]}',
    b'{"instances": [[1] [2]]}', b'{"instances": [[1 2]]}', b'{"instances": [[infinity]]}',
])
def test_fallback_outside_subset(body):
    assert parse_instances(body) is None


def test_large_body():
    X = np.random.default_rng(1).standard_normal((20000, 28))
    body = json.dumps({"instances": X.tolist()}).encode()
    assert _same(np.asarray(parse_instances(body)), X)


# ---------------------------------------------------------------- threaded
def _big_body(seed, rows=3000, cols=28):
    return _body(random.Random(seed), rows, cols)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_threaded_bit_exact(seed):
    """kf_parse_instances_mt (bodies >= 1 MB): the same matrix as json.loads
    and the one-thread parser, for any thread count (slice cuts land anywhere:
    inside numbers, whitespace, between rows)."""
    body = _big_body(seed)
    assert len(body) >= 1 << 20
    want = _ref(body)
    one = parse_instances(body, threads=1)
    assert _same(np.asarray(one), want)
    for t in (2, 3, 7, 8, 16):
        got = parse_instances(body, threads=t)
        assert got is not None and isinstance(got, JsonInstances), t
        assert _same(np.asarray(got), want), t


def test_threaded_rejects_what_one_thread_rejects():
    """Malformed bodies fall back whichever slice the damage lands in: a
    missing or doubled row comma, a ragged row, a stray bracket, trailing
    junk, a broken envelope."""
    body = _big_body(4).decode()
    rows_at = [i for i, ch in enumerate(body) if ch == "["][2:]   # row starts after the first
    rng = random.Random(5)
    cases = []
    for k in rng.sample(rows_at, 12):
        j = body.rfind(",", 0, k)                         # the comma before this row
        cases.append(body[:j] + body[j + 1:])             # missing comma
        cases.append(body[:j] + ",," + body[j + 1:])      # doubled comma
        e = body.find("]", k)
        c = body.rfind(",", k, e)
        cases.append(body[:c] + body[e:])                 # ragged: last value of the row dropped
        cases.append(body[:k] + "[" + body[k:])           # stray '[' (a nested row)
        cases.append(body[:e] + ",]" + body[e + 1:])      # trailing comma in a row
    cases.append(body + "x")
    last_close = body.rstrip().rstrip("}").rstrip().rfind("]")    # the instances list's ']'
    cases.append(body[:last_close] + "," + body[last_close:])     # trailing comma after the last row
    cases.append(body[:last_close] + ", " + body[last_close:])
    cases.append(body.replace('"instances"', '"instance"', 1))
    cases.append(body.rstrip()[:-1])                       # no closing brace
    for bad in cases:
        b = bad.encode()
        assert parse_instances(b, threads=1) is None
        for t in (2, 8):
            assert parse_instances(b, threads=t) is None, (t, bad[:80])
