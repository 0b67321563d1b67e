"""V2 inference protocol tensors on ``/v2/models/<name>/infer``.

The reference routes ``/v2/models/<name>/infer`` to the same handler as v1
``:predict`` (python/kfserving/kfserving/kfserver.py:77-78), so a v1-shaped
body still works there, and the protocol's tensor bodies
(docs/predict-api/v2/required_api.md:205-333) reach the plugins as dicts they
cannot read.  Here a body whose ``inputs`` are tensor objects
(``name``/``shape``/``datatype``/``data``) is decoded into a numpy array and
answered as a V2 inference response; any other body keeps the v1 path.

Two encodings of a tensor's contents:

* JSON ``data``: row-major, flat or nested (required_api.md:412-435);
* binary, the tensor-data extension the Triton clients speak (the reference's
  Triton sample requests it per output: docs/samples/v1beta1/triton/bert/
  bert_tokenizer_v2/bert_transformer_v2/bert_transformer.py:61-62; the
  extension is not part of the reference's KFServer).  The request carries an
  ``Inference-Header-Content-Length: n`` header.  The first n bytes of the
  body are the JSON header.  Each input whose ``parameters`` hold
  ``binary_data_size: k`` takes the next k bytes of the body, little-endian
  and row-major, in input order.  Outputs asked for with ``parameters:
  {"binary_data": true}`` (or the request parameter
  ``binary_data_output: true``) come back the same way.

This is the wire format with no number parsing at all: a float32 matrix goes
from the socket to the GPU kernel's float32 path as one ``np.frombuffer``.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Mapping, Optional, Tuple

import numpy as np

HEADER_LEN = "inference-header-content-length"

# required_api.md "Tensor Data Types" (BYTES is not a numeric tensor: the tree
# plugins cannot take it)
DTYPES = {
    "BOOL": np.bool_, "UINT8": np.uint8, "UINT16": np.uint16, "UINT32": np.uint32,
    "UINT64": np.uint64, "INT8": np.int8, "INT16": np.int16, "INT32": np.int32,
    "INT64": np.int64, "FP16": np.float16, "FP32": np.float32, "FP64": np.float64,
}
NAMES = {np.dtype(v): k for k, v in DTYPES.items()}


class V2Error(ValueError):
    """A malformed V2 request: answered 400 with {"error": message}."""


def is_tensor_request(obj: Any) -> bool:
    """A V2 inference request: ``inputs`` is a non-empty list of tensor objects."""
    if not isinstance(obj, dict):
        return False
    inputs = obj.get("inputs")
    return (isinstance(inputs, list) and len(inputs) > 0 and
            all(isinstance(i, dict) and "datatype" in i and "shape" in i for i in inputs))


def split_body(headers: Mapping[str, str], body: bytes) -> Tuple[bytes, bytes]:
    """(JSON header, binary tail) of a request body."""
    n = None
    for k, v in headers.items():
        if k.lower() == HEADER_LEN:
            try:
                n = int(v)
            except ValueError:
                raise V2Error(f"bad {HEADER_LEN}: {v!r}")
    if n is None:
        return body, b""
    if n < 0 or n > len(body):
        raise V2Error(f"{HEADER_LEN} {n} exceeds the body ({len(body)} bytes)")
    return body[:n], body[n:]


def _shape(t: Dict) -> Tuple[int, ...]:
    shape = t.get("shape")
    if not isinstance(shape, list) or not all(
            isinstance(d, int) and not isinstance(d, bool) and d >= 0 for d in shape):
        raise V2Error(f"input {t.get('name')!r}: shape must be a list of non-negative integers")
    count = 1
    for d in shape:           # Python ints: a product past int64 is an error, not a wrap
        count *= d
    if count >= 1 << 62:
        raise V2Error(f"input {t.get('name')!r}: shape {shape} is too large")
    return tuple(shape)


def decode_inputs(req: Dict, tail: bytes) -> List[Tuple[str, np.ndarray]]:
    """Every input tensor as (name, array of its shape and datatype)."""
    out = []
    off = 0
    for t in req["inputs"]:
        name = t.get("name")
        dt = DTYPES.get(t.get("datatype"))
        if dt is None:
            raise V2Error(f"input {name!r}: unsupported datatype {t.get('datatype')!r}")
        shape = _shape(t)
        count = 1
        for d in shape:
            count *= d
        params = t.get("parameters") or {}
        size = params.get("binary_data_size") if isinstance(params, dict) else None
        if size is not None:
            want = count * np.dtype(dt).itemsize
            if (not isinstance(size, int) or isinstance(size, bool) or size != want
                    or off + size > len(tail)):
                raise V2Error(f"input {name!r}: binary_data_size {size!r} does not match "
                              f"shape {list(shape)} x {t['datatype']} ({want} bytes) or the body")
            try:
                arr = np.frombuffer(tail, dtype=np.dtype(dt).newbyteorder("<"), count=count,
                                    offset=off).reshape(shape)
            except (TypeError, ValueError, OverflowError) as e:
                raise V2Error(f"input {name!r}: cannot read {list(shape)} x {t['datatype']}: {e}")
            off += size
        else:
            if "data" not in t:
                raise V2Error(f"input {name!r}: no data")
            try:
                arr = np.asarray(t["data"], dtype=dt)
            except (TypeError, ValueError, OverflowError) as e:
                raise V2Error(f"input {name!r}: data is not {t['datatype']}: {e}")
            if arr.size != count:
                raise V2Error(f"input {name!r}: {arr.size} values for shape {list(shape)}")
            try:
                arr = arr.reshape(shape)
            except (TypeError, ValueError, OverflowError) as e:
                raise V2Error(f"input {name!r}: cannot reshape to {list(shape)}: {e}")
        out.append((name, arr))
    if off != len(tail):
        raise V2Error(f"{len(tail) - off} bytes of binary data belong to no input")
    return out


def feature_matrix(inputs: List[Tuple[str, np.ndarray]]) -> np.ndarray:
    """The one input of a tree model as a [rows, features] matrix: a [N, F]
    tensor, or a [F] tensor as one row.  Integer and boolean tensors are
    read as float64; FP16 as float32; FP32 / FP64 keep their type (an FP32
    matrix takes the kernel's float32 path)."""
    if len(inputs) != 1:
        raise V2Error(f"a tree model takes one input tensor, got {len(inputs)}")
    name, X = inputs[0]
    if X.ndim == 1:
        X = X.reshape(1, -1)
    if X.ndim != 2:
        raise V2Error(f"input {name!r}: expected a [rows, features] tensor, got shape "
                      f"{list(X.shape)}")
    if X.dtype == np.float16:
        X = X.astype(np.float32)
    elif X.dtype not in (np.float32, np.float64):
        X = X.astype(np.float64)
    return np.ascontiguousarray(X)


def wants_binary(req: Dict, name: str) -> bool:
    params = req.get("parameters")
    if isinstance(params, dict) and params.get("binary_data_output") is True:
        return True
    for o in req.get("outputs") or []:
        if isinstance(o, dict) and o.get("name") == name:
            p = o.get("parameters") or {}
            return isinstance(p, dict) and p.get("binary_data") is True
    return False


def output_name(req: Dict) -> str:
    outs = req.get("outputs")
    if isinstance(outs, list) and outs and isinstance(outs[0], dict) and "name" in outs[0]:
        return str(outs[0]["name"])
    return "predict"


def encode_response(model_name: str, req: Dict, result: np.ndarray) -> Tuple[Dict[str, str], bytes]:
    """(extra headers, body) of the V2 inference response for one output."""
    name = output_name(req)
    arr = np.ascontiguousarray(result)
    dt = NAMES.get(arr.dtype)
    if dt is None:   # labels of another kind (e.g. strings): JSON values, BYTES
        dt = "BYTES"
    out: Dict[str, Any] = {"name": name, "shape": list(arr.shape), "datatype": dt}
    resp: Dict[str, Any] = {"model_name": model_name}
    if "id" in req:
        resp["id"] = req["id"]
    resp["outputs"] = [out]
    if dt != "BYTES" and wants_binary(req, name):
        raw = arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes()
        out["parameters"] = {"binary_data_size": len(raw)}
        head = json.dumps(resp).encode()
        return ({"Content-Type": "application/octet-stream",
                 "Inference-Header-Content-Length": str(len(head))}, head + raw)
    out["data"] = arr.reshape(-1).tolist()
    return {"Content-Type": "application/json"}, json.dumps(resp).encode()


def error_body(msg: str) -> bytes:
    """required_api.md:326-340: {"error": <message>}."""
    return json.dumps({"error": msg}).encode()


def parse_header(head: bytes) -> Optional[Dict]:
    try:
        obj = json.loads(head)
    except (json.JSONDecodeError, UnicodeDecodeError):
        return None
    return obj if is_tensor_request(obj) else None
