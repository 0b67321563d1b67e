"""Writes tests/golden/kfhttp_corpus.jsonl: the malformed-input corpus that
tests/test_asan_fuzz.py replays through libkfserve.so's native HTTP front end
(kh_*, include/kfhttp.h) and its body parsers (kf_parse_*, include/kfserve.h)
under AddressSanitizer + UndefinedBehaviorSanitizer.

Each line is one case:
  {"kind": "http", "name", "data": base64 bytes sent on one connection,
   "shut": half-close after sending, "expect": [allowed first status codes]
   (an empty list: any answer or none)}
  {"kind": "http_gen", "name", "recipe", "expect"}   -- large inputs built by
   tests/asan_replay.py from the named recipe (header floods, 1 MB lines)
  {"kind": "parse", "parser": "instances" | "instances_mt" | "inputs" | "v2",
   "name", "data": base64 body, "head_len" (v2), "cuts": replay every prefix}

The status contract is the reference's: a malformed request is 400
(python/kfserving/kfserving/handlers/http.py:68-74), a body over
--max_buffer_size 413 (kfserver.py:39); anything the native path does not
take is the application's answer.  Deterministic: rerun to regenerate.
"""
import base64
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "kfhttp_corpus.jsonl")
MODEL = "xgboost-iris"
PRED = f"/v1/models/{MODEL}:predict".encode()
INFER = f"/v2/models/{MODEL}/infer".encode()


def req(body: bytes, path=PRED, extra=b"", method=b"POST", version=b"HTTP/1.1") -> bytes:
    return (method + b" " + path + b" " + version + b"\r\nHost: x\r\n" + extra +
            b"Content-Length: %d\r\n\r\n" % len(body) + body)


def chunked(parts, path=PRED, tail=b"0\r\n\r\n") -> bytes:
    return (b"POST " + path + b" HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" +
            b"".join(b"%x\r\n" % len(p) + p + b"\r\n" for p in parts) + tail)


def main():
    good = b'{"instances": [[6.8, 2.8, 4.8, 1.4], [6.0, 3.4, 4.5, 1.6]]}'
    cases = []

    def http(name, data, expect=(), shut=True):
        cases.append({"kind": "http", "name": name, "data": base64.b64encode(data).decode(),
                      "shut": shut, "expect": list(expect)})

    def gen(name, recipe, expect=()):
        cases.append({"kind": "http_gen", "name": name, "recipe": recipe, "expect": list(expect)})

    def parse(parser, name, data, head_len=-1, cuts=True):
        cases.append({"kind": "parse", "parser": parser, "name": name,
                      "data": base64.b64encode(data).decode(), "head_len": head_len,
                      "cuts": cuts})

    # --- framing ---------------------------------------------------------
    http("good", req(good), [200])
    http("good_pipelined_x3", req(good) * 3, [200])
    http("chunked_good", chunked([good[:7], good[7:30], good[30:]]), [200])
    http("chunked_truncated_data", chunked([good])[:-25], [400])
    http("chunked_size_over_data", b"POST " + PRED + b" HTTP/1.1\r\nTransfer-Encoding: chunked"
         b"\r\n\r\n64\r\n" + good[:10], [400])
    http("chunked_size_huge", b"POST " + PRED + b" HTTP/1.1\r\nTransfer-Encoding: chunked"
         b"\r\n\r\nFFFFFFFFFFFFFFFFFFFF\r\n", [413])
    http("chunked_size_negative", b"POST " + PRED + b" HTTP/1.1\r\nTransfer-Encoding: chunked"
         b"\r\n\r\n-5\r\nhello\r\n0\r\n\r\n", [400])
    http("chunked_size_garbage", b"POST " + PRED + b" HTTP/1.1\r\nTransfer-Encoding: chunked"
         b"\r\n\r\nzz\r\n", [400])
    http("chunked_no_crlf_after_data", chunked([good]).replace(good + b"\r\n", good + b"XX"), [])
    http("chunked_many_tiny", chunked([good[i:i + 1] for i in range(len(good))]), [200])
    http("chunked_ext_and_trailer", chunked([good], tail=b"0;x=1\r\nTrailer: y\r\n\r\n"), [])
    http("content_length_overflow", b"POST " + PRED + b" HTTP/1.1\r\nContent-Length: "
         b"99999999999999999999999999\r\n\r\n", [413])
    http("content_length_negative", b"POST " + PRED + b" HTTP/1.1\r\nContent-Length: -1"
         b"\r\n\r\n", [400])
    http("content_length_garbage", b"POST " + PRED + b" HTTP/1.1\r\nContent-Length: 1e3"
         b"\r\n\r\n", [400])
    http("content_length_over_max", b"POST " + PRED + b" HTTP/1.1\r\nContent-Length: "
         b"104857601\r\n\r\n", [413])
    http("content_length_short_body", req(good).replace(b"Content-Length: %d" % len(good),
                                                        b"Content-Length: %d" % (len(good) + 40)),
         [400])
    http("duplicate_content_length", req(good, extra=b"Content-Length: 3\r\n"), [])
    http("duplicate_transfer_encoding", chunked([good]).replace(
        b"Transfer-Encoding: chunked\r\n", b"Transfer-Encoding: gzip\r\nTransfer-Encoding: chunked\r\n"),
        [200])
    http("te_and_cl", chunked([good]).replace(b"Host: x\r\n", b"Host: x\r\nContent-Length: 5\r\n"),
         [200])
    http("bad_request_line_2", b"GET /\r\n\r\n", [400])
    http("bad_request_line_4", b"GET / HTTP/1.1 x\r\n\r\n", [400])
    http("empty_lines", b"\r\n\r\n\r\n", [400])
    http("nul_bytes", b"\x00" * 64 + b"\r\n\r\n", [400])
    http("header_no_colon", req(good, extra=b"NoColonHere\r\n"), [200])
    http("header_bare_lf", req(good).replace(b"\r\n", b"\n"), [200])
    http("http10", req(good, version=b"HTTP/1.0"), [200])
    http("connection_close_then_more", req(good, extra=b"Connection: close\r\n") + req(good), [200])
    http("path_invalid_utf8", req(good, path=b"/v1/models/\xff\xfe:predict"), [])
    http("path_long_name", req(good, path=b"/v1/models/" + b"a" * 5000 + b":predict"), [404])
    http("header_invalid_utf8", req(good, extra=b"X-Bad: \xc3\x28\xa0\xa1\r\n"), [200])
    http("get_predict", req(b"", method=b"GET"), [])
    # --- bodies the native route parses --------------------------------
    for name, body in [
        ("nan_inf", b'{"instances": [[NaN, Infinity, -Infinity, 1]]}'),
        ("nan_lower", b'{"instances": [[nan, 1, 2, 3]]}'),
        ("infinity_suffix", b'{"instances": [[Infinityx, 1, 2, 3]]}'),
        ("invalid_utf8_body", b'{"instances": [[1, 2, 3, 4]], "\xff\xfe": 1}'),
        ("invalid_utf8_in_number", b'{"instances": [[1\xc3, 2, 3, 4]]}'),
        ("deep_nesting", b'{"instances": ' + b"[" * 3000 + b"1" + b"]" * 3000 + b"}"),
        ("ragged", b'{"instances": [[1, 2, 3, 4], [1, 2]]}'),
        ("long_digits", b'{"instances": [[' + b"1" * 400 + b'.5e-999, 2, 3, 4]]}'),
        ("exp_overflow", b'{"instances": [[1e400, -1e400, 1e-400, 4]]}'),
        ("not_a_list", b'{"instances": 3}'),
        ("empty_instances", b'{"instances": []}'),
        ("truncated_json", good[:-3]),
        ("trailing_garbage", good + b"xyz"),
        ("unterminated_string", b'{"instances": [[1, 2, 3, 4]], "a": "abc'),
        ("escaped_key", b'{"inst\\u0061nces": [[1, 2, 3, 4]]}'),
    ]:
        http("body_" + name, req(body), [])
    # --- V2 tensors and the binary extension -----------------------------
    v2 = json.dumps({"inputs": [{"name": "x", "shape": [2, 4], "datatype": "FP32",
                                 "data": [6.8, 2.8, 4.8, 1.4, 6.0, 3.4, 4.5, 1.6]}]}).encode()
    http("v2_json", req(v2, path=INFER), [200])
    raw = b"\x00\x00\x80\x3f" * 8
    head = json.dumps({"inputs": [{"name": "x", "shape": [2, 4], "datatype": "FP32",
                                   "parameters": {"binary_data_size": len(raw)}}]}).encode()
    ihcl = b"Inference-Header-Content-Length: %d\r\n"
    http("v2_binary", req(head + raw, path=INFER, extra=ihcl % len(head)), [200])
    big_claim = head.replace(b'"binary_data_size": %d' % len(raw), b'"binary_data_size": 1000000')
    http("v2_binary_size_over_body", req(big_claim + raw, path=INFER, extra=ihcl % len(big_claim)),
         [])
    neg_claim = head.replace(b'"binary_data_size": %d' % len(raw), b'"binary_data_size": -8')
    http("v2_binary_size_negative", req(neg_claim + raw, path=INFER, extra=ihcl % len(neg_claim)),
         [])
    http("v2_header_len_over_body", req(head + raw, path=INFER, extra=ihcl % 100000), [])
    http("v2_header_len_negative", req(head + raw, path=INFER,
                                       extra=b"Inference-Header-Content-Length: -3\r\n"), [])
    http("v2_header_len_garbage", req(head + raw, path=INFER,
                                      extra=b"Inference-Header-Content-Length: 1x\r\n"), [])
    http("v2_binary_odd_bytes", req(head + raw[:-3], path=INFER, extra=ihcl % len(head)), [])
    http("v2_shape_mismatch", req(v2.replace(b"[2, 4]", b"[3, 4]"), path=INFER), [])
    http("v2_shape_huge", req(v2.replace(b"[2, 4]", b"[4611686018427387904, 4]"), path=INFER), [])
    # --- large inputs built by the replay ---------------------------------
    gen("header_line_over_limit", "header_line_over_limit", [400])
    gen("request_line_over_limit", "request_line_over_limit", [400])
    gen("many_headers", "many_headers", [200])
    gen("body_cut_at_every_offset", "body_cut_at_every_offset", [])
    gen("slow_request_pipelined_megabytes", "slow_request_pipelined_megabytes", [200])
    # --- parsers, every prefix of each body -------------------------------
    for name, body in [("good", good), ("nan_inf", b'{"instances": [[NaN, -Infinity, 1e308, -0.0]]}'),
                       ("long_digits", b'{"instances": [[1.' + b"7" * 60 + b'e-20, 2]]}'),
                       ("deep", b'{"instances": ' + b"[" * 200 + b"1" + b"]" * 200 + b"}"),
                       ("utf8", b'{"instances": [[1, 2]], "\xe2\x82\xac": [1]}')]:
        parse("instances", name, body)
    inputs = json.dumps({"inputs": [{"sepal_width_(cm)": [2.8, None], "petal_length_(cm)": [4.8, 4.5],
                                     "x": {"nested": [1, 2]}, "sepal_length_(cm)": [True, False],
                                     "petal_width_(cm)": [1.4, 1.6]}]}).encode()
    parse("inputs", "mixed", inputs)
    parse("inputs", "dict_rows", json.dumps({"inputs": [{"sepal_length_(cm)": {"0": 5.1, "1": 4.9},
                                                         "petal_width_(cm)": {"0": 0.2, "1": 0.2}}]}
                                            ).encode())
    parse("v2", "json", v2)
    parse("v2", "id_and_params", json.dumps({"id": "r1", "parameters": {"binary_data_output": True},
                                             "inputs": json.loads(v2)["inputs"]}).encode())
    parse("v2", "binary", head + raw, head_len=len(head))
    parse("v2", "binary_claim_over", big_claim + raw, head_len=len(big_claim))
    with open(OUT, "w") as fh:
        for c in cases:
            fh.write(json.dumps(c) + "\n")
    print(f"{len(cases)} cases -> {OUT}")


if __name__ == "__main__":
    main()
