"""The sanitizer and fuzz recipe for libkfserve.so's network-facing code
(VERDICT r5 item 4): the native HTTP front end (kfhttp.cpp), the request
batcher (kfbatch.cpp) and the body parsers (kfserve_host.cpp), built with
AddressSanitizer + UndefinedBehaviorSanitizer (`__graft_entry__.build_host(
asan=True)` -> kfserving_amd/lib/asan/libkfserve.so), replay the committed
malformed-input corpus tests/golden/kfhttp_corpus.jsonl
(tests/golden/make_kfhttp_corpus.py) in a child process
(tests/asan_replay.py, LD_PRELOAD=libasan, KFSERVE_LIB=the sanitizer build).

Every case must give the reference's status (400 / 413,
python/kfserving/kfserving/handlers/http.py:68-74, kfserver.py:39) or the
application's answer, and no sanitizer report.  A canary run (a deliberate
read past a body) must be stopped by the sanitizer, so a green run cannot
come from an uninstrumented library.  Re-run by hand:

  python -c 'import __graft_entry__ as g; g.build_host(asan=True)'
  KFSERVE_LIB=kfserving_amd/lib/asan/libkfserve.so \\
  LD_PRELOAD=$(gcc -print-file-name=libasan.so) ASAN_OPTIONS=detect_leaks=0 \\
  python tests/asan_replay.py
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _asan_runtime():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                           text=True, check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def asan_env():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("no AddressSanitizer runtime (gcc's libasan.so) on this host")
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    srcs = [os.path.join(g.CSRC, f) for f in g.KFSERVE_SOURCES]
    srcs += glob.glob(os.path.join(ROOT, "include", "*.h")) + glob.glob(os.path.join(g.CSRC, "*.h"))
    lib = g.KFSERVE_ASAN_LIB
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(s) for s in srcs):
        g.build_host(asan=True)
    env = dict(os.environ)
    env.update(KFSERVE_LIB=lib, LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:exitcode=66",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               KF_NATIVE_HTTP="1", KF_NATIVE_BATCHER="1")
    return env


def _replay(env, *args):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tests", "asan_replay.py")] +
                          list(args), cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=600)


def test_sanitizer_catches_the_canary(asan_env):
    r = _replay(asan_env, "--canary")
    assert r.returncode == 66, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "AddressSanitizer" in r.stderr and "heap-buffer-overflow" in r.stderr or \
        "SUMMARY: AddressSanitizer" in r.stderr


def test_corpus_replay_under_asan_ubsan(asan_env):
    import json
    r = _replay(asan_env)
    report = "AddressSanitizer" in r.stderr or "runtime error:" in r.stderr
    assert r.returncode == 0 and not report, (r.returncode, r.stdout[-2000:], r.stderr[-6000:])
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["failures"] == [] and line["lib"].endswith("asan/libkfserve.so")
    assert line["parser_calls"] > 5000 and line["http_cases"] >= 60
    fe = line["front_end"]
    assert fe["native_requests"] > 0 and fe["python_requests"] > 0 and fe["bad_requests"] > 100
