"""C-ABI boundary checks that need no GPU: the library loads, exports every
entry point include/treeinfer.h declares, and the ctypes mirrors of the two
structs have the C layout (compiled with gcc against the header)."""
import ctypes
import os
import re
import subprocess

import pytest

from kfserving_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "treeinfer.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(ti_\w+)\(", src, re.M)))


def test_header_declares_the_binding_symbols():
    assert declared_functions() == sorted(engine.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = engine.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.ti_abi_version() == engine.ABI_VERSION
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ti_\w+)", out))
    assert set(declared_functions()) <= exported


def test_struct_layout_matches_header(tmp_path):
    prog = tmp_path / "layout.c"
    fields = [f for f, _ in engine._ForestDesc._fields_]
    ifields = [f for f, _ in engine._ForestInfo._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "treeinfer.h"', 'int main(){',
             'printf("desc %zu\\n", sizeof(ti_forest_desc));',
             'printf("info %zu\\n", sizeof(ti_forest_info));']
    lines += [f'printf("d.{f} %zu\\n", offsetof(ti_forest_desc, {f}));' for f in fields]
    lines += [f'printf("i.{f} %zu\\n", offsetof(ti_forest_info, {f}));' for f in ifields]
    lines += ['return 0;}']
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)],
                   check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.splitlines())
    assert int(got["desc"]) == ctypes.sizeof(engine._ForestDesc)
    assert int(got["info"]) == ctypes.sizeof(engine._ForestInfo)
    for f in fields:
        assert int(got[f"d.{f}"]) == getattr(engine._ForestDesc, f).offset, f
    for f in ifields:
        assert int(got[f"i.{f}"]) == getattr(engine._ForestInfo, f).offset, f


def test_abi_constants_match_python():
    from kfserving_amd import forest as F
    src = open(HEADER).read()
    consts = dict(re.findall(r"#define (TI_\w+)\s+(0x[0-9a-fA-F]+|-?\d+)", src))
    v = lambda k: int(consts[k], 0)
    assert (v("TI_F32"), v("TI_F64"), v("TI_I32")) == (F.TI_F32, F.TI_F64, F.TI_I32)
    assert (v("TI_NODE_NAN_LEFT"), v("TI_NODE_ZERO_FLIP"), v("TI_NODE_CATEGORICAL")) == \
        (F.NODE_NAN_LEFT, F.NODE_ZERO_FLIP, F.NODE_CATEGORICAL)
    assert (v("TI_OUTPUT_MARGIN"), v("TI_OUTPUT_PREDICT"), v("TI_OUTPUT_LEAF"),
            v("TI_OUTPUT_CONTRIB")) == (F.OUT_MARGIN, F.OUT_PREDICT, F.OUT_LEAF, F.OUT_CONTRIB)
    for name in ("IDENTITY", "SIGMOID", "SOFTMAX", "ARGMAX", "HINGE", "EXP", "SIGNSQUARE",
                 "LOG1PEXP", "STEP"):
        assert v("TI_TRANSFORM_" + name) == getattr(F, "T_" + name)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(engine.TreeInferError):
        engine.load_library(str(tmp_path / "nope.so"))


def test_kfserve_library_exports_its_header():
    from kfserving_amd.kfserving import fastjson
    src = open(os.path.join(ROOT, "include", "kfserve.h")).read()
    names = sorted(set(re.findall(r"^\s*int\s+(kf_\w+)\(", src, re.M)))
    assert names == ["kf_parse_inputs", "kf_parse_instances", "kf_parse_instances_mt",
                     "kf_parse_v2_tensor"]
    lib = fastjson.load_library()
    for n in names:
        assert hasattr(lib, n), n


def test_plugin_modules_import():
    """Every plugin module imports without a GPU (the device replica is lazy)."""
    import importlib
    for m in ("kfserving_amd.xgbserver.model", "kfserving_amd.lgbserver.model",
              "kfserving_amd.sklearnserver.model", "kfserving_amd.tree_model"):
        importlib.import_module(m)
