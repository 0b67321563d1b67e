import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# PyTorch-ROCm bundles its own libamdhip64 (soname libamdhip64.so.7, NEEDED as
# "libamdhip64.so").  Loading torch first makes libtreeinfer bind to that same
# runtime; loading libtreeinfer first would put two HIP runtimes in the process
# and torch would then see no GPU ("One HIP runtime").
try:
    import torch  # noqa: F401
except ImportError:
    pass

# the tests exercise every layout and A/B variant through libtreeinfer's
# developer knobs (TI_FORCE_LAYOUT, TI_TX_TOP, ...), which the library reads
# only under TI_DEV_KNOBS=1 (treeinfer.hip env_knob); tests/test_gpu_knob_gate.py
# checks that without it they change nothing
os.environ.setdefault("TI_DEV_KNOBS", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN
