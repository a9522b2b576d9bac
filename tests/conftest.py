"""pytest configuration: the `gpu` marker and shared paths.

`-m "not gpu"` runs here (no GPU): oracle vs goldens, host logic over a checker-backed index,
file format, and that libvs.so loads and exports every symbol of include/vs.h.
`-m gpu` runs on an MI355X: parity of the HIP path (through the C ABI) against the oracle.
"""
import os
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)
GOLDEN = os.path.join(TESTS, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libvs.so")
    # VS_TEST_K1_SCHEDULE=0|1: run the GPU suite under that K1 schedule (include/vs.h
    # vs_set_k1_schedule); unset = the library's default
    sched = os.environ.get("VS_TEST_K1_SCHEDULE")
    if sched is not None:
        from photo_search_engine_amd.index import set_k1_schedule
        set_k1_schedule(int(sched))


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
