import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pipeline2.0_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def gpu_available():
    """True with a HIP device; a library that does not load raises (HipDedispUnavailable
    names the cause, e.g. an undefined symbol) instead of reading as 'no device'."""
    from hipdedisp import _lib, device_count
    _lib.load()
    try:
        return device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine():
    """One device context for the whole GPU test session (one process on the card)."""
    from hipdedisp import Engine
    if not gpu_available():
        pytest.fail("no HIP device: GPU tests must run on the MI355X box (pytest -m gpu)")
    eng = Engine(0)
    yield eng
    eng.close()


def pytest_runtest_logreport(report):
    """A failing test's report printed at once: the session's engine closes at teardown, and a
    process that aborts there would otherwise take the failure summary with it."""
    if report.failed and report.when == "call":
        sys.stderr.write("\n==== failure of %s ====\n%s\n" % (report.nodeid, str(report.longrepr)[-6000:]))
        sys.stderr.flush()
