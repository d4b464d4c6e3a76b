import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def engine():
    from rifraf_amd.engine import Engine
    e = Engine(0)
    # small test launches would all take the latency-mode DP class
    # (RF_OPT_DP_LAT); the shared engine keeps the throughput classes, and the
    # DP tests parametrize latency mode explicitly (`dp_lat`).  Whole-run
    # parity tests take `run_engine`, which runs them in both modes.
    e.product_dp_lat = e.set_option("dp_lat", 0)
    assert e.product_dp_lat > 0, "the product default is latency mode for small calls"
    yield e
    e.close()


# DP modes of a whole-run parity test: "lat" is the product default (a call
# with at most RF_OPT_DP_LAT lean tasks runs them in k_dpx<false, false>, one
# task per wave -- every configs[0..2] realign and every small-cluster native
# run), "tp" the throughput classes (k_dpr, the c4 bench step's path)
DP_MODES = ("lat", "tp")


@pytest.fixture(params=DP_MODES)
def run_engine(engine, request):
    """The session engine in one DP mode (product default or throughput
    classes) for the test; restored afterwards."""
    old = engine.set_option("dp_lat", engine.product_dp_lat if request.param == "lat" else 0)
    yield engine
    engine.set_option("dp_lat", old)


_MEMO = {}


@pytest.fixture(scope="session")
def oracle_memo():
    """oracle_memo(key, fn): fn() once per session.  The oracle engine's
    result of a whole run does not depend on the HIP engine's DP mode, so the
    "lat" and "tp" variants of a parity test share one oracle run."""
    def get(key, fn):
        if key not in _MEMO:
            _MEMO[key] = fn()
        return _MEMO[key]
    return get


@pytest.fixture
def opts(engine):
    """Set engine options (rf_set_option) for one test; restored afterwards."""
    saved = {}

    def set_(name, value):
        old = engine.set_option(name, value)
        saved.setdefault(name, old)

    yield set_
    for k, v in saved.items():
        engine.set_option(k, v)
