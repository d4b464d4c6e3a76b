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
    # DP tests parametrize latency mode explicitly (`dp_lat`)
    e.set_option("dp_lat", 0)
    yield e
    e.close()


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
