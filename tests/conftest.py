"""Shared test fixtures.  `gpu`-marked tests need a real MI355X (run via gpurun)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-proof-of-work_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu on the GPU box")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "pow_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from _oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def miner():
    import distpow
    if distpow.device_count() == 0:
        pytest.fail("no HIP device visible: gpu tests must run on the GPU box")
    m = distpow.Miner(0)
    yield m
    m.close()
