"""Test configuration: `gpu` marker, import paths, shared helpers."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "duckdb-parquet-parser_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running full-size case")


@pytest.fixture(scope="session")
def ctx():
    from pqgpu import capi
    c = capi.Context(0)
    yield c
    c.close()
