"""pytest configuration: `gpu` marker, import paths, golden-fixture loader.

-m "not gpu"  runs here (no GPU): oracle vs golden fixtures, generator, host logic, ABI load/exports, gloo.
-m gpu        runs on an MI355X: parity of the HIP path (through the C ABI) against oracle + fixtures.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "gelly-streaming_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden
