import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(REPO, "tests")
for p in (REPO, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(TESTS, "golden")
STREAMS = os.path.join(GOLDEN, "streams")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP path)")
    config.addinivalue_line("markers", "slow: longer-running case")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the native library + the C oracle in-tree (no-op when up to date)."""
    from tiny_mp2v_dec_amd import build as B
    B.build()
    import _oracle
    _oracle.lib()


def load_manifest():
    with open(os.path.join(STREAMS, "manifest.json")) as f:
        return json.load(f)


def read_stream(entry):
    with open(os.path.join(STREAMS, entry["file"]), "rb") as f:
        return f.read()
