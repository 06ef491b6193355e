import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")
    # Build the in-tree libraries if they are missing (no-op when up to date).
    lib = os.path.join(REPO, "photonlibos_amd", "lib", "libphoton_checksum.so")
    ora = os.path.join(REPO, "oracle", "lib", "libcrc_oracle.so")
    if not (os.path.exists(lib) and os.path.exists(ora)):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(REPO, "photonlibos_amd", "csrc")])


@pytest.fixture(scope="session")
def golden_in():
    with open(os.path.join(GOLDEN, "checksum_in.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ref_vectors():
    with open(os.path.join(GOLDEN, "ref_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from tests import _oracle
    return _oracle


@pytest.fixture(scope="session")
def alphabet():
    return (b"abcdefghijklmnopqrstuvwxyz" * 200)[:5000]
