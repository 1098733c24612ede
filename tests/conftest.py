import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdifacto_amd.so)")


GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="session")
def rcv1():
    from difacto_amd import data
    return data.read_libsvm(os.path.join(GOLDEN, "rcv1_100.libsvm"))


@pytest.fixture(scope="session")
def known():
    import json
    with open(os.path.join(GOLDEN, "reference_known_answers.json")) as f:
        return json.load(f)
