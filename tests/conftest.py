import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: larger sizes")


class Golden:
    def __init__(self):
        self.manifest = json.load(open(os.path.join(GOLDEN, "golden.json")))
        self.blob = open(os.path.join(GOLDEN, "qlz_vectors.bin"), "rb").read()
        self.records_data = open(os.path.join(GOLDEN, "records.data"), "rb").read()

    def get(self, span):
        o, n = span
        return self.blob[o:o + n]

    @property
    def vectors(self):
        return self.manifest["vectors"]

    @property
    def records(self):
        return self.manifest["records"]


@pytest.fixture(scope="session")
def golden():
    return Golden()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU (run -m 'not gpu' here)")
    from gobeansdb_amd import build
    build.build()
    return torch.device("cuda:0")
