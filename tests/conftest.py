import os
import sys
from pathlib import Path

import pytest

# torch first: libtfrg then binds to the HIP runtime torch bundles (same soname). Loaded the other
# way round, the process holds two HIP/HSA runtimes and torch's finds no device.
import torch  # noqa: E402,F401

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "tfrecords-reader_amd"
for p in (str(PKG), str(REPO)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden_dir() -> Path:
    return REPO / "tests" / "golden"
