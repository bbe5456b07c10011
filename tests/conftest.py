import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return dict(np.load(GOLDEN / f"{name}.npz", allow_pickle=False))
    return load


@pytest.fixture(scope="session")
def built_lib():
    """Build (if stale) and load libisr.so."""
    from image_super_resolution_amd import _build, _lib
    _build.build()
    return _lib.load()


def t(a) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a))


os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
