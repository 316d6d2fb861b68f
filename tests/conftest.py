import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE) parity properties")


@pytest.fixture(scope="session")
def armi_lib():
    """libarmi.so, built in-tree if missing (hipcc cross-compiles for gfx950)."""
    from audio_rag_amd import build as armi_build
    from audio_rag_amd import _armi

    if not _armi.LIB_PATH.exists():
        armi_build.build()
    return _armi.load()


@pytest.fixture(scope="session")
def gpu(armi_lib):
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda is not available")
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle
