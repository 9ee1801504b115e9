import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

# Keep CPU tests off any GPU and hermetic.
os.environ.setdefault("TK8S_TEST", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: multi-second integration test")


@pytest.fixture(scope="session")
def native_build():
    """Build (incrementally) the in-tree native layer once per session."""
    from tritonk8ssupervisor_amd.utils.build_native import build

    return build()
