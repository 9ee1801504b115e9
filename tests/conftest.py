import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

# Keep CPU tests off any GPU and hermetic.
os.environ.setdefault("TK8S_TEST", "1")
# One host registry per test run (shared by its xdist workers, whose clusters must stay disjoint),
# so a cluster an earlier run leaked cannot hold this run's GPU.
os.environ.setdefault("TK8S_HOST_REGISTRY", os.path.join(
    os.environ.get("TMPDIR", "/tmp"), f"tk8s-hostreg-{os.environ.get('PYTEST_XDIST_TESTRUNUID') or os.getpid()}"))


def die_with_parent():
    """preexec_fn for a daemon a test starts: SIGTERM when the test process dies (an interrupted
    or timed-out pytest worker must not leave its control planes running)."""
    import ctypes

    prctl = ctypes.CDLL(None, use_errno=True).prctl

    def arm() -> None:
        prctl(1, 15)  # PR_SET_PDEATHSIG, SIGTERM

    return arm


@pytest.fixture(autouse=True)
def _restore_environ():
    """Setup.configure exports the cluster config into os.environ (the reference's exportVars,
    setup.sh:543-549): never let one test's TK8S_BACKEND/TK8S_PLATFORM leak into the next."""
    saved = dict(os.environ)
    yield
    os.environ.clear()
    os.environ.update(saved)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: multi-second integration test")


@pytest.fixture(scope="session")
def native_build():
    """Build (incrementally) the in-tree native layer once per session."""
    from tritonk8ssupervisor_amd.utils.build_native import build

    return build()


def pytest_sessionfinish(session, exitstatus):
    if not hasattr(session.config, "workerinput"):  # the controller, after every worker is done
        import shutil

        _teardown_leaked_clusters(Path(os.environ["TK8S_HOST_REGISTRY"]))
        shutil.rmtree(os.environ["TK8S_HOST_REGISTRY"], ignore_errors=True)


def _teardown_leaked_clusters(registry: Path) -> None:
    """A run interrupted by ``-x`` (xdist stops the other workers mid-test) skips fixture
    teardowns: every workspace still holding claims in this run's registry is torn down here,
    so no control plane or agent outlives the run (and keeps serving on an address the next
    run hands out again)."""
    import json
    import subprocess

    try:
        table = json.loads((registry / "claims.json").read_text())
    except (OSError, ValueError):
        return
    workspaces = {Path(c.get("alloc", "")).parent.parent for kind in ("ips", "gpus")
                  for c in (table.get(kind) or {}).values() if c.get("alloc")}
    for ws in sorted(workspaces):
        if (ws / "setup.sh").exists():
            subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, capture_output=True, timeout=120,
                           env={**os.environ, "PYTHONPATH": str(REPO)})
