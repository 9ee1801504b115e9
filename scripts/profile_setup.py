"""Host-side profile of one bring-up: run ./setup.sh under cProfile (TK8S_PROFILE) in a fresh
workspace and print the top functions by cumulative and own time. Usage:
    python3 scripts/profile_setup.py [--nodes N] > setup_profile.txt
"""
import argparse
import os
import pstats
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1)
    a = ap.parse_args()
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = Path(tempfile.mkdtemp(prefix="tk8s-prof-"))
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_PROFILE=str(ws / "setup.prof"))
    try:
        r = subprocess.run(["./setup.sh", "--nodes", str(a.nodes), "--yes", "--port", "0", "--rccl", "off"], cwd=ws,
                           env=env, capture_output=True, text=True, timeout=300)
        print(r.stdout[-1500:])
        if r.returncode != 0:
            print(r.stderr[-3000:])
            return r.returncode
        st = pstats.Stats(str(ws / "setup.prof"), stream=sys.stdout)
        st.sort_stats("cumulative").print_stats(45)
        st.sort_stats("tottime").print_stats(25)
    finally:
        env.pop("TK8S_PROFILE")
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, timeout=120)
        shutil.rmtree(ws, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
