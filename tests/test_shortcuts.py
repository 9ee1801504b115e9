"""TK8S_SHORTCUTS=0: one master switch for every start-up shortcut.

docs/architecture.md "Start-up shortcuts and their off-switches" lists each shortcut with its own
switch; the master switch sets all of them, for setup.sh (the ones acted on before Python starts)
and for every interpreter of the bring-up (tritonk8ssupervisor_amd/__init__.py). bench.py reports
the plain path's bring-up as plain_path_s (tests/test_bench_contract.py), and the GPU suite brings
it up on the MI355X (tests/test_kernels_gpu.py::test_setup_on_the_plain_path_on_a_real_gpu)."""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def test_the_master_switch_sets_every_shortcut_switch():
    from tritonk8ssupervisor_amd import SHORTCUT_SWITCHES

    env = {k: v for k, v in os.environ.items() if k not in SHORTCUT_SWITCHES}
    code = "import json, os, tritonk8ssupervisor_amd as t; print(json.dumps({k: os.environ.get(k) for k in t.SHORTCUT_SWITCHES}))"
    on = json.loads(subprocess.run([sys.executable, "-c", code], env={**env, "PYTHONPATH": str(REPO)}, cwd=REPO,
                                   capture_output=True, text=True, check=True).stdout)
    assert all(v is None for v in on.values()), on
    off = json.loads(subprocess.run([sys.executable, "-c", code], env={**env, "PYTHONPATH": str(REPO), "TK8S_SHORTCUTS": "0"},
                                    cwd=REPO, capture_output=True, text=True, check=True).stdout)
    assert off == SHORTCUT_SWITCHES


def test_every_documented_off_switch_is_in_the_master_switch():
    """Each row of the shortcut table names its switch; the master switch must cover it."""
    from tritonk8ssupervisor_amd import SHORTCUT_SWITCHES

    doc = (REPO / "docs" / "architecture.md").read_text()
    table = doc[doc.index("## Start-up shortcuts and their off-switches"):]
    named = set(re.findall(r"`(TK8S_[A-Z_]+)=", table)) - {"TK8S_FAULTS", "TK8S_ZYGOTE_TIMEOUT", "TK8S_BOOT_CONTROLPLANE",
                                                           "TK8S_BOOT_AGENT", "TK8S_SHORTCUTS"}
    assert named and named <= set(SHORTCUT_SWITCHES), named - set(SHORTCUT_SWITCHES)
    # and setup.sh sets the ones it acts on before any interpreter starts
    sh = (REPO / "setup.sh").read_text()
    for k in ("TK8S_HOST_BURNIN=0", "TK8S_NO_PYCACHE_PREFIX=1", "TK8S_SKIP_SITE=0"):
        assert k in sh


def test_plain_argv_drops_the_site_skip_only_when_asked(monkeypatch):
    from tritonk8ssupervisor_amd.utils.procs import plain_argv

    argv = ["/sup", "--", sys.executable, "-S", "-c", "import x", "-S"]
    monkeypatch.delenv("TK8S_SHORTCUTS", raising=False)
    monkeypatch.delenv("TK8S_SKIP_SITE", raising=False)
    assert plain_argv(argv) == argv
    assert plain_argv(argv, {"TK8S_SHORTCUTS": "0"}) == ["/sup", "--", sys.executable, "-c", "import x", "-S"]
    assert plain_argv(argv, {"TK8S_SKIP_SITE": "0"}) == ["/sup", "--", sys.executable, "-c", "import x", "-S"]
