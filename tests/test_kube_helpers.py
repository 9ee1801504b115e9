"""kube.py's copy of server-side apply's content type matches the control plane's, and importing
kube (setup's deploy task does, on the bring-up's critical path) leaves the wire module out."""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def test_apply_patch_content_type_matches_the_control_plane():
    from tritonk8ssupervisor_amd import kube
    from tritonk8ssupervisor_amd.controlplane import k8s_wire

    assert kube.APPLY_PATCH == k8s_wire.APPLY_PATCH


def test_importing_kube_does_not_import_the_wire_module():
    code = ("import sys, tritonk8ssupervisor_amd.kube\n"
            "print('tritonk8ssupervisor_amd.controlplane.k8s_wire' in sys.modules)")
    out = subprocess.run([sys.executable, "-S", "-c", code], cwd=REPO, capture_output=True, text=True, check=True,
                         env={"PYTHONPATH": str(REPO), "PATH": "/usr/bin:/bin"}).stdout.strip()
    assert out == "False"
