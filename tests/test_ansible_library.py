"""ansible/library/tk8s_*.py: the tk8s modules as real Ansible modules.

Ansible itself is not installed here (parity with a real ansible-playbook run is unpinned beyond
this): the modules run against tests/ansible_shim, a stand-in for ansible.module_utils.basic with
Ansible's argument-passing and exit contract. Pinned: every argument the shipped roles pass is in
the module's spec, and the modules do on the machine they run on what the in-repo engine does.
"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import pytest
import yaml

from tritonk8ssupervisor_amd.ansible_bridge import ARG_SPECS

REPO = Path(__file__).resolve().parents[1]
LIB = REPO / "ansible" / "library"
SHIM = REPO / "tests" / "ansible_shim"


def _role_uses():
    out = {}
    for f in (REPO / "ansible" / "roles").glob("*/tasks/main.yml"):
        for t in yaml.safe_load(f.read_text()) or []:
            for k, v in t.items():
                if k.startswith("tk8s_"):
                    out.setdefault(k, set()).update((v or {}).keys())
    return out


def test_library_matches_the_modules_the_roles_use():
    uses = _role_uses()
    assert set(uses) <= set(ARG_SPECS) and set(ARG_SPECS) == {p.stem for p in LIB.glob("tk8s_*.py")}
    for mod, args in uses.items():
        assert args <= set(ARG_SPECS[mod]), (mod, args - set(ARG_SPECS[mod]))


def _run(mod, args, tmp_path, check=False, env=None):
    f = tmp_path / f"{mod}-{time.monotonic_ns()}.json"
    f.write_text(json.dumps({"ANSIBLE_MODULE_ARGS": {**args, "_ansible_check_mode": check}}))
    e = dict(os.environ, PYTHONPATH=str(SHIM), TK8S_HOME=str(REPO), **(env or {}))
    r = subprocess.run([sys.executable, str(LIB / f"{mod}.py"), str(f)], env=e, capture_output=True, text=True,
                       timeout=60, cwd=tmp_path)
    return r.returncode, json.loads(r.stdout.strip().splitlines()[-1])


def test_gpu_facts_module(tmp_path):
    rc, out = _run("tk8s_gpu_facts", {"machine_dir": str(tmp_path / "m"), "gpus": "1"}, tmp_path,
                   env={"TK8S_FAKE_GPUS": "2"})
    assert rc == 0, out
    f = out["ansible_facts"]
    assert f["tk8s_host_gpus"] == 2 and f["tk8s_machine_gpus"] == [1] and "tk8s_rocm_version" in f


def test_daemon_module_lifecycle(tmp_path):
    m = {"machine_dir": str(tmp_path / "m"), "name": "sleeper"}
    rc, out = _run("tk8s_daemon", {**m, "argv": ["sh", "-c", "echo up; exec sleep 60"], "restart_policy": "no",
                                   "wait_for_log": "up", "timeout": 10}, tmp_path)
    assert rc == 0 and out["changed"] and out["running"], out
    pid = out["pid"]
    rc, out = _run("tk8s_daemon", {**m, "state": "query"}, tmp_path)
    assert rc == 0 and out["running"] and out["pid"] == pid
    rc, out = _run("tk8s_daemon", {**m, "state": "stopped"}, tmp_path, check=True)
    assert rc == 0 and out["changed"] and out["running"] is False  # check mode: would stop, did not
    rc, out = _run("tk8s_daemon", {**m, "state": "query"}, tmp_path)
    assert out["running"]
    rc, out = _run("tk8s_daemon", {**m, "state": "stopped"}, tmp_path)
    assert rc == 0 and out["changed"]
    rc, out = _run("tk8s_daemon", {**m, "state": "query"}, tmp_path)
    assert out["running"] is False


def test_argument_errors_are_ansible_errors(tmp_path):
    rc, out = _run("tk8s_daemon", {"machine_dir": str(tmp_path), "name": "x", "state": "bogus"}, tmp_path)
    assert rc == 1 and out["failed"] and "must be one of" in out["msg"]
    rc, out = _run("tk8s_burnin", {"machine_dir": str(tmp_path)}, tmp_path)
    assert rc == 1 and "command" in out["msg"]
    rc, out = _run("tk8s_kube", {"api": "x", "project": "y", "nope": 1}, tmp_path)
    assert rc == 1 and "Unsupported parameters" in out["msg"]


def test_burnin_module_without_gpus_is_a_noop(tmp_path):
    rc, out = _run("tk8s_burnin", {"machine_dir": str(tmp_path / "m"), "command": ["true"]}, tmp_path)
    assert rc == 0 and out.get("skipped") and "no GPUs" in out["msg"]


def test_library_files_are_the_generated_front_ends():
    """the five front ends are one template (ansible_bridge.LIBRARY_TEMPLATE) rendered
    per module; the shipped files must be exactly that output (regenerate with
    `python -m tritonk8ssupervisor_amd.ansible_bridge --write-library`)."""
    from tritonk8ssupervisor_amd.ansible_bridge import library_sources

    gen = library_sources()
    assert set(gen) == {p.stem for p in LIB.glob("tk8s_*.py")}
    for name, text in gen.items():
        assert (LIB / f"{name}.py").read_text() == text, name


def test_the_library_modules_document_every_option_for_ansible_doc():
    """What ansible-doc reads: DOCUMENTATION's options match ARG_SPECS (type, default, choices,
    required), every option has a real description, and EXAMPLES / RETURN are valid YAML."""
    import yaml

    from tritonk8ssupervisor_amd.ansible_bridge import ARG_SPECS

    lib = Path(__file__).resolve().parents[1] / "ansible" / "library"
    for name, spec in ARG_SPECS.items():
        src = (lib / f"{name}.py").read_text()
        ns: dict = {}
        exec(compile(src.split("def _home")[0], str(lib / f"{name}.py"), "exec"), ns)  # the module's constants only
        doc = yaml.safe_load(ns["DOCUMENTATION"])
        assert doc["module"] == name and set(doc["options"]) == set(spec), name
        for opt, o in doc["options"].items():
            assert o["type"] == spec[opt]["type"] and o["description"] != opt and len(o["description"]) > 15, (name, opt)
            assert o.get("required", False) == spec[opt].get("required", False), (name, opt)
            assert o.get("default") == spec[opt].get("default"), (name, opt)
            assert o.get("choices") == spec[opt].get("choices"), (name, opt)
        examples = yaml.safe_load(ns["EXAMPLES"])
        assert any(name in task for task in examples), name
        assert yaml.safe_load(ns["RETURN"]), name
