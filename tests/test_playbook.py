"""Playbook engine (the Ansible subset of ansible/clusterUp.yml + roles) and its Jinja subset.

Reference: ansible/clusterUp.yml:1-26, roles/*/tasks/main.yml; expressions like
``project_id['content'] | b64decode | replace('\\n', '')`` (rancherhost/tasks/main.yml:15).
"""
import json
import time
from pathlib import Path

import pytest
import yaml

from tritonk8ssupervisor_amd import templating as T
from tritonk8ssupervisor_amd.playbook import Playbook, _free_form, parse_inventory

REPO = Path(__file__).resolve().parents[1]


# ---- templating ----------------------------------------------------------------------------
def test_render_filters_and_types():
    v = {"p": {"content": "MWE3Cg=="}, "xs": [1, 2, 3], "name": "k8s dev", "n": "4"}
    assert T.render("{{ p['content'] | b64decode | replace('\\n', '') }}", v) == "1a7"
    assert T.render("{{ xs }}", v) == [1, 2, 3]  # a lone expression keeps its type
    assert T.render("id={{ xs | length }}", v) == "id=3"
    assert T.render("{{ (n | int) + 1 }}", v) == 5
    assert T.render("{{ n | int + 1 }}", v) == 5  # filters bind tighter than arithmetic (Jinja)
    assert T.render("{{ missing is defined }}", v) is False
    assert T.render("{{ p is not defined or xs | length > 2 }}", v) is True
    assert T.render("{{ name ~ '!' }}", v) == "k8s dev!"
    assert T.render("{{ missing | default('d') }}", v) == "d"
    assert T.render("{{ name | upper }}", v) == "K8S DEV"
    assert T.render("{{ xs | join(',') }}", v) == "1,2,3"
    assert T.render({"a": ["{{ name }}"]}, v) == {"a": ["k8s dev"]}
    assert T.render("{{ {'a': 1} | to_json }}", v) == '{"a": 1}'


def test_tests_and_truthiness():
    v = {"out": {"stdout": "rancher-agent up"}, "r": {"running": False}, "flag": "yes", "rc": 0}
    assert T.test("'rancher-agent' in out.stdout", v)
    assert T.test("not r.running", v)
    assert T.test("flag | bool", v)
    assert T.test("rc == 0 and out.stdout.find('up') > 0", v)
    assert not T.test("rc != 0 or 'x' in out.stdout", v)
    assert T.test(True, v) and not T.test(False, v)
    assert T.test(["rc == 0", "flag | bool"], v)  # list == all


def test_reference_inverted_when_is_not_needed():
    # dockersetup uses `when: docker_installed.stdout.find('Docker version')` (inverted truthiness,
    # ansible/roles/dockersetup/tasks/main.yml:10): -1 (absent) is truthy, 0 (found) falsy
    v = {"d": {"stdout": "Docker version 1.12.6"}}
    assert not T.test("d.stdout.find('Docker version')", v)
    v = {"d": {"stdout": ""}}
    assert T.test("d.stdout.find('Docker version')", v)


def test_undefined_and_sandbox():
    with pytest.raises(T.Undefined):
        T.render("{{ nope }}", {})
    with pytest.raises(T.TemplateError):
        T.evaluate("__import__('os').system('true')", {})
    with pytest.raises(T.TemplateError):
        T.evaluate("().__class__", {})


# ---- inventory / free-form ------------------------------------------------------------------
def test_inventory_groups_and_vars():
    inv = parse_inventory("[MASTER]\nkubemaster ansible_host=127.0.1.1\n[HOST]\nkubenode1 ansible_host=127.0.1.2\n"
                          "# comment\nkubenode2\n")
    assert inv["kubemaster"].groups == ["MASTER"] and inv["kubemaster"].address == "127.0.1.1"
    assert inv["kubenode2"].address == "kubenode2"
    assert [h for h in inv if "HOST" in inv[h].groups] == ["kubenode1", "kubenode2"]


def test_free_form_args():
    kv, free = _free_form('src="tmp/kubernetes_environment.id" mode=0644')
    assert kv == {"src": "tmp/kubernetes_environment.id", "mode": "0644"} and free == ""
    kv, free = _free_form("echo hi there")
    assert kv == {} and free == "echo hi there"


# ---- engine semantics ------------------------------------------------------------------------
def _play(tmp_path, plays, inventory="[MASTER]\nm1\n[HOST]\nh1\nh2\n", cfg="[defaults]\nforks = 0\n", roles=None, **kw):
    (tmp_path / "ansible.cfg").write_text(cfg)
    (tmp_path / "hosts").write_text(inventory)
    (tmp_path / "tmp").mkdir(exist_ok=True)
    for role, tasks in (roles or {}).items():
        d = tmp_path / "roles" / role / "tasks"
        d.mkdir(parents=True)
        (d / "main.yml").write_text(yaml.safe_dump(tasks))
    (tmp_path / "pb.yml").write_text(yaml.safe_dump(plays))
    lines = []
    pb = Playbook(tmp_path / "pb.yml", tmp_path / "hosts", out=lines.append, **kw)
    return pb, pb.run(), lines


def test_register_when_loop_set_fact(tmp_path):
    plays = [{"hosts": "all", "tasks": [
        {"name": "probe", "command": "echo {{ inventory_hostname }}", "register": "r"},
        {"name": "only masters", "set_fact": {"is_master": True}, "when": "'MASTER' in group_names"},
        {"name": "loop", "shell": "echo {{ item }}", "with_items": ["a", "b"], "register": "loop"},
        {"name": "skipped", "fail": {"msg": "never"}, "when": "r.stdout == 'nobody'"},
    ]}]
    pb, res, lines = _play(tmp_path, plays)
    assert res.ok, res.failures
    assert pb.hostvars["h1"]["r"]["stdout"] == "h1"
    assert pb.hostvars["m1"]["is_master"] is True and "is_master" not in pb.hostvars["h1"]
    assert [x["stdout"] for x in pb.hostvars["h2"]["loop"]["results"]] == ["a", "b"]
    assert res.stats["h1"]["skipped"] == 2 and res.stats["m1"]["skipped"] == 1
    assert any(l.startswith("PLAY RECAP") for l in lines)


def test_run_once_shares_result_and_failure_removes_host(tmp_path):
    plays = [{"hosts": "HOST", "tasks": [
        {"name": "once", "command": "date +%s%N", "run_once": True, "register": "o"},
        {"name": "fail h1", "fail": {"msg": "boom"}, "when": "inventory_hostname == 'h1'"},
        {"name": "after", "command": "true", "register": "after"},
    ]}]
    pb, res, _ = _play(tmp_path, plays)
    assert not res.ok and res.failures == ["h1: fail h1: boom"]
    assert pb.hostvars["h1"]["o"] == pb.hostvars["h2"]["o"]
    assert "after" in pb.hostvars["h2"] and "after" not in pb.hostvars["h1"]
    assert res.stats["h1"]["failed"] == 1


def test_ignore_errors_failed_when_changed_when(tmp_path):
    plays = [{"hosts": "m1", "tasks": [
        {"name": "ignored", "command": "false", "ignore_errors": True},
        {"name": "fw", "command": "echo ERROR", "register": "x", "failed_when": "'ERROR' in x.stdout", "ignore_errors": True},
        {"name": "cw", "command": "echo same", "register": "y", "changed_when": False},
    ]}]
    pb, res, _ = _play(tmp_path, plays)
    assert res.ok
    assert pb.hostvars["m1"]["x"]["failed"] is True and pb.hostvars["m1"]["x"]["ignored"] is True
    assert pb.hostvars["m1"]["y"]["changed"] is False


def test_until_retries_polls(tmp_path):
    # the reference polls `docker logs master` for "Listening on" (ranchermaster/tasks/main.yml:14-20)
    marker = tmp_path / "marker"
    plays = [{"hosts": "m1", "tasks": [
        {"name": "poll", "shell": f"n=$(cat {marker} 2>/dev/null || echo 0); echo $((n+1)) > {marker}; "
                                  f"[ $n -ge 2 ] && echo 'Listening on' || echo starting",
         "register": "logs", "until": "logs.stdout.find('Listening on') != -1", "retries": 5, "delay": 0.01},
    ]}]
    pb, res, _ = _play(tmp_path, plays)
    assert res.ok and pb.hostvars["m1"]["logs"]["attempts"] == 3
    plays[0]["tasks"][0]["retries"] = 0
    marker.unlink()
    (tmp_path / "roles").exists()
    pb2, res2, _ = _play(tmp_path / "again" if (tmp_path / "again").mkdir() is None else tmp_path, plays)
    assert not res2.ok and "until condition not met" in res2.failures[0]


def test_local_action_copy_slurp_stat(tmp_path):
    plays = [{"hosts": "m1", "tasks": [
        {"name": "store", "local_action": {"module": "copy", "content": "1a7", "dest": "{{ playbook_dir }}/tmp/env.id"}},
        {"name": "read", "local_action": "slurp src=tmp/env.id", "register": "pid"},
        {"name": "stat", "stat": {"path": "{{ playbook_dir }}/tmp/env.id"}, "register": "st", "delegate_to": "localhost"},
        {"name": "use", "debug": {"msg": "{{ pid['content'] | b64decode }}"}},
    ]}]
    pb, res, lines = _play(tmp_path, plays)
    assert res.ok, res.failures
    assert (tmp_path / "tmp" / "env.id").read_text() == "1a7"
    assert pb.hostvars["m1"]["st"]["stat"]["exists"] is True
    assert any("1a7" in l for l in lines)


def test_roles_and_vars_files(tmp_path):
    (tmp_path / "vars.yml").write_text("master: 10.0.0.1\nkubernetes_name: k8s dev\n")
    plays = [{"hosts": "MASTER", "vars_files": ["{{ playbook_dir }}/vars.yml"], "vars": {"playbook_dir": "$(pwd)"},
              "roles": ["r1"]}]
    roles = {"r1": [{"name": "uses vars", "set_fact": {"url": "http://{{ master }}:8080/{{ kubernetes_name }}"}}]}
    pb, res, lines = _play(tmp_path, plays, roles=roles)
    assert res.ok, res.failures
    assert pb.hostvars["m1"]["url"] == "http://10.0.0.1:8080/k8s dev"
    assert any("TASK [r1 : uses vars]" in l for l in lines)


def test_unknown_module_fails_cleanly(tmp_path):
    pb, res, _ = _play(tmp_path, [{"hosts": "m1", "tasks": [{"name": "x", "docker_container": {"name": "master"}}]}])
    assert not res.ok and "not supported" in res.failures[0]


def test_forks_bound_parallelism(tmp_path):
    inv = "[HOST]\n" + "".join(f"h{i}\n" for i in range(6))
    plays = [{"hosts": "all", "tasks": [{"name": "sleep", "command": "sleep 0.3"}]}]
    t = time.monotonic()
    _, res, _ = _play(tmp_path, plays, inventory=inv)  # forks=0 -> all 6 hosts at once
    all_at_once = time.monotonic() - t
    assert res.ok and all_at_once < 1.6  # one after another would be >= 1.8 s
    d = tmp_path / "f2"
    d.mkdir()
    t = time.monotonic()
    _, res, _ = _play(d, plays, inventory=inv, cfg="[defaults]\nforks = 2\n")  # 3 batches
    assert res.ok and time.monotonic() - t >= 0.85


def test_check_mode_on_shipped_cluster_playbook(tmp_path):
    """BASELINE.json config 1: `ansible-playbook --check clusterUp.yml` dry-run on localhost."""
    import shutil

    shutil.copytree(REPO / "ansible", tmp_path / "ansible")
    a = tmp_path / "ansible"
    (a / "hosts").write_text("[MASTER]\nkubemaster ansible_host=127.0.0.1\n[HOST]\nkubenode1 ansible_host=127.0.0.1\n")
    (a / "roles" / "ranchermaster" / "vars").mkdir(exist_ok=True)
    (a / "roles" / "ranchermaster" / "vars" / "vars.yml").write_text("master: 127.0.0.1\nkubernetes_name: k\nkubernetes_description: k\n")
    extra = {"tk8s_python": "python3", "tk8s_pythonpath": str(REPO), "tk8s_master_port": 1, "tk8s_bind_host": "127.0.0.1",
             "tk8s_cp_state_dir": str(tmp_path / "cp"), "tk8s_node_grace": 5, "tk8s_manifests": str(REPO / "manifests"),
             "tk8s_validation_command": ["true"], "tk8s_validation_pod_command": ["true", "--reuse", "x"],
             "tk8s_controlplane_argv": ["python3", "-m", "tritonk8ssupervisor_amd.controlplane"],
             "tk8s_validate": True, "tk8s_fake_gpus": "1"}
    lines = []
    res = Playbook(a / "clusterUp.yml", a / "hosts", extra_vars=extra, check=True, out=lines.append).run()
    assert res.ok, res.failures
    assert not (tmp_path / "cp").exists()  # nothing started / written
    assert not list((a / "tmp").glob("*.id"))
    plays = [l for l in lines if l.startswith("PLAY [")]
    assert len(plays) == 3


# ---- the fast subset agrees with real Jinja2 -----------------------------------------------------
CORPUS_VARS = {
    "project_id": {"content": "MWE3Cg=="}, "rancher_token_url": {"json": {"links": {"self": "http://m:8080/v1/t/1"}}},
    "joined": {"stat": {"exists": False}}, "agent": {"running": True}, "tk8s_validate": "yes", "group_names": ["HOST"],
    "tk8s_rocm_version": "7.0.0", "tk8s_fake_gpus": "", "tk8s_kfd": True, "tk8s_machine_gpus": [3],
    "kubernetes_template_id": {"json": {"data": [{"id": "1t5"}]}}, "env_id_file": {"stat": {"exists": True}},
    "master": "10.0.0.1", "tk8s_master_port": 8080, "inventory_hostname": "kubenode1", "xs": [1, 2, 3],
    "containerd_cfg": {"changed": True}, "k8s_sysctl": {"changed": False}, "n": "4", "name": "k8s dev",
    "cni": {"stdout": "daemonset.apps/kube-flannel-ds created"}, "groups": {"MASTER": ["kubemaster"]},
}
CORPUS = [
    "project_id['content'] | b64decode | replace('\\n', '')", "not joined.stat.exists",
    "not joined.stat.exists and not agent.running", "tk8s_validate | bool", "'HOST' in group_names",
    "tk8s_rocm_version != '' or tk8s_fake_gpus != ''", "tk8s_kfd or tk8s_fake_gpus != '' or (tk8s_machine_gpus | length) == 0",
    "kubernetes_template_id.json.data[0].id", "rancher_token_url.json['links']['self']", "xs | length > 2",
    "'restarted' if containerd_cfg is changed else 'started'", "k8s_sysctl is changed", "n | int + 1",
    "name ~ '!'", "missing | default('d')", "xs | join(',')", "name | upper", "groups['MASTER'][0]",
    "'created' in cni.stdout or 'configured' in cni.stdout", "master + ':' + tk8s_master_port | string",
    "tk8s_machine_gpus | first", "xs | last", "{'a': 1} | to_json", "true and not false", "none is none",
]


@pytest.mark.parametrize("expr", CORPUS)
def test_subset_agrees_with_jinja2(expr):
    fast = T._evaluate_subset(expr, CORPUS_VARS)
    assert fast == T.jinja_evaluate(expr, CORPUS_VARS), expr


def test_every_template_in_the_roles_parses():
    """Every {{ }} in the shipped playbooks and roles is either in the fast subset or valid Jinja2."""
    import re

    exprs = set()
    for f in [*(REPO / "ansible").glob("*.yml"), *(REPO / "ansible" / "roles").rglob("*.yml")]:
        exprs.update(m.strip() for m in re.findall(r"\{\{(.*?)\}\}", f.read_text(), re.S))
        for doc in yaml.safe_load(f.read_text()) or []:  # bare when/until/changed_when/failed_when
            for t in (doc.get("tasks") or [doc]) if isinstance(doc, dict) else []:
                for k in ("when", "until", "changed_when", "failed_when"):
                    if isinstance(t.get(k), str) and "{{" not in t[k]:
                        exprs.add(t[k].strip())
    assert len(exprs) > 45
    env = T._jinja_env(True)  # real Jinja2 + the Ansible filters/tests tk8s registers
    for e in exprs:
        try:
            T._rewrite(T._pyify(e))
        except T.TemplateError:
            pass
        env.compile_expression(e)  # raises on anything Jinja2 itself would reject


def test_outside_the_subset_goes_to_jinja2(tmp_path):
    v = {"xs": ["1", "2", "3"], "nodes": [{"a": {"g": "1"}}, {"a": {"g": "2"}}]}
    assert T.evaluate("xs | map('int') | sum", v) == 6  # map/sum: not in the subset
    assert T.evaluate("nodes | map(attribute='a') | map(attribute='g') | list", v) == ["1", "2"]
    (tmp_path / "t.yaml").write_text("image: {{ img }}\n")
    assert T.render("{{ lookup('template', p) }}", {"p": str(tmp_path / "t.yaml"), "img": "rocm/x"}) == "image: rocm/x\n"
    assert T.render("{% for x in xs %}{{ x }}{% endfor %}", v) == "123"
    with pytest.raises(T.Undefined):
        T.evaluate("nope | map('int') | list", {})


def test_cheap_tasks_on_local_machines_run_inline(tmp_path, monkeypatch):
    """Sandboxes of this host: file-only modules run host after host in the engine's thread;
    blocking modules, retries, loops, delegation and remote machines keep a thread per host."""
    plays = [{"hosts": "all", "gather_facts": False, "tasks": [
        {"name": "fact", "set_fact": {"x": "{{ inventory_hostname }}"}}]}]

    class Local:
        remote = False

    class Remote:
        remote = True

    pb, res, _ = _play(tmp_path, plays)
    assert res.ok and [pb.hostvars[h]["x"] for h in ("m1", "h1", "h2")] == ["m1", "h1", "h2"]
    pb.executor = Local()
    assert pb._inline({"set_fact": {"a": 1}}) and pb._inline({"ansible.builtin.copy": {"dest": "x", "content": ""}})
    assert not pb._inline({"command": "sleep 1"}) and not pb._inline({"uri": {"url": "http://x"}})
    assert not pb._inline({"stat": {"path": "x"}, "until": "r.stat.exists"})
    assert not pb._inline({"debug": {"msg": "x"}, "loop": [1, 2]})
    assert not pb._inline({"debug": {"msg": "x"}, "delegate_to": "localhost"})
    monkeypatch.setenv("TK8S_PLAY_INLINE", "0")
    assert not pb._inline({"set_fact": {"a": 1}})
    monkeypatch.delenv("TK8S_PLAY_INLINE")
    pb.executor = Remote()
    assert not pb._inline({"set_fact": {"a": 1}})


def test_pidfile_only_daemon_tasks_and_when_run_in_the_engine_thread(tmp_path, monkeypatch):
    """tk8s_daemon reads only pidfiles for a query, or for a start of a daemon already running
    on every host the task applies to: inline. `when:` is evaluated before any host goes to a
    thread, so a task that skips one host (the master) does not send the others to threads."""
    import threading

    class Local:
        remote = False

        def __init__(self):
            self.calls = []

        def daemon_status(self, host, name):
            self.calls.append((host, threading.get_ident()))
            return {"running": host != "m1", "pid": 1}

    pb, res, _ = _play(tmp_path, [{"hosts": "all", "gather_facts": False, "tasks": []}])
    ex = Local()
    pb.executor = ex
    assert pb._inline({"tk8s_daemon": {"name": "agent", "state": "query"}})
    hosts = [pb.hosts[h] for h in ("h1", "h2")]
    assert pb._inline({"tk8s_daemon": {"name": "agent", "argv": ["x"]}}, hosts)  # running on both
    assert not pb._inline({"tk8s_daemon": {"name": "agent", "argv": ["x"]}}, [pb.hosts["m1"], *hosts])
    assert not pb._inline({"tk8s_daemon": {"name": "{{ n }}", "argv": ["x"]}}, hosts)  # templated: undecided
    # a run: `when:` skips the master in the engine's thread; the two hosts left run inline
    ran = []
    monkeypatch.setattr(pb, "_exec", lambda task, mod, raw, v, host, deleg, local: (
        ran.append((host.name, threading.get_ident())) or {"changed": False}))
    task = {"name": "standby", "tk8s_daemon": {"name": "agent", "argv": ["x"]},
            "when": "inventory_hostname != 'm1'"}
    res = pb.run_task(task, [pb.hosts[h] for h in ("m1", "h1", "h2")], {})
    assert [r.status for r in res] == ["skipped", "ok", "ok"]
    assert sorted(h for h, _ in ran) == ["h1", "h2"] and {t for _, t in ran} == {threading.get_ident()}
