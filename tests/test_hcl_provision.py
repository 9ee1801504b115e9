"""HCL subset, rancher.tf rendering (setup.sh:162-198) and the provisioning engine
(terraform get/plan/apply/destroy, setup.sh:154-159, 498-503) over the local provider."""
import json
import os
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd import hcl
from tritonk8ssupervisor_amd.orchestrator import init_workspace
from tritonk8ssupervisor_amd.provider.local import LocalProvider
from tritonk8ssupervisor_amd.provision import Engine

REF = Path("/root/reference")


def test_parse_blocks_lists_maps_comments():
    b = hcl.parse('''
    # comment
    // another
    /* block
       comment */
    provider "triton" { account = "me"  url = "https://x" }
    module "m1" {
      source = "master"
      networks = ["a", "b",]
      n = 3
      ok = true
      tags = { role = "host", "k" = "v" }
      key = "${file("/etc/hostname")}"
    }
    ''')
    (p,) = b.children("provider")
    assert p.labels == ["triton"] and p.attrs == {"account": "me", "url": "https://x"}
    (m,) = b.children("module")
    assert m.attrs["networks"] == ["a", "b"] and m.attrs["n"] == 3 and m.attrs["ok"] is True
    assert m.attrs["tags"] == {"role": "host", "k": "v"}
    assert m.attrs["key"] == '${file("/etc/hostname")}'


def test_duplicate_attribute_is_reported():
    b = hcl.parse('resource "t" "r" {\n tags = { a = "1" }\n tags = { a = "2" }\n}\n')
    (r,) = b.children("resource")
    assert r.attrs["tags"] == {"a": "2"}
    assert r.duplicates  # the reference declares tags twice (terraform/master/main.tf:6-8, 33-35)


def test_parse_errors():
    with pytest.raises(hcl.HclError):
        hcl.parse('module "x" { a = ')
    with pytest.raises(hcl.HclError):
        hcl.parse("/* never closed")


def test_interpolation_types_and_functions(tmp_path):
    (tmp_path / "k.pub").write_text("ssh-ed25519 AAA me\n")
    ctx = {"var": {"networks": ["n1", "n2"], "hostname": "kubenode1"}, "__dir__": str(tmp_path),
           "tk8s_machine": {"host": {"primaryip": "127.0.1.2"}}}
    assert hcl.interpolate("${var.networks}", ctx) == ["n1", "n2"]  # exact interpolation keeps list type
    assert hcl.interpolate("nets=${var.networks}", ctx) == "nets=n1,n2"
    assert hcl.interpolate('${file("k.pub")}', ctx) == "ssh-ed25519 AAA me\n"
    assert hcl.interpolate("echo ${tk8s_machine.host.primaryip} >> hosts.ip", ctx) == "echo 127.0.1.2 >> hosts.ip"
    assert hcl.interpolate({"a": ["${var.hostname}"]}, ctx) == {"a": ["kubenode1"]}
    with pytest.raises(hcl.HclError):
        hcl.interpolate("${var.nope}", ctx)
    with pytest.raises(hcl.HclError):
        hcl.interpolate('${file("missing")}', ctx)


def test_render_root_golden():
    text = hcl.render_root("local", "me", "/k/id_ed25519", "/k/id_ed25519.pub", "SHA256:abc", "local://h",
                           "kubemaster", ["net-a"], ["kubenode1", "kubenode2"], ["net-a", "net-b"], "pkg-1")
    want = '''provider "local" {
    account = "me"
    key_material = "${file("/k/id_ed25519")}"
    key_id = "SHA256:abc"
    url = "local://h"
}

module "kubemaster" {
    source = "master"
    hostname = "kubemaster"
    networks = ["net-a"]
    root_authorized_keys = "${file("/k/id_ed25519.pub")}"
    package = "pkg-1"
}

module "kubenode1" {
    source = "host"
    hostname = "kubenode1"
    networks = ["net-a","net-b"]
    root_authorized_keys = "${file("/k/id_ed25519.pub")}"
    package = "pkg-1"
}

module "kubenode2" {
    source = "host"
    hostname = "kubenode2"
    networks = ["net-a","net-b"]
    root_authorized_keys = "${file("/k/id_ed25519.pub")}"
    package = "pkg-1"
}
'''
    assert text == want
    parsed = hcl.parse(text)
    assert [m.labels[0] for m in parsed.children("module")] == ["kubemaster", "kubenode1", "kubenode2"]


@pytest.mark.skipif(not (REF / "terraform").is_dir(), reason="reference checkout not mounted")
def test_parses_the_reference_terraform_modules():
    # the engine must read Terraform-0.9-era files like the reference's own modules
    for mod in ("master", "host"):
        b = hcl.parse_dir(REF / "terraform" / mod)
        (r,) = b.children("resource")
        assert r.labels[0] == "triton_machine"
        assert {"hostname", "networks", "root_authorized_keys", "image", "package"} <= {v.labels[0] for v in b.children("variable")}
        assert "tags" in r.duplicates
        kinds = [p.labels[0] for p in r.children("provisioner")]
        assert kinds == ["remote-exec", "local-exec"]


def test_own_modules_keep_reference_variables():
    for mod in ("master", "host"):
        b = hcl.parse_dir(Path(__file__).resolve().parents[1] / "terraform" / mod)
        assert {"hostname", "networks", "root_authorized_keys", "image", "package"} == {v.labels[0] for v in b.children("variable")}
        (r,) = b.children("resource")
        assert not r.duplicates


# ---- engine -------------------------------------------------------------------------------
@pytest.fixture
def ws(tmp_path, monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")
    monkeypatch.delenv("TK8S_FAULTS", raising=False)
    return init_workspace(tmp_path)


def _rancher_tf(ws, prov, nodes, package="mi355x-1gpu"):
    env = prov.env()
    key = prov.find_key(env["SDC_KEY_ID"])
    pub = prov.network_by_id_or_name("local-public").id
    text = hcl.render_root("local", env["SDC_ACCOUNT"], key, key + ".pub", env["SDC_KEY_ID"], env["SDC_URL"],
                           "kubemaster", [pub], [f"kubenode{i}" for i in range(1, nodes + 1)], [pub],
                           prov.package_by_id_or_name(package).id)
    (ws.tf / "rancher.tf").write_text(text)


def test_engine_get_plan_apply_destroy(ws):
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 3)
    eng = Engine(ws.tf, prov)
    assert eng.get() == ["kubemaster", "kubenode1", "kubenode2", "kubenode3"]
    assert (ws.tf / ".terraform" / "modules" / "kubenode1").resolve() == (ws.tf / "host").resolve()
    plan = eng.plan()
    assert [a.action for a in plan] == ["create"] * 4
    assert "Plan: 4 to add, 0 to change, 0 to destroy." in Engine.plan_summary(plan)
    res = eng.apply()
    assert res.ok and len(res.created) == 4
    ms = eng.machines()
    assert ms["kubemaster"].gpus == []  # the master never takes a GPU
    gpus = sorted(g for n in ("kubenode1", "kubenode2", "kubenode3") for g in ms[n].gpus)
    assert len(gpus) == 3 and len(set(gpus)) == 3  # exclusive GPU slices
    # hand-off files in module order, one IP per line (race-free rewrite of terraform/*/main.tf:30)
    assert (ws.tf / "masters.ip").read_text().split() == [ms["kubemaster"].primaryip]
    assert (ws.tf / "hosts.ip").read_text().split() == [ms[f"kubenode{i}"].primaryip for i in (1, 2, 3)]
    assert len({m.primaryip for m in ms.values()}) == 4 or os.environ.get("TK8S_SINGLE_IP") == "1"
    # second apply is a no-op
    assert [a.action for a in eng.plan()] == ["no-op"] * 4
    res2 = eng.apply()
    assert res2.ok and not res2.created and len(res2.unchanged) == 4
    # destroy frees everything
    assert len(eng.destroy()) == 4
    assert eng.state()["resources"] == {}
    assert prov.list_machines() == []
    alloc = json.loads((ws.state_dir / "alloc.json").read_text())
    assert alloc["machines"] == {} and alloc["gpus"] == {}


def test_engine_scale_down_plans_destroy(ws):
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 2)
    eng = Engine(ws.tf, prov)
    eng.get()
    assert eng.apply().ok
    _rancher_tf(ws, prov, 1)
    acts = {a.address: a.action for a in eng.plan()}
    assert acts["module.kubenode2.tk8s_machine.host"] == "destroy"


def test_engine_gpu_capacity_is_the_provisioning_limit(ws, monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "2")
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 3)
    eng = Engine(ws.tf, prov)
    eng.get()
    res = eng.apply()
    assert not res.ok and len(res.failed) == 1 and len(res.created) == 3
    assert "provisioning limit" in next(iter(res.failed.values()))


def test_engine_retries_injected_create_failure(ws, monkeypatch):
    monkeypatch.setenv("TK8S_FAULTS", "provision.create@kubenode2")
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 2)
    eng = Engine(ws.tf, prov, retries=1)
    eng.get()
    res = eng.apply()
    assert res.ok, res.failed  # first attempt fails, the retry succeeds


def test_engine_no_retries_marks_failure(ws, monkeypatch):
    monkeypatch.setenv("TK8S_FAULTS", "provision.create@kubenode1")
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 1)
    eng = Engine(ws.tf, prov, retries=0)
    eng.get()
    res = eng.apply()
    assert not res.ok and "module.kubenode1.tk8s_machine.host" in res.failed
    assert not (ws.tf / "hosts.ip").exists()  # missing hand-off file == setup.sh:117-120 error path


def test_engine_tainted_resource_is_replaced(ws):
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 1)
    eng = Engine(ws.tf, prov)
    eng.get()
    assert eng.apply().ok
    st = eng.state()
    st["resources"]["module.kubenode1.tk8s_machine.host"]["tainted"] = True
    (ws.tf / "terraform.tfstate").write_text(json.dumps(st))
    assert {a.address: a.action for a in eng.plan()}["module.kubenode1.tk8s_machine.host"] == "replace"
    res = eng.apply()
    assert res.ok and res.created == ["module.kubenode1.tk8s_machine.host"]


def test_engine_rejects_unknown_module_argument(ws):
    prov = LocalProvider(ws.state_dir)
    (ws.tf / "rancher.tf").write_text('module "x" {\n source = "host"\n hostname = "x"\n networks = []\n bogus = 1\n}\n')
    with pytest.raises(Exception, match="unknown arguments"):
        Engine(ws.tf, prov).specs()


def test_clusters_on_one_host_never_share_an_ip_or_a_gpu(tmp_path, monkeypatch):
    """Two workspaces on one host: the host registry keeps their loopback IPs (and so their DNS,
    ingress and NodePort sockets) and their GPUs disjoint, and frees them on delete or when the
    owner is gone."""
    monkeypatch.setenv("TK8S_HOST_REGISTRY", str(tmp_path / "hostreg"))
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")
    monkeypatch.setattr(LocalProvider, "_host_gpus", staticmethod(lambda: True))  # as on a real host
    a, b = LocalProvider(tmp_path / "a"), LocalProvider(tmp_path / "b")
    ma = a.create_machine("kubemaster", "cpu-only", ["local-public"], tags={"role": "master"})
    wa = a.create_machine("kubenode1", "mi355x-4gpu", ["local-public"])
    mb = b.create_machine("kubemaster", "cpu-only", ["local-public"], tags={"role": "master"})
    wb = b.create_machine("kubenode1", "mi355x-4gpu", ["local-public"])
    assert len({ma.primaryip, wa.primaryip, mb.primaryip, wb.primaryip}) == 4
    assert not set(wa.gpus) & set(wb.gpus) and len(wa.gpus + wb.gpus) == 8
    assert b.predict_gpus(1, 1) == []
    with pytest.raises(Exception, match="free"):
        b.create_machine("kubenode2", "mi355x-1gpu", ["local-public"])
    a.delete_machine(wa)  # released explicitly
    assert len(b.predict_gpus(4, 1)) == 4
    w2 = b.create_machine("kubenode2", "mi355x-4gpu", ["local-public"])
    assert sorted(w2.gpus) == sorted(wa.gpus)
    # a workspace deleted without teardown: its claims are reaped on the next allocation
    import shutil

    shutil.rmtree(tmp_path / "b")
    c = LocalProvider(tmp_path / "c")
    assert len(c.predict_gpus(4, 2)) == 8
    assert c.create_machine("kubemaster", "cpu-only", ["local-public"], tags={"role": "master"}).primaryip != ma.primaryip


# ---- the stock-Terraform form (terraform/compat: terraform_data + `tk8s machine`) ----------------
def _rancher_tf_form(ws, prov, nodes, form):
    env = prov.env()
    key = prov.find_key(env["SDC_KEY_ID"])
    pub = prov.network_by_id_or_name("local-public").id
    (ws.tf / "rancher.tf").write_text(hcl.render_root(
        "local", env["SDC_ACCOUNT"], key, key + ".pub", env["SDC_KEY_ID"], env["SDC_URL"], "kubemaster", [pub],
        [f"kubenode{i}" for i in range(1, nodes + 1)], [pub], prov.package_by_id_or_name("mi355x-1gpu").id, form=form))


def test_both_terraform_forms_plan_identically(ws):
    """the modules stock Terraform can load (terraform_data + local-exec calling
    `./tk8s machine create|delete`) plan exactly like the engine's tk8s_machine modules. Real
    terraform is not installed here: that it accepts the files is unpinned beyond the HCL2
    constructs they use (built-in terraform_data, list(string), join(), when = destroy)."""
    prov = LocalProvider(ws.state_dir)
    plans = {}
    for form in ("tk8s", "compat"):
        _rancher_tf_form(ws, prov, 2, form)
        eng = Engine(ws.tf, prov)
        eng.get()
        plans[form] = [(a.address.split(".")[1], a.action, a.attrs) for a in eng.plan()]
    assert plans["tk8s"] == plans["compat"]
    assert [p[0] for p in plans["compat"]] == ["kubemaster", "kubenode1", "kubenode2"]
    text = (ws.tf / "rancher.tf").read_text()
    assert 'source = "compat/host"' in text and 'provider "local"' not in text  # no provider to download
    compat = (hcl.parse_dir(ws.tf / "compat" / "host")).children("resource")[0]
    assert compat.labels == ["terraform_data", "host"]
    cmds = [p.attrs["command"] for p in compat.children("provisioner")]
    assert any("machine create" in c for c in cmds) and any("machine delete" in c for c in cmds)


def test_compat_form_applies_through_the_engine(ws):
    prov = LocalProvider(ws.state_dir)
    _rancher_tf_form(ws, prov, 2, "compat")
    eng = Engine(ws.tf, prov)
    eng.get()
    res = eng.apply()
    assert res.ok and len(res.created) == 3
    ms = eng.machines()
    assert (ws.tf / "hosts.ip").read_text().split() == [ms["kubenode1"].primaryip, ms["kubenode2"].primaryip]
    assert len(eng.destroy()) == 3 and prov.list_machines() == []


def test_machine_cli_is_what_the_compat_provisioners_run(ws):
    """The exact commands terraform/compat/host/main.tf's provisioners run, from terraform/."""
    import subprocess
    import sys

    repo = Path(__file__).resolve().parents[1]
    env = dict(os.environ, PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable)
    import shutil

    shutil.copy2(repo / "tk8s", ws.root / "tk8s")
    prov = LocalProvider(ws.state_dir)
    pub = prov.network_by_id_or_name("local-public").id
    pkg = prov.package_by_id_or_name("mi355x-1gpu").id
    run = lambda *a: subprocess.run(["../tk8s", "--workdir", "..", "machine", *a], cwd=ws.tf, env=env,
                                    capture_output=True, text=True, timeout=60)
    r = run("create", "--name", "kubenode1", "--package", pkg, "--networks", pub, "--role", "host", "--ip-file", "hosts.ip")
    assert r.returncode == 0, r.stderr
    m = json.loads(r.stdout)
    assert m["name"] == "kubenode1" and len(m["gpus"]) == 1
    assert (ws.tf / "hosts.ip").read_text().split() == [m["primaryip"]]
    assert [json.loads(x)["name"] for x in run("list").stdout.splitlines()] == ["kubenode1"]
    assert run("delete", "--name", "kubenode1").returncode == 0
    assert prov.list_machines() == []
    assert "already deleted" in run("delete", "--name", "kubenode1").stdout  # destroy is idempotent


def test_bootstrap_refuses_a_node_runtime_older_than_python_3_8(ws, tmp_path, monkeypatch):
    """The modules' bootstrap checks the machine's python3 by its --version (no interpreter start
    on the critical path): 3.8 and later pass, an older one fails the machine, tainted."""
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 1)
    old = tmp_path / "oldpy"
    old.mkdir()
    (old / "python3").write_text("#!/bin/sh\necho 'Python 3.6.9'\n")
    (old / "python3").chmod(0o755)
    monkeypatch.setenv("PATH", f"{old}:{os.environ['PATH']}")
    eng = Engine(ws.tf, prov, retries=0)
    eng.get()
    res = eng.apply()
    assert not res.ok and "python3 >= 3.8 required" in json.dumps(res.failed), res.failed
    assert any(r.get("tainted") for r in eng.state()["resources"].values())
    monkeypatch.setenv("PATH", os.environ["PATH"].split(":", 1)[1])
    (old / "python3").write_text("#!/bin/sh\necho 'Python 3.12.3'\n")
    monkeypatch.setenv("PATH", f"{old}:{os.environ['PATH']}")
    assert eng.apply().ok  # the tainted machines are replaced, and 3.12 passes
    eng.destroy()


@pytest.mark.parametrize("in_process", [True, False])
def test_bootstrap_in_process_and_its_off_switch(ws, monkeypatch, in_process):
    """A local machine's standard bootstrap is checked in the engine (no shell per machine);
    TK8S_INPROCESS_BOOTSTRAP=0 sends it to the provider's shell. Both refuse a sandbox whose
    directories are missing."""
    from tritonk8ssupervisor_amd import provision
    from tritonk8ssupervisor_amd.provider.base import Machine

    monkeypatch.setenv("TK8S_INPROCESS_BOOTSTRAP", "1" if in_process else "0")
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 2)
    scripts = []
    real = prov.exec
    monkeypatch.setattr(prov, "exec", lambda m, c, *a, **k: (scripts.append(c), real(m, c, *a, **k))[1])
    eng = Engine(ws.tf, prov, retries=0)
    eng.get()
    assert eng.apply().ok
    boots = [c for c in scripts if provision.BOOTSTRAP[0] in c]
    assert len(boots) == (0 if in_process else 3), scripts
    m = Machine(name="x", id="x", package="p", networks=[], primaryip="127.0.0.9", sandbox=str(ws.state_dir))
    done = provision._bootstrap_in_process(prov, m, list(provision.BOOTSTRAP))
    if in_process:
        assert done is not None and done[0] != 0 and "missing" in done[1]
    else:
        assert done is None
    eng.destroy()


def test_engine_reserves_all_machines_in_one_allocation(ws, monkeypatch):
    """The local provider allocates every planned machine's address and GPU slice under one take
    of the locks (reserve), and a machine whose create fails for good gives its reservation back."""
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 3)
    writes = []
    import tritonk8ssupervisor_amd.provider.local as local

    real = local.atomic_write_json
    monkeypatch.setattr(local, "atomic_write_json", lambda p, o: (writes.append(Path(p).name), real(p, o))[1])
    eng = Engine(ws.tf, prov)
    eng.get()
    assert eng.apply().ok
    assert writes.count("alloc.json") == 1, writes  # one allocation for the four machines
    eng.destroy()
    # a create that fails for good (injected, no retries): its reservation is released
    monkeypatch.setenv("TK8S_FAULTS", "provision.create@kubenode2")
    eng2 = Engine(ws.tf, LocalProvider(ws.state_dir), retries=0)
    res = eng2.apply()
    assert not res.ok and list(res.failed) == ["module.kubenode2.tk8s_machine.host"], res.failed
    alloc = json.loads((ws.state_dir / "alloc.json").read_text())
    assert sorted(alloc["machines"]) == ["kubemaster", "kubenode1", "kubenode3"], alloc["machines"]
    eng2.destroy()


def test_hcl_token_cache_round_trips_and_is_keyed_by_text(tmp_path, monkeypatch):
    """The parser's tokens are remembered across runs (utils/pcache.py, keyed by the file's whole
    text): a later process parses from the cache to the same tree, and a changed text is
    tokenized afresh."""
    from tritonk8ssupervisor_amd.utils.pcache import PersistentCache

    monkeypatch.setenv("TK8S_YAML_CACHE", str(tmp_path))
    monkeypatch.setattr(hcl, "_TOKEN_MEMO", {})
    monkeypatch.setattr(hcl, "_TOKEN_CACHE", None)
    text = 'module "m" {\n  source = "host"\n  n = 3\n  ok = true\n  nets = ["a", "${var.x}"]\n}\n'
    first = hcl.parse(text, cache=True)
    table = PersistentCache(f"hcl-tokens-{hcl._TOKENS_VERSION}")
    assert table.get(text) == hcl._tokens(text)
    monkeypatch.setattr(hcl, "_TOKEN_MEMO", {})  # a new process: from the file
    monkeypatch.setattr(hcl, "_TOKEN_CACHE", None)
    calls = []
    real = hcl._tokens
    monkeypatch.setattr(hcl, "_tokens", lambda t: (calls.append(t), real(t))[1])
    assert hcl.parse(text, cache=True) == first and calls == []
    assert hcl.parse(text.replace("3", "4"), cache=True).children("module")[0].attrs["n"] == 4 and len(calls) == 1
    assert hcl.parse(text) == first and len(calls) == 2  # the generated root: never cached


@pytest.mark.parametrize("serial", ["1", "0"])
def test_local_machines_master_first_and_the_state_holds_every_one(ws, monkeypatch, serial):
    """Local machines are created one after another, the master first (its control plane boots
    while the workers are made; profiles/r6_curve: 8 workers 0.0655 vs 0.0701 s with a thread per
    machine); TK8S_PROVISION_SERIAL=0 brings the threads back. Either way the state -- written
    through by one writer while the creations run -- ends up holding every machine."""
    import threading

    monkeypatch.setenv("TK8S_PROVISION_SERIAL", serial)
    prov = LocalProvider(ws.state_dir)
    _rancher_tf(ws, prov, 4)
    order, threads = [], set()
    real = prov.create_machine

    def create(name, *a, **kw):
        order.append(name)
        threads.add(threading.get_ident())
        return real(name, *a, **kw)

    monkeypatch.setattr(prov, "create_machine", create)
    eng = Engine(ws.tf, prov)
    eng.get()
    assert eng.apply().ok
    if serial == "1":
        assert order[0] == "kubemaster" and len(threads) == 1, (order, threads)
    st = json.loads((ws.tf / "terraform.tfstate").read_text())
    assert sorted(st["resources"]) == sorted(f"module.{m}.tk8s_machine.{'master' if m == 'kubemaster' else 'host'}"
                                           for m in ["kubemaster", "kubenode1", "kubenode2", "kubenode3", "kubenode4"])
    assert st["serial"] >= 5


def test_coalesced_state_writer_loses_no_record(ws):
    """_save_resource inside apply(): records arriving while another thread writes ride on its
    next write; after the final flush the file holds every one of 200 concurrent records."""
    import threading

    eng = Engine(ws.tf, LocalProvider(ws.state_dir))
    eng._mem, eng._dirty = {"version": 1, "resources": {}}, 0
    ts = [threading.Thread(target=lambda k=k: eng._save_resource(f"r{k}", {"k": k})) for k in range(200)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    eng._flush(wait=True)
    st = json.loads((ws.tf / "terraform.tfstate").read_text())
    assert len(st["resources"]) == 200 and st["serial"] == 200
