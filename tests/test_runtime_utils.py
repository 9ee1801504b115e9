"""Unit tests: pod runtime (restart policies, $(VAR) expansion, results), cluster keys, fs/event
helpers, fault parsing, and the Joyent `triton` provider driven by a fake `triton` CLI."""
import json
import os
import subprocess
import sys
import threading
import time
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd.agent.runtime import PodProc, PodRuntime, expand, last_json_line
from tritonk8ssupervisor_amd.provider import keys
from tritonk8ssupervisor_amd.utils import faults
from tritonk8ssupervisor_amd.utils.events import EventLog, read_events
from tritonk8ssupervisor_amd.utils.fsutil import atomic_write, atomic_write_json, file_lock, locked_append_line, read_json


# ---- pod runtime ---------------------------------------------------------------------------
def test_expand_kubernetes_style():
    env = {"A": "1", "JOB_COMPLETION_INDEX": "3"}
    assert expand("rank=$(JOB_COMPLETION_INDEX)", env) == "rank=3"
    assert expand("$(A)$(A)-$(MISSING)", env) == "11-$(MISSING)"
    assert expand("$$(A)", env) == "$(A)"


def test_last_json_line():
    assert last_json_line('noise\n{"ok": true}\nmore noise\n') == {"ok": True}
    assert last_json_line('{"a": 1}\n{"b": 2}\n') == {"b": 2}
    assert last_json_line("{broken\n") is None


def _runtime(tmp_path):
    events = []
    cond = threading.Condition()

    def on_status(pp, phase, extra):
        with cond:
            events.append((pp.key, phase, extra))
            cond.notify_all()

    def wait_for(pred, timeout=10):
        with cond:
            assert cond.wait_for(lambda: pred(events), timeout), events

    return PodRuntime(tmp_path / "pods", on_status), events, wait_for


def _pod(tmp_path, name, argv, policy):
    return PodProc(key=f"default/{name}", uid=name, dir=tmp_path / "pods" / name, argv=argv,
                   env=dict(os.environ), restart_policy=policy)


def test_pod_succeeds_with_result(tmp_path):
    rt, events, wait_for = _runtime(tmp_path)
    rt.start(_pod(tmp_path, "ok", [sys.executable, "-c", "print('hi'); print('{\"ok\": true, \"v\": 7}')"], "Never"))
    wait_for(lambda ev: any(p == "Succeeded" for _, p, _ in ev))
    final = [e for e in events if e[1] == "Succeeded"][0][2]
    assert final["exitCode"] == 0 and final["result"] == {"ok": True, "v": 7}
    assert (tmp_path / "pods" / "ok" / "log").read_text().startswith("hi")


def test_pod_onfailure_restarts_until_success(tmp_path):
    rt, events, wait_for = _runtime(tmp_path)
    cnt = tmp_path / "n"
    code = f"import pathlib,sys; p=pathlib.Path({str(cnt)!r}); n=int(p.read_text()) if p.exists() else 0; p.write_text(str(n+1)); sys.exit(0 if n>=2 else 1)"
    rt.start(_pod(tmp_path, "flaky", [sys.executable, "-c", code], "OnFailure"))
    wait_for(lambda ev: any(p == "Succeeded" for _, p, _ in ev))
    assert cnt.read_text() == "3"
    assert any(e[2].get("restarts") == 2 for e in events)


def test_pod_never_reports_failure_with_log_tail(tmp_path):
    rt, events, wait_for = _runtime(tmp_path)
    rt.start(_pod(tmp_path, "bad", ["sh", "-c", "echo boom >&2; exit 5"], "Never"))
    wait_for(lambda ev: any(p == "Failed" for _, p, _ in ev))
    extra = [e for e in events if e[1] == "Failed"][0][2]
    assert extra["exitCode"] == 5 and "boom" in extra["message"]


def test_pod_start_error_and_stop(tmp_path):
    rt, events, wait_for = _runtime(tmp_path)
    rt.start(_pod(tmp_path, "nope", ["/nonexistent/binary"], "Never"))
    wait_for(lambda ev: any(p == "Failed" and x.get("reason") == "StartError" for _, p, x in ev))
    pp = _pod(tmp_path, "sleeper", ["sleep", "600"], "Always")
    rt.start(pp)
    wait_for(lambda ev: any(k == "default/sleeper" and p == "Running" for k, p, _ in ev))
    t = time.monotonic()
    assert rt.stop("default/sleeper", grace=2.0) is pp
    assert pp.done.wait(5) and time.monotonic() - t < 5
    assert "default/sleeper" not in rt.running()


# ---- keys / fs / events / faults ----------------------------------------------------------------
def test_cluster_key_and_fingerprint_scan(tmp_path):
    priv, pub, fp = keys.ensure_cluster_key(tmp_path / "k")
    assert oct(priv.stat().st_mode & 0o777) == "0o600" and len(fp.split(":")) == 16
    assert keys.ensure_cluster_key(tmp_path / "k")[2] == fp  # stable
    assert keys.find_key(fp, [tmp_path / "nowhere", tmp_path / "k"]) == str(priv)
    assert keys.find_key("MD5:" + fp.upper(), [tmp_path / "k"]) == str(priv)
    assert keys.find_key("00:11", [tmp_path / "k"]) is None
    assert pub.read_text() != priv.read_text()  # machines get the public half, never the private key


def test_atomic_write_and_locked_append(tmp_path):
    atomic_write(tmp_path / "a" / "f", "x", mode=0o640)
    assert (tmp_path / "a" / "f").read_text() == "x" and oct((tmp_path / "a" / "f").stat().st_mode & 0o777) == "0o640"
    atomic_write_json(tmp_path / "j.json", {"k": [1, 2]})
    assert read_json(tmp_path / "j.json") == {"k": [1, 2]}
    assert read_json(tmp_path / "missing.json", 5) == 5
    (tmp_path / "bad.json").write_text("{")
    with pytest.raises(ValueError):  # corrupt state is loud, never silently "empty"
        read_json(tmp_path / "bad.json", "d")

    def writer(i):
        for j in range(50):
            locked_append_line(tmp_path / "ips", f"{i}-{j}")

    ts = [threading.Thread(target=writer, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    lines = (tmp_path / "ips").read_text().splitlines()
    assert len(lines) == 200 and len(set(lines)) == 200  # no torn / interleaved lines
    with file_lock(tmp_path / "l"):
        pass


def test_event_log_phases(tmp_path):
    ev = EventLog(tmp_path / "e.jsonl")
    with ev.phase("provision", n=2):
        ev.emit("machine_created", name="kubenode1")
    with pytest.raises(RuntimeError):
        with ev.phase("ansible"):
            raise RuntimeError("x")
    recs = read_events(tmp_path / "e.jsonl")
    assert [r["event"] for r in recs] == ["phase_start", "machine_created", "phase_end", "phase_start", "phase_end"]
    assert recs[2]["ok"] is True and recs[4]["ok"] is False
    assert set(ev.phases) == {"provision", "ansible"}


def test_fault_spec_parsing(monkeypatch):
    monkeypatch.setenv("TK8S_FAULTS", "provision.create@kubenode2,agent.crash@kubenode1:3,cp.delay:0.5")
    assert faults.fault("provision.create", "kubenode2") is True
    assert faults.fault("provision.create", "kubenode1") is None
    assert faults.fault("agent.crash", "kubenode1") == "3"
    assert faults.fault("cp.delay") == "0.5"
    with pytest.raises(faults.InjectedFault):
        faults.maybe_fail("provision.create", "kubenode2")
    monkeypatch.delenv("TK8S_FAULTS")
    assert faults.fault("provision.create", "kubenode2") is None


# ---- triton provider against a fake CLI ------------------------------------------------------------
FAKE_TRITON = r'''#!/usr/bin/env python3
import json, os, sys
a = sys.argv[1:]
with open(os.environ["FAKE_TRITON_LOG"], "a") as f:
    f.write(" ".join(a) + "\n")
if a[0] == "env":
    print('export SDC_URL="https://us-east-1.api.joyent.com"')
    print('export SDC_ACCOUNT="me"')
    print('export SDC_KEY_ID="%s"' % os.environ["FAKE_KEY_ID"])
elif a[0] == "networks":
    print("NAME                ID")
    print("Joyent-SDC-Public   1111-aaaa")
    print("Joyent-SDC-Private  2222-bbbb")
elif a[0] == "packages":
    print("NAME                  ID")
    print("k4-highcpu-kvm-7.75G  3333")
    print("g4-highcpu-1G         4444")
    print("k4-highcpu-kvm-1.75G  5555")
elif a[:2] == ["instance", "create"]:
    name = [x for x in a if x.startswith("--name=")][0].split("=", 1)[1]
    print(json.dumps({"id": "id-" + name, "name": name, "primaryIp": "10.0.0.9", "ips": ["10.0.0.9"]}))
elif a[:2] == ["instance", "delete"]:
    pass
else:
    sys.exit(2)
'''


def test_triton_provider_with_fake_cli(tmp_path, monkeypatch):
    from tritonk8ssupervisor_amd.provider.triton import TritonProvider

    bindir = tmp_path / "bin"
    bindir.mkdir()
    (bindir / "triton").write_text(FAKE_TRITON)
    (bindir / "triton").chmod(0o755)
    home = tmp_path / "home"
    (home / ".ssh").mkdir(parents=True)
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-f", str(home / ".ssh" / "id_ed25519")], check=True)
    md5 = subprocess.run(["ssh-keygen", "-E", "md5", "-lf", str(home / ".ssh" / "id_ed25519")], capture_output=True,
                         text=True, check=True).stdout.split()[1].removeprefix("MD5:")
    monkeypatch.setenv("PATH", f"{bindir}{os.pathsep}{os.environ['PATH']}")
    monkeypatch.setenv("HOME", str(home))
    monkeypatch.setenv("FAKE_TRITON_LOG", str(tmp_path / "calls"))
    monkeypatch.setenv("FAKE_KEY_ID", md5)
    # the VMs are configured over ssh with the discovered key (fake ssh: tests/fakessh.py)
    (tmp_path / "hosts" / "10.0.0.9" / ".ssh").mkdir(parents=True)
    (tmp_path / "hosts" / "10.0.0.9" / ".ssh" / "authorized_keys").write_text((home / ".ssh" / "id_ed25519.pub").read_text())
    monkeypatch.setenv("TK8S_SSH", f"{sys.executable} {Path(__file__).parent / 'fakessh.py'}")
    monkeypatch.setenv("FAKESSH_ROOT", str(tmp_path / "hosts"))
    monkeypatch.setenv("SDC_KEY", str(home / ".ssh" / "id_ed25519"))
    p = TritonProvider(tmp_path / "state")
    env = p.env()
    assert env == {"SDC_URL": "https://us-east-1.api.joyent.com", "SDC_ACCOUNT": "me", "SDC_KEY_ID": md5}
    # setup.sh:215-230: the private key whose MD5 fingerprint is SDC_KEY_ID
    assert p.find_key(md5) == str(home / ".ssh" / "id_ed25519")
    nets = p.networks()
    assert [n.name for n in nets] == ["Joyent-SDC-Private", "Joyent-SDC-Public"]  # sorted (setup.sh:257)
    assert next(i for i, n in enumerate(nets, 1) if n.name == p.default_network) == 2
    pk = p.packages()
    assert [x.name for x in pk] == ["k4-highcpu-kvm-1.75G", "k4-highcpu-kvm-7.75G"]  # -kvm- only (setup.sh:259)
    m = p.create_machine("kubenode1", "3333", ["1111-aaaa"], tags={"role": "host"})
    assert m.primaryip == "10.0.0.9" and m.id == "id-kubenode1"
    # node runtime installed on the VM, work dir made there; exec runs in it with the machine env
    assert Path(m.home, "tritonk8ssupervisor_amd", "executor.py").exists()
    assert m.sandbox == str(tmp_path / "hosts" / "10.0.0.9" / "tk8s" / "machine")
    rc, out = p.exec(m, "pwd; echo $TK8S_MACHINE")
    assert rc == 0 and out.split() == [m.sandbox, "kubenode1"]
    calls = [json.loads(x) for x in (tmp_path / "hosts" / "calls.jsonl").read_text().splitlines()]
    assert all(c["key"] == str(home / ".ssh" / "id_ed25519") and c["user"] == "root" for c in calls)
    assert all(c["opts"]["StrictHostKeyChecking"] == "accept-new" and c["opts"]["UserKnownHostsFile"] for c in calls)
    p.delete_machine(m)
    calls = (tmp_path / "calls").read_text().splitlines()
    assert any(c.startswith("instance create --wait --json --name=kubenode1 -N 1111-aaaa -t role=host") for c in calls)
    assert "instance delete --wait id-kubenode1" in calls


def test_triton_provider_without_cli_is_a_clear_error(tmp_path, monkeypatch):
    from tritonk8ssupervisor_amd.provider.base import ProvisionError
    from tritonk8ssupervisor_amd.provider.triton import TritonProvider

    monkeypatch.setenv("PATH", str(tmp_path))
    with pytest.raises(ProvisionError, match="CLI not found"):
        TritonProvider(tmp_path).networks()


def test_pmc_counter_pass_limits():
    """--rocprof-counters: one --pmc pass holds at most 8 SQ_, 4 TCC_ (FETCH_SIZE = 3), 2 GRBM_
    ... counters; asking for more makes rocprofv3 hang, so setup refuses before launching."""
    from tritonk8ssupervisor_amd.orchestrator import SetupError, check_pmc_counters

    check_pmc_counters(["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "GRBM_GUI_ACTIVE", "FETCH_SIZE",
                        "TCC_HIT_sum", "TCC_HIT_avr"])
    for bad in ([f"SQ_C{i}" for i in range(9)], ["FETCH_SIZE", "WRITE_SIZE"], ["GRBM_A", "GRBM_B", "GRBM_C"], ["XYZ_A"]):
        with pytest.raises(SetupError):
            check_pmc_counters(bad)


def test_pod_in_its_own_pid_namespace(tmp_path, monkeypatch):
    """P4: with unprivileged user namespaces, a CPU pod runs as init of its own PID namespace with
    its own /proc (it cannot see or signal the node's processes)."""
    from tritonk8ssupervisor_amd.agent import runtime

    monkeypatch.setattr(runtime, "_ISOLATION", None)
    avail, how = runtime.namespace_isolation("", str(tmp_path))
    if not avail:
        pytest.skip(f"no unprivileged namespaces here: {how}")
    rt, events, wait_for = _runtime(tmp_path)
    pp = _pod(tmp_path, "iso", ["sh", "-c", "echo pid=$$; ls /proc | grep -c '^[0-9]'"], "Never")
    pp.isolate = True
    rt.start(pp)
    wait_for(lambda ev: any(p == "Succeeded" for _, p, _ in ev))
    out = (tmp_path / "pods" / "iso" / "log").read_text().split()
    assert out[0] in ("pid=1", "pid=2") and int(out[1]) <= 4  # only the pod's own processes are visible


def test_local_provider_skips_addresses_something_already_serves_on():
    """A loopback address with a TCP listener or a bound UDP socket on it (a cluster this host's
    registry does not know about, e.g. one an interrupted run leaked) is never handed out."""
    import socket

    from tritonk8ssupervisor_amd.provider.local import LocalProvider

    u = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    t = socket.socket()
    c = socket.socket()
    try:
        u.bind(("127.0.9.77", 0))
        t.bind(("127.0.9.78", 0))
        t.listen(1)
        c.bind(("127.0.9.79", 0))  # bound but not listening: not serving
        seen = LocalProvider._bound_ips()
        assert {"127.0.9.77", "127.0.9.78"} <= seen and "127.0.9.79" not in seen
    finally:
        for s in (u, t, c):
            s.close()


def test_kill_pidfile_never_signals_a_stranger(tmp_path):
    """a pidfile whose process is gone (or whose pid now belongs to another process)
    is removed without signalling anything; the recorded start time is the identity."""
    import subprocess
    import sys

    from tritonk8ssupervisor_amd.utils.procs import kill_pidfile, proc_start_ticks, spawn_daemon

    pf = tmp_path / "d.pid"
    p = spawn_daemon([sys.executable, "-c", "import time; time.sleep(30)"], pidfile=str(pf))
    info = json.loads(pf.read_text())
    assert info["start"] == proc_start_ticks(p.pid)
    # the same pid with another start time: a reused pid -- left alone, the pidfile removed
    pf.write_text(json.dumps(dict(info, start=info["start"] - 1)))
    assert kill_pidfile(pf, grace=0.5) is False and not pf.exists() and p.poll() is None
    # a legacy pidfile (no start time) naming a process that is not tk8s's: left alone too
    stranger = subprocess.Popen(["sleep", "30"], start_new_session=True)
    pf.write_text(json.dumps({"pid": stranger.pid, "pgid": stranger.pid}))
    assert kill_pidfile(pf, grace=0.5) is False and stranger.poll() is None
    stranger.kill()
    stranger.wait()
    # the real owner is stopped
    pf.write_text(json.dumps(info))
    assert kill_pidfile(pf, grace=2.0) is True
    p.wait(5)


def test_fabric_visibility_needs_a_real_owner_job():
    """the agent checks a pod's Job ownerReference against the Job the control plane
    has (same uid), so a client-written ownerReference does not unlock node / host GPU views."""
    from tritonk8ssupervisor_amd.agent.agent import node_visibility_allowed

    pod = {"metadata": {"namespace": "kube-system", "ownerReferences": [{"kind": "Job", "name": "j", "uid": "u1"}]}}
    assert node_visibility_allowed(pod, lambda ns, name: "u1" if (ns, name) == ("kube-system", "j") else None)
    assert not node_visibility_allowed(pod, lambda ns, name: None)       # no such Job
    assert not node_visibility_allowed(pod, lambda ns, name: "u2")       # another Job of that name
    other_ns = {"metadata": {**pod["metadata"], "namespace": "default"}}
    assert not node_visibility_allowed(other_ns, lambda ns, name: "u1")


def test_init_containers_then_all_app_containers(tmp_path):
    """Init containers run in order to a zero exit before the app containers; every app container
    runs (each with its own log); the pod ends Succeeded once all of them exit 0, Failed if one
    does not; an init container that fails under restartPolicy Never fails the pod."""
    from tritonk8ssupervisor_amd.agent.runtime import PodProc, PodRuntime

    events = []
    rt = PodRuntime(tmp_path / "pods", lambda pp, phase, extra: events.append((phase, extra.get("reason"))))
    d = tmp_path / "pods" / "p"

    def proc(name, script, log="log"):
        return PodProc(key="default/p" if log == "log" else f"default/p/{name}", uid="u", dir=d, argv=["sh", "-c", script],
                       env={"PATH": "/usr/bin:/bin"}, restart_policy="Never", name=name, log_name=log)

    main = proc("main", "cat order.txt; echo main >> order.txt")
    main.init = [proc("i1", "echo i1 > order.txt", "log.i1"), proc("i2", "echo i2 >> order.txt", "log.i2")]
    main.sidecars = [proc("side", "sleep 0.3; echo side-done", "log.side")]
    rt.start(main)
    assert main.done.wait(20)
    assert events[-1] == ("Succeeded", None), events
    assert (d / "log").read_text() == "i1\ni2\n" and (d / "log.side").read_text() == "side-done\n"
    assert ("Pending", "PodInitializing") in events

    events.clear()
    d2 = tmp_path / "pods" / "q"
    bad = PodProc(key="default/q", uid="u", dir=d2, argv=["true"], env={"PATH": "/usr/bin:/bin"}, restart_policy="Never",
                  name="main")
    bad.sidecars = [PodProc(key="default/q/s", uid="u", dir=d2, argv=["sh", "-c", "exit 3"], env={"PATH": "/usr/bin:/bin"},
                            restart_policy="Never", name="s", log_name="log.s")]
    rt.start(bad)
    assert bad.done.wait(20) and events[-1][0] == "Failed"

    events.clear()
    d3 = tmp_path / "pods" / "r"
    never = PodProc(key="default/r", uid="u", dir=d3, argv=["true"], env={"PATH": "/usr/bin:/bin"}, restart_policy="Never",
                    name="main")
    never.init = [PodProc(key="default/r/i", uid="u", dir=d3, argv=["false"], env={"PATH": "/usr/bin:/bin"},
                          restart_policy="Never", name="i", log_name="log.i")]
    rt.start(never)
    assert never.done.wait(20) and events[-1] == ("Failed", "Init:Error")


def test_probe_handlers_and_prober(tmp_path):
    """httpGet / tcpSocket / exec handlers; readiness flips ready after its thresholds; a failing
    liveness probe kills the process."""
    import http.server
    import socketserver
    import threading as th
    import time as tm

    from tritonk8ssupervisor_amd.agent.probes import Prober, run_probe

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            self.send_response(200 if self.path == "/ok" else 503)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = socketserver.TCPServer(("127.0.0.1", 0), H)
    th.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    c = {"ports": [{"name": "web", "containerPort": port}]}
    try:
        assert run_probe({"httpGet": {"path": "/ok", "port": "web"}}, c, "127.0.0.1")[0]
        ok, msg = run_probe({"httpGet": {"path": "/bad", "port": port}}, c, "127.0.0.1")
        assert not ok and "503" in msg
        assert run_probe({"tcpSocket": {"port": port}}, c, "127.0.0.1")[0]
    finally:
        srv.shutdown()
        srv.server_close()
    assert not run_probe({"tcpSocket": {"port": port}}, c, "127.0.0.1")[0]
    assert run_probe({"exec": {"command": ["true"]}}, c, "127.0.0.1")[0]
    assert not run_probe({"exec": {"command": ["false"]}}, c, "127.0.0.1")[0]

    marker = tmp_path / "ready"
    changes, killed = [], []
    spec = {"readinessProbe": {"exec": {"command": ["test", "-f", str(marker)]}, "periodSeconds": 0.05,
                               "failureThreshold": 1},
            "livenessProbe": {"exec": {"command": ["test", "!", "-f", str(tmp_path / "dead")]}, "periodSeconds": 0.05,
                              "failureThreshold": 2}}
    alive = [True]
    p = Prober(spec, "127.0.0.1", lambda: alive[0], lambda: (killed.append(1), alive.__setitem__(0, False)),
               lambda: changes.append(1))
    assert not p.ready
    p.start()
    tm.sleep(0.2)
    assert not p.ready
    marker.touch()
    deadline = tm.monotonic() + 5
    while not p.ready and tm.monotonic() < deadline:
        tm.sleep(0.02)
    assert p.ready and changes
    (tmp_path / "dead").touch()
    deadline = tm.monotonic() + 5
    while not killed and tm.monotonic() < deadline:
        tm.sleep(0.02)
    assert killed and "livenessProbe failed 2 times" in p.last_message


def test_prestop_hook_sigterm_then_sigkill_after_the_grace_period(tmp_path):
    """Deleting a pod: preStop runs first, the container gets SIGTERM (a trainer's checkpoint
    window), and what ignores it is SIGKILLed when terminationGracePeriodSeconds runs out; the
    pod's GPUs stay held meanwhile."""
    rt, events, wait_for = _runtime(tmp_path)
    marks = tmp_path / "marks"
    code = ("import signal,time,pathlib\n"
            f"p=pathlib.Path({str(marks)!r})\n"
            "def term(*_):\n    p.open('a').write('term\\n')\n"
            "signal.signal(signal.SIGTERM, term)\n"
            "p.open('a').write('up\\n')\n"
            "while True: time.sleep(0.05)\n")
    pp = _pod(tmp_path, "trainer", [sys.executable, "-c", code], "Always")
    pp.grace, pp.gpu_ids = 1.5, ["gpu0"]
    pp.container = {"lifecycle": {"preStop": {"exec": {"command": ["sh", "-c", f"echo prestop >> {marks}"]}}}}
    rt.start(pp)
    wait_for(lambda ev: marks.exists() and "up" in marks.read_text())
    done = threading.Event()
    t = time.monotonic()
    rt.stop("default/trainer", wait=False, on_done=done.set)
    assert rt.is_terminating("default/trainer") and rt.held_gpus() == {"gpu0"}
    assert done.wait(10)
    took = time.monotonic() - t
    assert 1.4 < took < 6, took  # SIGTERM ignored: killed at the end of the grace period
    assert marks.read_text().split() == ["up", "prestop", "term"]
    assert not rt.is_terminating("default/trainer") and rt.held_gpus() == set()


def test_poststart_hook_failure_restarts_the_container(tmp_path):
    rt, events, wait_for = _runtime(tmp_path)
    n = tmp_path / "starts"
    pp = _pod(tmp_path, "hooked", ["sh", "-c", f"echo x >> {n}; sleep 30"], "Always")
    flag = tmp_path / "ok"
    pp.container = {"lifecycle": {"postStart": {"exec": {"command": ["sh", "-c", f"test -e {flag}"]}}}}
    rt.start(pp)
    wait_for(lambda ev: n.exists() and len(n.read_text().split()) >= 2)  # killed by the failing hook, restarted
    flag.write_text("")
    assert "FailedPostStartHook" in (tmp_path / "pods" / "hooked" / "log").read_text()
    rt.stop("default/hooked", grace=1.0)


def test_tty_pod_on_a_node_without_ptys_runs_with_its_stdin_pipe(tmp_path, monkeypatch):
    """`tty: true` where no pseudo-terminal can be had (the MI355X GPU boxes mount no devpts): the
    container runs as with `tty: false` -- its stdin a pipe when `stdin: true` -- and its log says
    why, instead of the pod failing to start."""
    import pty

    from tritonk8ssupervisor_amd.agent.runtime import PodProc, PodRuntime, close_stdin

    def no_pty():
        raise OSError("out of pty devices")

    monkeypatch.setattr(pty, "openpty", no_pty)
    rt = PodRuntime(tmp_path, on_status=lambda *a: None)
    pp = PodProc(key="default/t", uid="u1", dir=tmp_path / "pods" / "t", argv=["sh", "-c", "read x; echo got-$x"],
                 env={"PATH": "/usr/bin:/bin"}, restart_policy="Never", container={"tty": True, "stdin": True})
    p = rt._spawn(pp)
    assert pp.tty_master == -1 and pp.stdin_w >= 0
    os.write(pp.stdin_w, b"hi\n")
    close_stdin(pp)
    assert p.wait(10) == 0
    log = (pp.dir / "log").read_text()
    assert "no pseudo-terminal on this node" in log and "got-hi" in log, log
