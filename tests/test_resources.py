"""Pod and machine resource limits are enforced (VERDICT r3 missing-1, agent/resources.py).

The reference's machines were hard slices (a Triton KVM package,
/root/reference/terraform/host/main.tf:3) and its workloads Docker containers with cgroup limits
(/root/reference/ansible/roles/rancherhost/tasks/main.yml:26-34). Here: a pod over its
limits.memory is OOMKilled (exit 137) and restarted under its policy -- by the kernel in a
cgroup (cgroup1 on this dev box, as root in a v1 container), or by the agent's memory watchdog
(the GPU tier's unprivileged mode) -- and a GPU pod runs on its GPU's NUMA-local CPUs."""
import json
import os
import shutil
import subprocess
import sys
import time
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd.agent.resources import Enforcer, Limits, format_cpulist, parse_cpulist, pod_limits

REPO = Path(__file__).resolve().parents[1]

HOG = ("import time\nblocks = []\nfor _ in range(40):\n    blocks.append(bytearray(16 << 20))\n"
       "    for i in range(0, len(blocks[-1]), 4096):\n        blocks[-1][i] = 1\n    time.sleep(0.02)\n"
       "print('survived', flush=True)\n")


def test_limits_and_cpulists():
    pod = {"spec": {"containers": [{"resources": {"limits": {"memory": "64Mi", "cpu": "500m"}}},
                                   {"resources": {"limits": {"memory": "32Mi", "cpu": "1"}}}],
                    "initContainers": [{"resources": {"limits": {"memory": "512Mi"}}}]}}
    lim = pod_limits(pod)
    assert lim.memory == 512 << 20 and lim.cpu == 1.5  # the largest init container wins
    assert pod_limits({"spec": {"containers": [{}, {"resources": {"limits": {"memory": "1Gi"}}}]}}).memory is None
    assert parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"


def test_cgroup2_files_on_a_delegated_tree(tmp_path, monkeypatch):
    """The cgroup2 mode against a fake delegated subtree: the agent moves itself to a leaf,
    enables the controllers, writes the machine's package and each pod's limits, and reads an
    OOM kill from memory.events."""
    root = tmp_path / "cg"
    root.mkdir()
    for f, v in (("cgroup.controllers", "cpuset cpu io memory pids"), ("cgroup.subtree_control", ""),
                 ("cgroup.procs", f"{os.getpid()}\n")):
        (root / f).write_text(v)
    orig_mkdir = Path.mkdir

    def mkdir(self, *a, **kw):  # a cgroupfs directory comes with its interface files
        orig_mkdir(self, *a, **kw)
        if str(self).startswith(str(root)):
            for f in ("cgroup.procs", "cgroup.subtree_control", "memory.max", "memory.swap.max", "memory.oom.group",
                      "cpu.max", "cpuset.cpus", "cpuset.mems", "memory.events"):
                if not (self / f).exists():
                    (self / f).write_text("")

    monkeypatch.setattr(Path, "mkdir", mkdir)
    monkeypatch.setattr("tritonk8ssupervisor_amd.agent.resources._own_cgroups", lambda: {"": "/"})
    monkeypatch.setenv("TK8S_CGROUP_ROOT", str(root))
    monkeypatch.setenv("TK8S_POD_RESOURCES", "auto")
    e = Enforcer("kubenode1", Limits(memory=8 << 30, cpu=16, cpus="0-63"))
    assert e.mode == "cgroup2", e.why
    assert (root / "tk8s-agent" / "cgroup.procs").read_text().strip() == str(os.getpid())
    assert set((root / "cgroup.subtree_control").read_text().split()) == {"+memory", "+cpu", "+cpuset"}
    m = root / "tk8s-machine-kubenode1"  # (no scope given: the bare node name)
    assert (m / "agent" / "cgroup.procs").read_text().strip() == str(os.getpid())  # the agent lives in its machine
    assert (m / "memory.max").read_text().strip() == str(8 << 30) and (m / "cpu.max").read_text().strip() == "1600000 100000"
    assert (m / "cpuset.cpus").read_text().strip() == "0-63"
    opts = e.pod("default/web", Limits(memory=64 << 20, cpu=0.5, cpus="0-31"))
    d = m / "pod-default_web"
    assert opts == ["--cgroup-procs", str(d / "cgroup.procs")]  # the cpuset controller fences: no affinity
    assert (d / "memory.max").read_text().strip() == str(64 << 20) and (d / "cpu.max").read_text().strip() == "50000 100000"
    assert (d / "cpuset.cpus").read_text().strip() == "0-31" and (d / "memory.oom.group").read_text().strip() == "1"
    assert not e.oom_killed("default/web")
    (d / "memory.events").write_text("low 0\nhigh 0\nmax 3\noom 1\noom_kill 1\n")
    assert e.oom_killed("default/web")
    host = e.pod("kube-system/fabric", Limits(), in_machine=False)  # beside the machine slice
    assert host == ["--cgroup-procs", str(root / "pod-kube-system_fabric" / "cgroup.procs")]
    assert "cgroup2" in e.describe() and "memory 8192 MiB" in e.describe()


@pytest.fixture
def fake_sysfs(tmp_path):
    """GPUs 0-3 on CPUs 0-3, GPUs 4-7 on CPUs 4-7 (two sockets, as an MI355X node has)."""
    root = tmp_path / "sys"
    for i in range(8):
        d = root / "class" / "drm" / f"renderD{128 + i}" / "device"
        d.mkdir(parents=True)
        (d / "local_cpulist").write_text("0-3\n" if i < 4 else "4-7\n")
        (d / "numa_node").write_text("0\n" if i < 4 else "1\n")
    return root


def _cluster(tmp_path, env_extra):
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = tmp_path / "ws"
    ws.mkdir()
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_FAKE_GPUS="8", **env_extra)
    env.pop("TK8S_FAULTS", None)
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "2", "--rccl", "off"], cwd=ws,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]

    def kc(*a, check=True, stdin=None):
        p = subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=120, input=stdin)
        if check:
            assert p.returncode == 0, f"kubectl {' '.join(a)}: {p.stdout}{p.stderr}"
        return p

    return ws, env, kc


def _apply(kc, pod):
    kc("apply", "-f", "-", stdin=json.dumps({"apiVersion": "v1", "kind": "Pod", **pod}))


def _until(fn, timeout=60.0):
    deadline = time.monotonic() + timeout
    while True:
        v = fn()
        if v:
            return v
        assert time.monotonic() < deadline, "condition not met in time"
        time.sleep(0.1)


def _pod(kc, name):
    return json.loads(kc("get", "pod", name, "-o", "json").stdout)


@pytest.mark.parametrize("mode", ["auto", "watchdog"])
def test_a_pod_over_its_memory_limit_is_oomkilled_and_restarted(tmp_path, fake_sysfs, mode):
    ws, env, kc = _cluster(tmp_path, {"TK8S_POD_RESOURCES": mode, "TK8S_SYSFS_ROOT": str(fake_sysfs)})
    try:
        node = json.loads(kc("get", "node", "kubenode1", "-o", "json").stdout)
        enf = node["metadata"]["annotations"]["tk8s.amd.com/resource-enforcement"]
        if mode == "watchdog":
            assert enf.startswith("watchdog") and "duty cycle" in enf and "NOT enforced" not in enf, enf
        # the machine is its package's slice: capacity from the package (mi355x-1gpu = 1/8 host)
        assert float(node["status"]["capacity"]["cpu"]) == max(1, (os.cpu_count() or 8) // 8)
        (ws / "hog.py").write_text(HOG)
        _apply(kc, {"metadata": {"name": "hog"}, "spec": {"restartPolicy": "OnFailure", "containers": [{
            "name": "c", "command": [sys.executable, str(ws / "hog.py")],
            "resources": {"limits": {"memory": "64Mi"}}}]}})
        _apply(kc, {"metadata": {"name": "small"}, "spec": {"restartPolicy": "Never", "containers": [{
            "name": "c", "command": [sys.executable, "-c", "print('fits', flush=True)"],
            "resources": {"limits": {"memory": "256Mi"}}}]}})

        def restarted_oom():
            cs = (_pod(kc, "hog").get("status") or {}).get("containerStatuses") or [{}]
            last = (cs[0].get("lastState") or {}).get("terminated") or (cs[0].get("state") or {}).get("terminated") or {}
            return cs[0] if last.get("reason") == "OOMKilled" and cs[0].get("restartCount", 0) >= 1 else None

        c = _until(restarted_oom, 90)
        term = (c.get("lastState") or {}).get("terminated") or c["state"]["terminated"]
        assert term["exitCode"] == 137
        assert "survived" not in kc("logs", "hog").stdout
        d = kc("describe", "pod", "hog").stdout
        assert "Reason: OOMKilled, Exit Code: 137" in d and "memory 64 MiB" in d, d
        _until(lambda: _pod(kc, "small")["status"].get("phase") == "Succeeded")
        assert "fits" in kc("logs", "small").stdout
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, timeout=120)


@pytest.mark.parametrize("mode", ["auto", "watchdog"])
def test_a_gpu_pod_runs_on_its_gpus_numa_local_cpus(tmp_path, fake_sysfs, mode):
    if (os.cpu_count() or 0) < 8:
        pytest.skip("needs 8 CPUs for the two fake NUMA nodes")
    ws, env, kc = _cluster(tmp_path, {"TK8S_POD_RESOURCES": mode, "TK8S_SYSFS_ROOT": str(fake_sysfs)})
    try:
        for name in ("g1", "g2"):
            _apply(kc, {"metadata": {"name": name}, "spec": {"restartPolicy": "Never", "containers": [{
                "name": "c", "command": ["sh", "-c", "grep Cpus_allowed_list /proc/self/status"],
                "resources": {"limits": {"amd.com/gpu": 1}}}]}})
        for name in ("g1", "g2"):
            _until(lambda n=name: _pod(kc, n)["status"].get("phase") in ("Succeeded", "Failed"))
        for name in ("g1", "g2"):
            p = _pod(kc, name)
            ordinal = int(p["metadata"]["annotations"]["amd.com/gpu-ids"].split(",")[0].replace("gpu", ""))
            want = "0-3" if ordinal < 4 else "4-7"
            out = kc("logs", name).stdout
            node = json.loads(kc("get", "node", p["spec"]["nodeName"], "-o", "json").stdout)
            assert out.split()[-1] == want, (name, ordinal, out, p["metadata"]["annotations"].get("tk8s.amd.com/resources"),
                                             p["metadata"]["annotations"].get("tk8s.amd.com/gpu-isolation"),
                                             node["metadata"]["annotations"].get("tk8s.amd.com/resource-enforcement"))
            assert f"cpus {want}" in p["metadata"]["annotations"]["tk8s.amd.com/resources"]
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, timeout=120)


def test_a_half_set_up_cgroup_mode_leaves_nothing_behind(tmp_path, monkeypatch):
    """A cgroup mode that fails part way (another cluster's sweep removed a directory under it,
    a controller refused a write) falls through to the watchdog with none of its state: the GPU
    pod is then pinned by affinity, not left unfenced on a cpuset that is not there."""
    root = tmp_path / "cg"
    own = {"memory": "/jobs", "cpu": "/jobs", "cpuset": "/jobs"}
    for c in own:
        d = root / c / "jobs"
        d.mkdir(parents=True)
        (root / c / "cgroup.procs").write_text("")
        (d / "cgroup.procs").write_text("")
        if c == "cpuset":
            (d / "cpuset.cpus").write_text("0-7\n")
            (d / "cpuset.mems").write_text("0-1\n")
    orig_mkdir = Path.mkdir

    def mkdir(self, *a, **kw):
        orig_mkdir(self, *a, **kw)
        if str(self).startswith(str(root)):
            for f in ("cgroup.procs", "cpuset.cpus", "cpuset.mems", "memory.limit_in_bytes"):
                if not (self / f).exists():
                    (self / f).write_text("")

    def refuse(self, d, ctrl, lim):
        if ctrl == "cpuset":
            raise FileNotFoundError(2, "No such file or directory", str(d / "cpuset.cpus"))

    monkeypatch.setattr(Path, "mkdir", mkdir)
    monkeypatch.setattr("tritonk8ssupervisor_amd.agent.resources._own_cgroups", lambda: own)
    monkeypatch.setattr(Enforcer, "_limit", refuse)
    monkeypatch.setenv("TK8S_CGROUP_ROOT", str(root))
    monkeypatch.setenv("TK8S_POD_RESOURCES", "auto")
    e = Enforcer("kubenode1", Limits(cpus="0-3"))
    assert e.mode == "watchdog" and e.base == {}, (e.mode, e.base, e.why)
    assert "cgroup1" in e.why  # (its directories: rmdir'ed on a cgroupfs; here they hold plain files)
    assert e.pod("default/g", Limits(cpus="0-3")) == ["--cpus", "0-3"]


def test_the_sweep_spares_a_machine_cgroup_being_set_up(tmp_path, monkeypatch):
    from tritonk8ssupervisor_amd.agent import resources

    for n in ("new", "old"):
        (tmp_path / f"tk8s-machine-{n}").mkdir()
    monkeypatch.setattr(resources, "SWEEP_MIN_AGE_S", 60.0)
    resources._sweep(tmp_path)  # both just made: another agent may be about to move in
    assert sorted(p.name for p in tmp_path.iterdir()) == ["tk8s-machine-new", "tk8s-machine-old"]
    monkeypatch.setattr(resources, "SWEEP_MIN_AGE_S", -1.0)
    resources._sweep(tmp_path)  # old enough and empty: an agent that died without cleaning up
    assert list(tmp_path.iterdir()) == []


def test_usage_follows_children_that_leave_the_process_group(monkeypatch):
    """A container's processes are its session, its process group and their descendants: a child
    that moved to a new process group (job control) or a new session (setsid) still counts -- for
    kubectl top / the HPA, and for the memory watchdog's sum and kill."""
    from tritonk8ssupervisor_amd.agent.usage import _proc_table, members

    script = ("import os, time, sys\n"
              "if os.fork() == 0:\n    os.setsid()\n    time.sleep(30)\n    sys.exit(0)\n"
              "if os.fork() == 0:\n    os.setpgid(0, 0)\n    time.sleep(30)\n    sys.exit(0)\n"
              "print('forked', flush=True)\ntime.sleep(30)\n")
    p = subprocess.Popen([sys.executable, "-c", script], start_new_session=True, stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "forked"
        deadline = time.monotonic() + 10
        while True:
            table = _proc_table()
            kids = [q for q, v in table.items() if v[3] == p.pid]
            if len(kids) == 2 or time.monotonic() > deadline:
                break
            time.sleep(0.05)
        assert len(kids) == 2 and {table[k][0] for k in kids} != {p.pid}  # they left the group
        assert members(table, p.pid) == {p.pid, *kids}
        from tritonk8ssupervisor_amd.agent.resources import Enforcer

        monkeypatch.setenv("TK8S_POD_RESOURCES", "none")  # (no cgroup of the test's own)
        e = Enforcer("n", scope="t")
        e.kill_oom("default/p", [p.pid], sorted(members(table, p.pid)))
        assert p.wait(10) == -9
        for k in kids:
            deadline = time.monotonic() + 10
            while os.path.exists(f"/proc/{k}") and open(f"/proc/{k}/stat").read().split(") ")[1][0] != "Z":
                assert time.monotonic() < deadline, f"child {k} survived the kill"
                time.sleep(0.05)
    finally:
        if p.poll() is None:
            p.kill()


def test_numa_cpus_outside_the_agents_own_are_not_pinned(tmp_path, monkeypatch):
    """A GPU's NUMA-local CPUs that the agent may not use (a cpuset keeping it off that socket)
    are dropped: the pod runs unpinned instead of failing sched_setaffinity."""
    from tritonk8ssupervisor_amd.agent import resources

    d = tmp_path / "class" / "drm" / "renderD128" / "device"
    d.mkdir(parents=True)
    (d / "local_cpulist").write_text("0-3,8-11\n")
    monkeypatch.setenv("TK8S_SYSFS_ROOT", str(tmp_path))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: {2, 3, 4, 5})
    assert resources.gpu_local_cpus([128]) == "2-3"
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: {4, 5})
    assert resources.gpu_local_cpus([128]) == ""


BUSY = ("import os, time\nt = time.time()\nwhile time.time() - t < {secs}:\n    pass\n"
        "u = os.times()\nprint('cpu', round(u.user + u.system, 3), flush=True)\n")


def _cpu_of(pid: int) -> float:
    with open(f"/proc/{pid}/stat") as f:
        rest = f.read().rsplit(")", 1)[1].split()
    return (int(rest[11]) + int(rest[12])) / os.sysconf("SC_CLK_TCK")


def test_the_cpu_duty_cycle_holds_a_busy_loop_to_its_limit(monkeypatch):
    """VERDICT r4 next-3, unprivileged: a busy loop under a 250m limit gets <= 0.35 CPU over 5 s
    from the watchdog's SIGSTOP/SIGCONT duty cycle alone (no cgroup), and runs free once released."""
    import threading

    monkeypatch.setenv("TK8S_POD_RESOURCES", "watchdog")
    e = Enforcer("n", Limits(), scope="duty")
    assert e.mode == "watchdog" and "duty cycle" in e.describe() and "NOT enforced" not in e.describe()
    p = subprocess.Popen([sys.executable, "-c", BUSY.format(secs=30)], start_new_session=True)
    stop = threading.Event()
    try:
        e.pod("default/busy", Limits(cpu=0.25))
        th = threading.Thread(target=e.watch, args=(lambda: {"default/busy": [p.pid]}, stop), daemon=True)
        th.start()
        time.sleep(0.6)  # (the first /proc scan finds the pod)
        c0, t0 = _cpu_of(p.pid), time.monotonic()
        time.sleep(5.0)
        used = (_cpu_of(p.pid) - c0) / (time.monotonic() - t0)
        assert used <= 0.35, used
        assert used >= 0.1, used  # throttled, not starved
        assert e.throttle.stops > 10
        e.release("default/busy")  # released: it runs again at once
        time.sleep(0.2)
        c1 = _cpu_of(p.pid)
        time.sleep(1.0)
        assert _cpu_of(p.pid) - c1 > 0.5
    finally:
        stop.set()
        p.kill()
        p.wait(10)


def test_the_machine_memory_budget_oomkills_the_newest_pod(monkeypatch):
    """pods each within their own limits but together over the machine's
    package memory -- the newest one is OOMKilled, the older one keeps running."""
    import threading

    monkeypatch.setenv("TK8S_POD_RESOURCES", "watchdog")
    e = Enforcer("n", Limits(memory=160 << 20), scope="machine-mem")
    hold = ("import time\nb = bytearray({mb} << 20)\nfor i in range(0, len(b), 4096):\n    b[i] = 1\n"
            "print('holding', flush=True)\ntime.sleep(60)\n")
    old = subprocess.Popen([sys.executable, "-c", hold.format(mb=100)], start_new_session=True, stdout=subprocess.PIPE,
                           text=True)
    assert old.stdout.readline().strip() == "holding"
    e.pod("default/old", Limits(memory=512 << 20))
    new = subprocess.Popen([sys.executable, "-c", hold.format(mb=100)], start_new_session=True, stdout=subprocess.PIPE,
                           text=True)
    assert new.stdout.readline().strip() == "holding"
    e.pod("default/new", Limits(memory=512 << 20))
    stop = threading.Event()
    th = threading.Thread(target=e.watch, args=(lambda: {k: [q.pid] for k, q in (("default/old", old), ("default/new", new))
                                                         if q.poll() is None}, stop), daemon=True)
    th.start()
    try:
        assert new.wait(10) == -9
        assert e.oom_killed("default/new") and not e.oom_killed("default/old")
        time.sleep(1.0)
        assert old.poll() is None  # alone it fits the package
    finally:
        stop.set()
        for q in (old, new):
            if q.poll() is None:
                q.kill()
                q.wait(10)


def test_a_cpu_pod_gets_an_rlimit_data_backstop(monkeypatch):
    from tritonk8ssupervisor_amd.agent.resources import rlimit_data_for

    monkeypatch.setenv("TK8S_POD_RESOURCES", "watchdog")
    e = Enforcer("n", Limits(), scope="rlimit")
    assert e.pod("default/cpu", Limits(memory=64 << 20)) == ["--rlimit-data", str(rlimit_data_for(64 << 20))]
    assert e.pod("default/gpu", Limits(memory=64 << 20), gpu=True) == []  # the GPU runtime maps host memory
    assert e.pod("default/none", Limits()) == []


def test_oom_verdicts_count_only_kills_since_the_container_started(tmp_path, monkeypatch):
    """memory.events oom_kill is cumulative for the pod cgroup's life -- after one OOM
    kill, a later signal death of the restarted container is not reported OOMKilled again."""
    e = Enforcer.__new__(Enforcer)
    e.lock = __import__("threading").Lock()
    e.oom, e.oom_base = set(), {}
    d = tmp_path / "pod"
    d.mkdir()
    (d / "memory.events").write_text("oom 0\noom_kill 0\n")
    e.pods = {"default/p": {"": d}}
    e.reset_oom("default/p")
    assert not e.oom_killed("default/p")
    (d / "memory.events").write_text("oom 1\noom_kill 1\n")
    assert e.oom_killed("default/p")
    e.reset_oom("default/p")  # the container restarts
    assert not e.oom_killed("default/p")  # a liveness kill later is not an OOM
    (d / "memory.events").write_text("oom 2\noom_kill 2\n")
    assert e.oom_killed("default/p")


def test_cgroup2_moves_only_the_agent_itself(tmp_path, monkeypatch):
    """other processes in the agent's cgroup (other agents starting at the same
    moment) are not moved; with them there the mode is not taken, and the reason says so."""
    root = tmp_path / "cg"
    root.mkdir()
    for f, v in (("cgroup.controllers", "cpuset cpu io memory pids"), ("cgroup.subtree_control", ""),
                 ("cgroup.procs", f"{os.getpid()}\n4242\n")):
        (root / f).write_text(v)
    orig_mkdir = Path.mkdir

    def mkdir(self, *a, **kw):
        orig_mkdir(self, *a, **kw)
        if str(self).startswith(str(root)) and not (self / "cgroup.procs").exists():
            (self / "cgroup.procs").write_text("")

    monkeypatch.setattr(Path, "mkdir", mkdir)
    monkeypatch.setattr("tritonk8ssupervisor_amd.agent.resources._own_cgroups", lambda: {"": "/"})
    monkeypatch.setenv("TK8S_CGROUP_ROOT", str(root))
    monkeypatch.setenv("TK8S_POD_RESOURCES", "cgroup2")
    e = Enforcer("kubenode1", Limits(memory=1 << 30))
    assert e.mode == "none" and "4242" in e.why and "not this agent's" in e.why, e.why
    assert (root / "tk8s-agent" / "cgroup.procs").read_text().split() == [str(os.getpid())]  # 4242 never written


def test_a_watchdog_pod_over_its_cpu_limit_is_throttled_in_a_cluster(tmp_path, fake_sysfs):
    """The same through a bring-up: a pod with limits.cpu 250m spinning for 5 s of wall time gets
    <= 0.35 CPU (it reports its own CPU time), and describe node names the duty cycle."""
    ws, env, kc = _cluster(tmp_path, {"TK8S_POD_RESOURCES": "watchdog", "TK8S_SYSFS_ROOT": str(fake_sysfs)})
    try:
        node = json.loads(kc("get", "node", "kubenode1", "-o", "json").stdout)
        enf = node["metadata"]["annotations"]["tk8s.amd.com/resource-enforcement"]
        assert "duty cycle" in enf and "NOT enforced" not in enf, enf
        _apply(kc, {"metadata": {"name": "spin"}, "spec": {"restartPolicy": "Never", "containers": [{
            "name": "c", "command": [sys.executable, "-c", BUSY.format(secs=5)],
            "resources": {"limits": {"cpu": "250m"}}}]}})
        _until(lambda: _pod(kc, "spin")["status"].get("phase") in ("Succeeded", "Failed"), 60)
        out = kc("logs", "spin").stdout.split()
        used = float(out[out.index("cpu") + 1])
        assert used <= 0.35 * 5.0 + 0.2, out  # (+ the interpreter's start, before the first scan saw it)
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, timeout=120)


def test_signals_go_only_to_the_processes_the_scan_saw():
    """A pid (or process group id) reused since the watchdog's last /proc scan is never signalled:
    the recorded start time must still match."""
    import signal as _signal

    from tritonk8ssupervisor_amd.agent.resources import signal_ids
    from tritonk8ssupervisor_amd.utils.procs import proc_start_ticks

    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"], start_new_session=True)
    try:
        real = proc_start_ticks(p.pid)
        signal_ids([p.pid], [p.pid], _signal.SIGKILL, {p.pid: real + 1})  # "another process" with this pid
        time.sleep(0.2)
        assert p.poll() is None
        signal_ids([], [p.pid], _signal.SIGKILL, {})  # no record: left alone
        time.sleep(0.2)
        assert p.poll() is None
        signal_ids([p.pid], [], _signal.SIGKILL, {p.pid: real})
        assert p.wait(10) == -9
    finally:
        if p.poll() is None:
            p.kill()


def test_a_restarted_agent_ends_what_a_killed_one_left_behind(tmp_path):
    """runtime.reap_leftovers: an agent killed outright runs no stop_all, and its duty cycle may
    have left a pod SIGSTOPped; the next agent of the machine SIGCONTs and SIGKILLs each group
    its pidfile still names -- and leaves a pid that now belongs to another process alone."""
    import json
    import os
    import signal
    import subprocess
    import time

    from tritonk8ssupervisor_amd.agent.runtime import reap_leftovers
    from tritonk8ssupervisor_amd.utils.procs import proc_start_ticks

    pods = tmp_path / "pods"
    (pods / "a").mkdir(parents=True)
    (pods / "b").mkdir(parents=True)
    left = subprocess.Popen(["sleep", "60"], start_new_session=True)
    other = subprocess.Popen(["sleep", "60"], start_new_session=True)
    try:
        os.kill(left.pid, signal.SIGSTOP)
        (pods / "a" / "pod.pid").write_text(json.dumps({"pid": left.pid, "pgid": left.pid,
                                                        "start": proc_start_ticks(left.pid)}))
        (pods / "b" / "pod-side.pid").write_text(json.dumps({"pid": other.pid, "pgid": other.pid, "start": 1}))
        assert reap_leftovers(pods) == [left.pid]
        assert left.wait(timeout=10) == -signal.SIGKILL
        time.sleep(0.05)
        assert other.poll() is None  # start ticks differ: not the process the pidfile named
        assert not list(pods.glob("*/*.pid"))
        assert reap_leftovers(pods) == []
    finally:
        for p in (left, other):
            if p.poll() is None:
                p.kill()
                p.wait()


FORKER = ("import os, time\nt = time.time()\nwhile time.time() - t < {secs}:\n"
          "    pid = os.fork()\n    if pid == 0:\n        s = time.time()\n        while time.time() - s < 0.03:\n"
          "            pass\n        os._exit(0)\n    os.waitpid(pid, 0)\n")


def _cpu_with_children(pid: int) -> float:
    with open(f"/proc/{pid}/stat") as f:
        rest = f.read().rsplit(")", 1)[1].split()
    return sum(int(x) for x in rest[11:15]) / os.sysconf("SC_CLK_TCK")


def test_short_lived_children_cannot_escape_the_cpu_limit(monkeypatch):
    """a 250m pod that burns its CPU in a loop of short-lived children (30 ms each,
    gone before the next scan) is still held to its limit -- their CPU reaches the bill through the
    parent that reaps them (cutime/cstime)."""
    import threading

    monkeypatch.setenv("TK8S_POD_RESOURCES", "watchdog")
    e = Enforcer("n", Limits(), scope="forks")
    p = subprocess.Popen([sys.executable, "-c", FORKER.format(secs=30)], start_new_session=True)
    stop = threading.Event()
    try:
        e.pod("default/forks", Limits(cpu=0.25))
        th = threading.Thread(target=e.watch, args=(lambda: {"default/forks": [p.pid]}, stop), daemon=True)
        th.start()
        time.sleep(0.6)
        c0, t0 = _cpu_with_children(p.pid), time.monotonic()
        time.sleep(5.0)
        used = (_cpu_with_children(p.pid) - c0) / (time.monotonic() - t0)
        assert used <= 0.35, used
        assert e.throttle.stops > 5
    finally:
        stop.set()
        p.kill()
        p.wait(10)


def test_cgroup2_takes_the_agents_own_supervisor_along(tmp_path, monkeypatch):
    """the agent's restart supervisor (tk8s-supervise, its parent) shares its cgroup;
    it is moved into the leaf with the agent rather than counted as a stranger -- cgroup2 mode is
    taken, not dropped to the watchdog."""
    from tritonk8ssupervisor_amd.agent import resources

    root = tmp_path / "cg"
    root.mkdir()
    sup = 4343
    for f, v in (("cgroup.controllers", "cpuset cpu io memory pids"), ("cgroup.subtree_control", ""),
                 ("cgroup.procs", f"{os.getpid()}\n{sup}\n")):
        (root / f).write_text(v)
    orig_mkdir = Path.mkdir

    def mkdir(self, *a, **kw):
        orig_mkdir(self, *a, **kw)
        if str(self).startswith(str(root)) and not (self / "cgroup.procs").exists():
            (self / "cgroup.procs").write_text("")

    writes = []
    orig_write = resources._write

    def write(path, value):
        writes.append((Path(path).relative_to(root).as_posix(), str(value)))
        orig_write(path, value)

    monkeypatch.setattr(Path, "mkdir", mkdir)
    monkeypatch.setattr(resources, "_write", write)
    monkeypatch.setattr(resources, "_own_cgroups", lambda: {"": "/"})
    monkeypatch.setattr(resources, "_own_supervisor", lambda: sup)
    monkeypatch.setenv("TK8S_CGROUP_ROOT", str(root))
    monkeypatch.setenv("TK8S_POD_RESOURCES", "cgroup2")
    e = Enforcer("kubenode1", Limits(memory=1 << 30))
    assert e.mode == "cgroup2", e.why
    assert ("tk8s-agent/cgroup.procs", str(os.getpid())) in writes and ("tk8s-agent/cgroup.procs", str(sup)) in writes
    # a parent that is not tk8s-supervise is no excuse
    monkeypatch.setattr(resources, "_own_supervisor", lambda: None)
    (root / "cgroup.subtree_control").write_text("")
    e = Enforcer("kubenode2", Limits(memory=1 << 30))
    assert e.mode == "none" and str(sup) in e.why


def test_a_thread_heavy_cpu_pod_starts_under_a_small_limit():
    """RLIMIT_DATA counts virtual stacks and arenas, not the resident set: a 64Mi pod
    starting 40 threads (8 MiB stack each) must not fail at pthread_create under the backstop."""
    import resource

    from tritonk8ssupervisor_amd.agent.resources import rlimit_data_for

    lim = rlimit_data_for(64 << 20)
    assert lim >= 1 << 30
    code = ("import threading, time\nts = [threading.Thread(target=time.sleep, args=(0.2,)) for _ in range(40)]\n"
            "[t.start() for t in ts]\n[t.join() for t in ts]\nprint('ok')\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       preexec_fn=lambda: resource.setrlimit(resource.RLIMIT_DATA, (lim, lim)))
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-1000:]
