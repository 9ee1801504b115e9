"""Container images on an offline node (agent/images.py + native/tools/tk8s_container.cpp):
``./tk8s image load`` of a docker-save archive, the layers applied with their whiteouts, and a pod
naming the image running in its root file system with the image's entrypoint, env and working
directory -- the reference's Docker workloads (ansible/roles/rancherhost/tasks/main.yml:26-34),
without a registry. The test image is built here from this host's /bin/sh and its libraries."""
import json
import os
import shutil
import subprocess
import sys
import time
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd.agent.images import ImageStore, normalize, write_docker_archive

REPO = Path(__file__).resolve().parents[1]


def test_reference_normalisation():
    assert normalize("nginx") == "docker.io/library/nginx:latest"
    assert normalize("nginx:1.27") == "docker.io/library/nginx:1.27"
    assert normalize("rocm/k8s-device-plugin:1.31.0.6") == "docker.io/rocm/k8s-device-plugin:1.31.0.6"
    assert normalize("registry.local:5000/team/app") == "registry.local:5000/team/app:latest"
    assert normalize("localhost/x:2") == "localhost/x:2"
    assert normalize("busybox@sha256:abc") == "docker.io/library/busybox@sha256:abc"


def _host_files(*binaries: str) -> dict[str, bytes]:
    """The binaries and every library they load, at their own paths (a minimal root file system)."""
    files: dict[str, bytes] = {}
    for b in binaries:
        real = shutil.which(b)
        files[f"bin/{Path(b).name}"] = Path(real).read_bytes()
        out = subprocess.run(["ldd", real], capture_output=True, text=True).stdout
        for tok in out.split():
            if tok.startswith("/") and Path(tok).exists():
                files[tok.lstrip("/")] = Path(tok).resolve().read_bytes()
    return files


def _hello_archive(path: Path) -> str:
    base = _host_files("sh", "cat", "sleep", "uname")
    base.update({"etc/hello-release": b"tk8s hello 1\n", "etc/removed": b"gone in layer 1\n", "app/": b""})
    top = {"etc/.wh.removed": b"", "app/run.sh": (
        b"#!/bin/sh\necho greeting=$GREETING\necho cwd=$(pwd)\necho pid=$$\ncat /etc/hello-release\n"
        b"cat /etc/removed 2>/dev/null || echo removed=yes\necho args=$*\necho iso=$TK8S_GPU_ISOLATION\n"
        b"echo container=$TK8S_CONTAINER\necho written > /app/out.txt\n")}
    write_docker_archive(path, "hello:1", [base, top], {
        "Entrypoint": ["/bin/sh", "/app/run.sh"], "Cmd": ["default-arg"], "Env": ["GREETING=hi", "PATH=/bin"],
        "WorkingDir": "/app"})
    return "docker.io/library/hello:1"


def test_load_apply_whiteouts_and_kubernetes_command_rules(tmp_path):
    store = ImageStore(tmp_path / "store")
    ref = _hello_archive(tmp_path / "hello.tar")
    assert store.load(tmp_path / "hello.tar") == [ref]
    assert [i["ref"] for i in store.list()] == [ref] and store.get("hello:1") is not None
    root = store.rootfs("hello:1")
    assert (root / "etc" / "hello-release").read_text() == "tk8s hello 1\n"
    assert not (root / "etc" / "removed").exists() and (root / "app" / "run.sh").exists()
    assert store.rootfs("hello:1") == root  # built once
    # Kubernetes: command replaces ENTRYPOINT (and drops CMD), args replace CMD
    assert store.container_argv(ref, None, None) == (["/bin/sh", "/app/run.sh", "default-arg"],
                                                     {"GREETING": "hi", "PATH": "/bin"}, "/app")
    assert store.container_argv(ref, None, ["x"])[0] == ["/bin/sh", "/app/run.sh", "x"]
    assert store.container_argv(ref, ["/bin/cat"], ["/etc/hello-release"])[0] == ["/bin/cat", "/etc/hello-release"]
    assert store.remove("hello:1") and store.get(ref) is None


def test_layers_cannot_escape_the_root(tmp_path):
    import io
    import tarfile

    from tritonk8ssupervisor_amd.agent.images import apply_layer

    layer = tmp_path / "evil.tar"
    with tarfile.open(layer, "w") as t:
        for name, data in (("../escape.txt", b"x"), ("ok.txt", b"y")):
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            t.addfile(ti, io.BytesIO(data))
        ti = tarfile.TarInfo("link")
        ti.type, ti.linkname = tarfile.SYMTYPE, "/"
        t.addfile(ti)
        ti = tarfile.TarInfo("link/etc-escape")
        ti.size = 1
        t.addfile(ti, io.BytesIO(b"z"))
    root = tmp_path / "root"
    root.mkdir()
    apply_layer(layer, root)
    assert (root / "ok.txt").read_bytes() == b"y"
    assert not (tmp_path / "escape.txt").exists() and not Path("/etc-escape").exists()


@pytest.fixture
def ws(tmp_path):
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, tmp_path / f)
    yield tmp_path
    subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=_env(tmp_path), capture_output=True, timeout=120)


def _env(ws: Path) -> dict:
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_FAKE_GPUS="2",
               TK8S_IMAGE_STORE=str(ws / "images"))
    env.pop("TK8S_FAULTS", None)
    return env


def _probe_mode(mode: str) -> str:
    """What tk8s-container runs image pods with under --mode ``mode``: root/userns (namespaces),
    ptrace, or "" (skip: neither is available here)."""
    from tritonk8ssupervisor_amd.agent.runtime import CONTAINER

    if not CONTAINER.exists():
        return ""
    r = subprocess.run([str(CONTAINER), "--mode", mode, "--probe"], capture_output=True, text=True, timeout=20)
    info = json.loads(r.stdout or "{}")
    return info.get("how", "") if info.get("usable") else ""


@pytest.mark.parametrize("mode", ["auto", "ptrace"])
def test_a_pod_runs_in_its_image(ws, native_build, mode):
    """./tk8s image load, then a pod naming the image (no command): it runs the image's entrypoint
    in the image's root file system, with the image's env and working dir, writes into its own
    layer (the image stays pristine), and is GPU-jailed; describe pod says so. With namespaces it
    is pid 1 of its own PID namespace over an overlay; in ptrace mode (the GPU tier: no user
    namespaces -- native/tools/ptrace_root.h) its root is the pod's own tree of links to the image,
    by path translation, with the image's own loader."""
    how = _probe_mode(mode)
    if not how:
        pytest.skip(f"no container runtime for --mode {mode} here")
    env = _env(ws)
    if mode != "auto":
        env["TK8S_CONTAINER_MODE"] = mode
    ref = _hello_archive(ws / "hello.tar")
    r = subprocess.run(["./tk8s", "image", "load", "hello.tar"], cwd=ws, env=env, capture_output=True, text=True)
    assert r.returncode == 0 and f"Loaded image: {ref}" in r.stdout, r.stderr
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"], cwd=ws,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    (ws / "pod.json").write_text(json.dumps({
        "apiVersion": "v1", "kind": "Pod", "metadata": {"name": "hello"},
        "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "hello:1", "args": ["from-k8s"],
                                                           "env": [{"name": "GREETING", "value": "hello"}]}]}}))
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=60)
    assert kc("apply", "-f", "pod.json").returncode == 0
    deadline = time.monotonic() + 60
    phase = None
    while time.monotonic() < deadline:
        phase = json.loads(kc("get", "pod", "hello", "-o", "json").stdout)["status"].get("phase")
        if phase in ("Succeeded", "Failed"):
            break
        time.sleep(0.2)
    log = kc("logs", "hello").stdout
    assert phase == "Succeeded", (phase, log, kc("describe", "pod", "hello").stdout)
    lines = dict(x.split("=", 1) for x in log.split() if "=" in x)
    assert lines["greeting"] == "hello" and lines["cwd"] == "/app", log
    assert "tk8s hello 1" in log and lines["removed"] == "yes" and lines["args"] == "from-k8s", log
    assert lines["iso"].startswith("landlock:abi"), log
    # the write went to the pod's own layer, never into the shared image
    store = ImageStore(ws / "images")
    assert not (store.rootfs(ref) / "app" / "out.txt").exists()
    d = kc("describe", "pod", "hello").stdout
    assert "image hello:1" in d, d
    if how == "ptrace":
        assert lines["container"].startswith("ptrace:") and "rootfs:farm" in lines["container"], log
        assert "container: ptrace (path translation" in d and "own PID namespace" not in d, d
    else:
        assert lines["pid"] == "1" and "rootfs:overlay" in lines["container"], log
        assert "container: namespaces (root)" in d or "container: namespaces (userns)" in d, d
        assert "own PID namespace" in d, d


@pytest.mark.parametrize("mode", ["auto", "ptrace"])
def test_kubectl_exec_enters_the_container(ws, native_build, mode):
    """kubectl exec into an image pod runs inside its container (its root, its PID namespace --
    with namespaces --, the same GPU jail), not on the host."""
    how = _probe_mode(mode)
    if not how:
        pytest.skip(f"no container runtime for --mode {mode} here")
    env = _env(ws)
    if mode != "auto":
        env["TK8S_CONTAINER_MODE"] = mode
    _hello_archive(ws / "hello.tar")
    assert subprocess.run(["./tk8s", "image", "load", "hello.tar"], cwd=ws, env=env, capture_output=True).returncode == 0
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"], cwd=ws,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    (ws / "pod.json").write_text(json.dumps({
        "apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sleeper"},
        "spec": {"containers": [{"name": "c", "image": "hello:1", "command": ["/bin/sleep", "60"]}]}}))
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=60)
    assert kc("apply", "-f", "pod.json").returncode == 0
    deadline = time.monotonic() + 30
    while time.monotonic() < deadline:
        if json.loads(kc("get", "pod", "sleeper", "-o", "json").stdout)["status"].get("phase") == "Running":
            break
        time.sleep(0.2)
    time.sleep(0.5)  # the container's pid 1 has started
    r = kc("exec", "sleeper", "--", "/bin/sh", "-c", "cat /etc/hello-release; echo pid=$$; echo iso=$TK8S_GPU_ISOLATION")
    assert r.returncode == 0, r.stdout + r.stderr
    out = dict(x.split("=", 1) for x in r.stdout.split() if "=" in x)
    assert "tk8s hello 1" in r.stdout and out["iso"].startswith("landlock"), r.stdout
    assert how == "ptrace" or int(out["pid"]) < 100, r.stdout  # its own PID namespace
    assert kc("exec", "sleeper", "--", "/bin/cat", "/etc/removed").returncode != 0  # the image's view, not the host's


@pytest.mark.parametrize("mode", ["auto", "ptrace"])
def test_attach_to_an_image_pods_terminal(ws, native_build, mode):
    """`kubectl attach -it` to an image pod started with `stdin: true, tty: true`: its shell, in
    the image's root, reads the keystrokes from the pty the agent holds and answers on it -- through
    tk8s-container in either mode -- and its exit code ends the session."""
    from urllib.parse import urlsplit

    from tritonk8ssupervisor_amd.controlplane.wsclient import WSClient

    how = _probe_mode(mode)
    if not how:
        pytest.skip(f"no container runtime for --mode {mode} here")
    try:
        import pty

        for fd in pty.openpty():
            os.close(fd)
    except OSError as e:  # the GPU boxes mount no devpts: tty pods run without one (runtime._spawn_tty)
        pytest.skip(f"no pseudo-terminals on this host: {e}")
    env = _env(ws)
    if mode != "auto":
        env["TK8S_CONTAINER_MODE"] = mode
    _hello_archive(ws / "hello.tar")
    assert subprocess.run(["./tk8s", "image", "load", "hello.tar"], cwd=ws, env=env, capture_output=True).returncode == 0
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"], cwd=ws,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    (ws / "pod.json").write_text(json.dumps({
        "apiVersion": "v1", "kind": "Pod", "metadata": {"name": "term"},
        "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "image": "hello:1", "command": ["/bin/sh"],
                                                           "stdin": True, "tty": True}]}}))
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=60)
    assert kc("apply", "-f", "pod.json").returncode == 0
    deadline, phase = time.monotonic() + 30, None
    while time.monotonic() < deadline and phase != "Running":
        phase = json.loads(kc("get", "pod", "term", "-o", "json").stdout)["status"].get("phase")
        if phase in ("Succeeded", "Failed"):
            break
        time.sleep(0.2)
    assert phase == "Running", (phase, kc("logs", "term").stdout, kc("describe", "pod", "term").stdout)
    cfg = json.loads((ws / ".tk8s" / "kubeconfig.json").read_text())
    server = urlsplit(cfg["clusters"][0]["cluster"]["server"])
    w = WSClient.connect(server.hostname, server.port, f"{server.path}/api/v1/namespaces/default/pods/term/attach",
                         query=[("stdin", "true"), ("stdout", "true"), ("tty", "true")],
                         token=cfg["users"][0]["user"]["token"], protocols=("v5.channel.k8s.io",), timeout=30)
    w.send(b"\x00" + b"cat /etc/hello-release; [ -t 0 ] && echo tty=yes; cat /etc/removed || echo img=yes; exit 7\n")
    out, status, deadline = b"", None, time.monotonic() + 30
    while time.monotonic() < deadline and status is None:
        m = w.recv()
        if m is None:
            break
        if m[:1] == b"\x01":
            out += m[1:]
        elif m[:1] == b"\x03":
            status = json.loads(m[1:])
    w.close()
    text = out.decode(errors="replace")
    assert "tk8s hello 1" in text and "tty=yes" in text and "img=yes" in text, (text, kc("logs", "term").stdout,
                                                                                 kc("describe", "pod", "term").stdout)
    assert status and status["details"]["causes"][0]["message"] == "7", (status, text)


@pytest.mark.parametrize("mode", ["auto", "ptrace"])
def test_image_pod_volumes(ws, native_build, mode):
    """An image pod mounts its volumes where the spec says: a ConfigMap (read-only), a Secret, an
    emptyDir, a PersistentVolumeClaim (data kept for the next pod), the downward API; and gets
    its own hostname (UTS namespace; in ptrace mode uname's answer and the hostname files)."""
    if not _probe_mode(mode):
        pytest.skip(f"no container runtime for --mode {mode} here")
    env = _env(ws)
    if mode != "auto":
        env["TK8S_CONTAINER_MODE"] = mode
    _hello_archive(ws / "hello.tar")
    assert subprocess.run(["./tk8s", "image", "load", "hello.tar"], cwd=ws, env=env, capture_output=True).returncode == 0
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"], cwd=ws,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=60)
    script = ("cat /etc/app/app.conf; cat /etc/pw/password; echo; cat /info/name; echo; "
              "echo hostname=$(cat /proc/sys/kernel/hostname); echo uname=$(uname -n); cat /data/count 2>/dev/null || echo count=none; "
              "echo count=again > /data/count; echo x > /scratch/f && echo scratch=ok; "
              "echo y > /etc/app/new 2>/dev/null || echo cfg=readonly")

    def pod(name):
        return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                "spec": {"restartPolicy": "Never", "hostname": "box",
                         "containers": [{"name": "c", "image": "hello:1", "command": ["/bin/sh", "-c", script],
                                         "volumeMounts": [{"name": "cfg", "mountPath": "/etc/app"},
                                                          {"name": "pw", "mountPath": "/etc/pw"},
                                                          {"name": "info", "mountPath": "/info"},
                                                          {"name": "data", "mountPath": "/data"},
                                                          {"name": "scratch", "mountPath": "/scratch"}]}],
                         "volumes": [{"name": "cfg", "configMap": {"name": "cfg"}},
                                     {"name": "pw", "secret": {"secretName": "pw"}},
                                     {"name": "info", "downwardAPI": {"items": [
                                         {"path": "name", "fieldRef": {"fieldPath": "metadata.name"}}]}},
                                     {"name": "data", "persistentVolumeClaim": {"claimName": "data"}},
                                     {"name": "scratch", "emptyDir": {}}]}}

    (ws / "objs.json").write_text(json.dumps({"apiVersion": "v1", "kind": "List", "items": [
        {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cfg"}, "data": {"app.conf": "greeting=hi"}},
        {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "pw"}, "stringData": {"password": "s3cr3t"}},
        {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": "data"},
         "spec": {"resources": {"requests": {"storage": "1Gi"}}}},
        pod("first")]}))
    assert kc("apply", "-f", "objs.json").returncode == 0

    def wait(name):
        deadline = time.monotonic() + 60
        while time.monotonic() < deadline:
            phase = json.loads(kc("get", "pod", name, "-o", "json").stdout)["status"].get("phase")
            if phase in ("Succeeded", "Failed"):
                return phase
            time.sleep(0.2)
        return None

    assert wait("first") == "Succeeded", kc("describe", "pod", "first").stdout
    log = kc("logs", "first").stdout
    assert "greeting=hi" in log and "s3cr3t" in log and "first" in log and "hostname=box" in log, log
    assert "uname=box" in log, log
    assert "count=none" in log and "scratch=ok" in log and "cfg=readonly" in log, log
    (ws / "second.json").write_text(json.dumps(pod("second")))
    assert kc("apply", "-f", "second.json").returncode == 0
    assert wait("second") == "Succeeded"
    assert "count=again" in kc("logs", "second").stdout  # the claim kept the first pod's data
    assert "data" in kc("get", "pvc").stdout


def test_hardlink_to_a_symlinked_host_file_is_refused(tmp_path):
    """a layer's hard link must name a file of the image. ``s -> <host file>`` then a
    hard link ``h`` to ``s`` must not link the host file into the root (os.link follows links)."""
    import io
    import tarfile

    from tritonk8ssupervisor_amd.agent.images import apply_layer

    secret = tmp_path / "host-secret"
    secret.write_text("host only\n")
    layer = tmp_path / "evil.tar"
    with tarfile.open(layer, "w") as t:
        ti = tarfile.TarInfo("s")
        ti.type, ti.linkname = tarfile.SYMTYPE, str(secret)
        t.addfile(ti)
        ti = tarfile.TarInfo("h")
        ti.type, ti.linkname = tarfile.LNKTYPE, "s"
        t.addfile(ti)
        ti = tarfile.TarInfo("f")
        ti.size = 2
        t.addfile(ti, io.BytesIO(b"ok"))
        ti = tarfile.TarInfo("g")  # a hard link to a file of the image still works
        ti.type, ti.linkname = tarfile.LNKTYPE, "f"
        t.addfile(ti)
    root = tmp_path / "root"
    root.mkdir()
    apply_layer(layer, root)
    assert not (root / "h").exists() and os.stat(secret).st_nlink == 1
    assert (root / "g").read_bytes() == b"ok" and os.stat(root / "f").st_nlink == 2


@pytest.mark.parametrize("mode", ["auto", "ptrace"])
def test_mount_points_resolve_inside_the_image(ws, native_build, mode):
    """Debian/Ubuntu images ship /var/run -> /run. A volume (and the ServiceAccount
    token every image pod gets at /var/run/secrets/kubernetes.io/serviceaccount) mounted under it
    lands in the image's /run, resolved inside the image -- never on the host's /run."""
    how = _probe_mode(mode)
    if not how:
        pytest.skip(f"no container runtime for --mode {mode} here")
    env = _env(ws)
    if mode != "auto":
        env["TK8S_CONTAINER_MODE"] = mode
    base = _host_files("sh", "cat", "sleep", "ls")
    base.update({"var/": b"", "var/run": ("symlink", "/run"), "etc/os-release": b"debian-like\n"})
    write_docker_archive(ws / "deb.tar", "deb:1", [base], {"Env": ["PATH=/bin"], "WorkingDir": "/"})
    assert subprocess.run(["./tk8s", "image", "load", "deb.tar"], cwd=ws, env=env, capture_output=True).returncode == 0
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"], cwd=ws,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=60)
    host_before = os.path.exists("/run/tk8s-test-data")
    (ws / "pod.json").write_text(json.dumps({
        "apiVersion": "v1", "kind": "Pod", "metadata": {"name": "deb"},
        "spec": {"restartPolicy": "Never", "containers": [{
            "name": "c", "image": "deb:1", "command": ["/bin/sh", "-c",
                "echo tok=$(cat /var/run/secrets/kubernetes.io/serviceaccount/token); "
                "echo x > /var/run/tk8s-test-data/f && echo data=$(cat /run/tk8s-test-data/f); "
                "while read k v; do [ \"$k\" = CapBnd: ] && echo capbnd=$v; done < /proc/self/status; "
                "(echo 1 > /proc/sys/kernel/sysrq) 2>/dev/null && echo sysctl=written || echo sysctl=refused; "
                "(echo x > /sys/kernel/uevent_helper) 2>/dev/null && echo sysfs=written || echo sysfs=refused"],
            "volumeMounts": [{"name": "d", "mountPath": "/var/run/tk8s-test-data"}]}],
            "volumes": [{"name": "d", "emptyDir": {}}]}}))
    assert kc("apply", "-f", "pod.json").returncode == 0
    deadline = time.monotonic() + 60
    while True:
        o = json.loads(kc("get", "pod", "deb", "-o", "json").stdout)
        if o["status"].get("phase") in ("Succeeded", "Failed"):
            break
        assert time.monotonic() < deadline
        time.sleep(0.2)
    out = kc("logs", "deb").stdout
    assert o["status"]["phase"] == "Succeeded", (out, o["status"])
    assert "tok=tk8sb." in out and "data=x" in out, out  # the pod-bound token
    # the capability bounding set of a root pod is Docker's default set; host sysctl/sysfs stay read-only
    assert "sysctl=refused" in out and "sysfs=refused" in out, out
    if os.geteuid() == 0:
        assert "capbnd=00000000a80425fb" in out, out
    assert os.path.exists("/run/tk8s-test-data") == host_before  # nothing appeared on the host


@pytest.mark.gpu
def test_gpu_image_pod_runs_hip_in_its_image(tmp_path, native_build):
    """A GPU pod from an image: the image holds tk8s-gpuinfo, libtk8s and the C/C++ runtime; the
    node's ROCm comes in as a read-only hostPath volume (as a GPU container gets it). On the
    MI355X box (no namespaces) it runs in ptrace mode: HIP's device discovery -- /dev/kfd, its
    render node, the KFD topology in /sys, all through the path translation; the GPU ioctls
    themselves never stop -- finds the pod's one MI355X, and the jail keeps it to that one."""
    import shutil

    import torch

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    how = _probe_mode("auto")
    if not how:
        pytest.skip("no container runtime here")
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_IMAGE_STORE=str(tmp_path / "images"))
    gi = REPO / "tritonk8ssupervisor_amd" / "bin" / "tk8s-gpuinfo"
    files = {k: v for k, v in _host_files("sh", "cat").items()}
    files["opt/tk8s/bin/tk8s-gpuinfo"] = gi.read_bytes()
    files["opt/tk8s/lib/libtk8s.so"] = (REPO / "tritonk8ssupervisor_amd" / "lib" / "libtk8s.so").read_bytes()
    # the C/C++ runtime of the tool and of what HIP loads on its own (comgr: libzstd, libz, ...);
    # ROCm itself stays on the node
    rocm_lib = Path(os.path.realpath("/opt/rocm")) / "lib"
    for so in (gi, rocm_lib / "libamd_comgr.so.3", rocm_lib / "libhsa-runtime64.so.1", rocm_lib / "libamdhip64.so.7"):
        if not so.exists():
            continue
        for tok in subprocess.run(["ldd", str(so)], capture_output=True, text=True).stdout.split():
            if tok.startswith("/") and not tok.startswith("/opt/") and "tritonk8ssupervisor_amd" not in tok \
                    and Path(tok).exists():
                files[tok.lstrip("/")] = Path(tok).resolve().read_bytes()
    write_docker_archive(tmp_path / "gpu.tar", "gpuinfo:1", [files], {"Env": ["PATH=/bin"], "WorkingDir": "/"})
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True, text=True,
                                   timeout=60)
    try:
        assert subprocess.run(["./tk8s", "image", "load", "gpu.tar"], cwd=tmp_path, env=env,
                              capture_output=True).returncode == 0
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "120",
                            "--rccl", "off"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        (tmp_path / "pod.json").write_text(json.dumps({
            "apiVersion": "v1", "kind": "Pod", "metadata": {"name": "gpuinfo"},
            "spec": {"restartPolicy": "Never", "containers": [{
                "name": "c", "image": "gpuinfo:1", "command": ["/opt/tk8s/bin/tk8s-gpuinfo", "--no-links"],
                "env": [{"name": "LD_LIBRARY_PATH", "value": "/opt/tk8s/lib:/opt/rocm/lib"}],
                "resources": {"limits": {"amd.com/gpu": 1}},
                "volumeMounts": [{"name": "rocm", "mountPath": "/opt/rocm", "readOnly": True}]}],
                "volumes": [{"name": "rocm", "hostPath": {"path": os.path.realpath("/opt/rocm")}}]}}))
        assert kc("apply", "-f", "pod.json").returncode == 0
        deadline = time.monotonic() + 120
        phase = None
        while time.monotonic() < deadline:
            phase = json.loads(kc("get", "pod", "gpuinfo", "-o", "json").stdout)["status"].get("phase")
            if phase in ("Succeeded", "Failed"):
                break
            time.sleep(0.3)
        log = kc("logs", "gpuinfo").stdout
        assert phase == "Succeeded", (phase, log[-2000:], kc("describe", "pod", "gpuinfo").stdout[-3000:])
        info = json.loads(log.strip().splitlines()[-1])
        assert info["ok"] and len(info["devices"]) == 1 and info["devices"][0]["gfx"] == "gfx950", info
        d = kc("describe", "pod", "gpuinfo").stdout
        assert "image gpuinfo:1" in d and ("container: ptrace" in d or "container: namespaces" in d), d
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)
