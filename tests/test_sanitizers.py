"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the xGMI
allocator, the JSON/args helpers (native/tests/host_selftest.cpp) and the restart supervisor
(tk8s-supervise), built with g++ -fsanitize=address,undefined and exercised on the CPU."""
import json
import os
import shutil
import signal
import subprocess
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
NATIVE = REPO / "native"
SAN = ["-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _build(tmp_path, name, sources):
    out = tmp_path / name
    r = subprocess.run(["g++", *SAN, f"-I{NATIVE / 'include'}", *map(str, sources), "-o", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def test_host_selftest_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "selftest", [NATIVE / "tests" / "host_selftest.cpp", NATIVE / "src" / "topology.cpp"])
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=ENV, timeout=120)
    assert r.returncode == 0 and "host selftest ok" in r.stdout, r.stdout + r.stderr


def test_supervisor_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "tk8s-supervise", [NATIVE / "tools" / "tk8s_supervise.cpp"])
    cnt = tmp_path / "n"
    r = subprocess.run([str(exe), "--pidfile", str(tmp_path / "a.pid"), "--restart", "on-failure", "--max-restarts", "3",
                        "--backoff-ms", "5", "--", "sh", "-c", f"echo x >> {cnt}; exit 4"],
                       capture_output=True, text=True, env=ENV, timeout=60)
    assert r.returncode == 4 and cnt.read_text().count("x") == 4, r.stderr[-2000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    pf = tmp_path / "b.pid"
    p = subprocess.Popen([str(exe), "--pidfile", str(pf), "--log", str(tmp_path / "b.log"), "--", "sleep", "600"],
                         env=ENV, start_new_session=True, stderr=subprocess.PIPE, text=True)
    deadline = time.monotonic() + 10
    while not pf.exists() and time.monotonic() < deadline:
        time.sleep(0.01)
    child = json.loads(pf.read_text())["child"]
    os.kill(child, signal.SIGKILL)
    while json.loads(pf.read_text() or "{}").get("child") == child and time.monotonic() < deadline:
        time.sleep(0.01)
    p.send_signal(signal.SIGTERM)
    assert p.wait(20) == 0 or p.returncode in (128 + signal.SIGTERM, -signal.SIGTERM, 143)
    err = p.stderr.read() + (tmp_path / "b.log").read_text()
    assert "AddressSanitizer" not in err and "runtime error" not in err, err[-2000:]


def _fake_dri(root: Path) -> Path:
    dri = root / "dri"
    (dri / "by-path").mkdir(parents=True)
    for n in ("renderD128", "renderD129", "card0"):
        (dri / n).write_text("")
    os.symlink("../renderD128", dri / "by-path" / "pci-0000:01:00.0-render")
    return dri


def test_gpujail_under_asan_ubsan(tmp_path):
    """the pod jail's policy code (gpujail.h) and tk8s-gpujail under
    ASan/UBSan: --probe, --plan, and a real jail run against a fake DRI tree with deny,
    read-only and allow layers, symlinks and missing paths."""
    exe = _build(tmp_path, "tk8s-gpujail", [NATIVE / "tools" / "tk8s_gpujail.cpp"])
    r = subprocess.run([str(exe), "--probe"], capture_output=True, text=True, env=ENV, timeout=60)
    assert "landlock_abi" in r.stdout and "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    usable = json.loads(r.stdout)["usable"]
    dri = _fake_dri(tmp_path)
    st = tmp_path / "ws" / ".tk8s"
    (st / "machines" / "n1" / "pods" / "mine").mkdir(parents=True)
    (st / "machines" / "n1" / "pods" / "other").mkdir(parents=True)
    (st / "kubeconfig.json").write_text("admin")
    (st / "machines" / "n1" / "pods" / "other" / "token").write_text("tok")
    (tmp_path / "ws" / "config").write_text("cfg")
    os.symlink(str(st), tmp_path / "ws" / "state-link")
    policy = ["--dri-root", str(dri), "--allow-render", "129", "--deny", str(tmp_path / "ws" / "state-link"),
              "--read-only", str(tmp_path / "ws"), "--allow", str(st / "machines" / "n1" / "pods" / "mine"),
              "--deny", str(tmp_path / "missing"), "--scope-signals"]
    r = subprocess.run([str(exe), *policy, "--plan"], capture_output=True, text=True, env=ENV, timeout=60)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-2000:]
    plan = {x["path"]: x["access"] for x in map(json.loads, r.stdout.splitlines())}
    assert plan[str(st / "machines" / "n1" / "pods" / "mine")] == "rw" and plan[str(tmp_path / "ws" / "config")] == "r"
    assert str(dri / "renderD129") in plan and str(dri / "renderD128") not in plan and str(st) not in plan
    if not usable:
        pytest.skip("Landlock unavailable: the policy code ran, the jail itself cannot")
    mine = st / "machines" / "n1" / "pods" / "mine"
    script = (f"cat {st / 'kubeconfig.json'} 2>/dev/null && echo LEAK; cat {mine.parent / 'other' / 'token'} 2>/dev/null "
              f"&& echo LEAK; cat {tmp_path / 'ws' / 'config'} > /dev/null && echo cfg-read; "
              f"(echo x > {tmp_path / 'ws' / 'config'}) 2>/dev/null && echo LEAK; echo ok > {mine / 'out'} && cat {mine / 'out'}; "
              f"cat {dri / 'renderD128'} 2>/dev/null && echo LEAK; cat {dri / 'renderD129'} && echo render-ok")
    r = subprocess.run([str(exe), *policy, "--", "sh", "-c", script], capture_output=True, text=True, env=ENV, timeout=60)
    assert r.returncode == 0 and "LEAK" not in r.stdout, r.stdout + r.stderr
    assert "cfg-read" in r.stdout and "ok" in r.stdout and "render-ok" in r.stdout, r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-2000:]


def test_container_under_asan_ubsan(tmp_path):
    """tk8s-container under ASan/UBSan: --probe always; as root (a mount namespace without a
    user namespace), a run in a minimal root file system whose /var/run is a symlink to /run,
    with a read-only bind mounted under it and the jail inside."""
    exe = _build(tmp_path, "tk8s-container", [NATIVE / "tools" / "tk8s_container.cpp"])
    r = subprocess.run([str(exe), "--probe"], capture_output=True, text=True, env=ENV, timeout=60)
    assert "usable" in r.stdout and "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    if not json.loads(r.stdout)["usable"] or os.geteuid() != 0:
        pytest.skip("no mount namespace for this user: the probe ran, the container cannot")
    rootfs = tmp_path / "rootfs"
    for d in ("bin", "lib", "lib64", "usr", "etc", "var"):
        (rootfs / d).mkdir(parents=True, exist_ok=True)
    for d in ("lib", "lib64", "usr"):  # the host's libraries and binaries, read-only
        if Path("/" + d).is_dir():
            os.rmdir(rootfs / d)
            os.symlink("/host/" + d, rootfs / d)  # resolved inside the image: /host/<d> in it
    os.symlink("/run", rootfs / "var" / "run")
    (rootfs / "etc" / "hello").write_text("from the image\n")
    shutil.copy2(shutil.which("sh"), rootfs / "bin" / "sh")
    shutil.copy2(shutil.which("cat"), rootfs / "bin" / "cat")
    data = tmp_path / "data"
    data.mkdir()
    (data / "f").write_text("bound\n")
    binds = []
    for d in ("lib", "lib64", "usr"):
        if Path("/" + d).is_dir():
            binds += ["--bind-ro", f"/{d}:/host/{d}"]
    r = subprocess.run([str(exe), "--rootfs", str(rootfs), "--upper", str(tmp_path / "upper"), "--pid-ns",
                        *binds, "--bind-ro", f"{data}:/var/run/data",
                        "--", "/bin/sh", "-c", "cat /etc/hello; cat /run/data/f; echo pid=$$"],
                       capture_output=True, text=True, timeout=60,
                       # LeakSanitizer cannot run in the relaying parent: pivot_root moved its root
                       # too, and the /proc there is the container's PID namespace's, where the
                       # relay has no /proc/self for LSan's thread walk. ASan and UBSan stay on.
                       env={**ENV, "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "from the image" in r.stdout and "bound" in r.stdout and "pid=1" in r.stdout, r.stdout
    assert not Path("/run/data").exists()  # resolved in the image, never on the host
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-2000:]


def test_container_ptrace_mode_under_asan_ubsan(tmp_path):
    """tk8s-container's ptrace mode (native/tools/ptrace_root.h) under ASan/UBSan: the supervisor
    -- path resolution in the pod's tree, copy-up, loader and #! expansion, string mappings per
    thread, fork/vfork tracking -- on a small image with a script that forks, writes an image
    file and resolves an absolute symlink."""
    exe = _build(tmp_path, "tk8s-container", [NATIVE / "tools" / "tk8s_container.cpp"])
    r = subprocess.run([str(exe), "--mode", "ptrace", "--probe"], capture_output=True, text=True, env=ENV, timeout=60)
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    if not json.loads(r.stdout)["usable"]:
        pytest.skip(f"no ptrace supervision here: {r.stdout}")
    from test_images import _host_files

    img = tmp_path / "img"
    for rel, data in {**_host_files("sh", "cat", "ls"), "etc/hello": b"from the image\n"}.items():
        p = img / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(data)
        p.chmod(0o755 if data[:4] == b"\x7fELF" else 0o644)
    (img / "abs").symlink_to("/etc")
    (img / "run.sh").write_text("#!/bin/sh\ncat /abs/hello\n(cat /etc/hello) | cat\necho more >> /etc/hello\n"
                                "cat /etc/hello\nls / > /dev/null\n")
    (img / "run.sh").chmod(0o755)
    r = subprocess.run([str(exe), "--mode", "ptrace", "--rootfs", str(img), "--upper", str(tmp_path / "up"),
                        "--workdir", "/", "--no-gpu-jail", "--", "/run.sh"],
                       capture_output=True, text=True, timeout=120, env={**ENV, "PATH": "/bin"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("from the image") == 3 and "more" in r.stdout, r.stdout
    assert (img / "etc" / "hello").read_text() == "from the image\n"  # copied up, never written
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-2000:]
