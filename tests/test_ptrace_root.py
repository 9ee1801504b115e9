"""tk8s-container's ptrace mode (native/tools/ptrace_root.h): an image's root file system by path
translation under a seccomp-filtered supervisor, for nodes where no mount namespace can be had
(the MI355X GPU tier). Each test runs the tool directly on a small image built from this host's
binaries: the image's symlinks resolve inside it, writes to image files copy up (the unpacked
image is never written), host paths handed back by the kernel are mapped to guest paths, and
the Landlock jail keeps the host's tree read-only. Reference: the workloads of
ansible/roles/rancherhost/tasks/main.yml:26-34 ran in Docker containers."""
import json
import os
import signal
import subprocess
import time
from pathlib import Path

import pytest

from test_images import _host_files

REPO = Path(__file__).resolve().parents[1]
TOOL = REPO / "tritonk8ssupervisor_amd" / "bin" / "tk8s-container"


@pytest.fixture(scope="module")
def usable(native_build):
    if not TOOL.exists():
        pytest.skip("tk8s-container is not built")
    r = subprocess.run([str(TOOL), "--mode", "ptrace", "--probe"], capture_output=True, text=True, timeout=20)
    info = json.loads(r.stdout or "{}")
    if not info.get("usable"):
        pytest.skip(f"no ptrace supervision here: {info.get('error')}")
    return True


@pytest.fixture
def image(tmp_path, usable):
    root = tmp_path / "img"
    files = _host_files("sh", "cat", "readlink", "uname", "sleep", "ls", "chmod")
    files.update({"etc/hello-release": b"tk8s hello 1\n", "app/": b""})
    for rel, data in files.items():
        p = root / rel
        if rel.endswith("/"):
            p.mkdir(parents=True, exist_ok=True)
            continue
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(data)
        p.chmod(0o755 if data[:4] == b"\x7fELF" else 0o644)
    (root / "abs").symlink_to("/etc")                    # an absolute link: the image's /etc
    (root / "app" / "up").symlink_to("../../../../etc")  # ".." past the root stops at it
    return root


def _run(image: Path, upper: Path, script: str, *extra: str, timeout: float = 60) -> subprocess.CompletedProcess:
    (image / "app" / "t.sh").write_text("#!/bin/sh\n" + script)
    (image / "app" / "t.sh").chmod(0o755)
    return subprocess.run([str(TOOL), "--mode", "ptrace", "--rootfs", str(image), "--upper", str(upper),
                           "--workdir", "/app", *extra, "--", "/app/t.sh"], capture_output=True, text=True,
                          timeout=timeout, env={"PATH": "/bin"})


def test_symlinks_resolve_inside_the_image(image, tmp_path):
    r = _run(image, tmp_path / "up", "cat /abs/hello-release\ncat /app/up/hello-release\n"
                                     "cd /app && cat ../../../../etc/hello-release\nls /\n", "--no-gpu-jail")
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("tk8s hello 1") == 3, r.stdout
    listing = r.stdout.split()
    assert "app" in listing and "abs" in listing and "dev" in listing and "proc" in listing, r.stdout
    assert (tmp_path / "up" / "farm.complete").exists() and "farm.complete" not in listing


def test_writes_copy_up_and_the_image_stays_pristine(image, tmp_path):
    src = image / "etc" / "hello-release"
    before = (src.read_bytes(), src.stat().st_mode, src.stat().st_ino)
    r = _run(image, tmp_path / "up", "echo more >> /etc/hello-release\ncat /etc/hello-release\n"
                                     "chmod 600 /abs/hello-release\necho new > /app/new.txt\n", "--no-gpu-jail")
    assert r.returncode == 0, r.stderr
    assert "tk8s hello 1\nmore" in r.stdout, r.stdout
    assert (src.read_bytes(), src.stat().st_mode, src.stat().st_ino) == before  # the image's inode untouched
    pod = tmp_path / "up" / "farm" / "etc" / "hello-release"
    assert pod.read_bytes() == b"tk8s hello 1\nmore\n" and pod.stat().st_ino != before[2]
    assert oct(pod.stat().st_mode & 0o777) == oct(0o600)
    assert (tmp_path / "up" / "farm" / "app" / "new.txt").read_text() == "new\n"
    assert not (image / "app" / "new.txt").exists()
    # a file the pod has not written is still the image's own inode (a hard link, no copy)
    assert (tmp_path / "up" / "farm" / "bin" / "cat").stat().st_ino == (image / "bin" / "cat").stat().st_ino


def test_host_paths_come_back_as_guest_paths(image, tmp_path):
    r = _run(image, tmp_path / "up", "pwd\nreadlink /proc/self/cwd\nreadlink /proc/$$/exe\ncd /abs && pwd -P\n"
                                     "uname -n\ncat /etc/hostname\n", "--no-gpu-jail", "--hostname", "podx")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split()
    # the shell was started through the image's own loader, yet its exe is the shell
    assert lines[:6] == ["/app", "/app", "/bin/sh", "/etc", "podx", "podx"], r.stdout


def test_the_jail_keeps_the_host_read_only(image, tmp_path):
    secret = tmp_path / "secret"
    secret.mkdir()
    (secret / "key").write_text("s3cret\n")
    r = _run(image, tmp_path / "up",
             f"cat /proc/self/root{secret}/key && echo READ-SECRET\n"
             f"echo x > /proc/self/root{tmp_path}/evil.txt && echo WROTE-HOST\n"
             "echo y > /tmp/ok.txt && cat /tmp/ok.txt\necho iso=$TK8S_GPU_ISOLATION\n",
             "--deny", str(secret))
    assert r.returncode == 0, r.stderr
    assert "READ-SECRET" not in r.stdout and "WROTE-HOST" not in r.stdout and not (tmp_path / "evil.txt").exists()
    assert "y" in r.stdout.split() and "iso=landlock:abi" in r.stdout, r.stdout + r.stderr


def test_exit_status_and_stop_continue(image, tmp_path):
    """The container's exit status is its main process's; SIGSTOP/SIGCONT (the agent's CPU duty
    cycle) stop and resume a traced pod (PTRACE_LISTEN on its group-stop)."""
    (image / "app" / "t.sh").write_text("#!/bin/sh\nsleep 1\nexit 7\n")
    (image / "app" / "t.sh").chmod(0o755)
    p = subprocess.Popen([str(TOOL), "--mode", "ptrace", "--rootfs", str(image), "--upper", str(tmp_path / "up"),
                          "--workdir", "/app", "--no-gpu-jail", "--", "/app/t.sh"], start_new_session=True,
                         env={"PATH": "/bin"})
    time.sleep(0.3)
    os.killpg(p.pid, signal.SIGSTOP)
    time.sleep(1.2)
    assert p.poll() is None  # stopped: the sleep did not finish
    os.killpg(p.pid, signal.SIGCONT)
    assert p.wait(timeout=20) == 7


def test_children_and_a_missing_program(image, tmp_path):
    """Background children; a missing program is 127; a program without its execute bit is
    refused (126) although the supervisor would start it through the image's loader."""
    (image / "app" / "plain").write_bytes((image / "bin" / "cat").read_bytes())
    (image / "app" / "plain").chmod(0o644)
    r = _run(image, tmp_path / "up", "(cat /abs/hello-release) & (sleep 0.1; echo child) & wait\n"
                                     "/bin/nothere 2>/dev/null; echo rc=$?\n"
                                     "/app/plain /etc/hello-release 2>/dev/null; echo rc2=$?\n", "--no-gpu-jail")
    assert r.returncode == 0, r.stderr
    assert "tk8s hello 1" in r.stdout and "child" in r.stdout and "rc=127" in r.stdout, r.stdout
    assert "rc2=126" in r.stdout, r.stdout


THREADS_C = r"""
#include <fcntl.h>
#include <pthread.h>
#include <spawn.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>
extern char** environ;
static int bad[16];
static void* work(void* p) {
  long k = (long)p;
  char buf[64];
  for (int i = 0; i < 400; ++i) {
    int fd = open(i % 2 ? "/abs/hello-release" : "/etc/hello-release", O_RDONLY);
    if (fd < 0) { bad[k]++; continue; }
    ssize_t n = read(fd, buf, sizeof buf);
    close(fd);
    if (n != 13 || memcmp(buf, "tk8s hello 1\n", 13)) bad[k]++;
    struct stat st;
    if (stat("/app/../etc/hello-release", &st) != 0) bad[k]++;
  }
  return 0;
}
int main(void) {
  pthread_t t[16];
  for (long k = 0; k < 16; ++k) pthread_create(&t[k], 0, work, (void*)k);
  int spawned = 0;
  for (int i = 0; i < 8; ++i) {  /* posix_spawn: clone(CLONE_VM|CLONE_VFORK) while threads run */
    pid_t c;
    char* argv[] = {"cat", "/abs/hello-release", 0};
    if (posix_spawn(&c, "/bin/cat", 0, 0, argv, environ) == 0) {
      int st;
      waitpid(c, &st, 0);
      spawned += WIFEXITED(st) && WEXITSTATUS(st) == 0;
    }
  }
  int total = 0;
  for (int k = 0; k < 16; ++k) { pthread_join(t[k], 0); total += bad[k]; }
  printf("bad=%d spawned=%d\n", total, spawned);
  return total != 0 || spawned != 8;
}
"""


def test_threads_and_spawn_under_the_supervisor(image, tmp_path):
    """16 threads translating paths at once (each gets its own string mapping; a thread's
    strings are never overwritten while its syscall reads them) and posix_spawn's vfork-style
    children (running on the parent's mapping while it waits) alongside them."""
    import shutil

    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    src = tmp_path / "t.c"
    src.write_text(THREADS_C)
    exe = tmp_path / "threads"
    subprocess.run(["gcc", "-O2", "-pthread", "-o", str(exe), str(src)], check=True, capture_output=True)
    for rel, data in _host_files(str(exe)).items():
        p = image / rel
        if not p.exists():
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_bytes(data)
            p.chmod(0o755)
    r = _run(image, tmp_path / "up", "/bin/threads\n", "--no-gpu-jail", timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert "bad=0 spawned=8" in r.stdout, r.stdout


def test_a_duty_cycle_of_stops_never_strands_a_traced_pod(image, tmp_path):
    """The agent's unprivileged CPU limit stops and resumes a pod's process group many times a
    second. A traced pod's stop signals pass through the supervisor (itself stopped with the
    group); however the SIGSTOPs and SIGCONTs interleave, the pod ends up running and finishes."""
    import random

    (image / "app" / "t.sh").write_text("#!/bin/sh\ni=0; while [ $i -lt 100000 ]; do i=$((i+1)); done\n"
                                        "cat /etc/hello-release\n")
    (image / "app" / "t.sh").chmod(0o755)
    p = subprocess.Popen([str(TOOL), "--mode", "ptrace", "--rootfs", str(image), "--upper", str(tmp_path / "up"),
                          "--workdir", "/app", "--no-gpu-jail", "--", "/app/t.sh"], start_new_session=True,
                         stdout=subprocess.PIPE, text=True, env={"PATH": "/bin"})
    rnd = random.Random(7)
    for _ in range(30):
        os.killpg(p.pid, signal.SIGSTOP)
        time.sleep(rnd.uniform(0.001, 0.02))
        os.killpg(p.pid, signal.SIGCONT)
        time.sleep(rnd.uniform(0.001, 0.02))
    try:
        out, _ = p.communicate(timeout=60)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
    assert p.returncode == 0 and "tk8s hello 1" in out, out
