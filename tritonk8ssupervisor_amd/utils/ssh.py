"""SSH transport for remote machines (the reference's only channel to its VMs).

The reference reaches every machine over SSH: Terraform's remote-exec bootstrap as ``ubuntu``
with the private key (terraform/master/main.tf:13-27), every Ansible play as ``root``
(ansible/clusterUp.yml:4,10,20), and its readiness loop's ``ssh root@host docker ...`` probes
(setup.sh:72-78). Those ``ssh`` calls pass ``-o StrictHostKeyChecking=no`` and no key at all, so
the user's default identity is used and any host key is trusted. Here:

* the key the wizard discovered (``SDC_KEY``) or the inventory names is passed with ``-i`` and
  ``IdentitiesOnly=yes`` (no agent/default-key surprises);
* host keys go to a per-cluster known-hosts file with ``StrictHostKeyChecking=accept-new``:
  the first contact records the key, a later change is refused (trust on first use, not never);
* one multiplexed master connection per host (``ControlMaster=auto`` + ``ControlPersist``), so
  the hundreds of short commands a bring-up sends cost one TCP+auth handshake per host;
* ``BatchMode=yes``: a missing key fails instead of prompting on the orchestrator's tty.

``TK8S_SSH`` overrides the ssh program (tests point it at ``tests/fakessh.py``, which runs the
command in a per-host sandbox and checks the same options).
"""
from __future__ import annotations

import hashlib
import os
import shlex
import io
import subprocess
import tarfile
from pathlib import Path

from .record import field, record as dataclass


@dataclass(frozen=True)
class SSHTarget:
    host: str                      # address (or name ssh resolves)
    user: str = "root"
    port: int = 22
    key: str = ""                  # private key path ("" = ssh's default identities)
    known_hosts: str = ""          # per-cluster known-hosts file
    control_dir: str = ""          # where multiplexing sockets live ("" = no multiplexing)
    connect_timeout: int = 10
    extra_opts: tuple = field(default_factory=tuple)
    local: bool = False            # this very host (inventory ``connection: local``): no ssh at all

    def argv(self, command: str | None = None, *, tty: bool = False) -> list[str]:
        prog = shlex.split(os.environ.get("TK8S_SSH", "ssh"))
        a = list(prog)
        if self.key:
            a += ["-i", os.path.expanduser(self.key), "-o", "IdentitiesOnly=yes"]
        if self.port and int(self.port) != 22:
            a += ["-p", str(self.port)]
        a += ["-o", "BatchMode=yes", "-o", f"ConnectTimeout={self.connect_timeout}",
              "-o", "StrictHostKeyChecking=accept-new", "-o", "ServerAliveInterval=15"]
        if self.known_hosts:
            a += ["-o", f"UserKnownHostsFile={self.known_hosts}"]
        if self.control_dir:
            a += ["-o", "ControlMaster=auto", "-o", f"ControlPath={self.control_dir}/%C", "-o", "ControlPersist=120"]
        for o in self.extra_opts:
            a += ["-o", str(o)]
        if not tty:
            a.append("-T")
        a.append(f"{self.user}@{self.host}" if self.user else self.host)
        if command is not None:
            a.append(command)
        return a


def control_dir_for(state_dir: str | os.PathLike) -> str:
    """A short per-cluster directory for the multiplexing sockets (a Unix socket path must stay
    under 108 bytes, and ControlPath's %C alone is 40)."""
    tag = hashlib.sha1(str(Path(state_dir).resolve()).encode()).hexdigest()[:12]
    d = Path(os.environ.get("TMPDIR", "/tmp")) / f"tk8s-ssh-{os.getuid()}" / tag
    if len(str(d)) > 60:
        d = Path("/tmp") / f"tk8s-ssh-{os.getuid()}" / tag
    d.mkdir(parents=True, exist_ok=True, mode=0o700)
    return str(d)


def run(target: SSHTarget, command: str, *, timeout: float = 300, stdin: bytes | None = None,
        retries_on_connect: int = 0) -> tuple[int, str]:
    """Run ``command`` through the remote user's shell; (rc, stdout+stderr). rc 255 is ssh's own
    failure (unreachable, auth): retried ``retries_on_connect`` times (a machine still booting)."""
    import time

    if target.local:
        return _run_local(command, timeout=timeout, stdin=stdin)
    attempt = 0
    while True:
        try:
            r = subprocess.run(target.argv(command), input=stdin if stdin is not None else b"", capture_output=True,
                               timeout=timeout)
        except subprocess.TimeoutExpired:
            return 124, f"ssh {target.host}: timeout after {timeout}s"
        except OSError as e:
            return 255, f"ssh: {e}"
        out = (r.stdout or b"").decode(errors="replace") + (r.stderr or b"").decode(errors="replace")
        retries = int(os.environ.get("TK8S_SSH_CONNECT_RETRIES", retries_on_connect))
        if r.returncode == 255 and attempt < retries and "Permission denied" not in out:
            attempt += 1
            time.sleep(min(2.0 * attempt, 10.0))
            continue
        return r.returncode, out


def local_login_env() -> dict:
    """The environment a command gets on a ``connection: local`` host: what a login over ssh would
    give it (PATH, HOME, USER, LANG, SHELL), none of the orchestrator's own variables.
    ``TK8S_LOCAL_HOST_ROOT`` (CPU tests): the host is a fake root -- a directory laid out like
    tests/fakessh.py's (its ``bin/`` the whole PATH, ``sysroot/`` the system paths, ``.env`` its
    /etc/environment) -- so the kubeadm roles run against simulated tools."""
    import getpass

    env = {"PATH": os.environ.get("PATH", "/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin"),
           "HOME": os.path.expanduser("~"), "USER": getpass.getuser(), "LOGNAME": getpass.getuser(),
           "LANG": "C.UTF-8", "SHELL": "/bin/bash"}
    fake = os.environ.get("TK8S_LOCAL_HOST_ROOT")
    if fake:
        hd = Path(fake)
        env.update(HOME=str(hd), PATH=str(hd / "bin"), TK8S_SYSROOT=str(hd / "sysroot"))
        envf = hd / ".env"
        if envf.exists():
            for ln in envf.read_text().splitlines():
                if "=" in ln and not ln.startswith("#"):
                    k, v = ln.split("=", 1)
                    env[k.strip()] = v.strip()
    return env


def _run_local(command: str, *, timeout: float, stdin: bytes | None) -> tuple[int, str]:
    """``run`` on this host itself: the login shell's command in the login home, like ssh."""
    env = local_login_env()
    if os.environ.get("TK8S_LOCAL_HOST_ROOT"):  # a simulated root: nothing may touch the real system paths
        import re

        free = re.sub(r"\$\{?TK8S_SYSROOT(:-)?\}?/[^\s'\"]*", "",
                      re.sub(re.escape(env["TK8S_SYSROOT"]) + r"/[^\s'\"]*", "", command))
        for word in ("/etc/apt", "/etc/kubernetes", "/etc/containerd", "/etc/modules-load.d", "/etc/sysctl.d",
                     "/etc/fstab", "/opt/tk8s", "/root/.kube"):
            if word in free:
                return 126, f"local: refusing a system path outside the simulated root ({word})"
    try:
        r = subprocess.run(["bash", "-c", command], input=stdin if stdin is not None else b"", capture_output=True,
                           timeout=timeout, env=env, cwd=env["HOME"])
    except subprocess.TimeoutExpired:
        return 124, f"local: timeout after {timeout}s"
    except OSError as e:
        return 127, f"local: {e}"
    return r.returncode, (r.stdout or b"").decode(errors="replace") + (r.stderr or b"").decode(errors="replace")


def remote_script(command: str, *, cwd: str | None = None, env: dict | None = None) -> str:
    """``cd CWD && export K=V ...; exec bash -c COMMAND`` for the remote login shell."""
    parts = []
    if cwd:
        parts.append(f"cd {shlex.quote(cwd)} || exit 97")
    for k, v in (env or {}).items():
        parts.append(f"export {k}={shlex.quote(str(v))}")
    parts.append("exec bash -c " + shlex.quote(command))
    return "; ".join(parts)


# ---- tk8s distribution push (the "image" a bare-metal machine boots) --------------------------
DIST_EXCLUDE_DIRS = {"__pycache__", ".pytest_cache", "build", "obj"}
DIST_EXCLUDE_SUFFIXES = (".pyc", ".o", ".tmp")


def dist_files(repo: Path, package: str = "tritonk8ssupervisor_amd") -> list[Path]:
    """What a node needs to run the agent, the control plane and the validation tools: the Python
    package with its built native artefacts (bin/, lib/, the extension modules)."""
    out = []
    for root, dirs, files in os.walk(repo / package):
        dirs[:] = sorted(d for d in dirs if d not in DIST_EXCLUDE_DIRS)
        for f in sorted(files):
            if not f.endswith(DIST_EXCLUDE_SUFFIXES):
                out.append(Path(root) / f)
    return out


def dist_digest(repo: Path, files: list[Path]) -> str:
    h = hashlib.sha256()
    for f in files:
        st = f.stat()
        h.update(f"{f.relative_to(repo)}\0{st.st_size}\0{int(st.st_mtime_ns)}\0".encode())
    return h.hexdigest()[:16]


def dist_tarball(repo: Path, files: list[Path]) -> bytes:
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz", compresslevel=1) as tf:
        for f in files:
            tf.add(f, arcname=str(f.relative_to(repo)), recursive=False)
    return buf.getvalue()


def push_dist(target: SSHTarget, repo: Path, dest_root: str = ".tk8s/dist", timeout: float = 600) -> tuple[int, str, str]:
    """Install the tk8s distribution under ``~/<dest_root>/<digest>`` on the target (idempotent:
    an existing stamp skips the copy). Returns (rc, absolute install dir, output)."""
    files = dist_files(repo)
    digest = dist_digest(repo, files)
    d = f"{dest_root.rstrip('/')}/{digest}"
    probe = (f"mkdir -p {shlex.quote(d)} && cd {shlex.quote(d)} && pwd && "
             "if test -f .tk8s-dist-ok; then echo TK8S_PRESENT; fi")
    rc, out = run(target, probe, timeout=timeout, retries_on_connect=3)
    if rc != 0:
        return rc, "", out
    home = out.splitlines()[0].strip() if out.strip() else d
    if "TK8S_PRESENT" in out:
        return 0, home, "present"
    blob = dist_tarball(repo, files)
    cmd = f"cd {shlex.quote(home)} && tar -xzf - && echo {digest} > .tk8s-dist-ok"
    rc, out = run(target, cmd, timeout=timeout, stdin=blob)
    return rc, home, out
