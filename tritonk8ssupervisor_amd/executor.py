"""Machine executors: how the playbook engine and the orchestrator act "on" a machine.

The reference runs every play over SSH on the machines Terraform created (ansible/clusterUp.yml:
1-26, ``remote_user: root``) and probes/heals hosts with ``ssh root@host docker ...``
(setup.sh:72-78). One interface, two implementations:

``LocalExecutor``   machines are sandboxes on this host (the ``local`` provider): daemons are
                    spawned directly (process group + pidfile under the sandbox), files are
                    plain paths under the sandbox.
``RemoteExecutor``  machines are somewhere else (``baremetal``/``triton``): every operation is a
                    shell script sent through ``provider.exec`` (ssh), which runs it in the
                    machine's work directory with its machine environment. Daemons start with
                    ``setsid`` (+ ``tk8s-supervise`` for restart policies) ON the machine; their
                    pidfiles, logs, the burn-in markers and every file module act on the
                    machine's filesystem. Nothing is spawned by the controller.

The controller's layout (``REPO``, ``sys.executable``) appears in argv/env the roles render
(``tk8s_python``, ``tk8s_pythonpath``, validation commands); a remote executor translates it to
the machine's own install (``Machine.home``, ``Machine.python``) at the point of use, so one set
of playbook variables drives both kinds of machine.
"""
from __future__ import annotations

import os
import re
import shlex
import sys
import threading
import time
from pathlib import Path

from .provider.base import Machine, ProvisionError
from .utils.procs import kill_pidfile, pid_alive, read_pidfile, spawn_daemon

REPO = Path(__file__).resolve().parents[1]


# ---- filesystem views --------------------------------------------------------------------
class LocalFS:
    """Paths relative to ``base`` (the machine's sandbox, or the playbook dir for local tasks)."""

    def __init__(self, base: str | os.PathLike):
        self.base = Path(base)

    def path(self, p: str) -> Path:
        pp = Path(os.path.expanduser(str(p)))
        return pp if pp.is_absolute() else self.base / pp

    def read(self, p: str) -> bytes | None:
        try:
            return self.path(p).read_bytes()
        except OSError:
            return None

    def write(self, p: str, data: bytes, mode: int | None = None, check: bool = False) -> bool:
        dest = self.path(p)
        try:
            old = dest.read_bytes()
        except OSError:
            old = None
        changed = old != data
        if changed and not check:
            from .utils.fsutil import atomic_write

            atomic_write(dest, data)
        if mode is not None and not check and dest.exists():
            os.chmod(dest, mode)
        return changed

    def stat(self, p: str) -> dict:
        q = self.path(p)
        if not q.exists():
            return {"exists": False}
        st = q.stat()
        return {"exists": True, "isdir": q.is_dir(), "size": st.st_size, "mtime": st.st_mtime, "path": str(q)}

    def remove(self, p: str) -> bool:
        q = self.path(p)
        if not (q.exists() or q.is_symlink()):
            return False
        from .utils.fsutil import remove_paths

        remove_paths([q])
        return True

    def mkdir(self, p: str) -> bool:
        q = self.path(p)
        if q.is_dir():
            return False
        q.mkdir(parents=True, exist_ok=True)
        return True

    def touch(self, p: str) -> None:
        q = self.path(p)
        q.parent.mkdir(parents=True, exist_ok=True)
        q.touch()

    def search(self, p: str, regex: str | None) -> bool:
        data = self.read(p)
        if data is None:
            return False
        return not regex or re.search(regex, data.decode(errors="replace")) is not None


class RemoteFS:
    """The same operations as shell one-liners run on the machine (relative = its work dir)."""

    def __init__(self, ex: "RemoteExecutor", host: str):
        self.ex, self.host = ex, host

    def _sh(self, script: str, stdin: bytes | None = None, timeout: float = 120) -> tuple[int, str]:
        return self.ex.exec(self.host, script, timeout=timeout, stdin=stdin)

    def path(self, p: str) -> str:
        return str(p)

    def read(self, p: str) -> bytes | None:
        q = shlex.quote(str(p))
        rc, out = self._sh(f"test -f {q} || exit 3; base64 -w0 -- {q}")
        if rc != 0:
            return None
        import base64

        try:
            return base64.b64decode(out.strip())
        except ValueError:
            return None

    def write(self, p: str, data: bytes, mode: int | None = None, check: bool = False) -> bool:
        import hashlib

        q = shlex.quote(str(p))
        want = hashlib.md5(data).hexdigest()
        rc, out = self._sh(f"test -f {q} && md5sum -- {q} | cut -c1-32")
        changed = out.strip() != want
        if check:
            return changed
        if changed:
            script = (f'd=$(dirname -- {q}); mkdir -p "$d" && t="$d/.tk8s.$$.tmp" && cat > "$t" && mv -f "$t" {q}')
            rc, out = self._sh(script, stdin=data)
            if rc != 0:
                raise OSError(f"{self.host}: write {p}: {out.strip()[-300:]}")
        if mode is not None:
            self._sh(f"chmod {mode:o} {q}")
        return changed

    def stat(self, p: str) -> dict:
        q = shlex.quote(str(p))
        rc, out = self._sh(f"stat -c '%F|%s|%Y' -- {q} && readlink -f -- {q}")
        if rc != 0:
            return {"exists": False}
        lines = out.strip().splitlines()
        kind, size, mtime = lines[0].split("|")
        return {"exists": True, "isdir": kind == "directory", "size": int(size), "mtime": float(mtime),
                "path": lines[1] if len(lines) > 1 else str(p)}

    def remove(self, p: str) -> bool:
        q = shlex.quote(str(p))
        rc, _ = self._sh(f"test -e {q} || test -L {q} || exit 3; rm -rf -- {q}")
        return rc == 0

    def mkdir(self, p: str) -> bool:
        q = shlex.quote(str(p))
        rc, _ = self._sh(f"test -d {q} && exit 3; mkdir -p -- {q}")
        return rc == 0

    def touch(self, p: str) -> None:
        q = shlex.quote(str(p))
        self._sh(f'mkdir -p "$(dirname -- {q})" && touch -- {q}')

    def search(self, p: str, regex: str | None) -> bool:
        q = shlex.quote(str(p))
        if not regex:
            rc, _ = self._sh(f"test -e {q}")
        else:
            rc, _ = self._sh(f"grep -qE -- {shlex.quote(regex)} {q}")
        return rc == 0


# ---- executors ------------------------------------------------------------------------------
class _Base:
    remote = False

    def __init__(self, provider, machines: dict[str, Machine]):
        self.provider = provider
        self.machines = machines  # inventory host name -> Machine

    def _m(self, host: str) -> Machine:
        if host not in self.machines:
            raise ProvisionError(f"unknown machine {host}")
        return self.machines[host]

    def exec(self, host: str, cmd: str, env: dict | None = None, timeout: float = 600,
             stdin: bytes | None = None) -> tuple[int, str]:
        m = self._m(host)
        if stdin is None:
            return self.provider.exec(m, cmd, timeout=timeout, env=env)
        return self.provider.exec(m, cmd, timeout=timeout, env=env, stdin=stdin)

    def machine_dir(self, host: str) -> str:
        return self._m(host).sandbox

    def machine_gpus(self, host: str) -> list[int]:
        return list(self._m(host).gpus)

    def localize(self, host: str, s: str) -> str:  # controller layout -> machine layout
        return s


class LocalExecutor(_Base):
    """Machines are sandboxes of this host (local provider): spawn directly, act on local paths."""

    def __init__(self, provider, machines: dict[str, Machine]):
        super().__init__(provider, machines)
        sup = REPO / "tritonk8ssupervisor_amd" / "bin" / "tk8s-supervise"
        self.supervise = str(sup) if sup.exists() else None
        self._facts: tuple[float, dict] | None = None
        self._facts_lock = threading.Lock()

    def fs(self, host: str) -> LocalFS:
        return LocalFS(self._m(host).sandbox)

    def pid_alive(self, host: str, pid: int) -> bool:
        return pid_alive(int(pid))

    FACTS_TTL_S = 2.0

    def facts(self, host: str, timing: dict | None = None) -> dict:
        """Every machine here is a sandbox of this host: one gathering answers all of a play's
        hosts (at 8 workers nine concurrent KFD-topology walks were ~16 ms of play 1 on the
        MI355X host). Kept FACTS_TTL_S, so a later gathering sees a changed host. ``timing``
        receives the lock wait and, for the gathering call, its parts (nodefacts.node_facts)."""
        from .nodefacts import node_facts

        t = time.perf_counter()
        with self._facts_lock:
            if timing is not None:
                timing["lock_wait"] = round((time.perf_counter() - t) * 1e3, 3)
            now = time.monotonic()
            if self._facts is None or now - self._facts[0] > self.FACTS_TTL_S:
                self._facts = (now, node_facts(timing))
            return dict(self._facts[1])

    def _paths(self, host: str, name: str) -> tuple[Path, Path]:
        sb = Path(self._m(host).sandbox)
        return sb / "run" / f"{name}.pid", sb / "logs" / f"{name}.log"

    def daemon_status(self, host: str, name: str) -> dict:
        pidfile, _ = self._paths(host, name)
        info = read_pidfile(pidfile)
        if not info:
            return {"running": False}
        return {"running": pid_alive(int(info["pid"])), "pid": info["pid"]}

    def start_daemon(self, host: str, name: str, argv: list[str], env: dict, restart: str,
                     wait_for_log: str | None, timeout: float) -> dict:
        m = self._m(host)
        pidfile, log = self._paths(host, name)
        full_env = dict(os.environ)
        full_env.update(getattr(self.provider, "machine_env", lambda _m: {})(m))
        full_env.update(env)
        log.parent.mkdir(parents=True, exist_ok=True)
        offset = log.stat().st_size if log.exists() else 0
        if self.supervise and restart != "no":
            cmd = [self.supervise, "--pidfile", str(pidfile), "--log", str(log), "--restart", restart, "--", *argv]
            p = spawn_daemon(cmd, env=full_env, cwd=m.sandbox)
            deadline = time.monotonic() + 5
            while not pidfile.exists() and time.monotonic() < deadline and p.poll() is None:
                time.sleep(0.001)
        else:
            p = spawn_daemon(argv, env=full_env, cwd=m.sandbox, log_path=str(log), pidfile=str(pidfile))
        info = {"ok": True, "pid": p.pid, "log": str(log)}
        if wait_for_log:
            t = time.monotonic()
            deadline = t + timeout
            while time.monotonic() < deadline:
                try:
                    with open(log, "rb") as f:
                        f.seek(offset)
                        if wait_for_log.encode() in f.read():
                            info["wait_seconds"] = round(time.monotonic() - t, 6)
                            return info
                except OSError:
                    pass
                if p.poll() is not None:
                    break
                time.sleep(0.002)
            tail = log.read_text(errors="replace")[-600:] if log.exists() else ""
            return {"ok": False, "msg": f"{name} on {host} did not log {wait_for_log!r} within {timeout}s: {tail}"}
        return info

    def wait_log(self, host: str, name: str, text: str, timeout: float) -> dict:
        """A daemon that is already running: wait until its log has the ready line."""
        _, log = self._paths(host, name)
        t = time.monotonic()
        deadline = t + timeout
        want, seen, n = text.encode(), 0, 0
        while time.monotonic() < deadline:
            try:  # only what the log gained since the last look (a long log is not re-read)
                with open(log, "rb") as f:
                    f.seek(max(0, seen - len(want)))
                    chunk = f.read()
                    if want in chunk:
                        return {"ok": True, "wait_seconds": round(time.monotonic() - t, 6)}
                    seen = f.tell()
            except OSError:
                pass
            n += 1
            # a fine poll (the control plane's "Listening on" is on the bring-up's critical path);
            # whether the daemon died, every 10th look
            if n % 10 == 0 and not self.daemon_status(host, name).get("running"):
                break
            time.sleep(0.0005 if n < 2000 else 0.01)
        tail = log.read_text(errors="replace")[-600:] if log.exists() else ""
        return {"ok": False, "msg": f"{name} on {host} did not log {text!r} within {timeout}s: {tail}"}

    def stop_daemon(self, host: str, name: str) -> bool:
        pidfile, _ = self._paths(host, name)
        return kill_pidfile(pidfile)


# Shell helpers prepended to every daemon script (pidfiles are JSON, one key per line or not).
_SH_FUNCS = r"""
_pidof() { sed -n 's/.*"pid": *\([0-9][0-9]*\).*/\1/p' "$1" 2>/dev/null | head -n1; }
_pgidof() { g=$(sed -n 's/.*"pgid": *\([0-9][0-9]*\).*/\1/p' "$1" 2>/dev/null | head -n1); [ -n "$g" ] && echo "$g" || _pidof "$1"; }
_alive() { [ -n "$1" ] && kill -0 "$1" 2>/dev/null && [ "$(sed 's/.*) //' /proc/$1/stat 2>/dev/null | cut -c1)" != Z ]; }
"""


class RemoteExecutor(_Base):
    """Machines reached through ``provider.exec`` (ssh): every action is a script run there."""

    remote = True

    def fs(self, host: str) -> RemoteFS:
        return RemoteFS(self, host)

    def home(self, host: str) -> str:
        return self._m(host).home or str(REPO)

    def python(self, host: str) -> str:
        return self._m(host).python or "python3"

    def localize(self, host: str, s: str) -> str:
        s = str(s)
        if s == sys.executable:
            return self.python(host)
        return s.replace(str(REPO), self.home(host))

    def pid_alive(self, host: str, pid: int) -> bool:
        rc, _ = self.exec(host, _SH_FUNCS + f"_alive {int(pid)}", timeout=60)
        return rc == 0

    def facts(self, host: str, timing: dict | None = None) -> dict:
        import json

        rc, out = self.exec(host, f"{shlex.quote(self.python(host))} -S -m tritonk8ssupervisor_amd.nodefacts",
                            env={"PYTHONPATH": self.home(host)}, timeout=120)
        if rc != 0:
            raise ProvisionError(f"{host}: node facts failed rc={rc}: {out.strip()[-300:]}")
        return json.loads(out.strip().splitlines()[-1])

    def daemon_status(self, host: str, name: str) -> dict:
        pf = shlex.quote(f"run/{name}.pid")
        rc, out = self.exec(host, _SH_FUNCS + f'p=$(_pidof {pf}); [ -n "$p" ] || exit 3; echo "$p"; _alive "$p"',
                            timeout=60)
        pid = out.strip().splitlines()[0] if out.strip() else ""
        if rc == 3 or not pid.isdigit():
            return {"running": False}
        return {"running": rc == 0, "pid": int(pid)}

    def _wait_script(self, name: str, text: str, timeout: float, offset_var: str) -> str:
        log, pf = shlex.quote(f"logs/{name}.log"), shlex.quote(f"run/{name}.pid")
        return (f"end=$(( $(date +%s) + {int(timeout) + 1} ))\n"
                f"while :; do\n"
                f"  if tail -c +$(({offset_var}+1)) {log} 2>/dev/null | grep -qF -- {shlex.quote(text)}; then "
                f"echo TK8S_READY; exit 0; fi\n"
                f"  _alive \"$(_pidof {pf})\" || break\n"
                f"  [ $(date +%s) -ge $end ] && break\n"
                f"  sleep 0.005\n"
                f"done\n"
                f"echo TK8S_NOT_READY; tail -c 600 {log} 2>/dev/null; exit 1\n")

    def start_daemon(self, host: str, name: str, argv: list[str], env: dict, restart: str,
                     wait_for_log: str | None, timeout: float) -> dict:
        argv = [self.localize(host, a) for a in argv]
        env = {k: self.localize(host, v) for k, v in (env or {}).items()}
        env.setdefault("PYTHONPATH", self.home(host))  # the node's tk8s install is its "image"
        log, pf = shlex.quote(f"logs/{name}.log"), shlex.quote(f"run/{name}.pid")
        cmd = " ".join(shlex.quote(a) for a in argv)
        sup = shlex.quote(f"{self.home(host)}/tritonk8ssupervisor_amd/bin/tk8s-supervise")
        exports = "".join(f"export {k}={shlex.quote(str(v))}\n" for k, v in env.items())
        s = _SH_FUNCS + (
            f"mkdir -p run logs\n"
            f"off=$(stat -c %s {log} 2>/dev/null || echo 0)\n"
            f"rm -f {pf}\n{exports}")
        if restart != "no":
            s += (f"if [ -x {sup} ]; then\n"
                  f"  setsid {sup} --pidfile {pf} --log {log} --restart {shlex.quote(restart)} -- {cmd} "
                  f"</dev/null >/dev/null 2>&1 &\n"
                  f"  i=0; while [ ! -s {pf} ] && [ $i -lt 1000 ]; do sleep 0.005; i=$((i+1)); done\n"
                  f"else\n")
        s += (f"  setsid {cmd} </dev/null >>{log} 2>&1 &\n"
              f"  p=$!; printf '{{\"pid\": %s, \"pgid\": %s}}\\n' \"$p\" \"$p\" > {pf}.tmp && mv -f {pf}.tmp {pf}\n")
        if restart != "no":
            s += "fi\n"
        s += f'echo "TK8S_PID=$(_pidof {pf}) TK8S_OFF=$off"\n'
        if wait_for_log:
            s += self._wait_script(name, wait_for_log, timeout, "off")
        t = time.monotonic()
        rc, out = self.exec(host, s, timeout=max(60.0, float(timeout or 0) + 60.0))
        m = re.search(r"TK8S_PID=(\d*)", out)
        pid = int(m.group(1)) if m and m.group(1) else 0
        if not m or not pid:
            return {"ok": False, "msg": f"{name} on {host} failed to start (rc={rc}): {out.strip()[-600:]}"}
        info = {"ok": True, "pid": pid, "log": f"{self.machine_dir(host)}/logs/{name}.log"}
        if wait_for_log:
            if rc != 0 or "TK8S_READY" not in out:
                tail = out.split("TK8S_NOT_READY", 1)[-1].strip()[-600:]
                return {"ok": False, "msg": f"{name} on {host} did not log {wait_for_log!r} within {timeout}s: {tail}"}
            info["wait_seconds"] = round(time.monotonic() - t, 6)
        return info

    def wait_log(self, host: str, name: str, text: str, timeout: float) -> dict:
        t = time.monotonic()
        rc, out = self.exec(host, _SH_FUNCS + "off=0\n" + self._wait_script(name, text, timeout, "off"),
                            timeout=float(timeout) + 60.0)
        if rc == 0 and "TK8S_READY" in out:
            return {"ok": True, "wait_seconds": round(time.monotonic() - t, 6)}
        tail = out.split("TK8S_NOT_READY", 1)[-1].strip()[-600:]
        return {"ok": False, "msg": f"{name} on {host} did not log {text!r} within {timeout}s: {tail}"}

    def stop_daemon(self, host: str, name: str) -> bool:
        pf = shlex.quote(f"run/{name}.pid")
        rc, _ = self.exec(host, _SH_FUNCS + stop_group_script(pf), timeout=60)
        return rc == 0


def stop_group_script(pidfile_q: str, grace_ticks: int = 300) -> str:
    """SIGTERM the process group a pidfile names, wait (10 ms ticks), SIGKILL, drop the pidfile.
    Exit 1 when nothing ran."""
    return (f'g=$(_pgidof {pidfile_q}); [ -n "$g" ] || {{ rm -f {pidfile_q}; exit 1; }}\n'
            f'if ! kill -TERM -- -"$g" 2>/dev/null; then rm -f {pidfile_q}; exit 1; fi\n'
            f'i=0; while kill -0 -- -"$g" 2>/dev/null && [ $i -lt {grace_ticks} ]; do sleep 0.01; i=$((i+1)); done\n'
            f'kill -KILL -- -"$g" 2>/dev/null; rm -f {pidfile_q}; exit 0\n')


def executor_for(provider, machines: dict[str, Machine]):
    """The executor matching where the provider's machines live."""
    if getattr(provider, "colocated", False):
        return LocalExecutor(provider, machines)
    return RemoteExecutor(provider, machines)


# The orchestrator's historical name (used by `./tk8s ansible-playbook` and the boot hooks).
MachineExecutor = executor_for
