"""Pod runtime of the node agent: pods are process groups in the node sandbox.

The reference's nodes run Docker containers started by the Rancher agent (rancher/agent:v1.2.0,
ansible/roles/rancherhost/tasks/main.yml:26-34). Here a pod is a process group: its env gets the
device plugin's Allocate() result and the downward-API values, ``$(VAR)`` references in
command/args are expanded like Kubernetes does, stdout/stderr go to ``pods/<pod>/log``, and
restartPolicy Always/OnFailure/Never is honoured with capped exponential back-off; a restarted
container's previous log is kept as ``<log>.previous`` (``kubectl logs --previous``).

A pod's containers: ``initContainers`` run one after the other, each to a zero exit (retried
with back-off, or the pod fails with ``Init:Error`` under ``restartPolicy: Never``), then every
app container runs as its own process group. The first is the pod's ``PodProc`` (log ``log``);
the others are its ``sidecars`` (log ``log.<name>``), restarted under the same policy. The pod
ends once every app container has ended, Succeeded if all exited 0.

Lifecycle hooks and graceful termination, as the kubelet does them: a container's
``lifecycle.postStart`` (exec, httpGet or sleep) runs right after it starts -- a failing hook kills
the container, which restarts under the policy; deleting a pod runs every container's
``lifecycle.preStop`` hook, then SIGTERMs all its process groups and SIGKILLs what is left when
``terminationGracePeriodSeconds`` (default 30) runs out -- the window a training job gets to write
its checkpoint. Termination runs off the caller's thread (``stop(wait=False)``); the pod's GPUs
stay allocated until it is over.
"""
from __future__ import annotations

import contextlib
import json
import os
import re
import signal
import subprocess
import threading
import time
from pathlib import Path

from ..utils.faults import fault
from ..utils.fsutil import atomic_write_json
from ..utils.procs import kill_group, proc_start_ticks
from ..utils.record import field, record as dataclass
from ..utils.trace import trace

_VAR = re.compile(r"\$\(([A-Za-z_][A-Za-z0-9_]*)\)")
RUNNING_GRACE_S = 0.005  # a container that ends within this after its start never reports Running


def expand(s: str, env: dict) -> str:
    """Kubernetes `$(VAR)` expansion; `$$(VAR)` escapes; unknown refs stay verbatim."""
    out, i = [], 0
    while i < len(s):
        if s.startswith("$$(", i):
            out.append("$(")
            i += 3
            continue
        m = _VAR.match(s, i)
        if m:
            out.append(env.get(m.group(1), m.group(0)))
            i = m.end()
        else:
            out.append(s[i])
            i += 1
    return "".join(out)


def _tty_pump(pp, master: int, logfd: int) -> None:
    """Copy a tty container's output to its log and its attached sessions until every holder of
    the pty's slave side is gone (EIO); then the sessions get None: the container ended."""
    try:
        while True:
            try:
                data = os.read(master, 65536)
            except OSError:
                break
            if not data:
                break
            with contextlib.suppress(OSError):
                os.write(logfd, data)
            with pp.io_lock:
                subs = list(pp.io_subs)
            for q in subs:
                q.put(data)
    finally:
        os.close(logfd)
        with pp.io_lock:
            if pp.tty_master == master:
                pp.tty_master = -1
            subs = list(pp.io_subs)
        os.close(master)
        for q in subs:
            q.put(None)


def close_stdin(cp) -> None:
    """End a `stdin: true` container's input: EOF on its pipe (a tty's ends with the container)."""
    with cp.io_lock:
        w, cp.stdin_w = cp.stdin_w, -1
    if w >= 0:
        with contextlib.suppress(OSError):
            os.close(w)


def last_json_line(text: str) -> dict | None:
    for line in reversed(text.strip().splitlines()):
        line = line.strip()
        if line.startswith("{") and line.endswith("}"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


@dataclass
class PodProc:
    key: str                      # namespace/name
    uid: str
    dir: Path
    argv: list[str]
    env: dict
    restart_policy: str
    gpu_ids: list[str] = field(default_factory=list)
    ip: str = ""                  # the pod's own loopback IP (from the node's podCIDR)
    isolate: bool = False         # own user/pid/mount namespaces (see namespace_isolation())
    jail: list[str] = field(default_factory=list)  # GPU jail argv prefix (gpu_jail_argv), [] = none
    exec_prefix: list[str] = field(default_factory=list)  # image pods: `tk8s-container --exec-in` options
    name: str = ""                # the container's name
    log_name: str = "log"         # its log file in the pod dir (the first app container: "log")
    init: list = field(default_factory=list)      # init containers (PodProc each), run in order first
    sidecars: list = field(default_factory=list)  # the pod's other app containers (PodProc each)
    container: dict = field(default_factory=dict)  # its spec (probes, ports)
    prober: object = None         # agent/probes.Prober of the running process, if it has probes
    grace: float = 30.0           # terminationGracePeriodSeconds
    pod_key: str = ""             # the pod's key (sidecars' and init containers' too): its cgroup
    limit_opts: list[str] = field(default_factory=list)  # resources.py jail options, when no jail applies them
    oom_killed: bool = False      # the last instance ended in an out-of-memory kill
    last_term: dict | None = None  # the last instance's terminated state (lastState)
    proc: subprocess.Popen | None = None
    restarts: int = 0
    started: float = 0.0
    exit_code: int | None = None
    stopping: bool = False
    done: threading.Event = field(default_factory=threading.Event)
    tty_master: int = -1          # `tty: true`: the pty's master side (the pump reads it, attach writes it)
    stdin_w: int = -1             # `stdin: true` without a tty: the write end of the container's stdin
    io_subs: list = field(default_factory=list)  # attached sessions' output queues (tty containers)
    io_lock: threading.Lock = field(default_factory=threading.Lock)


class PodRuntime:
    def __init__(self, sandbox: Path, on_status, tool_dirs: list[str] | None = None):
        self.sandbox = Path(sandbox)
        self.enforcer = None              # resources.Enforcer: cgroups, OOM verdicts
        self.on_status = on_status        # callback(podproc, phase, extra: dict)
        self.pods: dict[str, PodProc] = {}
        self.terminating: dict[str, PodProc] = {}  # deleted, within their grace period
        self.lock = threading.Lock()
        self.tool_dirs = tool_dirs or []

    def start(self, pp: PodProc) -> None:
        with self.lock:
            self.pods[pp.key] = pp
        threading.Thread(target=self._run, args=(pp,), name=f"pod-{pp.key}", daemon=True).start()

    def _spawn(self, pp: PodProc) -> subprocess.Popen:
        pp.dir.mkdir(parents=True, exist_ok=True)
        env = dict(pp.env)
        if self.tool_dirs:
            env["PATH"] = os.pathsep.join(self.tool_dirs + [env.get("PATH", os.environ.get("PATH", ""))])
        argv = [*pp.jail, *pp.argv]  # nothing the pod runs can leave the jail
        if pp.isolate and namespace_isolation()[0]:  # outside the jail: a Landlocked process may not mount /proc
            argv = [*UNSHARE, "--", *argv]
        if pp.exit_code is not None:  # a restart: the last instance's log is `kubectl logs --previous`
            with contextlib.suppress(OSError):
                os.replace(pp.dir / pp.log_name, pp.dir / f"{pp.log_name}.previous")
        if self.enforcer is not None and pp.exit_code is not None:
            self.enforcer.reset_oom(pp.pod_key or pp.key)
        log = open(pp.dir / pp.log_name, "ab", buffering=0)
        c = pp.container or {}
        try:
            p = self._spawn_tty(pp, argv, env, log) if c.get("tty") else None
            if p is None and c.get("stdin"):
                r, w = os.pipe()
                try:
                    p = subprocess.Popen(argv, env=env, cwd=pp.dir, stdin=r, stdout=log, stderr=subprocess.STDOUT,
                                         start_new_session=True, close_fds=True)
                except BaseException:
                    os.close(w)
                    raise
                finally:
                    os.close(r)
                with pp.io_lock:
                    pp.stdin_w = w
            elif p is None:
                p = subprocess.Popen(argv, env=env, cwd=pp.dir, stdin=subprocess.DEVNULL, stdout=log,
                                     stderr=subprocess.STDOUT, start_new_session=True, close_fds=True)
        finally:
            log.close()
        if pp.limit_opts:  # no jail to join them: best effort right after the start
            _join_limits(p.pid, pp.limit_opts)
        atomic_write_json(pp.dir / _pidfile(pp), {"pid": p.pid, "pgid": p.pid, "argv": pp.argv,
                                                  "start": proc_start_ticks(p.pid)})
        return p

    def _spawn_tty(self, pp: PodProc, argv: list[str], env: dict, log) -> subprocess.Popen | None:
        """`tty: true`: the container gets a pty as its controlling terminal (stdin, stdout and
        stderr), like the kubelet's; a pump thread copies what it writes to the container's log and
        to every `kubectl attach` session, which write keystrokes and resizes to the master side.
        None on a node without pseudo-terminals (no devpts: the MI355X GPU boxes): the container
        then runs as with `tty: false`, and its log says so."""
        import fcntl
        import pty
        import termios

        try:
            if fault("node.no_pty") is not None:
                raise OSError("out of pty devices (injected: node.no_pty)")
            master, slave = pty.openpty()
        except OSError as e:
            log.write(f"tk8s: no pseudo-terminal on this node ({e}): the container runs without a tty\n".encode())
            return None

        env.setdefault("TERM", "xterm")
        try:
            p = subprocess.Popen(argv, env=env, cwd=pp.dir, stdin=slave, stdout=slave, stderr=slave,
                                 start_new_session=True, close_fds=True,
                                 preexec_fn=lambda: fcntl.ioctl(0, termios.TIOCSCTTY, 0))
        except BaseException:
            os.close(master)
            raise
        finally:
            os.close(slave)
        logfd = os.dup(log.fileno())
        with pp.io_lock:
            pp.tty_master = master
        threading.Thread(target=_tty_pump, args=(pp, master, logfd), name=f"tty-{pp.key}-{pp.name}", daemon=True).start()
        return p

    def _probe(self, cp: PodProc, pp: PodProc) -> None:
        """Start the container's probes for the process just spawned (agent/probes.py)."""
        if not any(k in cp.container for k in ("startupProbe", "livenessProbe", "readinessProbe")):
            cp.prober = None
            return
        from .probes import Prober

        proc = cp.proc
        cp.prober = Prober(cp.container, cp.ip, lambda: proc.poll() is None, lambda: kill_group(proc.pid, 1.0),
                           lambda: self.on_status(pp, "Running", {}), lambda cmd: container_exec_argv(cp, cmd),
                           env=dict(cp.env), cwd=str(cp.dir))
        cp.prober.start()

    def _init(self, pp: PodProc) -> bool:
        """Run the init containers in order; False when the pod stops or fails on one."""
        for i, ic in enumerate(pp.init):
            backoff = 0.1
            while True:
                if pp.stopping:
                    return False
                try:
                    ic.proc = self._spawn(ic)
                except OSError as e:
                    self.on_status(pp, "Failed", {"message": f"init container {ic.name}: {e}", "reason": "Init:StartError"})
                    return False
                self.on_status(pp, "Pending", {"reason": "PodInitializing", "message": f"Init:{i}/{len(pp.init)}"})
                rc = self._exited(ic, ic.proc.wait())
                (pp.dir / _pidfile(ic)).unlink(missing_ok=True)
                if rc == 0 or pp.stopping:
                    break
                if pp.restart_policy == "Never":
                    self.on_status(pp, "Failed", {"reason": "Init:Error", "exitCode": rc,
                                                  "message": f"init container {ic.name} exited {rc}"})
                    return False
                ic.restarts += 1
                time.sleep(backoff)
                backoff = min(backoff * 2, 10.0)
        return not pp.stopping

    def _run_sidecar(self, sc: PodProc, pp: PodProc) -> None:
        backoff = 0.1
        while not pp.stopping:
            sc.started = time.time()
            try:
                sc.proc = self._spawn(sc)
            except OSError:
                sc.exit_code = 127
                break
            self._post_start(sc, pp)
            self._probe(sc, pp)
            if pp.proc is not None and pp.proc.poll() is None:
                self.on_status(pp, "Running", {})  # its container statuses now include this one
            rc = self._exited(sc, sc.proc.wait())
            (pp.dir / _pidfile(sc)).unlink(missing_ok=True)
            if pp.stopping or not (pp.restart_policy == "Always" or (pp.restart_policy == "OnFailure" and rc != 0)):
                break
            sc.restarts += 1
            self.on_status(pp, "Running", {})
            time.sleep(backoff)
            backoff = min(backoff * 2, 10.0)
        sc.done.set()

    def _exited(self, cp: PodProc, rc: int) -> int:
        """Record a container's exit; an out-of-memory kill is exit 137, reason OOMKilled (the
        kernel's in a cgroup, or the memory watchdog's)."""
        close_stdin(cp)
        cp.oom_killed = bool(rc < 0 and self.enforcer is not None and self.enforcer.oom_killed(cp.pod_key or cp.key))
        if cp.oom_killed:
            rc = 137
        elif rc < 0:
            rc = 128 - rc  # killed by a signal: 128 + signo, as a shell reports it
        cp.exit_code = rc
        cp.last_term = {"exitCode": rc, "reason": "OOMKilled" if cp.oom_killed else ("Completed" if rc == 0 else "Error"),
                        "finishedAt": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
        return rc

    def _run(self, pp: PodProc) -> None:
        if pp.init and not self._init(pp):
            pp.done.set()
            return
        for sc in pp.sidecars:
            threading.Thread(target=self._run_sidecar, args=(sc, pp), name=f"pod-{pp.key}-{sc.name}", daemon=True).start()
        backoff = 0.1
        while not pp.stopping:
            pp.started = time.time()
            try:
                pp.proc = self._spawn(pp)
            except OSError as e:
                pp.exit_code = 127
                self.on_status(pp, "Failed", {"message": f"failed to start {pp.argv[0]!r}: {e}", "reason": "StartError"})
                break
            trace("runtime", f"spawned {pp.key}")
            self._post_start(pp, pp)
            self._probe(pp, pp)
            status = None
            if not pp.sidecars:  # a container done within the grace is reported once, as done: a
                status = _wait_briefly(pp.proc, RUNNING_GRACE_S)  # Running report first would only
                #                                 hold up its result (the validation pod's ~1 ms payload)
            if status is None:
                self.on_status(pp, "Running", {})
                status = pp.proc.wait()
            rc = self._exited(pp, status)
            trace("runtime", f"exited {pp.key} rc={rc}")
            (pp.dir / _pidfile(pp)).unlink(missing_ok=True)
            if pp.stopping:
                break
            ok = rc == 0
            again = pp.restart_policy == "Always" or (pp.restart_policy == "OnFailure" and not ok)
            if not again:
                for sc in pp.sidecars:  # the pod ends with its last container
                    while not sc.done.wait(0.5):
                        if pp.stopping:
                            break
                if pp.stopping:
                    break
                bad = [sc for sc in pp.sidecars if sc.exit_code not in (0, None)]
                if bad and ok:
                    ok, rc = False, bad[0].exit_code
                text = ""
                try:
                    text = (pp.dir / "log").read_text(errors="replace")
                except OSError:
                    pass
                extra = {"exitCode": rc, "result": last_json_line(text),
                         "message": "" if ok else text.strip()[-800:]}
                self.on_status(pp, "Succeeded" if ok else "Failed", extra)
                break
            pp.restarts += 1
            self.on_status(pp, "Running", {"restarts": pp.restarts, "lastExitCode": rc})
            time.sleep(backoff)
            backoff = min(backoff * 2, 10.0)
        pp.done.set()

    def _hook(self, cp: PodProc, hook: dict, timeout: float) -> str | None:
        """Run one lifecycle handler (exec / httpGet / sleep); None if it succeeded, else why not."""
        if timeout <= 0:
            return "no time left"
        if "exec" in hook:
            cmd = (hook["exec"] or {}).get("command") or []
            try:
                r = subprocess.run(container_exec_argv(cp, [expand(x, cp.env) for x in cmd]), env=dict(cp.env),
                                   cwd=cp.dir, capture_output=True, timeout=timeout)
            except (OSError, subprocess.TimeoutExpired) as e:
                return str(e)
            return None if r.returncode == 0 else f"exited {r.returncode}: {r.stderr.decode(errors='replace')[-200:]}"
        if "httpGet" in hook:
            import urllib.request

            h = hook["httpGet"] or {}
            port = h.get("port")
            if isinstance(port, str) and not port.isdigit():
                port = next((p.get("containerPort") for p in cp.container.get("ports") or [] if p.get("name") == port), port)
            url = f"{(h.get('scheme') or 'HTTP').lower()}://{h.get('host') or cp.ip or '127.0.0.1'}:{port}{h.get('path') or '/'}"
            try:
                with urllib.request.urlopen(url, timeout=timeout) as r:
                    return None if 200 <= r.status < 400 else f"HTTP {r.status}"
            except OSError as e:
                return str(e)
        if "sleep" in hook:
            time.sleep(min(float((hook["sleep"] or {}).get("seconds", 0)), timeout))
            return None
        return "unsupported handler"

    def _post_start(self, cp: PodProc, pp: PodProc) -> None:
        hook = (cp.container.get("lifecycle") or {}).get("postStart")
        if not hook or cp.proc is None:
            return
        why = self._hook(cp, hook, 30.0)
        if why is not None and cp.proc.poll() is None and not pp.stopping:
            trace("runtime", f"postStart hook of {cp.key} failed: {why}")
            with open(pp.dir / cp.log_name, "a") as f:
                f.write(f"[tk8s] FailedPostStartHook: {why}\n")
            kill_group(cp.proc.pid, 1.0)  # the container restarts under the pod's restartPolicy

    def _terminate(self, pp: PodProc, grace: float) -> None:
        """preStop hooks, SIGTERM to every container, SIGKILL at the end of the grace period."""
        deadline = time.monotonic() + grace
        conts = [c for c in (pp, *pp.sidecars) if c.proc is not None and c.proc.poll() is None]
        hooks = [threading.Thread(target=self._hook, args=(c, c.container["lifecycle"]["preStop"], grace), daemon=True)
                 for c in conts if (c.container.get("lifecycle") or {}).get("preStop")]
        for t in hooks:
            t.start()
        for t in hooks:
            t.join(max(0.0, deadline - time.monotonic()))
        groups = [c.proc.pid for c in (pp, *pp.sidecars, *pp.init) if c.proc is not None and c.proc.poll() is None]
        for g in groups:
            try:
                os.killpg(g, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
        for g in groups:  # the rest of the grace period, shared; kill_group SIGKILLs what outlives it
            kill_group(g, max(0.0, deadline - time.monotonic()), term=False)

    def stop(self, key: str, grace: float | None = None, wait: bool = True, on_done=None) -> PodProc | None:
        """Stop a pod: ``grace`` defaults to its terminationGracePeriodSeconds. ``wait=False``
        terminates in a thread (the pod is in ``terminating`` meanwhile) and calls ``on_done``."""
        with self.lock:
            pp = self.pods.pop(key, None)
            if pp is not None:
                self.terminating[key] = pp
        if pp is None:
            if on_done is not None:
                on_done()
            return None
        pp.stopping = True
        if self.enforcer is not None:  # a pod the CPU duty cycle stopped runs again for its SIGTERM
            self.enforcer.throttle.terminating(key)
        for c in (pp, *pp.sidecars):
            if c.prober is not None:
                c.prober.stop.set()

        def run():
            try:
                self._terminate(pp, pp.grace if grace is None else grace)
            finally:
                with self.lock:
                    if self.terminating.get(key) is pp:
                        del self.terminating[key]
                if on_done is not None:
                    on_done()

        if wait:
            run()
        else:
            threading.Thread(target=run, name=f"stop-{key}", daemon=True).start()
        return pp

    def is_terminating(self, key: str) -> bool:
        with self.lock:
            return key in self.terminating

    def terminating_gpus(self) -> set[str]:
        with self.lock:
            return {i for pp in self.terminating.values() for i in pp.gpu_ids}

    def held_gpus(self) -> set[str]:
        """GPUs of running pods and of pods still within their grace period."""
        with self.lock:
            return ({i for pp in self.pods.values() if not pp.done.is_set() for i in pp.gpu_ids}
                    | {i for pp in self.terminating.values() for i in pp.gpu_ids})

    def stop_all(self) -> None:
        """The agent is going away: every pod ends within a second, those already terminating too."""
        for key in list(self.pods):
            self.stop(key, grace=1.0)
        with self.lock:
            late = list(self.terminating.values())
        for pp in late:
            for c in (pp, *pp.sidecars, *pp.init):
                if c.proc is not None and c.proc.poll() is None:
                    kill_group(c.proc.pid, 1.0, term=False)

    def running(self) -> dict[str, PodProc]:
        with self.lock:
            return dict(self.pods)


def _wait_briefly(proc: subprocess.Popen, timeout: float) -> int | None:
    """The exit status if ``proc`` ends within ``timeout``, else None. Woken by the exit itself
    (a pidfd), not by Popen.wait's sleep-and-poll (0.5, 1, 2 ms...: up to ~1.5 ms late for a
    container that lives ~2 ms)."""
    import select

    try:
        fd = os.pidfd_open(proc.pid)
    except (AttributeError, OSError):  # an old kernel: the polling wait
        try:
            return proc.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            return None
    try:
        p = select.poll()
        p.register(fd, select.POLLIN)
        return proc.wait() if p.poll(max(0, int(timeout * 1000))) else None
    finally:
        os.close(fd)


def _join_limits(pid: int, opts: list[str]) -> None:
    """--cgroup-procs FILE / --cpus LIST for a process already started (no jail to do it)."""
    from .resources import parse_cpulist

    for flag, val in zip(opts[::2], opts[1::2]):
        try:
            if flag == "--cgroup-procs":
                with open(val, "w") as f:
                    f.write(f"{pid}\n")
            elif flag == "--cpus":
                os.sched_setaffinity(pid, parse_cpulist(val))
        except OSError:
            pass


def reap_leftovers(pods_dir: Path) -> list[int]:
    """A (re)starting agent's first act: the process groups an earlier agent of this machine
    started and left behind -- it was killed, so no ``stop_all`` ran -- are ended, each only while
    it is still the process its pidfile names (pid and start ticks; a reused pid is left alone).
    SIGCONT goes first: the watchdog's CPU duty cycle may have left them SIGSTOPped, and a stopped
    group would otherwise hold its GPUs and memory forever. The pods themselves come back from
    the control plane's desired state, so a leftover would only run twice. Returns the groups."""
    ended = []
    for pf in sorted(Path(pods_dir).glob("*/*.pid")):
        try:
            rec = json.loads(pf.read_text())
            pgid, start = int(rec.get("pgid") or rec["pid"]), rec.get("start")
        except (OSError, ValueError, KeyError, TypeError):
            continue
        if start is not None and proc_start_ticks(pgid) == start:
            for sig in (signal.SIGCONT, signal.SIGKILL):
                with contextlib.suppress(ProcessLookupError, PermissionError):
                    os.killpg(pgid, sig)
            ended.append(pgid)
        with contextlib.suppress(OSError):
            pf.unlink()
    return ended


def _pidfile(pp: PodProc) -> str:
    return "pod.pid" if pp.log_name == "log" else f"pod-{pp.name}.pid"


# A pod's own namespaces, when the kernel lets an unprivileged user create them: a user namespace
# mapping the agent's uid to itself, a PID namespace (the pod's processes see only each other;
# --kill-child: the pod dies with its init) and a mount namespace with its own /proc. The network
# namespace stays the host's: pods bind their own loopback IPs and Services/DNS answer there.
UNSHARE = ["unshare", "--user", "--map-current-user", "--pid", "--fork", "--mount-proc", "--kill-child"]
_ISOLATION: tuple[bool, str] | None = None


def namespace_isolation(readable: str = "", writable: str = "") -> tuple[bool, str]:
    """(available, description), probed once: ``unshare`` with the flags above must start, and
    inside it the tk8s install (``readable``) and the pods dir (``writable``) must still be
    usable -- a user namespace drops capabilities such as root's DAC override, which a node
    running as root may rely on to reach them."""
    global _ISOLATION
    if _ISOLATION is None:
        if os.environ.get("TK8S_POD_ISOLATION", "auto") == "none":
            _ISOLATION = (False, "disabled (TK8S_POD_ISOLATION=none)")
        else:
            check = "true"
            if readable:
                check += f" && test -r '{readable}'"
            if writable:
                check += f" && test -w '{writable}'"
            try:
                r = subprocess.run([*UNSHARE, "--", "sh", "-c", check], capture_output=True, text=True, timeout=10)
                ok = r.returncode == 0
                why = (r.stderr or "").strip().splitlines()[-1:] or [
                    f"the tk8s install or the pods dir is not accessible inside a user namespace (rc={r.returncode})"]
                _ISOLATION = (ok, "user,pid,mount" if ok else f"unavailable: {why[0]}")
            except (OSError, subprocess.TimeoutExpired) as e:
                _ISOLATION = (False, f"unavailable: {e}")
    return _ISOLATION


# The GPU jail (native/tools/tk8s_gpujail.cpp): Landlock keeps a pod from opening the DRM render
# nodes of GPUs it was not allocated, so its runtime enumerates exactly its GPUs whatever
# *_VISIBLE_DEVICES it sets and cannot map another GPU's memory -- the device-cgroup part of a
# container, with no privileges and no namespaces (both unavailable to the GPU tier's user).
JAIL = Path(__file__).resolve().parents[1] / "bin" / "tk8s-gpujail"
_JAIL: tuple[bool, str] | None = None
_JAIL_ABI = 0


def gpu_jail() -> tuple[bool, str]:
    """(available, description), probed once (``tk8s-gpujail --probe``); TK8S_GPU_JAIL=0 disables."""
    global _JAIL, _JAIL_ABI
    if _JAIL is None:
        if os.environ.get("TK8S_GPU_JAIL", "1") == "0":
            _JAIL = (False, "disabled (TK8S_GPU_JAIL=0)")
        elif not JAIL.exists():
            _JAIL = (False, "unavailable: tk8s-gpujail is not built")
        else:
            try:
                r = subprocess.run([str(JAIL), "--probe"], capture_output=True, text=True, timeout=10)
                info = json.loads(r.stdout or "{}")
                _JAIL = ((True, f"landlock (abi {info.get('landlock_abi')})") if r.returncode == 0 and info.get("usable")
                         else (False, f"unavailable: Landlock {info.get('error') or 'not usable'}"))
                _JAIL_ABI = int(info.get("landlock_abi") or 0)
            except (OSError, ValueError, subprocess.TimeoutExpired) as e:
                _JAIL = (False, f"unavailable: {e}")
    return _JAIL


def jail_signal_scoping() -> bool:
    """Does this kernel's Landlock scope signals (ABI >= 6)? Probed with gpu_jail()."""
    return gpu_jail()[0] and _JAIL_ABI >= 6


def gpu_jail_argv(gpus: list, *, deny=(), read_only=(), allow=(), scope_signals: bool = False,
                  extra=None) -> list[str]:
    """argv prefix that runs a command allowed to open only ``gpus`` (HostGpu records: KFD node +
    render minor), none of the ``deny`` paths, only for reading the ``read_only`` ones, and the
    ``allow`` paths beneath either (agent._jail_layers); ``scope_signals``: no signal to any process
    outside the pod. TK8S_GPU_JAIL_KFD_ROOT / TK8S_GPU_JAIL_DRI_ROOT point it at another tree (the
    CPU tests' fake GPUs)."""
    argv = [str(JAIL)]
    for opt, paths in (("--deny", deny), ("--read-only", read_only), ("--allow", allow)):
        for x in paths:
            argv += [opt, str(x)]
    if scope_signals:
        argv.append("--scope-signals")
    argv += list(extra or [])  # resources.py: --cgroup-procs FILE / --cpus LIST
    hide = os.environ.get("TK8S_GPU_JAIL_HIDE_TOPOLOGY") == "1"  # off: ROCm 7.2's thunk fails on it
    if hide:
        argv.append("--hide-topology")
    for g in gpus:
        if hide and getattr(g, "kfd_node", -1) >= 0:
            argv += ["--allow-node", str(g.kfd_node)]
        if getattr(g, "render_minor", -1) >= 0:
            argv += ["--allow-render", str(g.render_minor)]
    for opt, env in (("--kfd-root", "TK8S_GPU_JAIL_KFD_ROOT"), ("--dri-root", "TK8S_GPU_JAIL_DRI_ROOT")):
        if os.environ.get(env):
            argv += [opt, os.environ[env]]
    return argv + ["--"]


# Image pods (agent/images.py): tk8s-container (native/tools/tk8s_container.cpp) runs the
# command in the image's root file system -- mount namespace (+ a user namespace when not root,
# + a PID namespace for CPU pods), an overlay with the pod's own upper layer, the host's /dev /sys
# /proc, hostPath volumes -- with the same GPU jail as process pods inside. Where this user can
# make no namespace (the GPU tier), the same view by path translation under a seccomp-filtered
# ptrace supervisor (native/tools/ptrace_root.h): "ptrace" mode, host PID namespace.
# TK8S_CONTAINER_MODE=namespaces|ptrace picks one (default: namespaces when they can be had).
CONTAINER = Path(__file__).resolve().parents[1] / "bin" / "tk8s-container"
_CONTAINER: tuple[bool, str, str] | None = None


def _container_mode_opt() -> list[str]:
    m = os.environ.get("TK8S_CONTAINER_MODE", "")
    return ["--mode", m] if m in ("namespaces", "ptrace") else []


def _container_probe() -> tuple[bool, str, str]:
    global _CONTAINER
    if _CONTAINER is None:
        if not CONTAINER.exists():
            _CONTAINER = (False, "tk8s-container is not built", "")
        else:
            try:
                r = subprocess.run([str(CONTAINER), *_container_mode_opt(), "--probe"], capture_output=True, text=True,
                                   timeout=10)
                info = json.loads(r.stdout or "{}")
                how = info.get("how") or ""
                if r.returncode == 0 and info.get("usable"):
                    desc = ("ptrace (path translation under a seccomp-filtered supervisor; host PID namespace)"
                            if how == "ptrace" else f"namespaces ({how})")
                    _CONTAINER = (True, desc, "ptrace" if how == "ptrace" else "namespaces")
                else:
                    _CONTAINER = (False, info.get("error") or f"probe failed (rc={r.returncode})", "")
            except (OSError, ValueError, subprocess.TimeoutExpired) as e:
                _CONTAINER = (False, str(e), "")
    return _CONTAINER


def container_runtime() -> tuple[bool, str]:
    """(usable, description), probed once (``tk8s-container --probe``)."""
    ok, desc, _ = _container_probe()
    return ok, desc


def container_mode() -> str:
    """"namespaces", "ptrace", or "" (no container runtime on this node)."""
    return _container_probe()[2]


def container_argv(rootfs: str, upper: str, workdir: str, *, pid_ns: bool, gpus: list,
                   binds: list[tuple] = (), hostname: str = "", scope_signals: bool = False,
                   extra=None, layers: dict | None = None) -> list[str]:
    """argv prefix that runs a command as an image pod (see CONTAINER above). ``binds``:
    (source, path in the container[, read-only]) -- the pod's volume mounts (agent/volumes.py).
    ``layers``: the process pods' path layers (agent._jail_layers). In namespace mode the jail
    inside needs none and tk8s-container drops them: the host's tree is not the container's, and
    what the chroot leaves reachable of it (/proc/<pid>/root) is ptrace-guarded, which Landlock
    denies across domains. In ptrace mode the host's tree stays in view, so they hold there."""
    jail = gpu_jail_argv(gpus, **(layers or {}), scope_signals=scope_signals, extra=extra)[1:-1]  # options only
    argv = [str(CONTAINER), *_container_mode_opt(), "--rootfs", str(rootfs), "--upper", str(upper),
            "--workdir", workdir or "/"]
    if pid_ns:
        argv.append("--pid-ns")
    if hostname:
        argv += ["--hostname", hostname]
    for b in binds:
        src, dst, ro = (*b, False)[:3]
        argv += ["--bind-ro" if ro else "--bind", f"{src}:{dst}"]
    return argv + jail + ["--"]


def container_exec_argv(pp: "PodProc", command: list[str]) -> list[str]:
    """argv of ``kubectl exec`` into a running pod: inside its container (image pods), else under
    its GPU jail -- an exec never gets more of the node than the pod has."""
    if pp.exec_prefix and pp.proc is not None:
        return [str(CONTAINER), "--exec-in", str(pp.proc.pid), *pp.exec_prefix, *command]
    return [*pp.jail, *command]


def _sigterm_to_exit(*_):
    raise SystemExit(0)


def install_sigterm():
    signal.signal(signal.SIGTERM, _sigterm_to_exit)
