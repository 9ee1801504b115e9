"""Container probes (the kubelet's prober): ``startupProbe``, ``livenessProbe`` and
``readinessProbe`` with ``httpGet``, ``tcpSocket`` and ``exec`` handlers and the usual timing
fields (``initialDelaySeconds`` 0, ``periodSeconds`` 10, ``timeoutSeconds`` 1, ``failureThreshold``
3, ``successThreshold`` 1).

* startup: until it succeeds the other two do not run; ``failureThreshold`` failures kill the
  container (it restarts under the pod's restartPolicy).
* liveness: ``failureThreshold`` consecutive failures kill the container.
* readiness: decides the container's ``ready`` flag, hence the pod's Ready condition and whether
  Services send it traffic (controlplane/k8s_api.py ``_endpoints`` takes Ready pods only).

Ports are the container's (named ports resolve through ``ports[].name``), reached on the pod's
IP with the same low-port shift the pod's own listeners use (utils/net.host_port).
"""
from __future__ import annotations

import socket
import subprocess
import threading
import time
import urllib.error
import urllib.request
from typing import Callable

from ..utils.net import host_port


def _port(container: dict, port) -> int:
    if isinstance(port, str) and not port.isdigit():
        for p in container.get("ports") or []:
            if p.get("name") == port:
                return int(p["containerPort"])
        raise ValueError(f"no container port named {port!r}")
    return int(port)


def run_probe(probe: dict, container: dict, pod_ip: str, exec_argv: Callable[[list[str]], list[str]] | None = None,
              env: dict | None = None, cwd: str | None = None) -> tuple[bool, str]:
    """One probe attempt: (success, message)."""
    timeout = float(probe.get("timeoutSeconds", 1))
    try:
        if "httpGet" in probe:
            h = probe["httpGet"]
            host = h.get("host") or pod_ip
            scheme = (h.get("scheme") or "HTTP").lower()
            url = f"{scheme}://{host}:{host_port(_port(container, h.get('port', 80)))}{h.get('path') or '/'}"
            req = urllib.request.Request(url, headers={x["name"]: x["value"] for x in h.get("httpHeaders") or []})
            req.add_header("User-Agent", "kube-probe/tk8s")
            try:
                with urllib.request.urlopen(req, timeout=timeout) as r:
                    code = r.status
            except urllib.error.HTTPError as e:
                code = e.code
            return 200 <= code < 400, f"HTTP probe failed with statuscode: {code}" if not 200 <= code < 400 else ""
        if "tcpSocket" in probe:
            t = probe["tcpSocket"]
            with socket.create_connection((t.get("host") or pod_ip, host_port(_port(container, t.get("port")))), timeout):
                return True, ""
        if "exec" in probe:
            cmd = list(probe["exec"].get("command") or [])
            if not cmd:
                return False, "exec probe without a command"
            argv = exec_argv(cmd) if exec_argv else cmd
            r = subprocess.run(argv, env=env, cwd=cwd, capture_output=True, timeout=timeout)
            return r.returncode == 0, (r.stdout + r.stderr).decode(errors="replace")[-300:] if r.returncode else ""
        return False, f"probe handler {sorted(k for k in probe if k.endswith(('Get', 'Socket', 'exec', 'grpc')))} not supported"
    except (OSError, ValueError, subprocess.TimeoutExpired) as e:
        return False, str(e)


class Prober:
    """Runs one container's probes while its process lives; ``ready`` is what readiness says."""

    def __init__(self, container: dict, pod_ip: str, is_alive: Callable[[], bool], kill: Callable[[], None],
                 changed: Callable[[], None], exec_argv=None, env=None, cwd=None):
        self.c, self.ip = container, pod_ip
        self.is_alive, self.kill, self.changed = is_alive, kill, changed
        self.exec_argv, self.env, self.cwd = exec_argv, env, cwd
        self.ready = "readinessProbe" not in container
        self.started = "startupProbe" not in container
        self.last_message = ""
        self.stop = threading.Event()

    def start(self) -> None:
        if any(k in self.c for k in ("startupProbe", "livenessProbe", "readinessProbe")):
            threading.Thread(target=self._loop, name="prober", daemon=True).start()

    def _attempt(self, probe: dict) -> bool:
        ok, msg = run_probe(probe, self.c, self.ip, self.exec_argv, self.env, self.cwd)
        if not ok:
            self.last_message = msg
        return ok

    def _loop(self) -> None:
        state = {k: {"fail": 0, "ok": 0, "next": time.monotonic() + float(self.c[k].get("initialDelaySeconds", 0))}
                 for k in ("startupProbe", "livenessProbe", "readinessProbe") if k in self.c}
        while not self.stop.is_set() and self.is_alive():
            now = time.monotonic()
            for kind, st in state.items():
                if (kind != "startupProbe" and not self.started) or now < st["next"]:
                    continue
                p = self.c[kind]
                st["next"] = now + float(p.get("periodSeconds", 10))
                if kind == "startupProbe" and self.started:
                    continue
                ok = self._attempt(p)
                st["fail"], st["ok"] = (0, st["ok"] + 1) if ok else (st["fail"] + 1, 0)
                if kind == "readinessProbe":
                    want = self.ready
                    if ok and st["ok"] >= int(p.get("successThreshold", 1)):
                        want = True
                    elif not ok and st["fail"] >= int(p.get("failureThreshold", 3)):
                        want = False
                    if want != self.ready:
                        self.ready = want
                        self.changed()
                elif kind == "startupProbe" and ok:
                    self.started = True
                elif not ok and st["fail"] >= int(p.get("failureThreshold", 3)):
                    self.last_message = f"{kind} failed {st['fail']} times: {self.last_message}"
                    self.kill()  # the container restarts under the pod's restartPolicy
                    return
            nxt = min((st["next"] for st in state.values()), default=now + 1)
            self.stop.wait(max(0.02, min(1.0, nxt - time.monotonic())))
