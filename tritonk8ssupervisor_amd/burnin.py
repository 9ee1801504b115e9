"""Early GPU burn-in launcher (shared by the provisioning boot hook and the rocmsetup role).

Import-light on purpose: the boot hook runs inside provisioning, on the bring-up's critical
path, and must not pull in the playbook engine's HTTP/YAML stack before the burn-in starts.
"""
from __future__ import annotations

import os
from pathlib import Path


def start_burnin(ex, host: str, command: list, out: str = "run/gpu-burnin.json", name: str = "gpu-burnin",
                 env: dict | None = None) -> dict:
    """Start `command --out <out>` on a machine's GPUs as a one-shot daemon; idempotent (a burn-in
    that is running or has finished is left alone). Every file and process action goes through
    the machine's executor, so on a remote machine the burn-in, its markers and its result all
    live on that machine."""
    gpus = ex.machine_gpus(host)
    if not gpus:
        return {"changed": False, "skipped": True, "msg": "machine has no GPUs"}
    from .models.hostinfo import compose_visible_devices

    fs = ex.fs(host)
    pending = out + ".pending"
    if fs.stat(out)["exists"] or ex.daemon_status(host, name).get("running"):
        return {"changed": False, "msg": "GPU burn-in already started", "gpus": gpus, "out": out}
    marker = fs.read(pending)
    if marker is not None and _marker_pid(marker) and ex.pid_alive(host, _marker_pid(marker)):
        return {"changed": False, "msg": "GPU burn-in pending (host-level burn-in)", "gpus": gpus, "out": out}
    denv = dict(compose_visible_devices(gpus))
    denv["NODE_NAME"] = host
    denv.update({str(k): str(v) for k, v in (env or {}).items()})
    argv = [str(a) for a in command] + ["--out", out]
    tool = ex.localize(host, argv[0])
    if os.sep in tool and not fs.stat(tool)["exists"]:
        return {"changed": False, "skipped": True, "msg": f"{tool} is not built yet"}  # the pod probes itself
    fs.write(pending, b"")
    info = ex.start_daemon(host, name, argv, env=denv, restart="no", wait_for_log=None, timeout=0)
    if not info.get("ok"):
        fs.remove(pending)
        return {"failed": True, "msg": info.get("msg", "burn-in failed to start")}
    if not fs.stat(out)["exists"]:
        # the pid lets `--reuse` stop waiting if the burn-in dies without a result
        fs.write(pending, f"{info.get('pid', 0)}\n".encode())
    return {"changed": True, "pid": info.get("pid"), "gpus": gpus, "out": out}


def _marker_pid(data: bytes) -> int:
    try:
        return int(data.split()[0])
    except (ValueError, IndexError):
        return 0


def _pid_alive(pidfile: Path) -> bool:
    try:
        pid = int(pidfile.read_text().split()[0])
    except (OSError, ValueError, IndexError):
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except (OSError, IndexError):
        return True


def split_host_result(result: dict, burnin_gpus: list[int], machine_gpus: list[int],
                      report: dict | None = None) -> dict | None:
    """One machine's share of a host burn-in: the entries of its GPUs, renumbered in the order
    the machine sees them (its pods' device i = machine_gpus[i]). None if any GPU is missing.
    With peer pulls in the result, the share also carries ``xgmi``: the host-wide link verdict
    (xgmi.link_report) for the links into and out of this machine's GPUs."""
    pos = {g: i for i, g in enumerate(burnin_gpus)}
    if not machine_gpus or any(g not in pos for g in machine_gpus):
        return None
    devs = {d.get("device"): d for d in result.get("devices", [])}
    info = result.get("gpuinfo") or {}
    infos = {d.get("index"): d for d in info.get("devices", [])}
    links = info.get("links") or []
    sub_devs, sub_info = [], []
    mine = {pos[g] for g in machine_gpus}
    for i, g in enumerate(machine_gpus):
        d = devs.get(pos[g])
        if d is None:
            return None
        # The machine is judged on its own GPUs: their HBM/MD5/copy checks and the xGMI pulls
        # between them. Pulls from other machines' GPUs are the fabric's business (the RCCL Job
        # validates it cluster-wide once every node is Ready); they are kept for the record.
        peers = [p for p in d.get("peers") or [] if p.get("src_device") in mine]
        own = all((d.get(k) or {}).get("ok", True) for k in ("hbm", "md5", "copy")) and d.get("digest_ok", True)
        foreign_bad = any(not p.get("ok") for p in d.get("peers") or [] if p.get("src_device") not in mine)
        ok = bool(d.get("ok")) or bool(foreign_bad and own and all(p.get("ok") for p in peers) and "error" not in d)
        sub_devs.append({**d, "device": i, "host_index": g, "ok": ok, "peers": peers,
                         "host_peers": d.get("peers") or []})
        if pos[g] in infos:
            sub_info.append({**infos[pos[g]], "index": i, "host_index": g})
    idx = [pos[g] for g in machine_gpus]
    sub_links = [[links[a][b] for b in idx] for a in idx] if links and max(idx) < len(links) else []
    first = sub_devs[0]
    out = {"ok": all(d.get("ok") for d in sub_devs), "device": 0, "device_count": len(sub_devs),
           "probed": len(sub_devs), "devices": sub_devs, "host_burnin": True, "host_burnin_gpus": burnin_gpus,
           "timings_ms": result.get("timings_ms", {}),
           "gpuinfo": {**{k: v for k, v in info.items() if k not in ("devices", "links")}, "device_count": len(sub_info),
                       "devices": sub_info, "links": sub_links}}
    for key in ("hbm", "md5", "copy"):
        if key in first:
            out[key] = first[key]
    if "md5_expected" in result:
        out["md5_expected"] = result["md5_expected"]
    if report is None and any(d.get("peers") for d in result.get("devices", [])):
        from .xgmi import link_report

        report = link_report(result, burnin_gpus)
    if report is not None and report.get("pulls"):
        from .xgmi import node_view

        out["xgmi"] = node_view(report, machine_gpus)
    return out


# exit statuses of a payload that ended abnormally: abort (a GPU fault's SIGABRT), segfault, the
# watchdog / a time limit
_CRASH_RC = {-6, 134, -11, 139, 124, -9, 137}


def peer_fallback_reason(command: list, result: dict | None, rc: int | None, ngpus: int) -> str | None:
    """Why the HSA payload's pulls must be re-run through the HIP probe, or None.

    Only the HSA payload with pulls (``--peers``, two or more GPUs) falls back: it ended without a
    result (a crash, an abort, the watchdog), or one of its pulls errored -- a timeout of the
    bounded peer wait, a denied grant, a kernel error. A pull that ran and read wrong words is a
    link verdict, not a runtime failure: it is not re-run."""
    if ngpus < 2 or not command or os.path.basename(str(command[0])) != "tk8s-hsaprobe" or "--peers" not in command:
        return None
    if result is None:
        return f"the HSA payload ended without a result (exit {rc})"
    errs = [p.get("error") for d in result.get("devices") or [] for p in d.get("peers") or [] if p.get("error")]
    if errs:
        return f"{len(errs)} HSA pull(s) failed: {errs[0]}"[:300]
    if rc in _CRASH_RC:
        return f"the HSA payload exited {rc}"
    return None


def mark_hsa_peers_failed(reason: str) -> None:
    """Record in the host registry that the HSA payload's pulls failed here and the HIP probe's
    passed (earlyburn.hsa_peers_failed reads it)."""
    import json
    import time

    from .earlyburn import PEERS_MARK, registry_dir
    from .utils.fsutil import atomic_write

    try:
        os.makedirs(registry_dir(), exist_ok=True)
        atomic_write(os.path.join(registry_dir(), PEERS_MARK), json.dumps({"unix": time.time(), "reason": reason[:300]}))
    except OSError:
        pass


def merge_peer_fallback(result: dict | None, hip: dict | None, reason: str) -> dict | None:
    """The burn-in result with its pulls taken from the HIP probe's re-run. Without an HSA result
    at all, the HIP probe ran the whole validation and IS the result. Each device's ``peers`` are
    replaced, ``peers_runtime`` says "hip-fallback", and the HSA errors are kept."""
    if hip is None:
        return result
    if result is None:
        out = dict(hip)
        out["devices"] = [{**d, "peers": [{**p, "runtime": "hip"} for p in d.get("peers") or []]}
                          for d in hip.get("devices") or []]
        out.update(peers_runtime="hip-fallback", hsa_fallback_reason=reason)
        return out
    out = dict(result)
    by_dev = {i: d for i, d in enumerate(hip.get("devices") or [])}
    devs = []
    for i, d in enumerate(result.get("devices") or []):
        h = by_dev.get(i) or {}
        pulls = [{**p, "runtime": "hip"} for p in h.get("peers") or []]
        hsa_errs = [p.get("error") for p in d.get("peers") or [] if p.get("error")]
        devs.append({**d, "peers": pulls, "peers_ok": bool(h.get("peers_ok")) and bool(pulls),
                     **({"hsa_peer_errors": hsa_errs[:4]} if hsa_errs else {})})
    out.update(devices=devs, peers_runtime="hip-fallback", hsa_fallback_reason=reason)
    return out


def run_hip_peer_fallback(command: list, env: dict, full: bool, timeout: float | None = None) -> tuple[dict | None, int]:
    """Run the pulls (``full``: the whole validation) through the HIP probe in a FRESH child
    process -- never an exec of a GPU process -- bounded; returns (its JSON, exit status)."""
    import json
    import subprocess

    from .earlyburn import hip_peer_command

    if full:
        cmd = [str(a) for a in command]
        cmd[0] = os.path.join(os.path.dirname(cmd[0]), "tk8s-probe")
        cmd = [a for a in cmd if a != "--peers-host"]
        if "--no-peer-dma" not in cmd:
            cmd.append("--no-peer-dma")
    else:
        cmd = hip_peer_command(command)
    if timeout is None:
        try:
            sync = float(env.get("TK8S_GPU_SYNC_TIMEOUT_S") or 30.0)
        except ValueError:
            sync = 30.0
        timeout = 2 * sync + 60.0
    try:
        p = subprocess.run(cmd, env=env, stdin=subprocess.DEVNULL, capture_output=True, text=True, timeout=timeout,
                           start_new_session=True)
    except (OSError, subprocess.SubprocessError):
        return None, -1
    lines = [x for x in p.stdout.strip().splitlines() if x.startswith("{")]
    try:
        return (json.loads(lines[-1]) if lines else None), p.returncode
    except ValueError:
        return None, p.returncode


class HostBurnin:
    """One burn-in process for every GPU the workers of a bring-up are about to receive.

    A GPU process's runtime start is host-wide work serialised across processes: on the MI355X
    box hsa_init takes ~50 ms alone, ~90 / ~130-150 / ~200-240 ms when 2 / 4 / 8 processes start
    together, and the same with no GPU visible at all (profiles/r1_conc/): so N per-machine
    burn-ins at N workers would cost N-fold start-up contention on the bring-up's critical path.
    This launcher starts ONE ``tk8s-probe --all-devices`` over the predicted GPU set (the runtime
    starts once; one host thread per GPU), and when it exits hands every machine its own share:
    ``<sandbox>/run/gpu-burnin.json`` with exactly that machine's GPUs, which the machine's
    validation pod then reuses (``--reuse``). Until then the machine's ``.pending`` marker names
    this (the setup) process, so a pod waits while the split is outstanding and probes by itself
    if the setup dies. A machine whose GPUs the burn-in did not cover, or whose share did not
    pass, gets no file and probes itself -- nothing is ever skipped, only shared.
    """

    def __init__(self, command: list, gpus: list[int], state_dir: Path, env: dict | None = None,
                 out: str = "run/gpu-burnin.json", log=None):
        self.command = [str(a) for a in command]
        self.gpus = list(gpus)
        self.state_dir = Path(state_dir)
        self.env = env or {}
        self.out = out
        self.log = log or (lambda *_a, **_k: None)
        self.result_path = self.state_dir / "run" / "host-burnin.json"
        self.pidfile = self.state_dir / "run" / "host-burnin.pid"
        self.proc = None
        self.spawned_unix = 0.0  # wall clock of the burn-in's spawn
        self.done = False
        self.result: dict | None = None
        self.xgmi: dict | None = None  # host-wide link verdict (xgmi.link_report), with peer pulls
        self.machines: dict[str, tuple[Path, list[int]]] = {}
        import threading

        self.lock = threading.Lock()
        self.finished = threading.Event()

    def start(self) -> bool:
        import subprocess
        import threading
        import time

        from .models.hostinfo import compose_visible_devices

        if os.sep in self.command[0] and not os.access(self.command[0], os.X_OK):
            self._finish(None, -1)
            return False
        self.result_path.parent.mkdir(parents=True, exist_ok=True)
        self.result_path.unlink(missing_ok=True)
        env = dict(os.environ)
        env.update(compose_visible_devices(self.gpus))
        env["NODE_NAME"] = "host"
        env.update({str(k): str(v) for k, v in self.env.items()})
        log = open(self.state_dir / "run" / "host-burnin.log", "ab")
        try:
            self.proc = subprocess.Popen(self.command + ["--out", str(self.result_path)], env=env, stdin=subprocess.DEVNULL,
                                         stdout=subprocess.DEVNULL, stderr=log, start_new_session=True)
        except OSError:
            self._finish(None, -1)
            return False
        finally:
            log.close()
        self.spawned_unix = time.time()
        self.pidfile.write_text(f"{self.proc.pid}\n")
        threading.Thread(target=self._wait, name="host-burnin", daemon=True).start()
        return True

    def adopt(self, proc, spawned_unix: float = 0.0) -> None:
        """Take over a burn-in already running this exact command over these GPUs into
        ``result_path`` (earlyburn.py started it before the CLI imported anything)."""
        import threading

        self.proc = proc
        self.spawned_unix = spawned_unix
        self.pidfile.parent.mkdir(parents=True, exist_ok=True)
        self.pidfile.write_text(f"{proc.pid}\n")
        threading.Thread(target=self._wait, name="host-burnin", daemon=True).start()

    def register(self, name: str, sandbox: str, gpus: list[int]) -> bool:
        """A machine just booted: take its share when ready. False: not covered (probe yourself)."""
        if not gpus or any(g not in self.gpus for g in gpus):
            return False
        mdir = Path(sandbox)
        pending = mdir / (self.out + ".pending")
        pending.parent.mkdir(parents=True, exist_ok=True)
        with self.lock:
            if self.done:
                self._deliver(name, mdir, gpus)
                return True
            pending.write_text(f"{os.getpid()}\n")  # alive until the share is delivered
            self.machines[name] = (mdir, list(gpus))
        return True

    def _deliver(self, name: str, mdir: Path, gpus: list[int]) -> None:
        import json

        from .utils.fsutil import atomic_write

        share = split_host_result(self.result, self.gpus, gpus, self.xgmi) if self.result else None
        if share is not None and not share["ok"]:
            # Only a passing share is handed out: a failure (or a fault of the shared run itself)
            # makes the machine's validation pod probe its GPUs on its own, which then decides.
            self.log("gpu_burnin_share_failed", name=name, gpus=gpus)
            share = None
        if share is not None and not (os.environ.get("TK8S_FAKE_GPUS") and
                                      os.environ.get("TK8S_FAKE_BURNIN_CRASH") == name):
            # the probe's own format: one compact line, "ok" first (what --reuse prints and the
            # agent parses as the pod's result)
            atomic_write(mdir / self.out, json.dumps(share, separators=(",", ":")) + "\n")
            self.log("gpu_burnin_shared", name=name, gpus=gpus, ok=share["ok"])
        (mdir / (self.out + ".pending")).unlink(missing_ok=True)

    def _wait(self) -> None:
        import json

        import time

        # The probe writes its result (atomic rename) before it exits, and a GPU process's exit
        # (runtime teardown, the driver releasing its queues and memory) takes tens of ms more:
        # hand the shares out the moment the file appears, not when the process is gone.
        rc = None
        self.seen_unix = 0.0
        while not self.result_path.exists():
            rc = self.proc.poll()
            if rc is not None:
                break
            time.sleep(0.001)
        self.seen_unix = time.time()
        result = None
        try:
            result = json.loads(self.result_path.read_text())
        except (OSError, ValueError):
            pass
        if result is None and rc is None:
            rc = self.proc.poll()
        reason = peer_fallback_reason(self.command, result, rc, len(self.gpus))
        if reason is not None:
            result = self._fallback(result, rc, reason)
        elif result is not None and "--peers" in self.command and len(self.gpus) > 1:
            result.setdefault("peers_runtime", result.get("runtime", "hip"))
        self._finish(result, rc if rc is not None else 0)
        self.proc.wait()
        self.pidfile.unlink(missing_ok=True)

    def _fallback(self, result: dict | None, rc: int | None, reason: str) -> dict | None:
        """The HSA payload's peer phase failed: wait for it to be gone (its queues released), then
        re-run the pulls -- or, with no result at all, the whole validation -- through the HIP
        probe in a fresh child process."""
        import time

        from .models.hostinfo import compose_visible_devices

        try:
            self.proc.wait(timeout=30)
        except Exception:  # noqa: BLE001 - a payload that will not exit is killed
            self.stop()
        env = dict(os.environ)
        env.update(compose_visible_devices(self.gpus))
        env["NODE_NAME"] = "host"
        env.update({str(k): str(v) for k, v in self.env.items()})
        t0 = time.time()
        hip, hrc = run_hip_peer_fallback(self.command, env, full=result is None)
        self.log("gpu_burnin_peer_fallback", reason=reason, hip_rc=hrc, ok=bool(hip and hip.get("ok")),
                 seconds=round(time.time() - t0, 3))
        merged = merge_peer_fallback(result, hip, reason)
        if hip is not None and hip.get("ok"):
            mark_hsa_peers_failed(reason)  # the next bring-ups here pull through HIP directly
        if merged is not None:
            import json

            from .utils.fsutil import atomic_write

            atomic_write(self.result_path, json.dumps(merged) + "\n")  # what the record shows
        return merged

    def _finish(self, result: dict | None, rc: int) -> None:
        """Hand every registered machine its share (or release it to probe by itself)."""
        xg = None
        if result and any(d.get("peers") for d in result.get("devices", [])):
            from .xgmi import link_report

            xg = link_report(result, self.gpus)
        with self.lock:
            self.result, self.xgmi, self.done = result, xg, True
            for name, (mdir, gpus) in self.machines.items():
                self._deliver(name, mdir, gpus)
        extra = {}
        if xg is not None:
            extra = {"xgmi_pulls": xg["pulls"], "xgmi_median_gbps": xg["median_gbps"], "xgmi_min_gbps": xg["min_gbps"],
                     "xgmi_degraded": [f"{e['src']}->{e['dst']}" for e in xg["degraded"]]}
        timings = (result or {}).get("timings_ms") or {}
        self.log("gpu_burnin_host_done", rc=rc, ok=bool(result and result.get("ok")), gpus=self.gpus,
                 runtime_init_ms=timings.get("runtime_init", timings.get("hip_init")), peers_ms=timings.get("peers"),
                 **extra)
        self.finished.set()

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            try:
                os.killpg(self.proc.pid, 15)
            except OSError:
                pass


def stop_host_burnin(state_dir: Path) -> None:
    """Teardown: kill a host burn-in a failed or interrupted bring-up left running."""
    pidfile = Path(state_dir) / "run" / "host-burnin.pid"
    if _pid_alive(pidfile):
        try:
            os.killpg(int(pidfile.read_text().split()[0]), 15)
        except (OSError, ValueError):
            pass
    pidfile.unlink(missing_ok=True)
