"""Start the host GPU burn-in before the setup CLI has imported anything.

The bring-up's critical path is the GPU burn-in (burnin.HostBurnin): ~50 ms of host-wide HIP
runtime start, a first hardware queue, a few ms of kernels (profiles/r1_init_costs,
profiles/r1_bench21/events). Everything else -- provisioning, the three plays, the joins --
finishes inside it. The orchestrator can only start it once it has imported its modules and
run the wizard (~30 ms after ``./setup.sh`` started), so a non-interactive ``./setup.sh --answers
FILE`` starts it here instead, straight from ``cli/__main__.py``, with nothing but ``os``
loaded (JSON through the C scanner): the answers file says how many workers of which package, the KFD sysfs (no GPU runtime
in this process) and the host registry say which GPUs are free, and ``os.posix_spawn`` runs the
same ``tk8s-probe`` command the orchestrator would. The orchestrator then *adopts* the process
(``take()``): the provider prefers exactly these GPUs for the workers, and if its own plan
differs in any way (command, GPU set, result path) it kills the early run and starts its own,
so the early start can only save time, never change what is validated.

This module is import-light on purpose (it also holds the helpers the heavy modules share with
it: visibility env composition, the KFD GPU walk, the validation command, the registry path).
"""
from __future__ import annotations

import os
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(PKG, "bin")
KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _loads(text: str):
    """json.loads through the C scanner alone: ``import json`` pulls in ``re`` (~4-8 ms of
    interpreter work, the largest import on this path); ``_json`` is ~0.5 ms."""
    try:
        import _json
    except ImportError:  # pragma: no cover - CPython always has it
        import json

        return json.loads(text)

    class _Ctx:
        strict = True
        object_hook = object_pairs_hook = None
        parse_float, parse_int, parse_constant = float, int, float

    s = text.strip()
    if not s:
        raise ValueError("empty document")
    obj, end = _json.make_scanner(_Ctx())(s, 0)
    if end != len(s):
        raise ValueError("extra data")
    return obj


# ---- shared helpers (re-exported by models/hostinfo.py, provider/hostreg.py, orchestrator.py) ----
def probe_tool(peers: bool = False) -> str:
    """The validation payload binary: ``tk8s-hsaprobe`` (the same kernels and checks dispatched on
    ROCr directly, ~20 ms less start-up than HIP, native/tools/tk8s_hsaprobe.cpp) unless
    ``TK8S_PROBE_RUNTIME=hip`` says otherwise or its code objects are missing: then ``tk8s-probe``
    (HIP, the same checks and JSON).

    With xGMI pulls (``peers``: two or more GPUs) the HSA payload runs too (one
    burn-in runtime at every N -- the one the driver's measurements time), unless
    ``TK8S_PEERS_RUNTIME=hip``. Its peer grants (``hsa_amd_agents_allow_access`` on another GPU's
    VRAM) are new ground on a multi-GPU box, so they have a fallback instead of a veto (ADVICE
    r2): when the HSA payload's peer phase times out, faults or crashes, burnin.HostBurnin
    re-runs the pulls through the HIP probe (``hipDeviceEnablePeerAccess``, RCCL's own P2P path)
    in a fresh child process, and each link records which runtime validated it."""
    hsa = os.path.join(BIN, "tk8s-hsaprobe")
    lib = os.path.join(PKG, "lib")
    if peers and (os.environ.get("TK8S_PEERS_RUNTIME", "hsa") == "hip" or hsa_peers_failed()):
        return os.path.join(BIN, "tk8s-probe")
    if (os.environ.get("TK8S_PROBE_RUNTIME", "hsa") != "hip" and os.access(hsa, os.X_OK)
            and os.path.exists(os.path.join(lib, "tk8s_stream.co")) and os.path.exists(os.path.join(lib, "tk8s_md5.co"))):
        return hsa
    return os.path.join(BIN, "tk8s-probe")


PEERS_MARK = "hsa-peers-failed.json"
PEERS_MARK_TTL_S = 24 * 3600.0


def hsa_peers_failed(environ=None) -> bool:
    """The host burn-in had to fall back from the HSA payload's pulls to the HIP probe within the
    last day (burnin.HostBurnin records it in the host registry): the next bring-ups on this host
    pull through the HIP probe directly, so a fabric the HSA path cannot pull costs one bring-up
    the fallback, not every one. ``TK8S_PEERS_RUNTIME=hsa`` insists on the HSA path."""
    env = os.environ if environ is None else environ
    if env.get("TK8S_PEERS_RUNTIME") == "hsa":
        return False
    import time

    try:
        with open(os.path.join(registry_dir(env), PEERS_MARK)) as f:
            mark = _loads(f.read())
        return time.time() - float(mark.get("unix", 0)) < PEERS_MARK_TTL_S
    except (OSError, ValueError, AttributeError, TypeError, StopIteration):
        return False


def default_validation_command(hbm_bytes: int = 1 << 30, md5_bytes: int = 256 << 20, iters: int = 3,
                               peers: bool = True) -> list[str]:
    """The validation DaemonSet payload (and the burn-in): every GPU of a worker; ``peers``: also
    the xGMI pulls between them (workers of more than one GPU)."""
    if os.environ.get("TK8S_FAKE_GPUS"):
        return [sys.executable, "-m", "tritonk8ssupervisor_amd.ops.fakeprobe"]
    return [probe_tool(peers), "--all-devices", "--gpuinfo", *(["--peers"] if peers else []), "--hbm-bytes",
            str(hbm_bytes), "--md5-bytes", str(md5_bytes), "--iters", str(iters)]


PEER_CHECK_BYTES = 16 << 20  # the Ready path's pull per link: ~0.25 ms at xGMI rates


def host_burnin_command(command: list[str], gpus: list[int]) -> list[str]:
    """The host burn-in runs the validation command over every worker GPU at once, so it is the
    one place that owns both ends of every xGMI link: with two or more GPUs it also pulls every
    ordered pair (``--peers``, N7) before any node can be Ready -- also when each worker has a
    single GPU, where no per-machine probe could see a link. One GPU: nothing to pull, no flag."""
    cmd = [str(a) for a in command]
    if len(gpus) > 1 and "--peers" not in cmd:
        cmd.append("--peers")
        tool = probe_tool(peers=True)
        if cmd and os.path.basename(cmd[0]) != os.path.basename(tool) and \
                os.path.basename(cmd[0]) in ("tk8s-hsaprobe", "tk8s-probe"):
            cmd[0] = tool  # the pulls' runtime (probe_tool)
    if "--peers" in cmd and "--peer-bytes" not in cmd:
        # a link check, on the Ready path: 16 MiB kernel pulls, not the standalone probes' 32-64 MiB
        cmd += ["--peer-bytes", str(PEER_CHECK_BYTES)]
        if os.path.basename(cmd[0]) == "tk8s-probe":
            cmd.append("--no-peer-dma")  # (the HIP probe's SDMA timing per pair)
    return cmd


def hip_peer_command(command: list[str]) -> list[str]:
    """The pulls of a burn-in command again, through the HIP probe only (no HBM / MD5 / copy
    probes): the HSA payload's peer-phase fallback (burnin.HostBurnin)."""
    cmd = [str(a) for a in command]
    bytes_ = cmd[cmd.index("--peer-bytes") + 1] if "--peer-bytes" in cmd[:-1] else str(PEER_CHECK_BYTES)
    iters = cmd[cmd.index("--iters") + 1] if "--iters" in cmd[:-1] else "3"
    return [os.path.join(os.path.dirname(cmd[0]) or BIN, "tk8s-probe"), "--all-devices", "--peers", "--hbm-bytes", "0",
            "--skip-md5", "--copy-bytes", "0", "--peer-bytes", bytes_, "--no-peer-dma", "--iters", iters]


def registry_dir(environ=None) -> str:
    """Where the host-wide IP/GPU claims live (provider/hostreg.py)."""
    env = os.environ if environ is None else environ
    d = env.get("TK8S_HOST_REGISTRY")
    if d:
        return d
    return os.path.join(env.get("TMPDIR") or "/tmp", f"tk8s-host-{os.getuid()}")


def idx_list(val: str | None) -> list[int] | None:
    if val is None or val.strip() == "":
        return None
    return [int(t) for t in (x.strip() for x in val.split(",")) if t.isdigit()]


def visible_filter(n: int, environ=None) -> list[int] | None:
    """Indices (into the host's KFD GPU order) this process may use: ROCR_VISIBLE_DEVICES picks
    from the host's GPUs first, then HIP_/CUDA_VISIBLE_DEVICES from what ROCr left (the order
    the ROCm runtime applies them in)."""
    env = os.environ if environ is None else environ
    view = list(range(n))
    rocr = idx_list(env.get("ROCR_VISIBLE_DEVICES"))
    if rocr is not None:
        view = [view[i] for i in rocr if i < len(view)]
    hip = idx_list(env.get("HIP_VISIBLE_DEVICES")) or idx_list(env.get("CUDA_VISIBLE_DEVICES"))
    if hip is not None:
        view = [view[i] for i in hip if i < len(view)]
    return None if rocr is None and hip is None else view


def compose_visible_devices(ordinals: list[int], environ: dict | None = None) -> dict[str, str]:
    """Env for a child that must see exactly ``ordinals`` of this process's visible GPUs.

    The restriction is applied at the ROCr level (``ROCR_VISIBLE_DEVICES`` = host GPU indices),
    so the child's runtime only initialises its own GPUs -- on an 8-GPU node a HIP start that
    brings up all eight agents in every pod and burn-in would multiply start-up cost. The HIP /
    CUDA variables are reset to the identity over that list."""
    env = os.environ if environ is None else environ
    n_hint = max(ordinals, default=-1) + 1
    view = visible_filter(max(n_hint, 64), env)
    phys = [(view[i] if view is not None else i) for i in ordinals if view is None or i < len(view)]
    ident = ",".join(str(i) for i in range(len(phys)))
    return {"ROCR_VISIBLE_DEVICES": ",".join(map(str, phys)), "HIP_VISIBLE_DEVICES": ident,
            "CUDA_VISIBLE_DEVICES": ident}


def read_props(path: str) -> dict[str, int]:
    out = {}
    try:
        with open(path) as f:
            for line in f.read().splitlines():
                parts = line.split()
                if len(parts) == 2:
                    try:
                        out[parts[0]] = int(parts[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return out


def kfd_gpu_nodes(root: str = KFD_NODES) -> list[tuple[int, dict, str]]:
    """(kfd node id, properties, node dir) of every GPU node this process may open, in KFD
    order: a non-zero ``gfx_target_version`` and SIMDs, and a render node we can read and write
    (a container may see all GPUs in sysfs but be granted a subset)."""
    try:
        names = [n for n in os.listdir(root) if n.isdigit()]
    except OSError:
        return []
    out = []
    for name in sorted(names, key=int):
        d = os.path.join(root, name)
        p = read_props(os.path.join(d, "properties"))
        if not (p.get("gfx_target_version", 0) and p.get("simd_count", 0)):
            continue
        minor = p.get("drm_render_minor", -1)
        if minor >= 0:
            dev = f"/dev/dri/renderD{minor}"
            if not os.path.exists(dev) or not os.access(dev, os.R_OK | os.W_OK):
                continue
        out.append((int(name), p, d))
    return out


# ---- the early start ----------------------------------------------------------------------------
_VALUE_FLAGS = {"--answers", "--port", "--timeout", "--rccl-timeout", "--rccl", "--nodes", "--package", "--name",
                "--master-hostname", "--node-prefix", "--node-grace", "--rccl-max-bytes", "--rccl-op-timeout"}
_BOOL_FLAGS = {"--yes", "--json", "-v", "--verbose"}


def package_gpus(name) -> int | None:
    """GPUs per machine of a local package given by name (``mi355x-<k>gpu`` / ``cpu-only``)."""
    s = str(name)
    if s == "cpu-only":
        return 0
    if s.startswith("mi355x-") and s.endswith("gpu") and s[7:-3].isdigit():
        return int(s[7:-3])
    return None


def _host_claimed_gpus(environ=None) -> set[int]:
    try:
        with open(os.path.join(registry_dir(environ), "claims.json")) as f:
            return {int(k) for k in (_loads(f.read()) or {}).get("gpus", {})}
    except (OSError, ValueError, AttributeError, StopIteration):
        return set()


def plan(argv: list[str], environ=None, cwd: str | None = None, kfd_root: str = KFD_NODES) -> dict | None:
    """What to burn in for ``tk8s setup <argv>``, or None when this run is not a plain fresh
    non-interactive local bring-up (anything unusual is left to the orchestrator)."""
    env = os.environ if environ is None else environ
    if env.get("TK8S_HOST_BURNIN", "1") == "0" or env.get("TK8S_BACKEND", "local") != "local":
        return None
    opts: dict[str, str] = {}
    i = 0
    while i < len(argv):
        a = argv[i]
        if "=" in a and a.split("=", 1)[0] in _VALUE_FLAGS:
            k, v = a.split("=", 1)
            opts[k] = v
        elif a in _VALUE_FLAGS and i + 1 < len(argv):
            opts[a] = argv[i + 1]
            i += 1
        elif a not in _BOOL_FLAGS:
            return None  # --resume, --no-validate, probe sizes, rocprof, ...: the orchestrator decides
        i += 1
    answers_file = opts.get("--answers")
    if not answers_file:
        return None
    cwd = cwd or os.getcwd()
    ws = env.get("TK8S_WORKDIR") or cwd
    answers_path = os.path.join(cwd, answers_file)  # as the CLI opens it: relative to the cwd
    if (os.path.exists(os.path.join(ws, "config")) or os.path.exists(os.path.join(ws, "terraform", "rancher.tf"))
            or not answers_path.endswith(".json")):
        return None
    try:
        with open(answers_path) as f:
            answers = {str(k).lower(): v for k, v in _loads(f.read()).items()}
    except (OSError, ValueError, AttributeError, StopIteration):
        return None
    nodes = str(opts.get("--nodes", answers.get("nodes", 1)) or 1)
    per = package_gpus(opts.get("--package", answers.get("package") or "mi355x-1gpu"))
    if not (len(nodes) == 1 and nodes in "123456789") or per is None:
        return None
    count = int(nodes) * per
    free: list[int] = []
    cmd = None  # cpu-only workers: nothing to burn in, but the zygotes still pay off
    if count:
        fake = env.get("TK8S_FAKE_GPUS")
        if fake:
            free = list(range(int(fake)))
        else:
            n = len(kfd_gpu_nodes(kfd_root))
            vis = visible_filter(n, env)
            claimed = _host_claimed_gpus(env)
            free = [i for i in range(len(vis) if vis is not None else n) if i not in claimed]
        if len(free) < count:
            return None
        # the per-machine command (peers inside a multi-GPU machine), with the host-wide pulls added
        cmd = host_burnin_command(default_validation_command(peers=per > 1), free[:count])
    state = os.path.join(ws, ".tk8s")
    master = str(opts.get("--master-hostname", answers.get("master_hostname") or "kubemaster"))
    prefix = str(opts.get("--node-prefix", answers.get("node_prefix") or "kubenode"))
    return {"gpus": free[:count], "command": cmd, "state_dir": state,
            "workers": [f"{prefix}{i}" for i in range(1, int(nodes) + 1)] if _hostname_ok(prefix) else [],
            "result": os.path.join(state, "run", "host-burnin.json"),
            # the wizard's hostname rule (^[a-zA-Z][0-9a-zA-Z]+$); anything else: no zygote
            "master": master if _hostname_ok(master) else None}


def _hostname_ok(name: str) -> bool:
    """The wizard's hostname rule (^[a-zA-Z][0-9a-zA-Z]+$): only such names get a zygote."""
    return len(name) >= 2 and name.isascii() and name.isalnum() and name[0].isalpha()


class Spawned:
    """The early burn-in process (a child of this process, its own session): Popen's poll/wait."""

    def __init__(self, pid: int):
        self.pid = pid
        self.returncode: int | None = None

    def _status(self, flags: int) -> int | None:
        if self.returncode is None:
            try:
                pid, status = os.waitpid(self.pid, flags)
            except ChildProcessError:  # reaped elsewhere: its result file is what counts
                self.returncode = -1
                return self.returncode
            if pid:
                self.returncode = os.waitstatus_to_exitcode(status)
        return self.returncode

    def poll(self) -> int | None:
        return self._status(os.WNOHANG)

    def wait(self) -> int:
        return self._status(0)


class Early:
    def __init__(self, proc: Spawned, gpus: list[int], command: list[str], result: str, spawned_unix: float = 0.0):
        self.proc, self.gpus, self.command, self.result = proc, gpus, command, result
        self.spawned_unix = spawned_unix  # wall clock of the spawn (bench: launch -> burn-in start)

    def kill(self) -> None:
        try:
            os.killpg(self.proc.pid, 15)
        except OSError:
            pass


_LAUNCHED: Early | None = None
_ZYGOTE: dict | None = None


def controlplane_zygote(p: dict) -> dict | None:
    """Start the control plane's interpreter now, under its supervisor, in the master's future
    sandbox: it imports everything (asyncio alone is ~40-60 ms of interpreter work) while the
    orchestrator starts, provisions and runs play 1, then waits for its arguments -- the master's
    address and port, known only once the machine exists -- in ``run/controlplane.args``
    (``orchestrator._boot_controlplane`` writes them). Same pidfile and log as a control plane
    started by the boot hook or the ranchermaster role, so both find it running; a restart
    re-reads the same arguments. It gives up (and stops its supervisor) if no arguments come."""
    if not p.get("master") or os.environ.get("TK8S_BOOT_CONTROLPLANE", "1") == "0" \
            or os.environ.get("TK8S_CP_ZYGOTE", "1") == "0":
        return None
    sup = os.path.join(BIN, "tk8s-supervise")
    if not os.access(sup, os.X_OK):
        return None
    sb = os.path.join(p["state_dir"], "machines", p["master"])
    pidfile = os.path.join(sb, "run", "controlplane.pid")
    if os.path.exists(pidfile):  # something of an earlier run: leave it to the orchestrator
        return None
    os.makedirs(os.path.join(sb, "run"), exist_ok=True)
    os.makedirs(os.path.join(sb, "logs"), exist_ok=True)
    args = os.path.join(sb, "run", "controlplane.args")
    _mark_zygote(os.path.join(sb, "run", "controlplane.zygote"))
    argv = [sup, "--pidfile", pidfile, "--log", os.path.join(sb, "logs", "controlplane.log"), "--restart",
            "unless-stopped", "--", sys.executable, "-S", "-c", "import tritonk8ssupervisor_amd.controlplane.__main__",
            "--await-args", args]
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.dirname(PKG)] + [x for x in env.get("PYTHONPATH", "").split(os.pathsep) if x])
    pid = os.posix_spawn(sup, argv, env, setsid=True, file_actions=[
        (os.POSIX_SPAWN_OPEN, 0, os.devnull, os.O_RDONLY, 0),
        (os.POSIX_SPAWN_OPEN, 1, os.devnull, os.O_WRONLY, 0),
        (os.POSIX_SPAWN_OPEN, 2, os.devnull, os.O_WRONLY, 0),
    ])
    return {"pid": pid, "sandbox": sb, "args": args, "pidfile": pidfile}


def _mark_zygote(path: str) -> None:
    """``run/<daemon>.zygote``: this daemon's process is a zygote until ``run/<daemon>.args`` is
    written -- the mark that lets the playbook's daemon module replace one nobody ever handed its
    arguments (playbook_modules._orphaned_zygote)."""
    with open(path, "w") as f:
        f.write(f"{os.getpid()}\n")


AGENT_ENTRY = "import tritonk8ssupervisor_amd.agent.__main__"  # = workspace.AGENT_ENTRY
_AGENTS: dict[str, dict] = {}


def agent_zygotes(p: dict) -> None:
    """Start each planned worker's node agent interpreter now, under its supervisor, in the
    worker's future sandbox: it imports everything while the orchestrator provisions, then waits
    in ``run/agent.args`` for what only the created machine knows -- its argv (name, address) and
    environment (sandbox, GPUs) -- which the worker's boot hook (orchestrator._boot_agent) writes.
    The agent then runs exactly as if started then. The supervisors are started by ONE helper
    (``tk8s-supervise --spawn-list``): os.posix_spawn holds this interpreter's GIL through each
    vfork until the exec, so N spawns here were ~5 ms of the CLI's own start at 8 workers on the
    MI355X host (profiles/r6_curve/ab_agent_zygote). Their pids come from their pidfiles."""
    if os.environ.get("TK8S_AGENT_ZYGOTE", "1") == "0" or not p.get("workers"):
        return
    sup = os.path.join(BIN, "tk8s-supervise")
    if not os.access(sup, os.X_OK):
        return
    lines = []
    for name in p["workers"]:
        sb = os.path.join(p["state_dir"], "machines", name)
        pidfile = os.path.join(sb, "run", "agent.pid")
        try:
            if os.path.exists(pidfile):  # something of an earlier run: leave it to the orchestrator
                continue
            os.makedirs(os.path.join(sb, "run"), exist_ok=True)
            os.makedirs(os.path.join(sb, "logs"), exist_ok=True)
            args = os.path.join(sb, "run", "agent.args")
            _mark_zygote(os.path.join(sb, "run", "agent.zygote"))
        except OSError:
            continue
        argv = ["--pidfile", pidfile, "--log", os.path.join(sb, "logs", "agent.log"), "--restart", "unless-stopped",
                "--", sys.executable, "-S", "-c", AGENT_ENTRY, "--await-args", args]
        if any("\t" in a or "\n" in a for a in argv):
            continue  # (the list is tab-separated; such a path gets no zygote)
        lines.append("\t".join(argv))
        _AGENTS[os.path.realpath(sb)] = {"pid": None, "sandbox": sb, "args": args, "pidfile": pidfile}
    if not lines:
        return
    spec = os.path.join(p["state_dir"], "run", "agent-zygotes.list")
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.dirname(PKG)] + [x for x in env.get("PYTHONPATH", "").split(os.pathsep) if x])
    try:
        with open(spec, "w") as f:
            f.write("\n".join(lines) + "\n")
        os.posix_spawn(sup, [sup, "--spawn-list", spec], env, file_actions=[
            (os.POSIX_SPAWN_OPEN, 0, os.devnull, os.O_RDONLY, 0),
            (os.POSIX_SPAWN_OPEN, 1, os.devnull, os.O_WRONLY, 0),
            (os.POSIX_SPAWN_OPEN, 2, os.devnull, os.O_WRONLY, 0),
        ])
    except OSError:
        _AGENTS.clear()


def agent_zygote_for(sandbox: str, wait_s: float = 0.5) -> dict | None:
    """The node agent zygote started for this worker sandbox, if any (once), with its
    supervisor's pid from the pidfile the supervisor writes as it starts (waited for briefly)."""
    import time

    z = _AGENTS.pop(os.path.realpath(sandbox), None)
    if z is None:
        return None
    deadline = time.monotonic() + wait_s
    while True:
        try:
            with open(z["pidfile"]) as f:
                z["pid"] = int(_loads(f.read())["pid"])
            return z
        except (OSError, ValueError, KeyError, TypeError):
            if time.monotonic() > deadline:
                return None
            time.sleep(0.001)


def zygote_for(sandbox: str) -> dict | None:
    """The control plane zygote started for this master sandbox, if any (once)."""
    global _ZYGOTE
    z = _ZYGOTE
    if z is not None and os.path.realpath(z["sandbox"]) == os.path.realpath(sandbox):
        _ZYGOTE = None
        return z
    return None


def _spawn_burnin(p: dict) -> Early:
    run = os.path.join(p["state_dir"], "run")
    vis = dict(compose_visible_devices(p["gpus"]))
    vis["NODE_NAME"] = "host"
    cmd = p["command"] + ["--out", p["result"]]
    log = os.path.join(run, "host-burnin.log")
    import time

    pid = os.posix_spawn(cmd[0], cmd, {**os.environ, **vis}, setsid=True, file_actions=[
        (os.POSIX_SPAWN_OPEN, 0, os.devnull, os.O_RDONLY, 0),
        (os.POSIX_SPAWN_OPEN, 1, os.devnull, os.O_WRONLY, 0),
        (os.POSIX_SPAWN_OPEN, 2, log, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644),
    ])
    spawned = time.time()
    with open(os.path.join(run, "host-burnin.pid"), "w") as f:
        f.write(f"{pid}\n")
    return Early(Spawned(pid), p["gpus"], p["command"], p["result"], spawned)


def launch(argv: list[str]) -> Early | None:
    """Called first thing by ``./setup.sh`` (cli/fast.py) for ``setup ...``: the host burn-in
    (none for cpu-only workers) and the control-plane and node-agent zygotes."""
    global _LAUNCHED, _ZYGOTE
    try:
        p = plan(argv)
        if p is None:
            return None
        os.makedirs(os.path.join(p["state_dir"], "run"), exist_ok=True)
        try:
            os.unlink(p["result"])
        except FileNotFoundError:
            pass
        if p["command"] is None:  # nothing to burn in (cpu-only workers)
            _LAUNCHED = None
        else:
            _LAUNCHED = _spawn_burnin(p)
    except Exception:  # noqa: BLE001 - an optimisation only: the orchestrator starts its own
        return None
    try:
        _ZYGOTE = controlplane_zygote(p)
    except Exception:  # noqa: BLE001 - the boot hook starts the control plane the usual way
        _ZYGOTE = None
    try:
        agent_zygotes(p)
    except Exception:  # noqa: BLE001 - the boot hooks start the agents the usual way
        pass
    return _LAUNCHED


def take() -> Early | None:
    """Hand the early burn-in (if any) to the orchestrator, once."""
    global _LAUNCHED
    e, _LAUNCHED = _LAUNCHED, None
    return e
