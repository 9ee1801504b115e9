"""tk8s node agent: joins a worker to the control plane and runs its pods.

Plays the part of ``rancher/agent`` + kubelet on every HOST (ansible/roles/rancherhost/tasks/
main.yml:26-34 starts the agent with the registration URL as its only argument):

  0. (optional standby, --await-url)  start before the control plane exists; wait for the URL
  1. GET  <registrationUrl>          bootstrap (project, API prefix, heartbeat period)
  2. device plugin discovery          sysfs only — the agent never initialises the GPU
  3. POST <registrationUrl>          register the node (capacity incl. amd.com/gpu) -> node token
  4. heartbeat thread                 PUT nodes/<name>/status every period (the node lease)
  5. pod watch thread                 long-poll pods bound to this node; start/stop them via the
                                      pod runtime with the device plugin's Allocate() env

Fault points (utils/faults.py): ``agent.crash@<node>:N`` exits after registering, the first N
times (counted in the sandbox, so a restarted agent sees the count); ``agent.no_heartbeat@<node>``
stops heartbeats (lease expiry -> NotReady).
"""
from __future__ import annotations

import contextlib
import json
import os
import signal
import subprocess
import sys
import threading
import time
from pathlib import Path

from ..controlplane.client import ApiError, Client
from ..utils.faults import fault
from ..utils.k8senv import field_path, service_env
from ..utils.trace import trace
from .deviceplugin import DevicePlugin
from .volumes import VolumeError, env_name as volume_env_name, mounts as volume_mounts, volume_dirs
from .runtime import (
    PodProc, PodRuntime, container_argv, container_exec_argv, container_mode, container_runtime, gpu_jail, gpu_jail_argv,
    jail_signal_scoping,
    install_sigterm, namespace_isolation,
)

GPU = "amd.com/gpu"
ALL_GPUS = "tk8s.amd.com/all-gpus"
GPU_VISIBILITY = "tk8s.amd.com/gpu-visibility"
GPU_SCOPE = "tk8s.amd.com/gpu-scope"            # "host": the fabric Job's one process per host
HOST_LABEL = "tk8s.amd.com/host"                # which physical host a node's machine lives on
HOST_CLAIMS = "tk8s.amd.com/host-claims"        # set by the scheduler on host-scoped pods
HOST_DEVICES = "tk8s.amd.com/host-devices"
GPU_PEERS = "tk8s.amd.com/gpu-peers"            # "job": an Indexed Job's pods on one host open each other's GPUs
GPU_DEVICES = "tk8s.amd.com/gpu-devices"        # the GPUs a pod's agent gave it (node, id, host ordinal, render minor)
PEER_WAIT_S = 60.0                              # how long a gpu-peers pod waits for its peers' allocations
VALIDATION_LABEL = "tk8s.amd.com/validation"
TERMINAL = ("Succeeded", "Failed")
TK8S_HOME = str(Path(__file__).resolve().parents[2])  # this node's tk8s install root

# What of the agent's own environment a pod inherits (the rest of a pod's env is the pod spec, the
# downward API and the device plugin's Allocate()). A container starts from its image's env, not
# from the kubelet's: agent internals (TK8S_MACHINE*, TK8S_FAULTS, PYTHONPATH, credentials) never
# reach a pod. Kept: the login basics, the ROCm/HIP/HSA runtime knobs and the GPU view the node
# was given, RCCL tuning, and the tk8s fake-GPU/diagnostic switches the test tier relies on.
POD_ENV_KEEP = {"PATH", "HOME", "USER", "LOGNAME", "SHELL", "LANG", "LANGUAGE", "TZ", "TMPDIR", "TERM",
                "ROCM_PATH", "LD_LIBRARY_PATH", "CUDA_VISIBLE_DEVICES", "GPU_MAX_HW_QUEUES", "OMP_NUM_THREADS",
                "PYTORCH_ROCM_ARCH", "TK8S_TRACE", "TK8S_REMAP_PRIVILEGED_PORTS"}
POD_ENV_KEEP_PREFIXES = ("LC_", "HSA_", "HIP_", "ROCR_", "AMD_", "NCCL_", "RCCL_", "TK8S_FAKE_", "TK8S_PROBE_")


_STATE_DIRS: list[Path] | None = None


def operator_state_dirs() -> list[Path]:
    """What tk8s itself keeps for the operator outside the workspace and reads back later -- its
    state home (utils/pcache.state_home: parse/rewrite caches a poisoned entry of which the next
    ./setup.sh would run, the image store other pods' containers are made from), an explicit
    TK8S_YAML_CACHE / TK8S_IMAGE_STORE, the host registry of IP/GPU claims -- created if missing,
    so that a pod's jail can deny them (a Landlock rule needs the directory to exist)."""
    global _STATE_DIRS
    if _STATE_DIRS is not None:  # (once per agent: the agent's standby thread warms it)
        return _STATE_DIRS
    from ..provider.hostreg import registry_dir
    from ..utils.pcache import state_home

    dirs = [Path(state_home()), registry_dir()]
    for env in ("TK8S_YAML_CACHE", "TK8S_IMAGE_STORE"):
        v = os.environ.get(env, "")
        if v and v != "off":
            dirs.append(Path(v))
    home = Path.home()
    for d in dirs:
        try:
            d.mkdir(parents=True, exist_ok=True, mode=0o700)
        except OSError:
            pass
    for d in (home / ".cache", home / ".config" / "miopen"):  # the pod-writable ones (_jail_layers)
        try:  # (a rule needs them; under a read-only home a pod could not make them itself)
            d.mkdir(parents=True, exist_ok=True)
        except OSError:
            pass
    _STATE_DIRS = dirs
    return dirs


def unpacked_rccl_env(container_env: dict, merged: dict, library_dir=None) -> dict:
    """The fabric Job's ranks ask (``TK8S_RCCL_UNPACKED=1``) for RCCL with its gfx950 device code
    unpacked (utils/rccl_unpack.py): THIS node's copy -- checked against THIS node's ROCm -- goes
    in front of the library path the rank would otherwise have (the host's own path is
    kept, and a node whose copy is stale or missing loads its installed RCCL)."""
    if container_env.get("TK8S_RCCL_UNPACKED") != "1":
        return {}
    if library_dir is None:
        from ..utils.rccl_unpack import library_dir
    lib = library_dir()
    if lib is None:
        return {}
    rest = merged.get("LD_LIBRARY_PATH", "")
    return {"LD_LIBRARY_PATH": str(lib) + (":" + rest if rest else "")}


def pod_base_env(environ=None) -> dict:
    env = os.environ if environ is None else environ
    out = {k: v for k, v in env.items() if k in POD_ENV_KEEP or k.startswith(POD_ENV_KEEP_PREFIXES)}
    out["TK8S_HOME"] = TK8S_HOME
    out["TK8S_PYTHON"] = sys.executable
    return out


def node_visibility_allowed(pod: dict, job_uid=None) -> bool:
    """``gpu-visibility: node`` (a rank sees every GPU of the node, rccl-tests style) and
    ``gpu-scope: host`` are for the cluster's own fabric Jobs only: kube-system pods owned by a
    Job. ``job_uid(ns, name)`` looks the owner up (None: no such Job): an ownerReference a client
    wrote itself names no real Job, or one with another uid."""
    md = pod.get("metadata", {})
    if md.get("namespace") != "kube-system":
        return False
    owners = [r for r in md.get("ownerReferences") or [] if r.get("kind") == "Job"]
    if not owners:
        return False
    if job_uid is None:
        return True
    return any(r.get("uid") and job_uid("kube-system", r.get("name", "")) == r["uid"] for r in owners)


def host_id() -> str:
    """This host's identity for the ``tk8s.amd.com/host`` node label (a label value: at most 63
    characters of [A-Za-z0-9._-]): ``TK8S_HOST_ID`` if the provider set it, else the host name."""
    import re

    raw = os.environ.get("TK8S_HOST_ID") or os.uname().nodename or "localhost"
    v = re.sub(r"[^A-Za-z0-9._-]", "-", raw).strip("-._")[:63].strip("-._")
    return v or "localhost"


def pod_gpus(p: dict) -> int:
    total = 0
    for c in p.get("spec", {}).get("containers", []):
        r = c.get("resources", {})
        total += int(r.get("limits", {}).get(GPU, r.get("requests", {}).get(GPU, 0)) or 0)
    return total


SA_PATH = "/var/run/secrets/kubernetes.io/serviceaccount"


class _PodFail(Exception):
    """A container of the pod cannot run: the pod fails with this reason."""

    def __init__(self, reason: str, message: str):
        super().__init__(message)
        self.reason, self.message = reason, message


class ConfigError(Exception):
    """A pod's env refers to a ConfigMap/Secret (key) that does not exist (yet)."""


class Agent:
    def __init__(self, url: str | None, name: str, ip: str, sandbox: str, gpus: list[int],
                 labels: dict | None = None, tool_dirs: list[str] | None = None, timeout: float = 60.0,
                 smi_interval: float = 30.0, smi_delay: float = 5.0, device_plugin: str = "builtin"):
        self.reg_url = url
        self.name = name
        self.ip = ip
        self.sandbox = Path(sandbox)
        self.labels = dict(labels or {})
        self.labels.setdefault(HOST_LABEL, host_id())
        self.timeout = timeout
        self.plugin = DevicePlugin(gpus)
        self.runtime = PodRuntime(self.sandbox / "pods", self._on_status, tool_dirs)
        from .resources import Enforcer, Limits, gpu_local_cpus

        # the machine's shape (its package: TK8S_MACHINE_CPUS / _MEMORY_MB from the provider) and the
        # CPUs local to its GPUs, enforced on everything its pods run (agent/resources.py)
        self.shape = Limits(memory=int(float(os.environ.get("TK8S_MACHINE_MEMORY_MB", "0") or 0)) << 20 or None,
                            cpu=float(os.environ.get("TK8S_MACHINE_CPUS", "0") or 0) or None,
                            cpus=gpu_local_cpus([g.render_minor for g in self.plugin.inventory.gpus
                                                 if g.ordinal in set(gpus)]) if gpus else "")
        self.enforcer = Enforcer(name, self.shape, scope=str(self.sandbox.resolve()))
        self.runtime.enforcer = self.enforcer
        self.api: Client | None = None
        self.stop = threading.Event()
        self.hb_period = 1.0
        self.metrics_period = float(os.environ.get("TK8S_METRICS_PERIOD", "5"))
        self._sampler = None
        self._devices_dirty = False
        self._pods_meta: dict[str, dict] = {}
        self.pod_cidr = ""
        self._pod_ips: dict[str, str] = {}   # pod key -> IP
        self.smi_interval = smi_interval     # AMD SMI health period (0: off)
        self.smi_delay = smi_delay           # first sample after join, off the bring-up path
        self._annotations: dict[str, str] = {}
        self.device_plugin = device_plugin    # "builtin" (in-process core) or "grpc" (kubelet API)
        self.dp_client = None                 # kubelet-side handle on the gRPC plugin
        self.dp_servicer = None
        self.kubelet = None
        self._config_wait: dict[str, dict] = {}   # pods held in CreateContainerConfigError
        self._sa_tokens: dict[str, dict] = {}     # pod -> its bound ServiceAccount token (renewed by the heartbeat loop)
        # gpu-peers pods waiting for their Job's other pods on this host: their GPUs stay allocated
        # (published in GPU_DEVICES so the peers can find them) until the pod starts or goes away
        self._reserved: dict[str, tuple[list[str], dict, float]] = {}
        self._node_hosts: dict[str, str] = {}
        self._node_devs: dict[str, dict[str, int]] = {}
        self._peer_poller: threading.Thread | None = None
        self._registered_pods: dict | None = None   # the node's pods as the registration returned them
        self._start_lock = threading.RLock()
        self._execs_seen: set[str] = set()
        if url:
            self.set_url(url)

    def set_url(self, url: str) -> None:
        self.reg_url = url
        scheme_rest = url.split("://", 1)[1]
        self.base = "http://" + scheme_rest.split("/", 1)[0]
        self.reg_path = "/" + scheme_rest.split("/", 1)[1]

    def await_url(self, path: Path) -> None:
        """Standby (kubelet started before `join`): the interpreter, imports and device discovery
        are done before the control plane even exists; registration starts the moment the
        rancherhost role drops the registration URL into `path`."""
        delay = 0.0005
        while not self.stop.is_set():
            try:
                url = path.read_text().strip()
            except OSError:
                url = ""
            if url:
                trace(self.name, "registration url seen")
                self.set_url(url)
                return
            time.sleep(delay)
            delay = min(delay * 2, 0.001)  # one stat per ms while idle; the join starts <= 1 ms late
        raise SystemExit(0)

    # ---- device plugin over the kubelet API ----------------------------------------------
    def start_grpc_plugin(self) -> None:
        """``--device-plugin grpc``: serve the plugin core on the kubelet device-plugin API
        (agent/dp_grpc.py) and drive it from here the way the kubelet's device manager does
        (Register, ListAndWatch, GetPreferredAllocation, Allocate), over the Unix sockets."""
        from .dp_grpc import RESOURCE, GpuDevicePluginServicer, KubeletRegistry, PluginServer, socket_dir

        d = socket_dir(self.sandbox / "device-plugins")
        self.kubelet = KubeletRegistry(d).start()
        self.kubelet.on_update = lambda _c: setattr(self, "_devices_dirty", True)
        self.dp_servicer = GpuDevicePluginServicer(self.plugin, env_mode="process")
        server = PluginServer(self.dp_servicer, d, log=lambda m: print(f"{self.name}: {m}", flush=True))
        threading.Thread(target=server.serve_forever, args=(self.stop,), kwargs={"poll": 0.5},
                         name="device-plugin", daemon=True).start()
        c = self.kubelet.wait_plugin(RESOURCE, 10.0)
        if c is None or not c.wait(lambda c: c.updates > 0, 10.0):
            raise RuntimeError(f"{self.name}: the {RESOURCE} device plugin did not register over gRPC")
        self.dp_client = c
        print(f"{self.name}: kubelet device manager: {RESOURCE} via gRPC v1beta1, "
              f"{len(c.healthy())} healthy device(s)", flush=True)

    def _plugin_changed(self) -> None:
        self._devices_dirty = True
        if self.dp_servicer is not None:
            self.dp_servicer.notify()

    # ---- join -------------------------------------------------------------------------
    def join(self) -> None:
        c = Client(self.base, timeout=10.0)
        # a machine is its package's slice of the host (TK8S_MACHINE_CPUS / _MEMORY_MB): what the
        # scheduler may fit onto it, and what resources.py enforces
        cap = {"cpu": f"{self.shape.cpu:g}" if self.shape.cpu else str(os.cpu_count() or 1), "pods": "110"}
        try:
            cap["memory"] = (f"{self.shape.memory // 1024}Ki" if self.shape.memory else
                             f"{os.sysconf('SC_PAGE_SIZE') * os.sysconf('SC_PHYS_PAGES') // 1024}Ki")
        except (ValueError, OSError):
            pass
        body = {"name": self.name, "ip": self.ip, "capacity": cap, "labels": self.labels,
                "annotations": {"tk8s.amd.com/resource-enforcement": self.enforcer.describe()},
                "devices": self.plugin.devices(),
                "nodeInfo": {"osImage": _os_image(), "kernelVersion": os.uname().release,
                             "architecture": os.uname().machine, "containerRuntimeVersion": "tk8s-process://0.1",
                             "kubeletVersion": "tk8s-agent/0.1", "gpuInventory": self.plugin.inventory.source}}
        deadline = time.monotonic() + self.timeout
        delay = 0.01
        while True:  # (the registration itself is the reachability check: one request, not two)
            try:
                r = c.post(self.reg_path, body)
                break
            except (ApiError, OSError) as e:
                if isinstance(e, ApiError) and e.status < 500 or time.monotonic() > deadline:
                    raise RuntimeError(f"{self.name}: control plane unreachable at {self.base}: {e}") from e
                c.close()
                time.sleep(delay)
                delay = min(delay * 2, 1.0)
        self.hb_period = float(r.get("heartbeatSeconds", 1.0))
        self._registered_pods = r.get("pods")  # the watch's first list (watch_loop)
        self.api = Client(self.base, token=r["nodeToken"], prefix=r["apiPrefix"], timeout=10.0)
        self.pod_cidr = r.get("podCIDR") or ""
        c.close()
        try:  # lets a re-run of the rancherhost role see that this host has joined
            (self.sandbox / "run").mkdir(parents=True, exist_ok=True)
            (self.sandbox / "run" / "node-registered").write_text(f"{self.base} {r.get('projectId', '')}\n")
        except OSError:
            pass
        n = fault("agent.crash", self.name)
        if n is not None:
            counter = self.sandbox / "run" / "crash.count"
            count = int(counter.read_text()) if counter.exists() else 0
            if count < (int(n) if n is not True else 1):
                counter.parent.mkdir(parents=True, exist_ok=True)
                counter.write_text(str(count + 1))
                print(f"{self.name}: injected crash #{count + 1}", flush=True)
                os._exit(17)

    # ---- heartbeat --------------------------------------------------------------------
    def heartbeat_loop(self) -> None:
        api = Client(self.api.base, token=self.api.token, prefix=self.api.prefix, timeout=10.0)
        last_health = time.monotonic()
        # the first sample after one period: never on the bring-up's critical path
        next_metrics = time.monotonic() + self.metrics_period
        volume_period = float(os.environ.get("TK8S_VOLUME_SYNC_PERIOD", "10"))
        next_volumes = time.monotonic() + volume_period
        while not self.stop.is_set():
            if fault("agent.no_heartbeat", self.name) is None:
                body = {}
                if time.monotonic() - last_health > 10.0:
                    last_health = time.monotonic()
                    if self.plugin.refresh_health():
                        self._devices_dirty = True
                if self._devices_dirty:
                    self._devices_dirty = False
                    body["devices"] = self.plugin.devices()
                if self._annotations:
                    body["annotations"], self._annotations = self._annotations, {}
                if time.monotonic() >= next_metrics:  # CPU / memory for metrics.k8s.io (agent/usage.py)
                    next_metrics = time.monotonic() + self.metrics_period
                    body["metrics"] = self._usage_sample()
                for key, pod in list(self._config_wait.items()):  # kubelet retries config errors
                    if key not in self.runtime.running():
                        self._start_if_waiting(pod)
                if time.monotonic() >= next_volumes:  # ConfigMap/Secret/downwardAPI changes reach running pods
                    next_volumes = time.monotonic() + volume_period
                    self._sync_volumes()
                    self._renew_tokens(api)
                try:
                    api.put(api.k8s(f"/api/v1/nodes/{self.name}/status"), body)
                except ApiError as e:
                    if e.status in (401, 404):
                        print(f"{self.name}: node unknown to control plane ({e}); exiting for restart", flush=True)
                        os._exit(3)
                except OSError:
                    pass
            self.stop.wait(self.hb_period)

    def _usage_sample(self) -> dict:
        if self._sampler is None:
            from .usage import UsageSampler

            self._sampler = UsageSampler()
        groups = {}
        for key, pp in self.runtime.running().items():
            cs = {c.name or "main": c.proc.pid for c in (pp, *pp.sidecars) if c.proc is not None and c.proc.poll() is None}
            if cs:
                groups[key] = cs
        m = self._sampler.sample(groups)
        m["window"] = f"{self.metrics_period:g}s"
        # GPU busy % of each pod's GPUs (AMD SMI gfx activity, smi_loop): what a GPU-aware
        # HorizontalPodAutoscaler scales on (metrics_api.py, resource amd.com/gpu)
        busy = {d.id: (d.telemetry.get("activity") or {}).get("gfx_pct") for d in self.plugin.devices_}
        for key, pp in self.runtime.running().items():
            vals = [busy[i] for i in pp.gpu_ids if busy.get(i) is not None]
            if vals and key in m["pods"] and m["pods"][key]:
                m["pods"][key][0]["gpu_pct"] = sum(vals) / len(vals)
                m["pods"][key][0]["gpus"] = len(pp.gpu_ids)
        return m

    # ---- GPU health (AMD SMI) ------------------------------------------------------------
    def smi_loop(self) -> None:
        """Sample AMD SMI every ``smi_interval`` s through ``tk8s-smi`` (a separate process: the
        agent stays GPU-clean and a driver hiccup cannot take it down). A device with
        uncorrectable/deferred ECC errors goes Unhealthy -> leaves ``allocatable``."""
        if self.smi_interval <= 0 or not self.plugin.devices_:
            return
        if self.stop.wait(self.smi_delay):
            return
        while True:
            res = read_smi()
            if res is not None:
                changed = self.plugin.update_from_smi(res)
                self._devices_dirty = True  # telemetry rides along with the device list
                if changed:
                    self._plugin_changed()
                    bad = [d.id for d in self.plugin.devices_ if d.reason.startswith("ECC:")]
                    print(f"{self.name}: AMD SMI health changed; unhealthy: {bad or 'none'}", flush=True)
                self._annotations.update(self.plugin.telemetry_annotations())
            if self.stop.wait(self.smi_interval):
                return

    # ---- pods -------------------------------------------------------------------------
    def _pod_ip(self, key: str) -> str:
        """Next free address of this node's podCIDR (a /24 of 127.128.0.0/9; Linux answers on
        all of 127/8, so a pod can bind its own IP with no network set-up)."""
        if key in self._pod_ips:
            return self._pod_ips[key]
        if not self.pod_cidr:
            return self.ip
        base = self.pod_cidr.split("/")[0].rsplit(".", 1)[0]
        used = set(self._pod_ips.values())
        for host in range(2, 255):
            ip = f"{base}.{host}"
            if ip not in used:
                self._pod_ips[key] = ip
                return ip
        return self.ip

    def _free_devices(self) -> list[str]:
        used = set(self.runtime.held_gpus())  # (a deleted pod's GPUs stay held through its grace period)
        used.update(i for ids, _a, _t in self._reserved.values() for i in ids)
        if self.dp_client is not None:  # what the plugin's ListAndWatch last reported
            healthy = self.dp_client.healthy()
        else:
            healthy = [d["id"] for d in self.plugin.devices() if d["health"] == "Healthy"]
        return [i for i in healthy if i not in used]

    def _start_pod(self, pod: dict) -> None:
        with self._start_lock:  # the pod watch and the config-retry tick both start pods
            self._start_pod_locked(pod)

    def _start_if_waiting(self, pod: dict) -> None:
        """Retry a pod taken from a snapshot of ``_config_wait`` -- only if, under the start lock,
        it still waits there with the same uid: a pod deleted since (DELETED or a deletion
        timestamp, also handled under the lock) must not get its GPUs reserved again and start
        with no later event to stop it."""
        md = pod["metadata"]
        key = f"{md['namespace']}/{md['name']}"
        with self._start_lock:
            cur = self._config_wait.get(key)
            if cur is None or cur["metadata"].get("uid") != md.get("uid"):
                return
            self._start_pod_locked(cur)

    def _start_pod_locked(self, pod: dict) -> None:
        md, spec = pod["metadata"], pod["spec"]
        key = f"{md['namespace']}/{md['name']}"
        if key in self.runtime.running():
            return
        if self.runtime.is_terminating(key):  # the same name's previous pod is still shutting down
            self._config_wait[key] = pod
            return
        all_gpus = md.get("annotations", {}).get(ALL_GPUS) == "true"
        need = len(self.plugin.devices()) if all_gpus else pod_gpus(pod)
        # (namespaces are DNS labels, so "<ns>_<name>" cannot collide with a default-namespace pod)
        pp_dir = self.sandbox / "pods" / (md["name"] if md["namespace"] == "default" else f"{md['namespace']}_{md['name']}")
        pod_ip = self._pod_ip(key)
        # TK8S_MACHINE_DIR: the node's state dir (the hostPath the validation pod reads its
        # machine's burn-in result from)
        base = {"TK8S_HOME": TK8S_HOME, "TK8S_PYTHON": sys.executable, "TK8S_MACHINE_DIR": str(self.sandbox),
                "POD_NAME": md["name"], "POD_NAMESPACE": md["namespace"], "POD_UID": md.get("uid", ""),
                "HOSTNAME": spec.get("hostname") or md["name"],
                "POD_IP": pod_ip, "NODE_NAME": self.name, "NODE_IP": self.ip, "TK8S_API_URL": self.base,
                "TK8S_K8S_API": f"{self.base}{self.api.prefix}", "TK8S_KV_URL": f"{self.base}/v1/kv"}
        inits = list(spec.get("initContainers") or [])
        apps = list(spec["containers"])
        try:  # config first: a pod waiting for a ConfigMap must not hold GPUs
            vol_dirs = volume_dirs(pod, pp_dir, self.sandbox, self._fetch_object, pod_ip, self.ip)
            sa_dir = self._service_account_dir(pod, pp_dir)
            sa_mount = [(str(sa_dir), SA_PATH, True)] if sa_dir is not None else []
            cfg = {id(x): (self._container_env(pod, x, base, pod_ip), volume_mounts(x, vol_dirs) + [
                m for m in sa_mount if not any(v.get("mountPath") == SA_PATH for v in x.get("volumeMounts") or [])])
                for x in inits + apps}
        except (ConfigError, VolumeError) as e:
            if key not in self._config_wait:
                self._report(key, md["name"], md["namespace"], "Pending",
                             {"reason": "CreateContainerConfigError", "message": str(e)}, None)
            self._config_wait[key] = pod
            return
        self._config_wait.pop(key, None)
        trace(self.name, f"start {key}: config and volumes ready")
        ann = md.get("annotations", {})
        visibility = ann.get(GPU_VISIBILITY, "allocated")
        scope = ann.get(GPU_SCOPE, "node")
        if (visibility == "node" or scope == "host") and not node_visibility_allowed(pod, self._job_uid):
            what = f"{GPU_SCOPE}: host" if scope == "host" else f"{GPU_VISIBILITY}: node"
            self._report(key, md["name"], md["namespace"], "Failed",
                         {"reason": "Forbidden", "message": f"{what} is reserved for kube-system Jobs (the cluster's "
                                                            "RCCL fabric check)"}, None)
            return
        others: list[dict] = []
        if scope == "host":  # one process over GPUs of several nodes of this host (scheduler.py)
            try:
                claims = json.loads(ann.get(HOST_CLAIMS) or "{}")
                others = [d for d in json.loads(ann.get(HOST_DEVICES) or "[]") if d.get("node") != self.name]
                need = int(claims.get(self.name, 0))
            except (ValueError, AttributeError, TypeError):
                self._report(key, md["name"], md["namespace"], "Failed",
                             {"reason": "UnexpectedAdmissionError", "message": f"unreadable {HOST_CLAIMS}"}, None)
                return
        peers = ann.get(GPU_PEERS)
        if peers is not None and key not in self._reserved:  # (admitted once: its GPUs are reserved)
            try:
                why = self._peers_forbidden(pod, peers, need, scope, visibility)
            except (ApiError, OSError) as e:  # the control plane is busy: try again on the next tick
                if key not in self._config_wait:
                    print(f"{self.name}: {key}: cannot check its Job yet ({e})", flush=True)
                self._config_wait[key] = pod
                return
            if why:
                self._report(key, md["name"], md["namespace"], "Failed", {"reason": "Forbidden", "message": why}, None)
                return
        free = self._free_devices()
        if key in self._reserved:  # a gpu-peers pod back from waiting: it keeps what it was given
            ids, alloc, _since = self._reserved[key]
            free = list(ids)
        if need > len(free) and need <= len(free) + len(self.runtime.terminating_gpus()):
            # a deleted pod is still shutting down (its grace period): wait for its GPUs
            if key not in self._config_wait:
                self._report(key, md["name"], md["namespace"], "Pending",
                             {"reason": "ContainerCreating",
                              "message": f"waiting for {GPU} released by a terminating pod"}, None)
            self._config_wait[key] = pod
            return
        if need > len(free):
            self._report(key, md["name"], md["namespace"], "Failed",
                         {"reason": "UnexpectedAdmissionError",
                          "message": f"Allocate failed: requested {need} {GPU}, {len(free)} free"}, None)
            return
        try:
            if key in self._reserved:
                pass
            elif need and self.dp_client is not None:
                ids = self.dp_client.preferred(free, [], need)
                alloc = self.dp_client.allocate(ids)
            else:
                ids = self.plugin.preferred(free, [], need) if need else []
                alloc = self.plugin.allocate(ids) if ids else {"env": {}, "devices": [], "annotations": {}}
        except Exception as e:  # noqa: BLE001 - grpc.RpcError / allocator errors fail the pod
            self._report(key, md["name"], md["namespace"], "Failed",
                         {"reason": "UnexpectedAdmissionError", "message": f"Allocate failed: {e}"}, None)
            return
        trace(self.name, f"start {key}: allocated {','.join(ids) or 'no GPU'}")
        ordinals = [self._ordinal(i) for i in ids]
        peer_devs: list[dict] = []
        if peers is not None:
            peer_devs = self._gather_peers(pod, key, ids, alloc)
            if peer_devs is None:  # still waiting (the pod is in _config_wait, its GPUs reserved)
                return
        env = pod_base_env()
        if scope == "host":
            ordinals += [int(d["ordinal"]) for d in others]
            env.update(host_scope_env(ordinals))
        elif peer_devs:
            env.update(peer_gpu_env(ordinals, [int(d["ordinal"]) for d in peer_devs]))
            others = peer_devs  # opened and named like a host-scoped pod's other devices
        else:
            env.update(pod_gpu_env(alloc["env"], ordinals, visibility))
        env.update(base)
        env.update({volume_env_name(n): str(d) for n, (d, _ro) in vol_dirs.items()})
        if sa_dir is not None:  # process pods: the token where a client can find it (image pods: SA_PATH)
            env.update(TK8S_SERVICEACCOUNT_DIR=str(sa_dir), TK8S_SERVICEACCOUNT_TOKEN_FILE=str(sa_dir / "token"))
        env.update({"TK8S_GPU_IDS": ",".join(ids + [f"{d['node']}/{d['id']}" for d in others]),
                    "TK8S_GPU_COUNT": str(len(ordinals))})
        # GPU pods stay in the host PID namespace: HIP/RCCL inter-process sharing (dmabuf handles
        # passed by pid, RCCL's pid-keyed shared memory) needs the peers' real pids.
        gpu_pod = bool(ids) or all_gpus or visibility == "node" or bool(others)
        avail, how = namespace_isolation(str(Path(TK8S_HOME) / "tritonk8ssupervisor_amd" / "__init__.py"),
                                         str(self.sandbox / "pods"))
        isolation = "none: GPU pod (shares the host PID namespace for HIP/RCCL IPC)" if gpu_pod else how if avail \
            else f"none: {how}"
        # GPU isolation, whatever the pod does with *_VISIBLE_DEVICES: it can open exactly the
        # GPUs it holds (none for a pod without an amd.com/gpu request)
        jail_ok, jail_how = gpu_jail()
        by_ord = {g.ordinal: g for g in self.plugin.inventory.gpus}
        # node visibility (rccl-tests style ranks): the pod's runtime sees the node's GPUs
        view = [d.ordinal for d in self.plugin.devices_] if visibility == "node" and scope != "host" else ordinals
        if peer_devs:
            view = ordinals + [int(d["ordinal"]) for d in peer_devs]
        mine = [by_ord[o] for o in view if o in by_ord]
        gpu_isolation = (f"{jail_how}: may open {', '.join(f'gpu{g.ordinal}' for g in mine) or 'no GPU'}" if jail_ok
                         else f"none: {jail_how}")
        if peers is not None:
            gpu_isolation += ("; Job peers on this host: " + ", ".join(f"{d['node']}/{d['id']}" for d in peer_devs)
                              if peer_devs else "; no Job peer on this host")
        trace(self.name, f"start {key}: isolation probed")
        layers = self._jail_layers(pod, pp_dir, vol_dirs)
        clash = hostpath_clashes(layers["deny"], [v["hostPath"].get("path", "") for v in spec.get("volumes") or []
                                                  if "hostPath" in v])
        if clash:  # the jail's most specific layer wins: such a volume would re-open what is denied
            self._report(key, md["name"], md["namespace"], "Failed",
                         {"reason": "HostPathDenied",
                          "message": f"hostPath {clash[0]} is at or beneath {clash[1]}, which no pod may reach (the "
                                     "node's state, the operator's keys and caches); whatever the namespace's level"},
                         None)
            return
        from .resources import gpu_local_cpus, pod_limits

        lim = pod_limits(pod)
        if gpu_pod and scope != "host":  # on the CPUs of its GPUs' NUMA node (all_gpus: the machine's)
            own = set(ordinals)
            lim.cpus = gpu_local_cpus([g.render_minor for g in mine if g.ordinal in own or not peer_devs]) or self.shape.cpus
        try:
            limit_opts = self.enforcer.pod(key, lim, in_machine=scope != "host", gpu=gpu_pod)
        except OSError as e:
            self._report(key, md["name"], md["namespace"], "Failed",
                         {"reason": "CreateContainerError", "message": f"pod cgroup: {e}"}, None)
            return
        resources = (f"{self.enforcer.mode}: " + ", ".join(x for x in (
            f"memory {lim.memory >> 20} MiB" if lim.memory else "", f"cpu {lim.cpu:g}" if lim.cpu else "",
            f"cpus {lim.cpus}" if lim.cpus else "") if x)) if self.enforcer.mode != "none" else "none"
        if jail_ok:
            shares_pids = gpu_pod or not avail  # (image pods of CPU workloads: a PID namespace of their own)
            gpu_isolation += f"; node state denied ({', '.join(layers['deny'])})" + (
                "; signals scoped to the pod" if shares_pids and jail_signal_scoping() else
                "; shares the host PID namespace: signals not scoped (Landlock ABI < 6)" if shares_pids else "")
        trace(self.name, f"start {key}: limits set")
        procs = []
        for n, cont in enumerate(inits + apps):
            first_app = cont is apps[0]
            try:
                built = self._container_cmd(pod, cont, env, cfg[id(cont)], mine, gpu_pod, jail_ok, pp_dir, first_app,
                                            layers, limit_opts, scope_signals=gpu_pod or not avail)
            except _PodFail as e:
                self._report(key, md["name"], md["namespace"], "Failed", {"reason": e.reason, "message": e.message}, None)
                return
            if built["image"] is not None and first_app:
                isolation = f"container: {container_runtime()[1]}, image {built['image']}" + (
                    "" if gpu_pod or container_mode() != "namespaces" else ", own PID namespace")
            procs.append(PodProc(key=key if first_app else f"{key}/{cont.get('name')}", uid=md.get("uid", ""), dir=pp_dir,
                                 argv=built["argv"], env=built["env"], restart_policy=spec.get("restartPolicy", "Always"),
                                 gpu_ids=ids if first_app else [], ip=pod_ip,
                                 isolate=avail and not gpu_pod and built["image"] is None, jail=built["jail"],
                                 exec_prefix=built["exec_prefix"], name=cont.get("name") or f"c{n}", container=cont,
                                 log_name="log" if first_app else f"log.{cont.get('name') or n}",
                                 grace=float(spec.get("terminationGracePeriodSeconds", 30)), pod_key=key,
                                 limit_opts=[] if jail_ok or built["image"] is not None else limit_opts))
        pp = procs[len(inits)]
        pp.init, pp.sidecars = procs[:len(inits)], procs[len(inits) + 1:]
        self._pods_meta[key] = {"name": md["name"], "namespace": md["namespace"], "pod": pod,
                                "images": {x.get("name"): x.get("image") or "" for x in inits + apps},
                                "validation": md.get("labels", {}).get(VALIDATION_LABEL) == "true",
                                "annotations": {**alloc["annotations"], "tk8s.amd.com/log-path": str(pp_dir / "log"),
                                                "tk8s.amd.com/isolation": isolation,
                                                "tk8s.amd.com/gpu-isolation": gpu_isolation,
                                                "tk8s.amd.com/resources": resources}}
        trace(self.name, f"start {key}: handed to the runtime")
        self.runtime.start(pp)

    def _peers_forbidden(self, pod: dict, value: str, need: int, scope: str, visibility: str) -> str | None:
        """Why a ``gpu-peers`` pod may not run (None: it may). Only ``job``, only for a pod that
        holds GPUs and belongs to an Indexed Job (the real one: its uid checked against the
        control plane), never together with the fabric's own node/host GPU views. Raises
        ApiError/OSError when the control plane could not answer (the caller retries)."""
        md = pod["metadata"]
        if value != "job":
            return f'{GPU_PEERS}: only "job" is supported, not "{value}"'
        if not need:
            return f"{GPU_PEERS}: job needs an {GPU} request"
        if scope == "host" or visibility == "node":
            return f"{GPU_PEERS}: job does not combine with {GPU_SCOPE} / {GPU_VISIBILITY}"
        owners = [r for r in md.get("ownerReferences") or [] if r.get("kind") == "Job"]
        job = None
        if owners:
            try:
                job = self.api.get(self.api.k8s(f"/apis/batch/v1/namespaces/{md['namespace']}/jobs/{owners[0]['name']}"))
            except ApiError as e:
                if e.status != 404:
                    raise
                job = None
        if job is None or job["metadata"].get("uid") != owners[0].get("uid"):
            return f"{GPU_PEERS}: job is for the pods of a Job, and this pod's Job does not exist"
        if (job.get("spec") or {}).get("completionMode") != "Indexed":
            return f"{GPU_PEERS}: job is for Indexed Jobs (completionMode: Indexed)"
        return None

    def _node_host(self, node: str) -> str:
        """The physical host a node's machine lives on (its ``tk8s.amd.com/host`` label)."""
        if node == self.name:
            return self.labels[HOST_LABEL]
        if node not in self._node_hosts:
            n = self.api.get(self.api.k8s(f"/api/v1/nodes/{node}"))
            self._node_hosts[node] = (n["metadata"].get("labels") or {}).get(HOST_LABEL, f"node:{node}")
        return self._node_hosts[node]

    def _node_devices(self, node: str) -> dict[str, int]:
        """A node's GPUs as it registered them (its Node's ``status.devices``): id -> host ordinal."""
        if node == self.name:
            return {d.id: d.ordinal for d in self.plugin.devices_}
        if node not in self._node_devs:
            n = self.api.get(self.api.k8s(f"/api/v1/nodes/{node}"))
            self._node_devs[node] = {str(d.get("id")): int(d.get("ordinal", -1))
                                     for d in (n.get("status") or {}).get("devices") or [] if d.get("id")}
        return self._node_devs[node]

    def _peer_record(self, o: dict, node: str, published: str, host: str) -> list[dict]:
        """A peer pod's published GPUs, each one checked before this pod may open it:
        the record must name a GPU that the peer's node allocated to that pod (``amd.com/gpu-ids``,
        which only that node writes: admission refuses it in pods and pod templates) and that the
        node registered as its own; the ordinal and render minor are taken from the node's
        registration and this host's inventory, never from the record."""
        ann = o["metadata"].get("annotations") or {}
        given = {x for x in (ann.get("amd.com/gpu-ids") or "").split(",") if x}
        owned = self._node_devices(node)
        by_ord = {g.ordinal: g for g in self.plugin.inventory.gpus}
        out = []
        for d in json.loads(published):
            gid = str(d.get("id"))
            if d.get("node") != node or gid not in given or gid not in owned or owned[gid] not in by_ord:
                print(f"{self.name}: ignoring a gpu-devices entry of pod {o['metadata']['name']} that its node "
                      f"{node} did not allocate to it: {d}", flush=True)
                continue
            ordinal = owned[gid]
            out.append({"node": node, "id": gid, "ordinal": ordinal, "host": host,
                        "renderMinor": getattr(by_ord[ordinal], "render_minor", -1)})
        return out

    def _gather_peers(self, pod: dict, key: str, ids: list[str], alloc: dict) -> list[dict] | None:
        """The GPUs of the other live pods of this pod's Job on this host, or None while some of
        them (bound here, or not yet bound) have no GPUs yet -- for up to PEER_WAIT_S, after which
        the pod starts with the peers it found. The pod's own GPUs are published first (reserved,
        and in its GPU_DEVICES annotation), so peers started on other agents wait for each other
        without a deadlock."""
        md = pod["metadata"]
        host = self.labels[HOST_LABEL]
        if key not in self._reserved:
            self._reserved[key] = (list(ids), alloc, time.monotonic())
            by_ord = {g.ordinal: g for g in self.plugin.inventory.gpus}
            mine = [{"node": self.name, "id": i, "ordinal": self._ordinal(i), "host": host,
                     "renderMinor": getattr(by_ord.get(self._ordinal(i)), "render_minor", -1)} for i in ids]
            md.setdefault("annotations", {})[GPU_DEVICES] = json.dumps(mine, sort_keys=True)
            self._report(key, md["name"], md["namespace"], "Pending",
                         {"reason": "ContainerCreating",
                          "message": f"waiting for the GPUs of the Job's pods on this host ({GPU_PEERS}: job)"},
                         None, {**(alloc.get("annotations") or {}), GPU_DEVICES: md["annotations"][GPU_DEVICES]})
        since = self._reserved[key][2]  # (set above: deletions pop it under the same lock)
        job = next(r for r in md.get("ownerReferences") or [] if r.get("kind") == "Job")
        devices, waiting = [], []
        try:
            lst = self.api.get(self.api.k8s(f"/api/v1/namespaces/{md['namespace']}/pods"),
                               query={"labelSelector": f"job-name={job['name']}"})
            for o in lst.get("items") or []:
                om = o["metadata"]
                if (om["name"] == md["name"] or om.get("deletionTimestamp")
                        or (o.get("status") or {}).get("phase") in TERMINAL
                        or not any(r.get("uid") == job.get("uid") for r in om.get("ownerReferences") or [])):
                    continue
                nn = o["spec"].get("nodeName")
                if not nn:
                    waiting.append(om["name"])
                    continue
                if self._node_host(nn) != host:
                    continue  # on another host: RCCL reaches it over the network, nothing to open
                published = (om.get("annotations") or {}).get(GPU_DEVICES)
                if published:  # (written by that node's agent: only its own GPUs are taken)
                    devices += self._peer_record(o, nn, published, host)
                else:
                    waiting.append(om["name"])
        except (ApiError, OSError, ValueError, KeyError) as e:
            waiting.append(f"(pod list: {e})")
        if waiting and time.monotonic() - since < PEER_WAIT_S:
            self._config_wait[key] = pod
            if self._peer_poller is None or not self._peer_poller.is_alive():
                self._peer_poller = threading.Thread(target=self._poll_peers, name="gpu-peers", daemon=True)
                self._peer_poller.start()
            return None
        if waiting:
            print(f"{self.name}: {key} starts without Job peers {', '.join(waiting)} (not placed after "
                  f"{PEER_WAIT_S:.0f}s)", flush=True)
        self._reserved.pop(key, None)  # (under _start_lock: nothing allocates before the pod starts)
        return sorted(devices, key=lambda d: (d["node"], d["id"]))

    def _poll_peers(self) -> None:
        """Retry the gpu-peers pods waiting for their peers every 0.1 s (not on the 1 s config
        tick): a Job's ranks start within a poll of each other."""
        while not self.stop.wait(0.1):
            waiting = [self._config_wait.get(k) for k in list(self._reserved)]
            waiting = [p for p in waiting if p is not None]
            if not waiting:
                return
            for p in waiting:
                self._start_if_waiting(p)

    def _jail_layers(self, pod: dict, pp_dir: Path, vol_dirs: dict) -> dict:
        """What a jailed pod may not read, may only read, and may write again beneath those
        (gpujail.h; the most specific path decides):

        * denied: the node's state root (the workspace's ``.tk8s/``: admin kubeconfig and token,
          the cluster key, every machine's registration URL, other pods' directories with their
          ServiceAccount tokens and secret volumes), the workspace's Terraform state and
          ``ansible/tmp``, the operator's ``~/.ssh``, tk8s's parse caches and the host registry
          (``operator_state_dirs``: what the operator's next bring-up reads back);
        * read-only: the tk8s install, the workspace and the operator's home (the operator runs
          them: a pod that could rewrite them would run as the operator), except its ``~/.cache``
          and MIOpen's ``~/.config/miopen``;
        * read-write: the pod's own directory, its hostPath volumes (read-only ones read-only);
          validation pods (kube-system, the DaemonSet's label) consume their machine's ``run/``
          burn-in result."""
        md = pod["metadata"]
        sb = self.sandbox.resolve()
        state = sb.parent.parent if sb.parent.name == "machines" else sb
        deny, ro, rw = [str(state)], [TK8S_HOME], [str(pp_dir)]
        if state.name == ".tk8s":
            ws = state.parent
            ro.append(str(ws))
            deny += [str(x) for x in sorted((ws / "terraform").glob("terraform.tfstate*"))] + [str(ws / "ansible" / "tmp")]
        home = Path.home()
        deny += [str(home / ".ssh"), *(str(d) for d in operator_state_dirs())]
        if str(home) != "/":
            # the operator's home, read-only: its shell start-up files, ~/.local/bin on its PATH
            # and the user site-packages its interpreters load are ways into the operator's next
            # login or bring-up; the workloads' caches (~/.cache: MIOpen, torch, HF) stay writable
            ro.append(str(home))
            rw += [str(home / ".cache"), str(home / ".config" / "miopen")]  # (made by operator_state_dirs)
        for d, read_only in vol_dirs.values():
            (ro if read_only else rw).append(str(d))
        if md.get("namespace") == "kube-system" and (md.get("labels") or {}).get(VALIDATION_LABEL) == "true":
            rw.append(str(self.sandbox / "run"))  # it consumes the result (renames it: single use)
        return {"deny": deny, "read_only": ro, "allow": rw}

    def _container_cmd(self, pod: dict, c: dict, pod_env: dict, cfg: tuple, mine: list, gpu_pod: bool, jail_ok: bool,
                       pp_dir: Path, first_app: bool, layers: dict | None = None, limit_opts: list | None = None,
                       scope_signals: bool | None = None) -> dict:
        """One container's process: argv, env, and the prefix it runs under (GPU jail, or
        tk8s-container for a loaded image); raises _PodFail with the pod's failure reason."""
        md, spec = pod["metadata"], pod["spec"]
        cenv, mounts = cfg
        env = {**pod_env, **cenv}
        if scope_signals is None:
            scope_signals = gpu_pod
        argv = [_expand(str(x), env) for x in (c.get("command") or []) + (c.get("args") or [])]
        image = self._image(c.get("image"))
        if image is not None:  # a loaded image (agent/images.py): its root file system, entrypoint, env
            ok, why = container_runtime()
            if not ok:
                raise _PodFail("ContainerCannotRun", f"image {c.get('image')!r} needs a mount namespace or ptrace "
                                                     f"supervision on this node: {why}")
            store, ref = image
            img_argv, img_env, _wd = store.container_argv(ref, c.get("command"), c.get("args"))
            for k, v in img_env.items():  # the image's env, under what the pod spec sets itself
                if k not in cenv:
                    env[k] = v
            argv = [_expand(str(x), env) for x in img_argv]
        elif not c.get("command"):
            from ..apps import resolve

            entry = resolve(c.get("image"))
            if entry:  # the image's entrypoint: a built-in app (apps/__init__.py), the image's own env
                env.setdefault("PYTHONPATH", TK8S_HOME)
                argv = entry + [_expand(str(x), env) for x in (c.get("args") or [])]
        if not argv:
            raise _PodFail("ErrImageNeverPull", f"container {c.get('name')!r} has no command and image {c.get('image')!r} "
                                                "is neither loaded on this node (./tk8s image load) nor in the tk8s app "
                                                "catalogue (tritonk8ssupervisor_amd/apps)")
        # signals scoped to the pod wherever no PID namespace of its own fences them (GPU pods, and
        # CPU pods on a node without user namespaces): it cannot signal the agent or other pods
        jail = gpu_jail_argv(mine, **(layers or {}), scope_signals=scope_signals, extra=limit_opts) if jail_ok else []
        if jail and image is None and "TMPDIR" not in cenv:
            # its own temporary directory: /tmp may be on the way to a denied path (gpujail.h)
            (pp_dir / "tmp").mkdir(parents=True, exist_ok=True)
            env["TMPDIR"] = str(pp_dir / "tmp")
        exec_prefix: list[str] = []
        if image is not None:  # tk8s-container: namespaces, the image's root, the same GPU jail inside
            store, ref = image
            try:
                rootfs = store.rootfs(ref)
            except Exception as e:  # noqa: BLE001 - an unreadable image fails the pod, not the agent
                raise _PodFail("ErrImageUnpack", str(e)[:500]) from e
            workdir = c.get("workingDir") or store.container_argv(ref, None, None)[2]
            cname = str(c.get("name") or "")
            if "/" in cname or cname in ("", ".", ".."):  # a path component only (the API admits DNS labels)
                raise _PodFail("InvalidContainerName", f"container name {cname!r} is not a DNS label")
            upper = pp_dir / ("rootfs" if first_app else f"rootfs-{cname}")
            # ptrace mode keeps the host PID namespace and the host's tree in view: signals scoped
            # and the process pods' path layers, as for a process pod
            traced = container_mode() == "ptrace"
            scoped = gpu_pod or traced
            jail = container_argv(str(rootfs), str(upper), workdir, pid_ns=not gpu_pod, gpus=mine,
                                  binds=mounts, hostname=spec.get("hostname") or md["name"], scope_signals=scoped,
                                  extra=limit_opts, layers=layers)
            exec_prefix = ["--workdir", workdir, *gpu_jail_argv(mine, **(layers or {}), scope_signals=scoped,
                                                                extra=limit_opts)[1:-1], "--"]
        return {"argv": argv, "env": env, "jail": jail, "exec_prefix": exec_prefix,
                "image": image[1] if image is not None else None}

    # ---- container env (kubelet semantics) ------------------------------------------------
    def _container_env(self, pod: dict, c: dict, base: dict, pod_ip: str) -> dict:
        """Service links, then envFrom (ConfigMap/Secret, optional prefix), then env (value with
        $(VAR) expansion, or valueFrom configMapKeyRef/secretKeyRef/fieldRef) -- later wins."""
        ns = pod["metadata"]["namespace"]
        out: dict[str, str] = {}
        if pod["spec"].get("enableServiceLinks", True):
            try:
                svcs = self.api.get(self.api.k8s(f"/api/v1/namespaces/{ns}/services"))["items"]
            except (ApiError, OSError):
                svcs = []
            out.update(service_env(svcs, self.base))
        for src in c.get("envFrom") or []:
            prefix = src.get("prefix", "")
            for kind, ref in (("configmaps", src.get("configMapRef")), ("secrets", src.get("secretRef"))):
                if ref:
                    for k, v in (self._config_data(kind, ns, ref["name"], ref.get("optional", False)) or {}).items():
                        out[prefix + k] = v
        merged = {**pod_base_env(), **base, **out}
        for e in c.get("env") or []:
            if "valueFrom" in e:
                v = self._value_from(e["valueFrom"], pod, ns, pod_ip)
                if v is None:
                    continue
            else:
                v = _expand(str(e.get("value", "")), merged)
            out[e["name"]] = merged[e["name"]] = v
        out.update(unpacked_rccl_env(out, merged))
        return out

    def _service_account_dir(self, pod: dict, pp_dir: Path) -> Path | None:
        """The pod's ServiceAccount token, namespace and CA files (kubelet's projected token
        volume), unless ``automountServiceAccountToken: false``. The token is a BOUND one
        (TokenRequest): made for this pod (its uid), for the API server's audience,
        expiring after ``TK8S_SA_TOKEN_TTL_S`` (default 1 h) and renewed by the heartbeat loop at
        80 % of its life; deleting the pod revokes it -- not the namespace-wide ``<sa>-token``
        Secret every pod of the ServiceAccount used to share."""
        spec, ns = pod["spec"], pod["metadata"]["namespace"]
        if spec.get("automountServiceAccountToken") is False:
            return None
        sa = spec.get("serviceAccountName") or spec.get("serviceAccount") or "default"
        tok = self._request_token(pod, sa)
        if tok is None:
            return None
        d = pp_dir / "serviceaccount"
        d.mkdir(parents=True, exist_ok=True)
        for name, data in (("token", tok[0].encode()), ("namespace", ns.encode()), ("ca.crt", b"")):
            (d / name).write_bytes(data)
            os.chmod(d / name, 0o600 if name == "token" else 0o644)
        md = pod["metadata"]
        self._sa_tokens[f"{ns}/{md['name']}"] = {"dir": d, "sa": sa, "pod": pod, "exp": tok[1], "iat": time.time()}
        return d

    def _request_token(self, pod: dict, sa: str, api=None) -> tuple[str, float] | None:
        """A bound token for ``pod`` as ServiceAccount ``sa`` (POST .../serviceaccounts/<sa>/token)."""
        md = pod["metadata"]
        ttl = float(os.environ.get("TK8S_SA_TOKEN_TTL_S", "3600"))
        body = {"apiVersion": "authentication.k8s.io/v1", "kind": "TokenRequest",
                "spec": {"expirationSeconds": int(ttl),
                         "boundObjectRef": {"kind": "Pod", "apiVersion": "v1", "name": md["name"], "uid": md.get("uid", "")}}}
        api = api or self.api
        try:
            r = api.post(api.k8s(f"/api/v1/namespaces/{md['namespace']}/serviceaccounts/{sa}/token"), body)
        except (ApiError, OSError) as e:
            print(f"{self.name}: {md['namespace']}/{md['name']}: no ServiceAccount token ({e})", flush=True)
            return None
        st = (r or {}).get("status") or {}
        if not st.get("token"):
            return None
        left = float(((r.get("spec") or {}).get("expirationSeconds")) or ttl)
        return st["token"], time.time() + left

    def _renew_tokens(self, api) -> None:
        """Renew every running pod's bound token at 80 % of its life (kubelet's rule); drop the
        entries of pods that are gone."""
        running = self.runtime.running()
        now = time.time()
        for key, t in list(self._sa_tokens.items()):
            if key not in running:
                self._sa_tokens.pop(key, None)
                continue
            if now < t["iat"] + 0.8 * (t["exp"] - t["iat"]):
                continue
            tok = self._request_token(t["pod"], t["sa"], api)
            if tok is None:
                continue
            from ..utils.fsutil import atomic_write

            atomic_write(t["dir"] / "token", tok[0], mode=0o600)
            t.update(exp=tok[1], iat=now)

    def _fetch_object(self, kind: str, ns: str, name: str) -> dict | None:
        """A namespaced object the pod's volumes need (None: it does not exist)."""
        try:
            return self.api.get(self.api.k8s(f"/api/v1/namespaces/{ns}/{kind}/{name}"))
        except ApiError as e:
            if e.status == 404:
                return None
            raise VolumeError(f"{kind[:-1]} {name}: {e}") from e
        except OSError as e:
            raise VolumeError(f"{kind[:-1]} {name}: {e}") from e

    def _config_data(self, kind: str, ns: str, name: str, optional: bool) -> dict | None:
        try:
            o = self.api.get(self.api.k8s(f"/api/v1/namespaces/{ns}/{kind}/{name}"))
        except ApiError as e:
            if e.status == 404:
                if optional:
                    return None
                raise ConfigError(f'{kind[:-1]} "{name}" not found') from e
            raise ConfigError(f"{kind[:-1]} {name}: {e}") from e
        except OSError as e:
            raise ConfigError(f"{kind[:-1]} {name}: {e}") from e
        data = dict(o.get("data") or {})
        if kind == "secrets":
            import base64

            data = {k: base64.b64decode(v).decode(errors="replace") for k, v in data.items()}
        return data

    def _value_from(self, vf: dict, pod: dict, ns: str, pod_ip: str) -> str | None:
        if "fieldRef" in vf:
            try:
                return field_path(pod, vf["fieldRef"].get("fieldPath", ""), pod_ip, self.ip)
            except ValueError as e:
                raise ConfigError(str(e)) from e
        for kind, key in (("configmaps", "configMapKeyRef"), ("secrets", "secretKeyRef")):
            ref = vf.get(key)
            if ref:
                data = self._config_data(kind, ns, ref["name"], ref.get("optional", False))
                if data is None:
                    return None
                if ref["key"] not in data:
                    if ref.get("optional"):
                        return None
                    raise ConfigError(f"couldn't find key {ref['key']} in {kind[:-1]} {ns}/{ref['name']}")
                return data[ref["key"]]
        if "resourceFieldRef" in vf:
            r = vf["resourceFieldRef"].get("resource", "")
            lim = pod["spec"]["containers"][0].get("resources", {})
            kind, _, res = r.partition(".")
            return str(lim.get(kind, {}).get(res, "0"))
        return None

    def _on_status(self, pp: PodProc, phase: str, extra: dict) -> None:
        meta = self._pods_meta.get(pp.key, {})
        result = extra.get("result")
        if meta.get("validation") and phase in TERMINAL and isinstance(result, dict):
            result["_allocated_ids"] = pp.gpu_ids
            self.plugin.update_from_probe(result)
            self._plugin_changed()
        trace(self.name, f"report {pp.key} {phase}")
        self._report(pp.key, meta.get("name", pp.key.split("/")[1]), meta.get("namespace", "default"), phase, extra,
                     pp, meta.get("annotations"))

    def _report(self, key: str, name: str, ns: str, phase: str, extra: dict, pp: PodProc | None,
                annotations: dict | None = None) -> None:
        st = {"phase": phase, "hostIP": self.ip, "podIP": (pp.ip if pp is not None and pp.ip else self.ip)}
        if pp is not None:
            def cstatus(cp: PodProc, image: str = "") -> dict:
                alive = cp.proc is not None and cp.proc.poll() is None
                ready = alive and (cp.prober is None or cp.prober.ready)
                if alive:
                    state = {"running": {"startedAt": _rfc3339(cp.started)}}
                elif cp.exit_code is not None and phase in ("Running", "Pending") and cp.last_term:
                    # between two instances: the kubelet's back-off wait, the last exit in lastState
                    state = {"waiting": {"reason": "CrashLoopBackOff",
                                         "message": f"back-off restarting failed container {cp.name or 'main'}"}}
                elif cp.exit_code is not None:
                    state = {"terminated": {"exitCode": cp.exit_code, "reason": _term_reason(cp)}}
                else:
                    state = {"waiting": {"reason": "PodInitializing" if phase == "Pending" else "ContainerCreating"}}
                out = {"name": cp.name or "main", "image": image, "restartCount": cp.restarts, "state": state,
                       "ready": ready, "started": alive and (cp.prober is None or cp.prober.started)}
                if cp.last_term and (alive or "terminated" not in state):
                    out["lastState"] = {"terminated": dict(cp.last_term)}
                if cp.prober is not None and cp.prober.last_message and not ready:
                    out["lastProbeMessage"] = cp.prober.last_message[-300:]
                return out

            images = self._pods_meta.get(key, {}).get("images") or {}
            main = cstatus(pp, images.get(pp.name, ""))
            if phase in ("Succeeded", "Failed") and "terminated" not in main["state"]:
                main["state"] = {"terminated": {"exitCode": extra.get("exitCode", pp.exit_code),
                                                "reason": "Completed" if phase == "Succeeded" else _term_reason(pp)}}
            if (phase == "Running" and "running" not in main["state"] and pp.proc is not None
                    and (main["state"].get("waiting") or {}).get("reason") != "CrashLoopBackOff"):
                main.update(state={"running": {"startedAt": _rfc3339(pp.started)}}, ready=pp.prober is None or pp.prober.ready,
                            started=True)
            st["containerStatuses"] = [main] + [cstatus(sc, images.get(sc.name, "")) for sc in pp.sidecars]
            if pp.init:
                st["initContainerStatuses"] = [cstatus(ic, images.get(ic.name, "")) for ic in pp.init]
            st["startTime"] = _rfc3339(pp.started)
        for k in ("message", "reason", "result"):
            if extra.get(k) is not None:
                st[k] = extra[k]
        body = {"status": st}
        if annotations:
            body["annotations"] = annotations
        try:
            self.api.put(self.api.k8s(f"/api/v1/namespaces/{ns}/pods/{name}/status"), body)
            trace(self.name, f"reported {key} {phase}")
        except (ApiError, OSError) as e:
            print(f"{self.name}: status report for {key} failed: {e}", flush=True)

    def watch_loop(self) -> None:
        api = Client(self.api.base, token=self.api.token, prefix=self.api.prefix, timeout=40.0)
        path = api.k8s("/api/v1/pods")
        q = {"fieldSelector": f"spec.nodeName={self.name}"}
        rv = 0
        first = True
        while not self.stop.is_set():
            try:
                if first:
                    lst, self._registered_pods = self._registered_pods or api.get(path, query=q), None
                    rv = int(lst.get("resourceVersion") or lst["metadata"]["resourceVersion"])
                    for pod in lst["items"]:
                        self._handle("ADDED", pod)
                    first = False
                rv, events = api.watch(path, rv, timeout=20.0, query=q)
                for ev in events:
                    self._handle(ev["type"], ev["object"])
            except (ApiError, OSError) as e:
                if self.stop.is_set():
                    return
                print(f"{self.name}: watch error {e}; retrying", flush=True)
                first = True
                self.stop.wait(0.2)

    def exec_loop(self) -> None:
        """Exec requests for this node's pods (kubectl exec): run the command with the pod's env
        in the pod's directory, post stdout/stderr/exit code back."""
        api = Client(self.api.base, token=self.api.token, prefix=self.api.prefix, timeout=40.0)
        path = api.k8s(f"/api/v1/nodes/{self.name}/execs")
        while not self.stop.is_set():
            try:
                items = api.get(path, query={"timeoutSeconds": "20"})["items"]
            except (ApiError, OSError):
                if self.stop.wait(0.5):
                    return
                continue
            for x in items:
                threading.Thread(target=self._run_exec, args=(x,), name="exec", daemon=True).start()

    def _run_exec(self, x: dict) -> None:
        xid = x["metadata"]["name"]
        if xid in self._execs_seen:
            return
        self._execs_seen.add(xid)
        pp = self.runtime.running().get(f"{x['namespace']}/{x['pod']}")
        if x.get("stream"):
            (self._run_attach_stream if x.get("attach") else self._run_exec_stream)(x, pp)
            return
        if pp is None or pp.done.is_set():
            res = {"stdout": "", "stderr": f"pod {x['pod']} is not running on {self.name}\n", "exitCode": 1}
        else:
            env = dict(pp.env)
            if self.runtime.tool_dirs:
                env["PATH"] = os.pathsep.join(self.runtime.tool_dirs + [env.get("PATH", os.environ.get("PATH", ""))])
            import base64

            # bytes both ways (kubectl cp streams tar archives through exec)
            stdin = base64.b64decode(x["stdin_b64"]) if x.get("stdin_b64") else str(x.get("stdin", "")).encode()
            try:
                r = subprocess.run(container_exec_argv(pp, list(x["command"])), input=stdin, env=env, cwd=pp.dir,
                                   capture_output=True, timeout=float(x.get("timeoutSeconds", 60)))
                res = {"stdout_b64": base64.b64encode(r.stdout).decode(), "stderr_b64": base64.b64encode(r.stderr).decode(),
                       "exitCode": r.returncode}
            except FileNotFoundError as e:
                res = {"stdout": "", "stderr": f"exec: {e}\n", "exitCode": 127}
            except subprocess.TimeoutExpired as e:
                res = {"stdout_b64": base64.b64encode(e.stdout or b"").decode(),
                       "stderr": f"exec: timed out after {e.timeout}s\n", "exitCode": 124}
        try:
            self.api.put(self.api.k8s(f"/api/v1/nodes/{self.name}/execs/{xid}"), res)
        except (ApiError, OSError) as e:
            print(f"{self.name}: exec {xid} result not delivered: {e}", flush=True)

    def _run_exec_stream(self, x: dict, pp) -> None:
        """An interactive exec (``kubectl exec -it``): the command runs on a pseudo-terminal
        inside the pod's container or GPU jail (container_exec_argv, like every exec), and its
        bytes stream over a WebSocket to the control plane (k8s_api.h_exec_stream), which relays
        them to the client with the channel bytes of the Kubernetes protocol: 0 stdin and 4
        resize ({"Width", "Height"}) come in, 1 the terminal's output and 3 the final Status go
        out. [255, 0] (the client closed stdin) is the terminal's end of file; the client going
        away (0xfe from the relay, or the stream closing) hangs the terminal up (SIGHUP)."""
        import fcntl
        import pty
        import struct
        import termios
        from urllib.parse import urlsplit

        from ..controlplane.k8s_api import exec_status
        from ..controlplane.wsclient import WSClient

        xid = x["metadata"]["name"]
        u = urlsplit(self.api.base)
        try:
            ws = WSClient.connect(u.hostname, u.port or 80, f"{self.api.prefix}/api/v1/nodes/{self.name}/execs/{xid}/stream",
                                  token=self.api.token, protocols=("tk8s.exec.v1",))
        except OSError as e:
            print(f"{self.name}: exec {xid}: stream not opened: {e}", flush=True)
            return
        send_lock = threading.Lock()

        def send(b: bytes) -> None:
            with send_lock:
                try:
                    ws.send(b)
                except OSError:
                    pass

        if pp is None or pp.done.is_set():
            send(b"\x01" + f"pod {x['pod']} is not running on {self.name}\r\n".encode())
            send(b"\x03" + json.dumps(exec_status(1)).encode())
            ws.close()
            return
        env = dict(pp.env)
        env.setdefault("TERM", "xterm")
        if self.runtime.tool_dirs:
            env["PATH"] = os.pathsep.join(self.runtime.tool_dirs + [env.get("PATH", os.environ.get("PATH", ""))])
        try:
            if fault("node.no_pty", self.name) is not None:
                raise OSError("out of pty devices (injected: node.no_pty)")
            master, slave = pty.openpty()
        except OSError as e:  # a node without pseudo-terminals (no devpts: the MI355X GPU boxes)
            self._run_exec_pipes(x, pp, ws, send, env, e)
            return

        def controlling_tty():  # the child's own session, the terminal as its controlling tty
            os.setsid()
            fcntl.ioctl(0, termios.TIOCSCTTY, 0)

        try:
            proc = subprocess.Popen(container_exec_argv(pp, list(x["command"])), stdin=slave, stdout=slave, stderr=slave,
                                    env=env, cwd=pp.dir, preexec_fn=controlling_tty, close_fds=True)
        except OSError as e:
            os.close(master)
            os.close(slave)
            send(b"\x01" + f"exec: {e}\r\n".encode())
            send(b"\x03" + json.dumps(exec_status(127)).encode())
            ws.close()
            return
        os.close(slave)

        def inbound():  # stdin and resizes from the client
            while True:
                m = ws.recv()
                if m is not None and m[:2] == b"\xff\x00":  # stdin closed: ^D, end of file on the terminal
                    try:
                        os.write(master, b"\x04")
                    except OSError:
                        pass
                    continue
                if m is None or m[:1] == b"\xfe":
                    if proc.poll() is None:  # the client hung up: so does the terminal
                        try:
                            os.killpg(proc.pid, signal.SIGHUP)
                        except OSError:
                            pass
                    return
                ch, data = m[:1], m[1:]
                try:
                    if ch == b"\x00" and data:
                        os.write(master, data)
                    elif ch == b"\x04" and data:
                        sz = json.loads(data)
                        fcntl.ioctl(master, termios.TIOCSWINSZ,
                                    struct.pack("HHHH", int(sz.get("Height", 24)), int(sz.get("Width", 80)), 0, 0))
                except (OSError, ValueError, TypeError):
                    pass

        threading.Thread(target=inbound, name=f"exec-{xid}-in", daemon=True).start()
        while True:  # the terminal's output until the command has exited and the pty is drained
            try:
                data = os.read(master, 65536)
            except OSError:  # EIO: every slave end is closed
                break
            if not data:
                break
            send(b"\x01" + data)
        code = proc.wait()
        os.close(master)
        send(b"\x03" + json.dumps(exec_status(code if code >= 0 else 128 - code)).encode())
        ws.close()

    def _run_exec_pipes(self, x: dict, pp, ws, send, env: dict, why: Exception) -> None:
        """``exec -it`` on a node with no pseudo-terminal (no devpts): the command runs on pipes
        instead -- the keystrokes to its stdin, its stdout and stderr back as they come, [255, 0]
        its end of file, the client going away its SIGHUP -- a line-based session rather than a
        terminal, which its first line says."""
        from ..controlplane.k8s_api import exec_status

        send(b"\x01" + f"(no pseudo-terminal on node {self.name}: {why}; running without a tty)\r\n".encode())
        try:
            proc = subprocess.Popen(container_exec_argv(pp, list(x["command"])), stdin=subprocess.PIPE,
                                    stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, cwd=pp.dir,
                                    start_new_session=True, close_fds=True)
        except OSError as e:
            send(b"\x01" + f"exec: {e}\r\n".encode())
            send(b"\x03" + json.dumps(exec_status(127)).encode())
            ws.close()
            return

        def inbound():
            while True:
                m = ws.recv()
                if m is None or m[:1] == b"\xfe":
                    if proc.poll() is None:
                        with contextlib.suppress(OSError):
                            os.killpg(proc.pid, signal.SIGHUP)
                    return
                with contextlib.suppress(OSError, ValueError):
                    if m[:2] == b"\xff\x00":  # the client closed its stdin
                        proc.stdin.close()
                    elif m[:1] == b"\x00" and len(m) > 1:
                        proc.stdin.write(m[1:])
                        proc.stdin.flush()

        threading.Thread(target=inbound, name=f"exec-{x['metadata']['name']}-in", daemon=True).start()
        while True:
            try:
                data = os.read(proc.stdout.fileno(), 65536)
            except OSError:
                break
            if not data:
                break
            send(b"\x01" + data)
        code = proc.wait()
        send(b"\x03" + json.dumps(exec_status(code if code >= 0 else 128 - code)).encode())
        ws.close()

    def _run_attach_stream(self, x: dict, pp) -> None:
        """``kubectl attach -i [-t]`` (and ``kubectl run -it``): a session on the stdin and output
        of a container started with ``stdin: true`` (runtime._spawn: a pipe) or ``tty: true`` (a
        pty and its output pump), over the same node stream as an interactive exec. Channel 0
        writes to the container, 4 resizes its terminal, [255, 0] ends its input when the
        container has ``stdinOnce`` (for a tty: ^D); the output goes out on channel 1 -- the pty's
        bytes, or the container log's new bytes without a tty -- and when the container ends, its
        exit status on channel 3. A client that goes away detaches: the container runs on (with
        ``stdinOnce`` its input is closed, as the kubelet does after the first session)."""
        import fcntl
        import queue
        import struct
        import termios
        from urllib.parse import urlsplit

        from ..controlplane.k8s_api import exec_status
        from ..controlplane.wsclient import WSClient
        from .runtime import close_stdin

        xid = x["metadata"]["name"]
        u = urlsplit(self.api.base)
        try:
            ws = WSClient.connect(u.hostname, u.port or 80, f"{self.api.prefix}/api/v1/nodes/{self.name}/execs/{xid}/stream",
                                  token=self.api.token, protocols=("tk8s.exec.v1",))
        except OSError as e:
            print(f"{self.name}: attach {xid}: stream not opened: {e}", flush=True)
            return
        send_lock = threading.Lock()

        def send(b: bytes) -> None:
            with send_lock:
                try:
                    ws.send(b)
                except OSError:
                    pass

        cp = None
        if pp is not None and not pp.done.is_set():
            cp = next((c for c in (pp, *pp.sidecars) if c.name == x.get("container")), pp) if x.get("container") else pp
        proc = cp.proc if cp is not None else None
        if proc is None or proc.poll() is not None:
            send(b"\x01" + f"container {x.get('container') or x['pod']} is not running on {self.name}\r\n".encode())
            send(b"\x03" + json.dumps(exec_status(1)).encode())
            ws.close()
            return
        once = bool(cp.container.get("stdinOnce"))
        tty = bool(x.get("tty")) and cp.tty_master >= 0
        detached = threading.Event()
        q: queue.Queue = queue.Queue()
        if tty:
            with cp.io_lock:
                if cp.tty_master >= 0:
                    cp.io_subs.append(q)
                else:
                    q.put(None)

        def to_container(data: bytes) -> None:
            with cp.io_lock:  # a dup: the pump may close the master while this write blocks
                fd = os.dup(cp.tty_master) if cp.tty_master >= 0 else (os.dup(cp.stdin_w) if cp.stdin_w >= 0 else -1)
            if fd < 0:
                return
            try:
                os.write(fd, data)
            finally:
                os.close(fd)

        def inbound():
            while True:
                m = ws.recv()
                if m is None or m[:1] == b"\xfe":
                    detached.set()
                    q.put(b"")
                    if once:
                        close_stdin(cp)
                    return
                ch, data = m[:1], m[1:]
                try:
                    if m[:2] == b"\xff\x00":  # the client closed its stdin
                        if once:
                            to_container(b"\x04") if tty else close_stdin(cp)
                    elif ch == b"\x00" and data and x.get("stdin", True):
                        to_container(data)
                    elif ch == b"\x04" and data and tty:
                        sz = json.loads(data)
                        with cp.io_lock:
                            if cp.tty_master >= 0:
                                fcntl.ioctl(cp.tty_master, termios.TIOCSWINSZ,
                                            struct.pack("HHHH", int(sz.get("Height", 24)), int(sz.get("Width", 80)), 0, 0))
                except (OSError, ValueError, TypeError):
                    pass

        f = None
        if not tty:  # the container log's new bytes: from before the first keystroke can reach it
            try:
                f = open(cp.dir / cp.log_name, "rb")
                f.seek(0, os.SEEK_END)
            except OSError:
                pass
        threading.Thread(target=inbound, name=f"attach-{xid}-in", daemon=True).start()
        try:
            if tty:
                while not detached.is_set():
                    data = q.get()
                    if data is None:  # the pty's last holder is gone
                        break
                    if data:
                        send(b"\x01" + data)
            elif f is not None:
                while not detached.is_set():
                    ended = proc.poll() is not None  # before the read: what it wrote last is in it
                    chunk = f.read(1 << 20)
                    if chunk:
                        send(b"\x01" + chunk)
                    elif ended:
                        break
                    else:
                        time.sleep(0.05)
            else:
                while not detached.is_set() and proc.poll() is None:
                    time.sleep(0.05)
        finally:
            if f is not None:
                f.close()
            with cp.io_lock:
                if q in cp.io_subs:
                    cp.io_subs.remove(q)
        if not detached.is_set():
            try:
                code = proc.wait(timeout=10.0)
            except subprocess.TimeoutExpired:
                code = 1
            send(b"\x03" + json.dumps(exec_status(code if code >= 0 else 128 - code)).encode())
        ws.close()

    def _handle(self, etype: str, pod: dict) -> None:
        md = pod["metadata"]
        key = f"{md['namespace']}/{md['name']}"
        if etype == "DELETED":
            with self._start_lock:  # (a waiting pod is retried under it: see _start_if_waiting)
                self._config_wait.pop(key, None)
                self._reserved.pop(key, None)
                self._pods_meta.pop(key, None)
            self.runtime.stop(key, wait=False, on_done=lambda: self._terminated(key))
            return
        if md.get("deletionTimestamp"):  # graceful deletion: stop it, then confirm the delete
            with self._start_lock:
                self._config_wait.pop(key, None)
                self._reserved.pop(key, None)
            if self.runtime.is_terminating(key):
                return  # already under way; its end confirms
            cur = self.runtime.running().get(key)
            uid = md.get("uid", "")
            if cur is not None and (not uid or cur.uid == uid):
                self.runtime.stop(key, grace=float(md.get("deletionGracePeriodSeconds", 30)), wait=False,
                                  on_done=lambda: (self._confirm_deleted(md["namespace"], md["name"], uid),
                                                   self._terminated(key)))
            else:
                self._confirm_deleted(md["namespace"], md["name"], uid)
            return
        phase = pod.get("status", {}).get("phase", "Pending")
        if phase in TERMINAL:
            return
        cur = self.runtime.running().get(key)
        if cur is not None and key in self._pods_meta and cur.uid == md.get("uid", cur.uid):
            self._pods_meta[key]["pod"] = pod  # its labels/annotations, for downwardAPI volumes
        if cur is not None and md.get("uid") and cur.uid and cur.uid != md["uid"]:
            # the same name, a new pod (a StatefulSet's replacement) whose deletion event this
            # watch did not see: the old process goes first (the new one starts when it is gone)
            self.runtime.stop(key, wait=False, on_done=lambda: self._terminated(key))
        if key not in self.runtime.running():
            trace(self.name, f"watch {etype} {key}")
            self._start_pod(pod)

    def _sync_volumes(self) -> None:
        from .volumes import has_dynamic, refresh

        for key, pp in self.runtime.running().items():
            pod = self._pods_meta.get(key, {}).get("pod")
            if pod is None or not has_dynamic(pod):
                continue
            try:
                changed = refresh(pod, pp.dir, self._fetch_object, pp.ip, self.ip)
            except OSError as e:
                print(f"{self.name}: volumes of {key} not refreshed: {e}", flush=True)
                continue
            if changed:
                trace(self.name, f"volumes of {key} updated: {','.join(changed)}")

    def _confirm_deleted(self, ns: str, name: str, uid: str) -> None:
        """The kubelet's last word on a gracefully deleted pod: its containers are gone."""
        try:
            self.api.delete(self.api.k8s(f"/api/v1/namespaces/{ns}/pods/{name}"), query={"gracePeriodSeconds": "0"},
                            body={"apiVersion": "v1", "kind": "DeleteOptions", "gracePeriodSeconds": 0,
                                  **({"preconditions": {"uid": uid}} if uid else {})})
        except ApiError as e:
            if e.status not in (404, 409):
                print(f"{self.name}: pod {ns}/{name} not confirmed deleted: {e}", flush=True)
        except OSError as e:
            print(f"{self.name}: pod {ns}/{name} not confirmed deleted: {e}", flush=True)

    def _pod_groups(self) -> dict[str, list[int]]:
        """Pod key -> the process groups of its running containers (the memory watchdog's view)."""
        out = {}
        for key, pp in self.runtime.running().items():
            gs = [c.proc.pid for c in (pp, *pp.sidecars, *pp.init) if c.proc is not None and c.proc.poll() is None]
            if gs:
                out[key] = gs
        return out

    def _terminated(self, key: str) -> None:
        """A pod's termination is over: its IP is free, and a successor of the same name may start."""
        # under the start lock: a successor of the same name (a DaemonSet's re-created pod) may be
        # between its set-up -- its cgroup, its IP, both keyed by the name -- and its start
        with self._start_lock:
            if key not in self.runtime.running():
                self._pod_ips.pop(key, None)
                self.enforcer.release(key)
        for k, nxt in list(self._config_wait.items()):  # its name, its GPUs: what waited may start now
            if k not in self.runtime.running():
                self._start_if_waiting(nxt)

    # ---- lifecycle --------------------------------------------------------------------
    def _probe_isolation(self) -> None:
        """The pod runtime's one-time probes (the GPU jail's Landlock ABI, user namespaces), each a
        child process: run while the agent waits for its registration URL, not when the first pod
        (the validation pod, on the bring-up's critical path) starts."""
        gpu_jail()
        namespace_isolation(str(Path(TK8S_HOME) / "tritonk8ssupervisor_amd" / "__init__.py"), str(self.sandbox / "pods"))
        operator_state_dirs()
        trace(self.name, "isolation probed")

    def run(self, await_url: Path | None = None) -> int:
        install_sigterm()
        from .runtime import reap_leftovers

        left = reap_leftovers(self.sandbox / "pods")  # an earlier agent of this machine was killed
        if left:
            print(f"{self.name}: ended {len(left)} process group(s) a previous agent left running: {left}", flush=True)
        threading.Thread(target=self._probe_isolation, name="isolation-probe", daemon=True).start()
        if self.device_plugin == "grpc":  # before the URL wait: off the join's critical path
            self.start_grpc_plugin()
        if not self.reg_url and await_url is not None:
            self.await_url(await_url)
        t0 = time.monotonic()
        self.join()
        trace(self.name, "joined")
        print(f"{self.name}: registered in {time.monotonic() - t0:.3f}s "
              f"({len(self.plugin.devices())} GPU, inventory={self.plugin.inventory.source})", flush=True)
        threads = [threading.Thread(target=self.heartbeat_loop, name="heartbeat", daemon=True),
                   threading.Thread(target=self.smi_loop, name="smi", daemon=True),
                   threading.Thread(target=self.watch_loop, name="pods", daemon=True),
                   threading.Thread(target=self.exec_loop, name="exec", daemon=True),
                   threading.Thread(target=self.enforcer.watch, args=(self._pod_groups, self.stop),
                                    name="memory-watchdog", daemon=True)]
        for t in threads:
            t.start()
        try:
            while not self.stop.is_set():
                self.stop.wait(1.0)
        except (SystemExit, KeyboardInterrupt):
            pass
        finally:
            self.stop.set()
            self.runtime.stop_all()
            self.enforcer.close()
            if self.kubelet is not None:
                self.kubelet.stop()
        return 0

    def _image(self, ref: str | None):
        """(store, ref) when ``ref`` is an image loaded on this node, else None."""
        if not ref:
            return None
        from .images import ImageStore

        store = ImageStore()
        return (store, ref) if store.get(ref) is not None else None

    def _job_uid(self, ns: str, name: str) -> str | None:
        """uid of the Job ns/name as the control plane has it (None: there is none)."""
        try:
            return self.api.get(self.api.k8s(f"/apis/batch/v1/namespaces/{ns}/jobs/{name}"))["metadata"].get("uid")
        except (ApiError, OSError, KeyError):
            return None

    def _ordinal(self, dev_id: str) -> int:
        return next(d.ordinal for d in self.plugin.devices_ if d.id == dev_id)


def hostpath_clashes(deny: list[str], volumes: list) -> tuple[str, str] | None:
    """The first (volume, denied path) pair where a pod's volume directory is a denied path or lies
    beneath one: in gpujail.h's layers the most specific path decides, so such a
    read-write -- or read-only -- grant would re-open the admin token, the cluster key or other
    pods' ServiceAccount tokens. A volume ABOVE a denied path is fine: the deny stays deeper."""
    if not volumes:
        return None
    den = [Path(d).resolve() for d in deny]
    for v in volumes:
        rv = Path(v).resolve()
        for d in den:
            if rv == d or d in rv.parents:
                return str(rv), str(d)
    return None


def host_scope_env(ordinals: list[int]) -> dict:
    """GPU env of a host-scoped pod: its runtime sees exactly the claimed GPUs of the host (its
    own node's and the other claimed nodes', host ordinals), named 0..n-1 in TK8S_GPU_DEVICES."""
    from ..earlyburn import compose_visible_devices

    env = compose_visible_devices(ordinals)
    env["TK8S_GPU_DEVICES"] = ",".join(str(i) for i in range(len(ordinals)))
    env["TK8S_GPU_DEVICE"] = "0" if ordinals else ""
    return env


def _rfc3339(t: float) -> str:
    """A Kubernetes timestamp (what client-go parses), from a time.time() value."""
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


def peer_gpu_env(own: list[int], peers: list[int]) -> dict:
    """GPU env of a ``gpu-peers`` pod: its runtime sees its own GPUs first (devices 0..k-1,
    TK8S_GPU_DEVICE(S)) and then its Job peers' on this host (TK8S_GPU_PEER_DEVICES) -- RCCL's
    P2P transport over xGMI connects GPUs that every rank's runtime can see."""
    from ..earlyburn import compose_visible_devices

    env = compose_visible_devices(own + peers)
    env["TK8S_GPU_DEVICES"] = ",".join(str(i) for i in range(len(own)))
    env["TK8S_GPU_DEVICE"] = "0" if own else ""
    env["TK8S_GPU_PEER_DEVICES"] = ",".join(str(len(own) + i) for i in range(len(peers)))
    return env


def pod_gpu_env(alloc_env: dict, ordinals: list[int], visibility: str = "allocated") -> dict:
    """GPU env of a pod. ``allocated`` (default): the device plugin's Allocate env, so the pod's
    runtime initialises only its own GPUs. ``node``: the pod still owns exactly its allocated GPUs
    but sees the agent's whole view, with its devices named in TK8S_GPU_DEVICE(S) -- what
    rccl-tests style ranks need, since RCCL's peer-to-peer transport over xGMI only connects
    GPUs that are visible to each rank's runtime."""
    if visibility == "node":
        return {"TK8S_GPU_DEVICES": ",".join(map(str, ordinals)),
                "TK8S_GPU_DEVICE": str(ordinals[0]) if ordinals else ""}
    return dict(alloc_env)


def _term_reason(cp) -> str:
    """A terminated container's reason, as the kubelet words it."""
    if cp.oom_killed:
        return "OOMKilled"
    return "Completed" if cp.exit_code == 0 else "Error"


def read_smi(timeout: float = 20.0) -> dict | None:
    """One AMD SMI sample (tk8s-smi, or the fake twin under TK8S_FAKE_GPUS); None if unavailable."""
    if os.environ.get("TK8S_FAKE_GPUS"):
        cmd = [sys.executable, "-S", "-m", "tritonk8ssupervisor_amd.ops.fakesmi", "--no-links"]
    else:
        tool = Path(__file__).resolve().parents[1] / "bin" / "tk8s-smi"
        if not tool.exists():
            return None
        cmd = [str(tool), "--no-links"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        return json.loads(r.stdout) if r.stdout.strip() else None
    except (OSError, subprocess.TimeoutExpired, ValueError):
        return None


def _os_image() -> str:
    """PRETTY_NAME of /etc/os-release (what kubelet reports); `platform` costs ~8 ms to import."""
    try:
        for line in Path("/etc/os-release").read_text().splitlines():
            if line.startswith("PRETTY_NAME="):
                return line.split("=", 1)[1].strip().strip('"')
    except OSError:
        pass
    return f"{os.uname().sysname} {os.uname().release}"


def _expand(s: str, env: dict) -> str:
    from .runtime import expand

    return expand(s, env)


_STR_OPTS = {"--url": "url_opt", "--name": "name", "--ip": "ip", "--sandbox": "sandbox", "--gpus": "gpus",
             "--labels": "labels", "--device-plugin": "device_plugin", "--await-url": "await_url"}
_FLOAT_OPTS = {"--timeout": "timeout", "--smi-interval": "smi_interval", "--smi-delay": "smi_delay"}


def _defaults() -> dict:
    return {"url": None, "url_opt": None, "name": os.environ.get("TK8S_MACHINE", os.uname().nodename),
            "ip": os.environ.get("TK8S_MACHINE_IP", "127.0.0.1"), "sandbox": os.environ.get("TK8S_MACHINE_DIR", "."),
            "gpus": os.environ.get("TK8S_MACHINE_GPUS", ""), "labels": "", "tool_dir": [], "timeout": 60.0,
            "smi_interval": float(os.environ.get("TK8S_SMI_INTERVAL", "30")),
            "smi_delay": float(os.environ.get("TK8S_SMI_DELAY", "5")),
            "device_plugin": os.environ.get("TK8S_DEVICE_PLUGIN", "builtin"), "await_url": None}


def _parse_fast(argv: list[str]) -> dict | None:
    """The agent's arguments without argparse (~2 ms of its start, which the bring-up waits for):
    ``--opt value`` pairs and one optional positional URL; None for anything else (``--help``,
    ``--opt=value``, unknown options, bad values), which argparse then handles."""
    a = _defaults()
    i = 0
    while i < len(argv):
        tok = argv[i]
        if not tok.startswith("-"):
            if a["url"] is not None:
                return None
            a["url"] = tok
            i += 1
            continue
        if i + 1 >= len(argv) or argv[i + 1].startswith("-"):
            return None
        val = argv[i + 1]
        if tok in _STR_OPTS:
            a[_STR_OPTS[tok]] = val
        elif tok in _FLOAT_OPTS:
            try:
                a[_FLOAT_OPTS[tok]] = float(val)
            except ValueError:
                return None
        elif tok == "--tool-dir":
            a["tool_dir"].append(val)
        else:
            return None
        i += 2
    if a["device_plugin"] not in ("builtin", "grpc"):
        return None
    return a


def _parse_argparse(argv: list[str] | None) -> dict:
    import argparse

    d = _defaults()
    ap = argparse.ArgumentParser(prog="tk8s-agent", description="tk8s node agent")
    ap.add_argument("url", nargs="?", help="registration URL (http://master:port/v1/scripts/TOKEN)")
    ap.add_argument("--url", dest="url_opt")
    ap.add_argument("--name", default=d["name"])
    ap.add_argument("--ip", default=d["ip"])
    ap.add_argument("--sandbox", default=d["sandbox"])
    ap.add_argument("--gpus", default=d["gpus"])
    ap.add_argument("--labels", default="")
    ap.add_argument("--tool-dir", action="append", default=[])
    ap.add_argument("--timeout", type=float, default=60.0)
    ap.add_argument("--smi-interval", type=float, default=d["smi_interval"],
                    help="AMD SMI health sampling period in s (0 disables)")
    ap.add_argument("--smi-delay", type=float, default=d["smi_delay"],
                    help="first AMD SMI sample this many s after joining")
    ap.add_argument("--device-plugin", choices=["builtin", "grpc"], default=d["device_plugin"],
                    help="builtin: in-process plugin core; grpc: the kubelet device-plugin API over Unix sockets")
    ap.add_argument("--await-url", default=None,
                    help="standby: wait for a file holding the registration URL (relative to --sandbox)")
    a = vars(ap.parse_args(argv))
    if not (a["url_opt"] or a["url"]) and not a["await_url"]:
        ap.error("registration URL (or --await-url FILE) is required")
    return a


def main(argv: list[str] | None = None) -> int:
    trace("agent", "imported")
    argv = sys.argv[1:] if argv is None else argv
    from .. import shortcut_on

    a = _parse_fast(argv) if shortcut_on("TK8S_FAST_ARGS") else None
    if a is None or not (a["url_opt"] or a["url"] or a["await_url"]):
        a = _parse_argparse(argv)
    url = a["url_opt"] or a["url"]
    gpus = [int(x) for x in a["gpus"].split(",") if x.strip() != ""]
    labels = dict(kv.split("=", 1) for kv in a["labels"].split(",") if "=" in kv)
    tools = a["tool_dir"] or [str(Path(__file__).resolve().parents[1] / "bin")]
    wait = Path(a["sandbox"]) / a["await_url"] if a["await_url"] else None
    return Agent(url, a["name"], a["ip"], a["sandbox"], gpus, labels, tools, a["timeout"],
                 smi_interval=a["smi_interval"], smi_delay=a["smi_delay"], device_plugin=a["device_plugin"]).run(wait)


if __name__ == "__main__":
    sys.exit(main())
