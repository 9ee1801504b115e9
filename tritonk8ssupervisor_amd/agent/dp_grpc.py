"""``amd.com/gpu`` device plugin on the kubelet's gRPC API (device-plugin ``v1beta1``).

The kubelet-facing half of N2. The plugin core is the one the tk8s agent uses
(``deviceplugin.DevicePlugin``: KFD-sysfs discovery that never initialises HIP, AMD SMI ECC
health, xGMI-aware preferred allocation in C++); this module serves it on a Unix socket in the
kubelet's device-plugin directory and registers it with ``kubelet.sock``, so a stock kubelet
(kubeadm / k3s / RKE2 worker on an MI355X host) schedules ``amd.com/gpu`` through it:

  plugin   serve DevicePlugin on <dir>/tk8s-amd-gpu.sock, then Registration.Register on
           <dir>/kubelet.sock (version v1beta1, resource amd.com/gpu, preferred allocation on)
  kubelet  ListAndWatch            device list, re-sent whenever a device's health changes
           GetPreferredAllocation  xGMI-connected sets (max weakest link, then total link weight)
           Allocate                /dev/kfd + the allocated /dev/dri/renderD* nodes, env, annotations

A restarting kubelet wipes the directory; ``PluginServer.serve_forever`` notices (its socket is
gone, or ``kubelet.sock`` was replaced) and serves + registers again.

Env mode. In a container (``container``, the CLI default) the runtime exposes only the allocated
render nodes, so ROCm enumerates exactly those GPUs and no ``*_VISIBLE_DEVICES`` is set (host
indices would be wrong inside the container's view). The tk8s agent's process pods share the
host's ``/dev`` (``process``): the plugin then sets ``ROCR_VISIBLE_DEVICES`` to host indices, as
the agent's built-in path does.

``KubeletRegistry`` + ``PluginClient`` are the kubelet's side (Registration service + device
manager). The tk8s agent uses them in ``--device-plugin grpc`` mode, so the local backend drives
the plugin over the same wire protocol a real kubelet speaks; the tests do too.

Reference anchor: ansible/roles/rancherhost/tasks/main.yml:26-34 joins nodes through
``rancher/agent``; the reference has no device plugin or accelerator scheduling at all.
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import tempfile
import threading
from concurrent import futures
from pathlib import Path

import grpc

from .deviceplugin import DevicePlugin
from .dp_proto import DEVICE_PLUGIN_PATH, HEALTHY, KUBELET_SOCKET, SERVICES, VERSION, codec, method_path, pb

RESOURCE = "amd.com/gpu"
ENDPOINT = "tk8s-amd-gpu.sock"
_SUN_PATH_MAX = 107  # sockaddr_un.sun_path minus its terminating NUL


def numa_node(render_minor: int) -> int:
    """NUMA node of a GPU from its DRM device (-1 if unknown)."""
    if render_minor < 0:
        return -1
    try:
        return int(Path(f"/sys/class/drm/renderD{render_minor}/device/numa_node").read_text().strip())
    except (OSError, ValueError):
        return -1


def socket_dir(path: str | os.PathLike) -> Path:
    """``path`` if the kubelet and plugin sockets fit in sun_path there, else a short private dir
    named after it (``/tmp/tk8s-dp-<uid>/<hash>``: the same one on every restart, so nothing piles
    up; ``KubeletRegistry.stop`` removes it)."""
    import hashlib

    p = Path(path).absolute()
    if len(str(p)) + 1 + max(len(ENDPOINT), len(KUBELET_SOCKET)) <= _SUN_PATH_MAX:
        p.mkdir(parents=True, exist_ok=True)
        return p
    base = Path(tempfile.gettempdir())
    if len(str(base)) > 40:
        base = Path("/tmp")
    d = base / f"tk8s-dp-{os.getuid()}" / hashlib.sha1(str(p).encode()).hexdigest()[:12]
    d.mkdir(parents=True, exist_ok=True, mode=0o700)
    return d


def _is_private_socket_dir(d: Path) -> bool:
    return d.parent.name == f"tk8s-dp-{os.getuid()}"


def _unix(path: Path) -> str:
    return f"unix://{Path(path).absolute()}"


def _generic_handler(impl, service: str) -> grpc.GenericRpcHandler:
    table = {}
    for meth, _, _, stream in SERVICES[service]:
        req, resp, _ = codec(service, meth)
        make = grpc.unary_stream_rpc_method_handler if stream else grpc.unary_unary_rpc_method_handler
        table[meth] = make(getattr(impl, meth), request_deserializer=req.FromString,
                           response_serializer=resp.SerializeToString)
    return grpc.method_handlers_generic_handler(f"{VERSION}.{service}", table)


def _stub(channel: grpc.Channel, service: str, meth: str):
    req, resp, stream = codec(service, meth)
    make = channel.unary_stream if stream else channel.unary_unary
    return make(method_path(service, meth), request_serializer=req.SerializeToString,
                response_deserializer=resp.FromString)


def _ident(p: Path):
    try:
        st = p.stat()
        return st.st_dev, st.st_ino, st.st_ctime_ns
    except OSError:
        return None


# ---- plugin side ------------------------------------------------------------------------------
class GpuDevicePluginServicer:
    """The DevicePlugin service over the plugin core (method names are the wire names)."""

    def __init__(self, core: DevicePlugin, env_mode: str = "container", health_interval: float = 5.0):
        if env_mode not in ("container", "process"):
            raise ValueError(f"env_mode must be 'container' or 'process', not {env_mode!r}")
        self.core = core
        self.env_mode = env_mode
        self.health_interval = health_interval
        self.cv = threading.Condition()
        self.generation = 0
        self.stopping = False
        self.allocations: list[list[str]] = []

    def notify(self) -> None:
        """The device list changed (health, SMI, validation): every ListAndWatch stream re-sends it."""
        with self.cv:
            self.generation += 1
            self.cv.notify_all()

    def _wake(self) -> None:
        with self.cv:
            self.cv.notify_all()

    def stop(self) -> None:
        with self.cv:
            self.stopping = True
            self.cv.notify_all()

    def resume(self) -> None:
        with self.cv:
            self.stopping = False

    def device_list(self):
        resp = pb.ListAndWatchResponse()
        for d in self.core.devices_:
            dev = resp.devices.add(ID=d.id, health=d.health)
            node = numa_node(d.render_minor)
            if node >= 0:
                dev.topology.nodes.add(ID=node)
        return resp

    def GetDevicePluginOptions(self, request, context):
        return pb.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        context.add_callback(self._wake)  # the kubelet went away: end the stream now
        sent = -1
        while True:
            with self.cv:
                while sent == self.generation and not self.stopping and context.is_active():
                    if not self.cv.wait(self.health_interval) and self.core.refresh_health():
                        self.generation += 1
                if self.stopping or not context.is_active():
                    return
                sent = self.generation
                msg = self.device_list()
            yield msg

    def GetPreferredAllocation(self, request, context):
        resp = pb.PreferredAllocationResponse()
        for cr in request.container_requests:
            try:
                ids = self.core.preferred(list(cr.available_deviceIDs), list(cr.must_include_deviceIDs),
                                          int(cr.allocation_size))
            except (KeyError, ValueError) as e:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"GetPreferredAllocation: {e}")
            resp.container_responses.add(deviceIDs=ids)
        return resp

    def Allocate(self, request, context):
        resp = pb.AllocateResponse()
        by_id = {d.id: d for d in self.core.devices_}
        for cr in request.container_requests:
            ids = list(cr.devices_ids)
            unknown = [i for i in ids if i not in by_id]
            if unknown:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unknown {RESOURCE} device(s) {unknown}")
            sick = [i for i in ids if by_id[i].health != HEALTHY]
            if sick:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, f"unhealthy {RESOURCE} device(s) {sick}")
            a = self.core.allocate(ids)
            c = resp.container_responses.add()
            if self.env_mode == "process":
                c.envs.update(a["env"])
            c.annotations.update(a["annotations"])
            for path in a["devices"]:
                c.devices.add(container_path=path, host_path=path, permissions="rw")
            self.allocations.append(ids)
        return resp

    def PreStartContainer(self, request, context):
        return pb.PreStartContainerResponse()


class PluginServer:
    """Serves one plugin on ``<dir>/<endpoint>`` and keeps it registered with the kubelet."""

    def __init__(self, servicer: GpuDevicePluginServicer, plugin_dir: str | os.PathLike = DEVICE_PLUGIN_PATH,
                 endpoint: str = ENDPOINT, resource: str = RESOURCE, log=print):
        self.servicer = servicer
        self.dir = Path(plugin_dir)
        self.endpoint = endpoint
        self.resource = resource
        self.log = log
        self.server: grpc.Server | None = None
        self.registrations = 0
        self._kubelet = None

    @property
    def socket(self) -> Path:
        return self.dir / self.endpoint

    @property
    def kubelet_socket(self) -> Path:
        return self.dir / KUBELET_SOCKET

    def start(self) -> None:
        self.dir.mkdir(parents=True, exist_ok=True)
        self.socket.unlink(missing_ok=True)
        self.servicer.resume()
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=8, thread_name_prefix="amd-gpu-dp"))
        self.server.add_generic_rpc_handlers((_generic_handler(self.servicer, "DevicePlugin"),))
        self.server.add_insecure_port(_unix(self.socket))
        self.server.start()

    def register(self, timeout: float = 10.0) -> None:
        ident = _ident(self.kubelet_socket)
        with grpc.insecure_channel(_unix(self.kubelet_socket)) as ch:
            _stub(ch, "Registration", "Register")(
                pb.RegisterRequest(version=VERSION, endpoint=self.endpoint, resource_name=self.resource,
                                   options=pb.DevicePluginOptions(get_preferred_allocation_available=True)),
                timeout=timeout, wait_for_ready=True)
        self._kubelet = ident
        self.registrations += 1

    def stop(self, grace: float = 0.2) -> None:
        self.servicer.stop()
        if self.server is not None:
            self.server.stop(grace).wait()
            self.server = None
        self.socket.unlink(missing_ok=True)

    def kubelet_restarted(self) -> bool:
        return not self.socket.exists() or _ident(self.kubelet_socket) != self._kubelet

    def serve_forever(self, stop: threading.Event, poll: float = 1.0, register_timeout: float = 10.0) -> None:
        try:
            while not stop.is_set():
                if self.server is None or self.kubelet_restarted():
                    if self.server is not None:
                        self.log(f"tk8s device plugin: kubelet restarted; registering {self.resource} again")
                        self.stop()
                    if self.kubelet_socket.exists():
                        self.start()
                        try:
                            self.register(register_timeout)
                            self.log(f"tk8s device plugin: {self.resource} registered with the kubelet "
                                     f"({len(self.servicer.core.devices_)} device(s), endpoint {self.socket})")
                        except grpc.RpcError as e:
                            self.log(f"tk8s device plugin: registration failed ({e.code().name}: {e.details()}); "
                                     "retrying")
                            self.stop()
                stop.wait(poll)
        finally:
            self.stop()


# ---- kubelet side -----------------------------------------------------------------------------
class PluginClient:
    """The kubelet device manager's handle on one registered plugin."""

    def __init__(self, socket: Path, resource: str, options):
        self.resource = resource
        self.options = options
        self.channel = grpc.insecure_channel(_unix(socket))
        self._rpc = {m: _stub(self.channel, "DevicePlugin", m) for m, *_ in SERVICES["DevicePlugin"]}
        self.cv = threading.Condition()
        self.devices: dict[str, str] = {}       # device id -> health
        self.numa: dict[str, list[int]] = {}
        self.updates = 0
        self.closed = False
        self.on_update = None
        self._stream = None

    def watch(self) -> None:
        self._stream = self._rpc["ListAndWatch"](pb.Empty())
        threading.Thread(target=self._consume, name=f"listandwatch-{self.resource}", daemon=True).start()

    def _consume(self) -> None:
        try:
            for resp in self._stream:
                with self.cv:
                    self.devices = {d.ID: d.health for d in resp.devices}
                    self.numa = {d.ID: [n.ID for n in d.topology.nodes] for d in resp.devices}
                    self.updates += 1
                    self.cv.notify_all()
                if self.on_update is not None:
                    self.on_update(self)
        except grpc.RpcError:
            pass
        with self.cv:  # the plugin is gone: its devices are no longer allocatable
            self.devices, self.closed = {}, True
            self.updates += 1
            self.cv.notify_all()
        if self.on_update is not None:
            self.on_update(self)

    def wait(self, pred, timeout: float) -> bool:
        with self.cv:
            return self.cv.wait_for(lambda: pred(self), timeout)

    def healthy(self) -> list[str]:
        with self.cv:
            return sorted(i for i, h in self.devices.items() if h == HEALTHY)

    def get_options(self, timeout: float = 10.0):
        return self._rpc["GetDevicePluginOptions"](pb.Empty(), timeout=timeout)

    def preferred(self, available: list[str], must_include: list[str], size: int, timeout: float = 10.0) -> list[str]:
        req = pb.PreferredAllocationRequest(container_requests=[pb.ContainerPreferredAllocationRequest(
            available_deviceIDs=list(available), must_include_deviceIDs=list(must_include),
            allocation_size=int(size))])
        return list(self._rpc["GetPreferredAllocation"](req, timeout=timeout).container_responses[0].deviceIDs)

    def allocate(self, ids: list[str], timeout: float = 10.0) -> dict:
        req = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=list(ids))])
        c = self._rpc["Allocate"](req, timeout=timeout).container_responses[0]
        return {"env": dict(c.envs), "devices": [d.host_path for d in c.devices],
                "annotations": dict(c.annotations),
                "mounts": [{"containerPath": m.container_path, "hostPath": m.host_path, "readOnly": m.read_only}
                           for m in c.mounts]}

    def close(self) -> None:
        if self._stream is not None:
            self._stream.cancel()
        self.channel.close()


class KubeletRegistry:
    """The kubelet's Registration service on ``<dir>/kubelet.sock`` plus its device manager."""

    def __init__(self, plugin_dir: str | os.PathLike):
        self.dir = Path(plugin_dir)
        self.plugins: dict[str, PluginClient] = {}
        self.cv = threading.Condition()
        self.server: grpc.Server | None = None
        self.on_update = None

    def start(self) -> "KubeletRegistry":
        self.dir.mkdir(parents=True, exist_ok=True)
        sock = self.dir / KUBELET_SOCKET
        sock.unlink(missing_ok=True)
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4, thread_name_prefix="kubelet-reg"))
        self.server.add_generic_rpc_handlers((_generic_handler(self, "Registration"),))
        self.server.add_insecure_port(_unix(sock))
        self.server.start()
        return self

    def Register(self, request, context):
        if request.version != VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          f"unsupported device plugin API version {request.version!r} (kubelet speaks {VERSION})")
        if not request.endpoint or "/" in request.endpoint:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"invalid endpoint {request.endpoint!r}")
        if "/" not in request.resource_name:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                          f"{request.resource_name!r} is not an extended resource name (domain/resource)")
        client = PluginClient(self.dir / request.endpoint, request.resource_name, request.options)
        client.on_update = self.on_update
        with self.cv:
            old = self.plugins.get(request.resource_name)
            self.plugins[request.resource_name] = client
            self.cv.notify_all()
        if old is not None:
            old.close()
        client.watch()
        return pb.Empty()

    def wait_plugin(self, resource: str, timeout: float) -> PluginClient | None:
        with self.cv:
            self.cv.wait_for(lambda: resource in self.plugins, timeout)
            return self.plugins.get(resource)

    def stop(self, wipe: bool = True) -> None:
        """Stop serving; ``wipe`` removes every socket in the directory, as a restarting kubelet does."""
        with self.cv:
            plugins, self.plugins = list(self.plugins.values()), {}
        for c in plugins:
            c.close()
        if self.server is not None:
            self.server.stop(0).wait()
            self.server = None
        if wipe:
            for s in self.dir.glob("*.sock"):
                s.unlink(missing_ok=True)
            if _is_private_socket_dir(self.dir):  # the short /tmp stand-in for a too-long path
                import shutil

                shutil.rmtree(self.dir, ignore_errors=True)


# ---- CLI: the DaemonSet payload on a kubelet-managed MI355X node ------------------------------
def _smi_loop(core: DevicePlugin, servicer: GpuDevicePluginServicer, interval: float, stop: threading.Event) -> None:
    if interval <= 0:
        return
    from .agent import read_smi

    while True:
        res = read_smi()
        if res is not None and core.update_from_smi(res):
            servicer.notify()
        if stop.wait(interval):
            return


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="tk8s-device-plugin",
                                 description="amd.com/gpu device plugin for the kubelet (device-plugin API v1beta1)")
    ap.add_argument("--plugin-dir", default=os.environ.get("TK8S_DEVICE_PLUGIN_DIR", DEVICE_PLUGIN_PATH))
    ap.add_argument("--gpus", default="all", help="host GPU ordinals to advertise, e.g. 0,1 (default: all)")
    ap.add_argument("--env-mode", choices=["container", "process"], default="container")
    ap.add_argument("--health-interval", type=float, default=5.0, help="render-node presence check period (s)")
    ap.add_argument("--smi-interval", type=float, default=30.0, help="AMD SMI ECC health period (s, 0 = off)")
    ap.add_argument("--poll", type=float, default=1.0, help="kubelet restart detection period (s)")
    a = ap.parse_args(argv)
    from ..models.hostinfo import discover

    inv = discover()
    gpus = [g.ordinal for g in inv.gpus] if a.gpus == "all" else [int(x) for x in a.gpus.split(",") if x.strip()]
    core = DevicePlugin(gpus, inventory=inv)
    servicer = GpuDevicePluginServicer(core, a.env_mode, a.health_interval)
    server = PluginServer(servicer, a.plugin_dir, log=lambda m: print(m, flush=True))
    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    threading.Thread(target=_smi_loop, args=(core, servicer, a.smi_interval, stop), name="smi", daemon=True).start()
    print(f"tk8s device plugin: {len(gpus)} x {RESOURCE} ({inv.source}); kubelet socket {server.kubelet_socket}",
          flush=True)
    server.serve_forever(stop, poll=a.poll)
    return 0


if __name__ == "__main__":
    sys.exit(main())
