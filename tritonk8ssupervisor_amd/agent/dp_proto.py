"""Kubelet device-plugin API ``v1beta1`` message/service definitions, built without protoc.

The image has grpcio and protobuf but no ``grpc_tools``/``protoc``, so the
schema of ``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto`` is declared here as a
``FileDescriptorProto`` and the message classes come from protobuf's message factory. Only field
numbers and wire types reach the wire, so these classes are byte-compatible with the kubelet's
Go structs: a real kubelet can register and drive the plugin in ``dp_grpc.py``.

Two services (method paths ``/v1beta1.<Service>/<Method>``):

  Registration  Register(RegisterRequest) -> Empty                     (served by the kubelet)
  DevicePlugin  GetDevicePluginOptions(Empty) -> DevicePluginOptions   (served by the plugin)
                ListAndWatch(Empty) -> stream ListAndWatchResponse
                GetPreferredAllocation(PreferredAllocationRequest) -> PreferredAllocationResponse
                Allocate(AllocateRequest) -> AllocateResponse
                PreStartContainer(PreStartContainerRequest) -> PreStartContainerResponse

Reference anchor: the reference joins a worker with ``rancher/agent`` (ansible/roles/rancherhost/
tasks/main.yml:26-34) and never advertises accelerators; this is the kubelet-facing half of N2.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET = "kubelet.sock"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

_F = descriptor_pb2.FieldDescriptorProto
_STR, _BOOL, _I32, _I64, _MSG = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT32, _F.TYPE_INT64, _F.TYPE_MESSAGE
_ONE, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

# name -> [(field, number, type, label, message type or None)]
_MESSAGES: dict[str, list[tuple]] = {
    "DevicePluginOptions": [("pre_start_required", 1, _BOOL, _ONE, None),
                            ("get_preferred_allocation_available", 2, _BOOL, _ONE, None)],
    "RegisterRequest": [("version", 1, _STR, _ONE, None), ("endpoint", 2, _STR, _ONE, None),
                        ("resource_name", 3, _STR, _ONE, None),
                        ("options", 4, _MSG, _ONE, "DevicePluginOptions")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, _MSG, _REP, "Device")],
    "TopologyInfo": [("nodes", 1, _MSG, _REP, "NUMANode")],
    "NUMANode": [("ID", 1, _I64, _ONE, None)],
    "Device": [("ID", 1, _STR, _ONE, None), ("health", 2, _STR, _ONE, None),
               ("topology", 3, _MSG, _ONE, "TopologyInfo")],
    "PreStartContainerRequest": [("devices_ids", 1, _STR, _REP, None)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, _MSG, _REP, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, _STR, _REP, None),
                                            ("must_include_deviceIDs", 2, _STR, _REP, None),
                                            ("allocation_size", 3, _I32, _ONE, None)],
    "PreferredAllocationResponse": [("container_responses", 1, _MSG, _REP, "ContainerPreferredAllocationResponse")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, _STR, _REP, None)],
    "AllocateRequest": [("container_requests", 1, _MSG, _REP, "ContainerAllocateRequest")],
    "ContainerAllocateRequest": [("devices_ids", 1, _STR, _REP, None)],
    "CDIDevice": [("name", 1, _STR, _ONE, None)],
    "AllocateResponse": [("container_responses", 1, _MSG, _REP, "ContainerAllocateResponse")],
    "ContainerAllocateResponse": [("envs", 1, _MSG, _REP, "ContainerAllocateResponse.EnvsEntry"),
                                  ("mounts", 2, _MSG, _REP, "Mount"),
                                  ("devices", 3, _MSG, _REP, "DeviceSpec"),
                                  ("annotations", 4, _MSG, _REP, "ContainerAllocateResponse.AnnotationsEntry"),
                                  ("cdi_devices", 5, _MSG, _REP, "CDIDevice")],
    "Mount": [("container_path", 1, _STR, _ONE, None), ("host_path", 2, _STR, _ONE, None),
              ("read_only", 3, _BOOL, _ONE, None)],
    "DeviceSpec": [("container_path", 1, _STR, _ONE, None), ("host_path", 2, _STR, _ONE, None),
                   ("permissions", 3, _STR, _ONE, None)],
}
_MAPS = {"ContainerAllocateResponse": ("EnvsEntry", "AnnotationsEntry")}   # map<string, string>

# service -> [(method, input, output, server_streaming)]
SERVICES: dict[str, list[tuple[str, str, str, bool]]] = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
                     ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
                     ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
                     ("Allocate", "AllocateRequest", "AllocateResponse", False),
                     ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False)],
}


def _field(msg: descriptor_pb2.DescriptorProto, name: str, num: int, ftype: int, label: int, tname) -> None:
    f = msg.field.add(name=name, number=num, type=ftype, label=label)
    if tname:
        f.type_name = f".{VERSION}.{tname}"


def file_descriptor() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="deviceplugin/v1beta1/api.proto", package=VERSION,
                                            syntax="proto3")
    for name, fields in _MESSAGES.items():
        m = fd.message_type.add(name=name)
        for entry in _MAPS.get(name, ()):
            e = m.nested_type.add(name=entry)
            e.options.map_entry = True
            _field(e, "key", 1, _STR, _ONE, None)
            _field(e, "value", 2, _STR, _ONE, None)
        for f in fields:
            _field(m, *f)
    for svc, methods in SERVICES.items():
        s = fd.service.add(name=svc)
        for meth, inp, out, stream in methods:
            s.method.add(name=meth, input_type=f".{VERSION}.{inp}", output_type=f".{VERSION}.{out}",
                         server_streaming=stream)
    return fd


_POOL = descriptor_pool.DescriptorPool()
_POOL.Add(file_descriptor())


class _Messages:
    """Attribute access to the generated classes: ``pb.RegisterRequest(...)``."""

    def __init__(self):
        for name in _MESSAGES:
            setattr(self, name, message_factory.GetMessageClass(_POOL.FindMessageTypeByName(f"{VERSION}.{name}")))


pb = _Messages()


def method_path(service: str, method: str) -> str:
    return f"/{VERSION}.{service}/{method}"


def codec(service: str, method: str) -> tuple[type, type, bool]:
    """(request class, response class, server_streaming) of one RPC."""
    for meth, inp, out, stream in SERVICES[service]:
        if meth == method:
            return getattr(pb, inp), getattr(pb, out), stream
    raise KeyError(f"{service}.{method}")
