"""Kubelet device-plugin API v1beta1 over gRPC: the hand-built schema is pinned
against hand-encoded wire bytes, then the kubelet flow (Register -> ListAndWatch ->
GetPreferredAllocation -> Allocate) runs against the plugin on Unix sockets, with health updates
and a kubelet restart. Fake gfx950 inventory (TK8S_FAKE_GPUS), no GPU needed."""
import threading

import grpc
import pytest

from tritonk8ssupervisor_amd.agent.deviceplugin import DevicePlugin
from tritonk8ssupervisor_amd.agent.dp_grpc import (RESOURCE, GpuDevicePluginServicer, KubeletRegistry, PluginServer,
                                                   socket_dir)
from tritonk8ssupervisor_amd.agent.dp_proto import KUBELET_SOCKET, pb
from tritonk8ssupervisor_amd.models.hostinfo import fake_inventory


def test_wire_format_matches_the_kubelet_proto():
    d = pb.Device(ID="gpu0", health="Healthy", topology=pb.TopologyInfo(nodes=[pb.NUMANode(ID=1)]))
    assert d.SerializeToString() == b"\x0a\x04gpu0\x12\x07Healthy\x1a\x04\x0a\x02\x08\x01"
    r = pb.RegisterRequest(version="v1beta1", endpoint="x.sock", resource_name="amd.com/gpu",
                           options=pb.DevicePluginOptions(get_preferred_allocation_available=True))
    assert r.SerializeToString() == b"\x0a\x07v1beta1\x12\x06x.sock\x1a\x0bamd.com/gpu\x22\x02\x10\x01"
    c = pb.ContainerAllocateResponse(envs={"A": "1"}, devices=[
        pb.DeviceSpec(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")])
    assert c.SerializeToString() == b"\x0a\x06\x0a\x01A\x12\x011" + b"\x1a\x18\x0a\x08/dev/kfd\x12\x08/dev/kfd\x1a\x02rw"
    p = pb.ContainerPreferredAllocationRequest(available_deviceIDs=["a"], must_include_deviceIDs=["b"],
                                               allocation_size=2)
    assert p.SerializeToString() == b"\x0a\x01a\x12\x01b\x18\x02"
    # and back: the kubelet's bytes decode into the same message
    assert pb.Device.FromString(d.SerializeToString()).topology.nodes[0].ID == 1


@pytest.fixture
def kubelet(tmp_path):
    reg = KubeletRegistry(socket_dir(tmp_path / "dp")).start()
    yield reg
    reg.stop()


@pytest.fixture
def fake8(monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")  # fake inventory: refresh_health skips /dev checks


def _plugin(reg, gpus=(0, 1, 2, 3), env_mode="process", n=8):
    core = DevicePlugin(list(gpus), inventory=fake_inventory(n))
    srv = PluginServer(GpuDevicePluginServicer(core, env_mode=env_mode, health_interval=0.2), reg.dir,
                       log=lambda m: None)
    stop = threading.Event()
    t = threading.Thread(target=srv.serve_forever, args=(stop,), kwargs={"poll": 0.05}, daemon=True)
    t.start()
    return core, srv, stop, t


def test_kubelet_flow_register_list_prefer_allocate(kubelet, fake8, native_build):
    core, srv, stop, t = _plugin(kubelet)
    try:
        c = kubelet.wait_plugin(RESOURCE, 10)
        assert c is not None and c.options.get_preferred_allocation_available
        assert c.wait(lambda c: len(c.devices) == 4, 10)
        assert c.healthy() == ["gpu0", "gpu1", "gpu2", "gpu3"]
        assert c.get_options().get_preferred_allocation_available
        ids = c.preferred(["gpu1", "gpu2", "gpu3"], ["gpu3"], 2)
        assert len(ids) == 2 and "gpu3" in ids
        a = c.allocate(["gpu2"])
        assert a["env"]["ROCR_VISIBLE_DEVICES"] == "2" and a["env"]["HIP_VISIBLE_DEVICES"] == "0"
        assert a["devices"] == ["/dev/kfd", "/dev/dri/renderD130"]
        assert a["annotations"]["amd.com/gpu-ids"] == "gpu2"
        assert srv.servicer.allocations == [["gpu2"]]
        with pytest.raises(grpc.RpcError) as e:
            c.allocate(["gpu7"])  # on the host, but not this plugin's
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    finally:
        stop.set()
        t.join(5)


def test_container_mode_leaves_visibility_to_the_device_nodes(kubelet, fake8):
    _, _, stop, t = _plugin(kubelet, env_mode="container")
    try:
        c = kubelet.wait_plugin(RESOURCE, 10)
        a = c.allocate(["gpu1"])
        assert "ROCR_VISIBLE_DEVICES" not in a["env"] and a["devices"] == ["/dev/kfd", "/dev/dri/renderD129"]
    finally:
        stop.set()
        t.join(5)


def test_health_changes_are_streamed_and_block_allocation(kubelet, monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "4")
    from tritonk8ssupervisor_amd.ops import fakesmi

    core, srv, stop, t = _plugin(kubelet, gpus=(0, 1), n=4)
    try:
        c = kubelet.wait_plugin(RESOURCE, 10)
        assert c.wait(lambda c: c.healthy() == ["gpu0", "gpu1"], 10)
        monkeypatch.setenv("TK8S_FAKE_SMI_UE", "1:2")  # host GPU 1: 2 uncorrectable ECC errors
        assert core.update_from_smi(fakesmi.report(4))
        srv.servicer.notify()
        assert c.wait(lambda c: c.devices.get("gpu1") == "Unhealthy", 10)
        assert c.healthy() == ["gpu0"]
        with pytest.raises(grpc.RpcError) as e:
            c.allocate(["gpu1"])
        assert e.value.code() == grpc.StatusCode.FAILED_PRECONDITION
    finally:
        stop.set()
        t.join(5)


def test_plugin_registers_again_after_a_kubelet_restart(tmp_path, fake8):
    d = socket_dir(tmp_path / "dp")
    reg = KubeletRegistry(d).start()
    _, srv, stop, t = _plugin(reg)
    try:
        assert reg.wait_plugin(RESOURCE, 10) is not None
        _until(lambda: srv.registrations == 1)  # the plugin counts once its Register RPC returned
        reg.stop()  # the kubelet exits and wipes the socket directory
        reg = KubeletRegistry(d).start()
        c = reg.wait_plugin(RESOURCE, 10)
        assert c is not None
        _until(lambda: srv.registrations == 2)
        assert c.wait(lambda c: len(c.healthy()) == 4, 10)
    finally:
        stop.set()
        t.join(5)
        reg.stop()
    assert not srv.socket.exists()


def _until(pred, timeout=10.0):
    import time

    deadline = time.monotonic() + timeout
    while not pred():
        assert time.monotonic() < deadline, "condition not met in time"
        time.sleep(0.01)


def test_registry_rejects_a_wrong_api_version(kubelet):
    from tritonk8ssupervisor_amd.agent.dp_grpc import _stub

    with grpc.insecure_channel(f"unix://{kubelet.dir / KUBELET_SOCKET}") as ch:
        with pytest.raises(grpc.RpcError) as e:
            _stub(ch, "Registration", "Register")(
                pb.RegisterRequest(version="v1alpha", endpoint="x.sock", resource_name=RESOURCE), timeout=5)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_socket_dir_falls_back_when_the_path_is_too_long(tmp_path):
    from tritonk8ssupervisor_amd.agent.dp_grpc import KubeletRegistry

    long = tmp_path / ("d" * 120)
    d = socket_dir(long)
    assert d != long and socket_dir(long) == d  # the same stand-in every time: nothing piles up
    assert socket_dir(tmp_path / "dp") == (tmp_path / "dp").absolute()
    reg = KubeletRegistry(d).start()
    reg.stop()
    assert not d.exists()  # the stand-in is removed with the kubelet side
