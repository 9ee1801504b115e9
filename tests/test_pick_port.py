"""utils.net.pick_port: the API port is drawn outside the kernel's ephemeral range and the NodePorts."""
import socket

from tritonk8ssupervisor_amd.utils import net


def test_port_is_below_the_ephemeral_range_and_free():
    low = min(net._ephemeral_low(), net.NODE_PORT_LOW)
    for _ in range(20):
        p = net.pick_port()
        assert net.PRIV_PORT_BASE + 1024 <= p < low
        with socket.socket() as s:  # still free: the picker closed its probe socket
            s.bind(("127.0.0.1", p))


def test_taken_candidates_are_skipped(monkeypatch):
    held = socket.socket()
    held.bind(("127.0.0.1", 0))
    taken = held.getsockname()[1]
    monkeypatch.setattr(net, "_ephemeral_low", lambda: taken + 1)
    monkeypatch.setattr(net, "NODE_PORT_LOW", 1 << 16)
    monkeypatch.setattr(net, "PRIV_PORT_BASE", taken - 1024 - 256)  # 257 candidates, one of them held
    try:
        ports = {net.pick_port() for _ in range(200)}
    finally:
        held.close()
    assert taken not in ports and all(taken - 256 <= p <= taken for p in ports)


def test_no_room_below_the_range_falls_back_to_any_port(monkeypatch):
    monkeypatch.setattr(net, "_ephemeral_low", lambda: net.PRIV_PORT_BASE + 1100)
    p = net.pick_port()
    assert p > 0
