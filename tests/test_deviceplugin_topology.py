"""amd.com/gpu device plugin core: sysfs discovery, xGMI-aware preferred
allocation (C++ ``_tk8s_topo``, checked against a brute-force Python oracle), Allocate env."""
import itertools
import random

import pytest

from tritonk8ssupervisor_amd.agent.deviceplugin import DevicePlugin, link_matrix
from tritonk8ssupervisor_amd.models import hostinfo
from tritonk8ssupervisor_amd.models.hostinfo import compose_visible_devices, discover, fake_inventory


@pytest.fixture(scope="module")
def topo(native_build):
    from tritonk8ssupervisor_amd.ops import topo as _topo

    return _topo()


def _oracle(n, w, avail, must, size):
    best = None
    for combo in itertools.combinations(sorted(avail), size):
        if not set(must) <= set(combo):
            continue
        vals = [min(w[i * n + j], w[j * n + i]) for a, i in enumerate(combo) for j in combo[a + 1:]]
        mn, tot = min(vals, default=0), sum(vals)
        key = (-mn, -tot, combo)
        if best is None or key < best[0]:
            best = (key, combo, mn, tot)
    return list(best[1]), best[2], best[3]


def _islands(n=8, split=4):
    links = [[{"type": "self" if i == j else ("xgmi" if (i < split) == (j < split) else "pcie"), "hops": 0 if i == j else 1}
              for j in range(n)] for i in range(n)]
    return link_matrix(links)


def test_link_weights(topo):
    assert topo.link_weight("xgmi", 1) > topo.link_weight("pcie", 1) > 0
    w = link_matrix([[{"type": "self", "hops": 0}, {"type": "xgmi", "hops": 1}],
                     [{"type": "pcie", "hops": 2}, {"type": "self", "hops": 0}]])
    assert w == [1000, 100, 5, 1000]


def test_fully_connected_prefers_lowest(topo):
    w = link_matrix(fake_inventory(8).links)
    r = topo.preferred_allocation(8, w, list(range(8)), [], 4)
    assert list(r["devices"]) == [0, 1, 2, 3] and r["exhaustive"]


def test_islands_keep_a_set_on_one_xgmi_island(topo):
    w = _islands()
    r = topo.preferred_allocation(8, w, [2, 3, 4, 5, 6, 7], [], 4)
    assert list(r["devices"]) == [4, 5, 6, 7]
    r = topo.preferred_allocation(8, w, list(range(8)), [5], 2)
    assert 5 in r["devices"] and all(d >= 4 for d in r["devices"])


def test_must_include_and_errors(topo):
    w = link_matrix(fake_inventory(4).links)
    assert 3 in topo.preferred_allocation(4, w, [0, 1, 2, 3], [3], 2)["devices"]
    with pytest.raises(ValueError):
        topo.preferred_allocation(4, w, [0, 1], [], 3)  # not satisfiable
    with pytest.raises(ValueError):
        topo.preferred_allocation(4, w, [0, 9], [], 1)  # out of range
    with pytest.raises(ValueError):
        topo.preferred_allocation(4, w[:-1], [0, 1], [], 1)  # bad matrix
    with pytest.raises(ValueError):
        topo.preferred_allocation(4, w, [0, 1], [2], 1)  # must_include not available


def test_matches_bruteforce_oracle_on_random_topologies(topo):
    rng = random.Random(0)
    for _ in range(150):
        n = rng.randint(2, 8)
        w = [0] * (n * n)
        for i in range(n):
            w[i * n + i] = 1000
            for j in range(i + 1, n):
                w[i * n + j] = rng.choice([1, 5, 10, 50, 100])
                w[j * n + i] = w[i * n + j] if rng.random() < 0.8 else rng.choice([1, 5, 10, 50, 100])
        avail = sorted(rng.sample(range(n), rng.randint(1, n)))
        size = rng.randint(1, len(avail))
        must = rng.sample(avail, rng.randint(0, min(size, 2)))
        r = topo.preferred_allocation(n, w, avail, must, size)
        devs, mn, tot = _oracle(n, w, avail, must, size)
        assert (r["min_link"], r["total_link"]) == (mn, tot), (n, w, avail, must, size)
        assert list(r["devices"]) == devs


# ---- sysfs discovery ---------------------------------------------------------------------
def _fake_kfd(root, gpus, links):
    """KFD topology: node 0 = CPU, nodes 1.. = gfx950 GPUs; links[(a, b)] = io_link type."""
    (root / "0").mkdir(parents=True)
    (root / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\ngfx_target_version 0\n")
    for k in range(1, gpus + 1):
        d = root / str(k)
        (d / "io_links").mkdir(parents=True)
        (d / "properties").write_text(f"simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\nlocation_id {k * 256}\n")
        for m, ((a, b), t) in enumerate((kv for kv in links.items() if kv[0][0] == k)):
            (d / "io_links" / str(m)).mkdir()
            (d / "io_links" / str(m) / "properties").write_text(f"type {t}\nnode_from {a}\nnode_to {b}\n")


def test_discover_reads_kfd_sysfs(tmp_path, monkeypatch):
    monkeypatch.delenv("TK8S_FAKE_GPUS", raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    links = {(a, b): (11 if (a <= 2) == (b <= 2) else 2) for a in range(1, 5) for b in range(1, 5) if a != b}
    _fake_kfd(tmp_path, 4, links)
    inv = discover(tmp_path)
    assert inv.count == 4 and inv.source == "kfd-sysfs"
    assert all(g.gfx == "gfx950" and g.cu_count == 256 for g in inv.gpus)
    assert inv.links[0][1]["type"] == "xgmi" and inv.links[0][2]["type"] == "pcie"
    assert inv.links[3][3]["type"] == "self"
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,3")
    inv = discover(tmp_path)
    assert inv.count == 2 and [g.kfd_node for g in inv.gpus] == [3, 4] and [g.ordinal for g in inv.gpus] == [0, 1]
    assert inv.links[0][1]["type"] == "xgmi"
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1,2,3")  # ROCr first: host 1,2,3; then HIP 2,3 -> host 3 only
    inv = discover(tmp_path)
    assert [g.kfd_node for g in inv.gpus] == [4]


def test_discover_fake_and_empty(tmp_path, monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")
    inv = discover(tmp_path)
    assert inv.count == 8 and inv.source == "fake"
    monkeypatch.delenv("TK8S_FAKE_GPUS")
    assert discover(tmp_path / "missing").count == 0


def test_compose_visible_devices_nests_views():
    # restriction at the ROCr level (the child initialises only its own GPUs), HIP = identity
    assert compose_visible_devices([1, 3], {}) == {"ROCR_VISIBLE_DEVICES": "1,3", "HIP_VISIBLE_DEVICES": "0,1",
                                                   "CUDA_VISIBLE_DEVICES": "0,1"}
    # an agent that itself only sees host GPUs 4-7 (through HIP) hands out host indices
    assert compose_visible_devices([0, 2], {"HIP_VISIBLE_DEVICES": "4,5,6,7"})["ROCR_VISIBLE_DEVICES"] == "4,6"
    # ... and through ROCr then HIP: ROCR 2,3,5,7 -> HIP 1,3 -> host 3,7 -> ordinal 1 -> host 7
    env = {"ROCR_VISIBLE_DEVICES": "2,3,5,7", "HIP_VISIBLE_DEVICES": "1,3"}
    assert compose_visible_devices([1], env)["ROCR_VISIBLE_DEVICES"] == "7"
    # nesting a child's own view again is stable
    child = compose_visible_devices([1, 3], {})
    assert compose_visible_devices([1], child)["ROCR_VISIBLE_DEVICES"] == "3"


# ---- plugin ------------------------------------------------------------------------------
def test_plugin_list_allocate_and_probe_feedback(monkeypatch, native_build):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    p = DevicePlugin([2, 3, 9])
    devs = p.devices()
    assert [d["id"] for d in devs] == ["gpu2", "gpu3", "gpu9"]
    assert [d["health"] for d in devs] == ["Healthy", "Healthy", "Unhealthy"]  # gpu9 is not on the host
    a = p.allocate(["gpu3"])
    assert a["env"]["ROCR_VISIBLE_DEVICES"] == "3" and a["env"]["HIP_VISIBLE_DEVICES"] == "0"
    assert a["devices"][0] == "/dev/kfd"
    assert a["annotations"]["amd.com/gpu-ids"] == "gpu3"
    assert p.preferred(["gpu2", "gpu3"], [], 2) == ["gpu2", "gpu3"]
    assert p.preferred(["gpu2", "gpu3"], ["gpu3"], 1) == ["gpu3"]
    p.update_from_probe({"ok": True, "_allocated_ids": ["gpu2"],
                         "gpuinfo": {"devices": [{"pci_bus_id": "0000:23:00.0", "uuid": "u2", "gfx": "gfx950"}]}})
    assert p.devices()[0]["pciBusId"] == "0000:23:00.0"
    p.update_from_probe({"ok": False, "_allocated_ids": ["gpu3"]})
    assert p.devices()[1]["health"] == "Unhealthy" and p.devices()[1]["reason"] == "probe failed"


def test_smi_health_marks_ecc_devices_unhealthy_by_pci_id(monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "4")
    from tritonk8ssupervisor_amd.agent.deviceplugin import DevicePlugin
    from tritonk8ssupervisor_amd.models.hostinfo import fake_inventory
    from tritonk8ssupervisor_amd.ops import fakesmi

    plugin = DevicePlugin([2, 3], inventory=fake_inventory(4))
    assert [d["pciBusId"] for d in plugin.devices()] == ["0000:12:00.0", "0000:13:00.0"]
    monkeypatch.setenv("TK8S_FAKE_SMI_UE", "3:5,0:1")  # host GPU 0 is not this node's: ignored
    assert plugin.update_from_smi(fakesmi.report(4)) is True
    health = {d["id"]: (d["health"], d["reason"]) for d in plugin.devices()}
    assert health == {"gpu2": ("Healthy", ""), "gpu3": ("Unhealthy", "ECC: 5 uncorrectable, 0 deferred")}
    ann = plugin.telemetry_annotations()
    assert ann["amd.com/gpu-ecc-uncorrectable"] == "5" and ann["amd.com/gpu-temp-hotspot-max-c"] == "43"
    assert plugin.update_from_smi(fakesmi.report(4)) is False  # same sample: no change
    monkeypatch.setenv("TK8S_FAKE_SMI_UE", "")
    assert plugin.update_from_smi(fakesmi.report(4)) is True
    assert all(d["health"] == "Healthy" for d in plugin.devices())
    # a failed validation probe is sticky: SMI health never overrides it
    plugin.update_from_probe({"ok": False, "_allocated_ids": ["gpu2"]})
    assert plugin.update_from_smi(fakesmi.report(4)) is False
    assert plugin.devices()[0]["reason"] == "probe failed"
    assert plugin.update_from_smi({"ok": False, "error": "AMD SMI found no GPU"}) is False


def test_pci_bus_id_from_kfd_location():
    from tritonk8ssupervisor_amd.models.hostinfo import HostGpu

    assert HostGpu(ordinal=0, location_id=(0xa4 << 8) | (1 << 3) | 2, domain=1).pci_bus_id == "0001:a4:01.2"
