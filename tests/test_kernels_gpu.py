"""Numerics of the gfx950 HIP kernels against exact host / PyTorch fp32 references (GPU only)."""
import json

import numpy as np
import pytest

from tritonk8ssupervisor_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def nat(native_build):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tritonk8ssupervisor_amd.ops import native

    return native()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_gpuinfo_reports_gfx950(nat):
    info = json.loads(nat.gpuinfo_json(True))
    assert info["ok"] and info["device_count"] >= 1
    d0 = info["devices"][0]
    assert d0["gfx"] == "gfx950"
    assert d0["wavefront_size"] == 64
    assert d0["cu_count"] >= 256
    assert d0["total_mem_bytes"] > 250 * 2**30
    assert len(info["links"]) == info["device_count"]


@pytest.mark.parametrize("nbytes", [16, 4096, 3 * 2**20 + 48])
def test_philox_fill_matches_host(nat, nbytes):
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    nat.philox_fill(buf.data_ptr(), nbytes, 0x1234_5678_9ABC, _stream())
    torch.cuda.synchronize()
    assert bytes(buf.cpu().numpy()) == ref.philox_bytes(nbytes, 0x1234_5678_9ABC)


@pytest.mark.parametrize("nbytes,chunk", [(0, 1024), (16, 1024), (1024, 1024), (1040, 1024), (16384, 1024),
                                          (17408, 1024), (65536, 1024), (70000 * 16, 1024), (100000, 192),
                                          (2**20, 256), (5 * 2**20 + 32, 4096)])
def test_md5_tree_matches_hashlib(nat, nbytes, chunk):
    data = ref.philox_bytes(nbytes, seed=11) if nbytes else b""
    src = torch.frombuffer(bytearray(data) or bytearray(16), dtype=torch.uint8).cuda()
    ws = max(nat.md5_tree_workspace(nbytes, chunk), 16)
    wa = torch.empty(ws, dtype=torch.uint8, device="cuda")
    wb = torch.empty(ws, dtype=torch.uint8, device="cuda")
    out = torch.zeros(16, dtype=torch.uint8, device="cuda")
    nat.md5_tree(src.data_ptr(), nbytes, chunk, wa.data_ptr(), wb.data_ptr(), out.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()) == ref.md5_tree(data, chunk)


@pytest.mark.parametrize("mode", ["nontemporal", "plain"])
def test_hbm_fill_and_verify(nat, mode):
    n = 64 * 2**20 + 16 * 5
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    nat.hbm_fill(buf.data_ptr(), n, 0xDEADBEEF, mode, _stream())
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    nat.verify_fill(buf.data_ptr(), n, 0xDEADBEEF, bad.data_ptr(), _stream())
    torch.cuda.synchronize()
    words = buf.view(torch.int32).cpu().numpy().view(np.uint32)
    assert (words == 0xDEADBEEF).all()
    assert int(bad.item()) == 0
    # verify must catch a corrupted word
    buf[4096:4100] = 0
    nat.verify_fill(buf.data_ptr(), n, 0xDEADBEEF, bad.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert int(bad.item()) == 1


@pytest.mark.parametrize("dtype,tdt", [("float32", torch.float32), ("bfloat16", torch.bfloat16)])
def test_allreduce_fill_and_check_vs_torch(nat, dtype, tdt):
    count, nranks = 1_000_003, 8
    bufs = []
    for r in range(nranks):
        b = torch.empty(count, dtype=tdt, device="cuda")
        nat.ar_fill(b.data_ptr(), count, r, dtype, _stream())
        bufs.append(b)
    total = torch.stack([b.float() for b in bufs]).sum(0)  # plain PyTorch fp32 reduction
    expect = torch.from_numpy(ref.allreduce_expected(count, nranks)).cuda()
    assert torch.equal(total, expect)
    summed = total.to(tdt)
    stats = torch.zeros(2, dtype=torch.int64, device="cuda")
    nat.ar_check(summed.data_ptr(), count, nranks, dtype, 0.0, stats.data_ptr(), stats.data_ptr() + 8, _stream())
    torch.cuda.synchronize()
    assert int(stats[1].item()) == 0 and int(stats[0].item()) == 0
    summed[12345] += 4
    stats.zero_()
    nat.ar_check(summed.data_ptr(), count, nranks, dtype, 0.0, stats.data_ptr(), stats.data_ptr() + 8, _stream())
    torch.cuda.synchronize()
    max_err = np.array([int(stats[0].item())], dtype=np.uint64).astype(np.uint32).view(np.float32)[0]
    assert int(stats[1].item()) == 1 and max_err == pytest.approx(4.0)


def test_stream_copy_matches_torch(nat):
    n = 32 * 2**20
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    nat.stream_copy(dst.data_ptr(), src.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    assert torch.equal(src, dst)


def test_probes_json(nat):
    h = json.loads(nat.hbm_write_probe(256 * 2**20, 3, "nontemporal", 0, 0))
    assert h["ok"] and h["bad_words"] == 0 and h["gbps"] > 500
    m = json.loads(nat.md5_probe(16 * 2**20, 1024, 5, 2, 0))
    assert m["ok"]
    assert m["digest"] == ref.md5_tree(ref.philox_bytes(16 * 2**20, 5), 1024).hex()
    c = json.loads(nat.copy_probe(0, 0, 64 * 2**20, 3))
    assert c["ok"] and c["kernel_gbps"] > 100


def test_rccl_single_gpu(nat):
    r = json.loads(nat.rccl_allreduce([0], 8, 1 << 20, 16, 3, 1, "float32", True))
    assert r["ok"], r
    assert r["nranks"] == 1 and all(x["bad"] == 0 for x in r["results"])


@pytest.mark.parametrize("n16", [1, 3, 1023, 4097, 1_000_003])
def test_slab_kernels_handle_ragged_tails(nat, n16):
    n = 16 * n16
    buf = torch.zeros(n, dtype=torch.uint8, device="cuda")
    nat.hbm_fill(buf.data_ptr(), n, 0x01020304, "plain", _stream())
    dst = torch.empty_like(buf)
    nat.stream_copy(dst.data_ptr(), buf.data_ptr(), n, _stream())
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    nat.verify_fill(dst.data_ptr(), n, 0x01020304, bad.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert int(bad.item()) == 0 and torch.equal(buf, dst)
    dst[-1] = 0  # the very last word belongs to the last slab's tail loop
    nat.verify_fill(dst.data_ptr(), n, 0x01020304, bad.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert int(bad.item()) == 1


def _probe(*args, timeout=120):
    import subprocess

    from tritonk8ssupervisor_amd.ops import tool

    r = subprocess.run([str(tool("tk8s-probe")), *args], capture_output=True, text=True, timeout=timeout)
    return r.returncode, json.loads(r.stdout.strip().splitlines()[-1])


def test_probe_cli_all_devices_known_answer(nat):
    rc, out = _probe("--all-devices", "--gpuinfo", "--peers", "--iters", "2", "--copy-bytes", str(64 << 20),
                     "--peer-bytes", str(16 << 20))
    assert rc == 0 and out["ok"], out
    assert out["probed"] == out["device_count"] >= 1
    assert out["md5_expected"] == "6a21931a145024b03ee4405e01204ce2"  # host oracle, 256 MiB seed 0
    for d in out["devices"]:
        assert d["ok"] and d["digest_ok"] and d["hbm"]["bad_words"] == 0
        assert d["hbm"]["gbps"] > 3000 and d["copy"]["kernel_gbps"] > 1500
        assert len(d.get("peers", [])) == out["device_count"] - 1
    assert out["gpuinfo"]["devices"][0]["gfx"] == "gfx950"
    assert out["timings_ms"]["total"] >= out["timings_ms"]["hip_init"] > 0


def test_probe_cli_out_and_reuse(nat, tmp_path):
    f = tmp_path / "burn.json"
    (tmp_path / "burn.json.pending").write_text("")
    rc, out = _probe("--out", str(f), "--hbm-bytes", str(64 << 20), "--md5-bytes", str(1 << 20), "--iters", "1")
    assert rc == 0 and out["ok"] and f.exists() and not (tmp_path / "burn.json.pending").exists()
    rc2, again = _probe("--reuse", str(f), "--hbm-bytes", "16")
    assert rc2 == 0 and again == out  # the pod reports the burn-in's result verbatim


def test_smi_health_matches_kfd_and_hip_views(nat):
    """tk8s-smi (AMD SMI, no HIP) sees the GPU HIP sees, under the same PCI bus id the agent's
    KFD sysfs discovery computes — the join key of device health."""
    import subprocess

    from tritonk8ssupervisor_amd.models.hostinfo import discover
    from tritonk8ssupervisor_amd.ops import tool

    r = subprocess.run([str(tool("tk8s-smi"))], capture_output=True, text=True, timeout=60)
    out = json.loads(r.stdout)
    assert out["ok"] and out["gpu_count"] >= 1, out
    assert r.returncode in (0, 1)
    smi_ids = {g["pci_bus_id"].lower() for g in out["gpus"]}
    kfd_ids = {g.pci_bus_id.lower() for g in discover(cache=False).gpus}
    assert kfd_ids and kfd_ids <= smi_ids, (kfd_ids, smi_ids)
    hip_ids = {d["pci_bus_id"].lower() for d in json.loads(nat.gpuinfo_json(False))["devices"]}
    assert hip_ids <= smi_ids, (hip_ids, smi_ids)
    g = out["gpus"][0]
    assert g["vram_total_bytes"] > 250 * 2**30 and "ecc" in g and "hotspot" in g["temp_c"]


def test_setup_on_a_real_gpu(tmp_path):
    """./setup.sh with one MI355X worker: the real tk8s-probe validates the GPU before Ready."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable, TK8S_SMI_DELAY="0.1", TK8S_SMI_INTERVAL="1")
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "120"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["gpus_allocatable"] == 1 and s["nodes_validated"] == 1
        k = subprocess.run(["./kubectl", "get", "node", "kubenode1", "-o", "json"], cwd=tmp_path, env=env,
                           capture_output=True, text=True, timeout=60)
        node = json.loads(k.stdout)
        assert float(node["metadata"]["annotations"]["tk8s.amd.com/hbm-write-gbps"]) > 3000
        assert node["status"]["devices"][0]["gfx"] == "gfx950"
        # the agent's AMD SMI health sample reaches the node (device joined by PCI bus id)
        import time

        deadline = time.monotonic() + 20
        while time.monotonic() < deadline:
            node = json.loads(subprocess.run(["./kubectl", "get", "node", "kubenode1", "-o", "json"], cwd=tmp_path,
                                             env=env, capture_output=True, text=True, timeout=60).stdout)
            if "telemetry" in node["status"]["devices"][0]:
                break
            time.sleep(0.2)
        dev = node["status"]["devices"][0]
        assert "telemetry" in dev, node
        assert dev["health"] == "Healthy" and dev["telemetry"]["ecc"]["uncorrectable"] == 0
        assert node["metadata"]["annotations"]["amd.com/gpu-health-source"] == "amdsmi"
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_setup_with_grpc_device_plugin_and_rccl_on_a_real_gpu(tmp_path):
    """The kubelet device-plugin API path on real hardware: the agent serves amd.com/gpu over gRPC
    v1beta1 (real KFD inventory, NUMA topology from sysfs), allocates the validation pod and the
    RCCL rank through it, and the rank finds its GPU as --device $(TK8S_GPU_DEVICE)."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable, TK8S_DEVICE_PLUGIN="grpc")
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "120",
                            "--rccl", "on", "--rccl-max-bytes", str(4 << 20)],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["gpus_allocatable"] == 1 and s["nodes_validated"] == 1 and s["rccl"]["ok"]
        log = (tmp_path / ".tk8s" / "machines" / "kubenode1" / "logs" / "agent.log").read_text()
        assert "via gRPC v1beta1" in log, log[-2000:]
        # the rank used RCCL with its device code unpacked (utils/rccl_unpack.py): no 5.3 GB inflation
        assert s["rccl"]["rccl_library"] == "unpacked", s["rccl"]
        assert s["rccl"]["comm_init_ms_max"] < 1500, s["rccl"]
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_unpacked_rccl_starts_faster_on_a_real_gpu(native_build):
    """RCCL with its gfx950 device code unpacked once (utils/rccl_unpack.py)
    loads, all-reduces exactly, and starts its communicator without inflating the 5.3 GB bundle:
    well under the installed library's ~1.8 s."""
    import os
    import subprocess
    from pathlib import Path

    from tritonk8ssupervisor_amd.utils.rccl_unpack import library_dir

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lib = library_dir()
    assert lib is not None, native_build.get("rccl-unpacked")
    tool = Path(__file__).resolve().parents[1] / "tritonk8ssupervisor_amd" / "bin" / "tk8s-rccl"
    args = [str(tool), "--ngpus", "1", "--max-bytes", str(1 << 20), "--iters", "3", "--warmup", "1"]
    out = {}
    for name, extra in (("installed", {}), ("unpacked", {"LD_LIBRARY_PATH": str(lib)})):
        r = subprocess.run(args, capture_output=True, text=True, timeout=120, env={**os.environ, **extra})
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        out[name] = json.loads(r.stdout.strip().splitlines()[-1])
        out[name]["path"] = next((ln.split(":", 1)[1].strip() for ln in r.stdout.splitlines()
                                  if ln.startswith("Librccl path")), "")
    assert out["unpacked"]["ok"] and all(x["bad"] == 0 for x in out["unpacked"]["results"])
    assert out["unpacked"]["path"].startswith(str(lib)), out["unpacked"]["path"]
    assert out["unpacked"]["comm_init_ms"] < 1000.0 < out["installed"]["comm_init_ms"], \
        (out["unpacked"]["comm_init_ms"], out["installed"]["comm_init_ms"])


def test_setup_with_host_burnin_on_a_real_gpu(tmp_path):
    """The host-level burn-in (one tk8s-probe for every worker GPU, split per machine) on real
    hardware (the default for every GPU count)."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable)
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "120"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["gpus_allocatable"] == 1 and s["nodes_validated"] == 1
        burn = json.loads((tmp_path / ".tk8s" / "machines" / "kubenode1" / "run" / "gpu-burnin.json.consumed").read_text())
        assert burn["ok"] and burn["host_burnin"] and burn["devices"][0]["host_index"] == 0
        assert burn["md5"]["digest"] == burn["md5_expected"] and burn["gpuinfo"]["devices"][0]["gfx"] == "gfx950"
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_torch_rccl_allreduce_single_rank(tmp_path):
    """The PyTorch (RCCL) twin of tk8s-rccl, rendezvous through a real control-plane KV."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    from test_controlplane import _start, _stop

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p, c = _start(tmp_path)
    try:
        r = subprocess.run([sys.executable, "-m", "tritonk8ssupervisor_amd.parallel.dist_allreduce", "--backend", "nccl",
                            "--rank", "0", "--nranks", "1", "--kv-url", f"{c.base}/v1/kv/t/addr", "--max-bytes", str(16 << 20)],
                           cwd=Path(__file__).resolve().parents[1], capture_output=True, text=True, timeout=180,
                           env={**os.environ, "TK8S_KV_TOKEN": c.token})  # the KV answers no anonymous caller
    finally:
        _stop(p)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["ok"] and out["backend"] == "nccl", r.stderr[-2000:]
    assert all(x["bad"] == 0 for x in out["results"])


def test_setup_rccl_job_under_rocprof(tmp_path):
    """BASELINE.json config 5 on one GPU: the RCCL Job's rank runs under rocprofv3
    --kernel-trace --stats and the per-kernel summary lands in the setup summary."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable, TMPDIR="/tmp")
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "240",
                            "--rccl", "on", "--rocprof", "--rccl-max-bytes", str(16 << 20)],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=400)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["rccl"]["ok"] and s["rccl"]["nranks"] == 1
        prof = s["rccl"]["rocprof"]
        assert prof["ranks"], prof
        kernels = [k["kernel"] for ks in prof["ranks"].values() for k in ks]
        assert kernels and all(k["calls"] > 0 for ks in prof["ranks"].values() for k in ks)
        out = Path(os.environ.get("GRAFT_REPO_ROOT", repo)) / "gpurun_out" / "rccl_rocprof"
        out.mkdir(parents=True, exist_ok=True)
        (out / "summary.json").write_text(json.dumps(s["rccl"], indent=1))
        for f in Path(prof["dir"]).rglob("*_kernel_stats.csv"):
            shutil.copy2(f, out / f.name)
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def _gpu_count():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X (xGMI)")
def test_multi_gpu_rccl_single_process_all_devices(nat):
    n = _gpu_count()
    r = json.loads(nat.rccl_allreduce(list(range(n)), 1024, 64 << 20, 4, 5, 2, "bfloat16", True))
    assert r["ok"] and r["nranks"] == n, r
    assert all(x["bad"] == 0 for x in r["results"])
    from tritonk8ssupervisor_amd.xgmi import fabric_floors

    assert r["peak_busbw_gbps"] > fabric_floors(n)["allreduce_busbw_gbps"], r  # xGMI, not PCIe / host memory


@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X (xGMI)")
def test_multi_gpu_peer_probe(nat):
    rc, out = _probe("--all-devices", "--peers", "--hbm-bytes", str(64 << 20), "--md5-bytes", str(1 << 20),
                     "--copy-bytes", str(64 << 20), "--peer-bytes", str(64 << 20), "--iters", "2")
    assert rc == 0 and out["ok"], out
    from tritonk8ssupervisor_amd.xgmi import fabric_floors

    floor = fabric_floors(out["device_count"])["peer_pull_gbps"]
    for d in out["devices"]:
        assert len(d["peers"]) == out["device_count"] - 1
        assert all(p["ok"] and p["kernel_gbps"] > floor for p in d["peers"]), (floor, d["peers"])
    # every pair is a direct xGMI link in the KFD topology (a PCIe pair would say "pcie")
    links = json.loads(nat.gpuinfo_json(True))["links"]
    assert all(links[i][j]["type"] == "xgmi" for i in range(len(links)) for j in range(len(links)) if i != j), links


@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X (xGMI)")
def test_multi_gpu_setup_with_rccl_job(tmp_path):
    """BASELINE.json config 4 in small: 2 workers x 1 MI355X, validated, RCCL Job across both."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    # the ranks log their transports: every channel must be P2P over xGMI
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable, NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,P2P")
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "2", "--yes", "--json", "--port", "0", "--timeout", "240",
                            "--rccl-max-bytes", str(64 << 20)], cwd=tmp_path, env=env, capture_output=True, text=True,
                           timeout=400)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        rc = s["rccl"]
        assert s["gpus_allocatable"] == 2 and rc["ok"] and rc["nranks"] == 2
        assert rc["transport"]["logged"] and rc["transport"]["p2p"] > 0, rc["transport"]
        assert rc["transport"]["shm"] == 0 and rc["transport"]["net"] == 0, rc["transport"]  # no host fallback
        from tritonk8ssupervisor_amd.xgmi import fabric_floors

        assert rc["peak_busbw_gbps"] > fabric_floors(2)["allreduce_busbw_gbps"], rc  # one xGMI link at 64 MiB
        assert rc["init_spread_ms"] < 5000, rc  # the ranks' runtimes came up together
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X (xGMI)")
def test_multi_gpu_node_fabric_job_is_one_process_per_node(tmp_path):
    """A 2-GPU worker: the RCCL Job is one pod holding both GPUs, its one process driving them as
    ranks 0 and 1 (tk8s-rccl --group-index/--devices), P2P over xGMI."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable, NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,P2P")
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--package", "mi355x-2gpu", "--rccl", "on", "--yes", "--json",
                            "--port", "0", "--timeout", "240", "--rccl-max-bytes", str(64 << 20)], cwd=tmp_path, env=env,
                           capture_output=True, text=True, timeout=400)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
        rc = json.loads(r.stdout.strip().splitlines()[-1])["rccl"]
        assert rc["ok"] and rc["nranks"] == 2 and rc["pods"] == 1 and rc["gpus_per_pod"] == 2, rc
        assert rc["transport"]["p2p"] > 0 and rc["transport"]["shm"] == 0, rc["transport"]
        from tritonk8ssupervisor_amd.xgmi import fabric_floors

        assert rc["peak_busbw_gbps"] > fabric_floors(2)["allreduce_busbw_gbps"], rc
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_rccl_rank_group_cli_on_one_gpu(tmp_path):
    """tk8s-rccl's per-node shape with one device (what the fabric Job runs on 1-GPU nodes)."""
    import subprocess

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tritonk8ssupervisor_amd.ops import BIN

    r = subprocess.run([str(BIN / "tk8s-rccl"), "--group-index", "0", "--devices", "0", "--nranks", "1",
                        "--uid-file", str(tmp_path / "uid"), "--max-bytes", str(4 << 20), "--iters", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["nranks"] == 1 and out["first_rank"] == 0 and out["local_ranks"] == 1
    assert all(x["bad"] == 0 for x in out["results"])
    bad = subprocess.run([str(BIN / "tk8s-rccl"), "--group-index", "1", "--devices", "0", "--nranks", "1",
                          "--uid-file", str(tmp_path / "uid"), "--uid-timeout", "5"], capture_output=True, text=True,
                         timeout=60)
    assert bad.returncode != 0  # rank 1 of a 1-rank communicator is refused, not a hang


@pytest.mark.gpu
def test_setup_from_an_answers_file_adopts_the_early_burnin_on_a_real_gpu(tmp_path):
    """``./setup.sh --answers FILE`` (the bench's path): the real tk8s-probe is spawned before the
    CLI imports anything, the orchestrator adopts it, and the control plane zygote serves."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    (tmp_path / "answers.json").write_text(json.dumps({"nodes": 1, "package": "mi355x-1gpu", "confirm": "yes"}))
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable, TK8S_HOST_REGISTRY=str(tmp_path / "hostreg"))
    try:
        r = subprocess.run(["./setup.sh", "--answers", "answers.json", "--yes", "--json", "--port", "0", "--timeout", "120"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["gpus_allocatable"] == 1 and s["nodes_validated"] == 1
        events = [json.loads(x) for x in (tmp_path / ".tk8s" / "events.jsonl").read_text().splitlines()]
        started = [e for e in events if e["event"] == "gpu_burnin_host_started"]
        assert len(started) == 1 and started[0].get("early"), started
        assert any(e["event"] == "controlplane_boot_started" and e.get("zygote") for e in events)
        burn = json.loads((tmp_path / ".tk8s" / "machines" / "kubenode1" / "run" / "gpu-burnin.json.consumed").read_text())
        assert burn["ok"] and burn["host_burnin"] and burn["gpuinfo"]["devices"][0]["gfx"] == "gfx950"
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def _hsaprobe(*args, timeout=120, env=None):
    import os
    import subprocess

    from tritonk8ssupervisor_amd.ops import BIN

    r = subprocess.run([str(BIN / "tk8s-hsaprobe"), *args], capture_output=True, text=True, timeout=timeout,
                       env=None if env is None else {**os.environ, **env})
    return r.returncode, json.loads(r.stdout.strip().splitlines()[-1])


def test_hsaprobe_digests_match_the_host_oracle(nat):
    """tk8s-hsaprobe dispatches the same kernels on ROCr with hand-built AQL packets: the MD5 tree
    of the Philox stream must match the host oracle, bit for bit, at a ragged and a full size."""
    from tritonk8ssupervisor_amd.ops import reference as ref

    for nbytes in (1 << 20, 3 * (1 << 20) + 4096):
        rc, out = _hsaprobe("--hbm-bytes", str(16 << 20), "--md5-bytes", str(nbytes), "--copy-bytes", str(1 << 20),
                            "--iters", "1")
        assert rc == 0 and out["ok"] and out["runtime"] == "hsa", out
        assert out["md5"]["digest"] == ref.md5_tree(ref.philox_bytes(nbytes, 0), 1024).hex()
        assert out["hbm"]["bad_words"] == 0 and out["copy"]["bad_words"] == 0


def test_hsaprobe_known_answer_and_gpuinfo_agree_with_the_hip_probe(nat):
    rc, hsa = _hsaprobe("--all-devices", "--gpuinfo", "--iters", "2")
    assert rc == 0 and hsa["ok"], hsa
    assert hsa["md5_expected"] == "6a21931a145024b03ee4405e01204ce2" and hsa["md5"]["digest"] == hsa["md5_expected"]
    for d in hsa["devices"]:
        assert d["ok"] and d["digest_ok"] and d["hbm"]["gbps"] > 3000 and d["copy"]["kernel_gbps"] > 1500
    rc, hip = _probe("--all-devices", "--gpuinfo", "--iters", "1", "--hbm-bytes", str(64 << 20))
    assert rc == 0
    for a, b in zip(hsa["gpuinfo"]["devices"], hip["gpuinfo"]["devices"]):
        assert a["gfx"] == b["gfx"] == "gfx950"
        assert a["pci_bus_id"] == b["pci_bus_id"] and a["cu_count"] == b["cu_count"]


def test_hsaprobe_skips_the_cpu_cache_walk_and_still_passes(nat):
    """The probe hides the per-CPU sysfs cache directories from the thunk's hsa_init walk
    (profiles/r2_hsainit/); the runtime must come up with the same agents and the burn-in must
    give the same answers as with the walk kept (TK8S_HSA_CPU_CACHES=1)."""
    import os

    args = ("--all-devices", "--gpuinfo", "--hbm-bytes", str(64 << 20), "--md5-bytes", str(256 << 20), "--iters", "1")
    rc, fast = _hsaprobe(*args)
    assert rc == 0 and fast["ok"], fast
    assert fast["timings_ms"]["cpu_cache_walk"] == "skipped"
    if os.path.isdir("/sys/devices/system/cpu/cpu0/cache"):
        assert fast["timings_ms"]["cpu_cache_dirs_hidden"] > 0
    rc, kept = _hsaprobe(*args, env={"TK8S_HSA_CPU_CACHES": "1"})
    assert rc == 0 and kept["ok"], kept
    assert kept["timings_ms"]["cpu_cache_walk"] == "kept" and kept["timings_ms"]["cpu_cache_dirs_hidden"] == 0
    assert fast["device_count"] == kept["device_count"]
    assert fast["md5"]["digest"] == kept["md5"]["digest"] == fast["md5_expected"]
    assert [d["pci_bus_id"] for d in fast["gpuinfo"]["devices"]] == [d["pci_bus_id"] for d in kept["gpuinfo"]["devices"]]


def test_hip_probe_skips_the_cpu_cache_walk(nat):
    rc, out = _probe("--iters", "1", "--hbm-bytes", str(64 << 20))
    assert rc == 0 and out["ok"] and out["timings_ms"]["cpu_cache_walk"] == "skipped", out


def test_hsaprobe_peers_on_one_gpu_is_a_no_op(nat):
    """--peers with a single GPU: no pair to pull over, nothing dispatched for it, result unchanged."""
    n = _gpu_count()
    rc, out = _hsaprobe("--all-devices", "--peers", "--hbm-bytes", str(64 << 20), "--md5-bytes", str(1 << 20),
                        "--copy-bytes", str(16 << 20), "--iters", "1")
    assert rc == 0 and out["ok"], out
    assert out["peer_rounds"] == n - 1
    for d in out["devices"]:
        assert d["peers_ok"] and len(d["peers"]) == n - 1
    if n == 1:
        assert out["timings_ms"]["peers"] < 1.0, out["timings_ms"]


def test_hsaprobe_pull_from_granted_non_local_memory(nat):
    """The peer-pull mechanism from a source the GPU does not own: host memory granted with
    hsa_amd_agents_allow_access, pulled by the stream copy kernel at system-scope acquire and
    checked against the source's pattern (the part of N7 a one-GPU box can run)."""
    rc, out = _hsaprobe("--peers-host", "--peer-bytes", str(8 << 20), "--hbm-bytes", str(16 << 20),
                        "--md5-bytes", str(1 << 20), "--copy-bytes", str(1 << 20), "--iters", "1")
    assert rc == 0 and out["ok"], out
    hp = out["devices"][0]["host_pull"]
    assert hp["ok"] and hp["access"] == "allowed" and hp["bad_words"] == 0 and hp["src_device"] == -1, hp
    assert 1.0 < hp["kernel_gbps"] < 1000.0, hp  # PCIe/host-link rate, not a local-HBM copy


def test_hsaprobe_multi_device_path_on_one_gpu(nat):
    """--devices 0,0,0: three queues and arenas on the one GPU run the multi-device path end to
    end -- a thread per device, the peer grants (hsa_amd_agents_allow_access on each source
    arena for the other devices' agents), two rounds of pulls at system-scope acquire, each
    checked against its source's pattern -- and the result splits and judges as a host burn-in's
    would (burnin.split_host_result, xgmi.link_report). Only the cross-GPU mapping itself needs
    a second GPU."""
    from tritonk8ssupervisor_amd.burnin import split_host_result
    from tritonk8ssupervisor_amd.xgmi import link_report

    rc, out = _hsaprobe("--devices", "0,0,0", "--gpuinfo", "--peers", "--peer-bytes", str(16 << 20),
                        "--hbm-bytes", str(256 << 20), "--md5-bytes", str(16 << 20), "--copy-bytes", str(16 << 20),
                        "--iters", "2")
    assert rc == 0 and out["ok"], out
    assert out["peer_rounds"] == 2 and [d["device"] for d in out["devices"]] == [0, 0, 0]
    for d in out["devices"]:
        assert d["ok"] and d["peers_ok"] and len(d["peers"]) == 2, d
        for p in d["peers"]:
            assert p["ok"] and p["access"] == "allowed" and p["bad_words"] == 0 and p["kernel_gbps"] > 50, p
    # three queues on one GPU contend for its HBM, so their rates say nothing about links: the
    # verdict is asked for dead pulls only (fraction 0), which none may be
    rep = link_report(out, [0, 1, 2], fraction=0.0)
    assert rep["pulls"] == 6 and not rep["degraded"], rep
    share = split_host_result(out, [0, 1, 2], [0], rep)  # (every entry names GPU 0)
    assert share is not None and share["ok"] and share["device_count"] == 1
    rc, bad = _hsaprobe("--devices", "0,x", "--iters", "1")
    assert rc == 2 and not bad["ok"] and "--devices" in bad["error"]


def test_hip_peer_pull_path_on_one_gpu(nat, monkeypatch):
    """The HIP probe's xGMI pull path (copy_probe with src != dst) keeps its buffers per device --
    a source filled once and only read, a destination held for the pull -- instead of a
    hipMalloc/hipFree per pull (hipFree synchronises the whole device). TK8S_PROBE_PEER_PATH=1
    routes a copy within one GPU through that path: repeated pulls, a larger one (the source
    buffer regrows and is refilled), the SDMA pass, and the local copy afterwards."""
    monkeypatch.setenv("TK8S_PROBE_PEER_PATH", "1")
    for nbytes in (16 << 20, 16 << 20, 48 << 20, 16 << 20):
        c = json.loads(nat.copy_probe(0, 0, nbytes, 3))
        assert c["ok"] and c["probe"] == "xgmi_peer_copy" and c["bad_words"] == 0, c
        assert c["kernel_gbps"] > 100 and c["dma_gbps"] > 10, c
    monkeypatch.delenv("TK8S_PROBE_PEER_PATH")
    c = json.loads(nat.copy_probe(0, 0, 16 << 20, 3))
    assert c["ok"] and c["probe"] == "local_copy" and c["bad_words"] == 0, c


def test_hsaprobe_md5_unpinned_for_other_inputs(nat):
    rc, out = _hsaprobe("--md5-bytes", str(1 << 20), "--hbm-bytes", str(16 << 20), "--copy-bytes", str(1 << 20),
                        "--iters", "1")
    assert rc == 0 and out["md5_pinned"] is False
    rc, out = _hsaprobe("--hbm-bytes", str(16 << 20), "--copy-bytes", str(1 << 20), "--iters", "1")
    assert rc == 0 and out["md5_pinned"] is True and out["md5"]["digest"] == out["md5_expected"]


@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X (xGMI)")
def test_multi_gpu_hsaprobe_peer_matrix(nat):
    """Every ordered pair pulled once over its own link, pattern-checked, at xGMI rates."""
    n = _gpu_count()
    rc, out = _hsaprobe("--all-devices", "--peers", "--hbm-bytes", str(64 << 20), "--md5-bytes", str(1 << 20),
                        "--copy-bytes", str(16 << 20), "--iters", "2")
    assert rc == 0 and out["ok"], out
    pairs = {(p["src_device"], p["dst_device"]) for d in out["devices"] for p in d["peers"]}
    assert pairs == {(a, b) for a in range(n) for b in range(n) if a != b}
    for d in out["devices"]:
        assert d["peers_ok"]
        assert all(p["ok"] and p["access"] == "allowed" and p["kernel_gbps"] > 20 for p in d["peers"]), d["peers"]
    from tritonk8ssupervisor_amd import xgmi

    rep = xgmi.link_report(out)
    assert rep["pulls"] == n * (n - 1) and not rep["degraded"], rep


@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X (xGMI)")
def test_multi_gpu_degraded_link_keeps_its_nodes_not_ready(tmp_path):
    """N7 before Ready on real links: the host burn-in pulls every ordered pair; a link reported at
    a tenth of its measured rate (TK8S_FAULTS=xgmi.degrade@0-1:0.1, applied to the measurement)
    keeps both of its nodes NotReady with XGMILinkDegraded, and setup fails fast."""
    import os
    import shutil
    import subprocess
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable)
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "2", "--yes", "--json", "--port", "0", "--timeout", "120",
                            "--rccl", "off"], cwd=tmp_path, env={**env, "TK8S_FAULTS": "xgmi.degrade@0-1:0.1"},
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 2 and "XGMILinkDegraded" in r.stderr, r.stdout[-2000:] + r.stderr[-2000:]
        out = subprocess.run(["./kubectl", "get", "nodes"], cwd=tmp_path, env=env, capture_output=True,
                             text=True).stdout
        assert out.count("NotReady") == 2, out
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_doctor_passes_on_the_mi355x_host():
    """./tk8s doctor on the GPU box: the KFD is usable and exposes gfx950 GPUs, the build is there."""
    import os
    import subprocess
    from pathlib import Path

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env["PYTHONPATH"] = str(repo)
    r = subprocess.run([str(repo / "tk8s"), "doctor", "--json"], cwd=repo, env=env, capture_output=True, text=True,
                       timeout=120)
    checks = {c["check"]: c for c in json.loads(r.stdout)}
    assert checks["/dev/kfd"]["status"] == "OK" and checks["rocm"]["status"] == "OK", checks
    assert checks["gpus"]["status"] == "OK" and "gfx950" in checks["gpus"]["detail"], checks["gpus"]
    assert checks["native build"]["status"] == "OK"
    assert r.returncode == 0 or any(c["status"] == "FAIL" and c["check"] == "free gpus" for c in checks.values()), checks


def _real_ws(tmp_path):
    import os
    import shutil
    import sys
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k not in ("TK8S_FAKE_GPUS", "TK8S_FAULTS")}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable)
    return env


def test_gpu_jail_on_a_real_gpu():
    """the GPU jail (Landlock) decides what a process's runtime can open. Denied the
    GPU's render node, HIP finds no device -- even with HIP/ROCR_VISIBLE_DEVICES pointing at it;
    allowed it, the GPU works (profiles/r3_gpujail/)."""
    import os
    import subprocess

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tritonk8ssupervisor_amd.agent.runtime import JAIL, gpu_jail
    from tritonk8ssupervisor_amd.models.hostinfo import discover
    from tritonk8ssupervisor_amd.ops import tool

    ok, how = gpu_jail()
    assert ok, how
    g = discover(cache=False).gpus[0]
    info = str(tool("tk8s-gpuinfo"))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0", ROCR_VISIBLE_DEVICES="0")
    r = subprocess.run([str(JAIL), "--", info, "--no-links"], capture_output=True, text=True, timeout=60, env=env)
    assert json.loads(r.stdout.strip().splitlines()[-1])["device_count"] == 0, r.stdout + r.stderr
    r = subprocess.run([str(JAIL), "--allow-render", str(g.render_minor), "--", info, "--no-links"],
                       capture_output=True, text=True, timeout=60)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] and out["device_count"] == 1 and out["devices"][0]["gfx"] == "gfx950", out


def test_pods_see_only_their_gpus_on_a_real_gpu(tmp_path):
    """VERDICT r2 #5 on the cluster: a pod without an amd.com/gpu request gets device_count 0 from
    tk8s-gpuinfo (it clears nothing, the jail decides); a pod holding the GPU sees it; `kubectl
    describe pod` names the isolation."""
    import subprocess
    import time

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tritonk8ssupervisor_amd.ops import tool

    env = _real_ws(tmp_path)
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=60)
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "120"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        st = tmp_path / ".tk8s"
        secrets = [st / "kubeconfig.json", st / "admin-token", *sorted((st / "keys").glob("*"))]
        # a GPU pod, too, gets EACCES on the cluster's credentials -- and its GPU
        # still works under the same jail (the gpuinfo line is its last output)
        steal = "".join(f'if cat {f} > /dev/null 2>&1; then echo "read {f}"; else echo "denied {f}"; fi; '
                        for f in secrets)
        for name, gpus in (("no-gpu", 0), ("one-gpu", 1)):
            (tmp_path / f"{name}.json").write_text(json.dumps({
                "apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                "spec": {"restartPolicy": "Never", "containers": [{
                    "name": "c", "command": ["sh", "-c", steal + f"exec {tool('tk8s-gpuinfo')} --no-links"],
                    "env": [{"name": "HIP_VISIBLE_DEVICES", "value": "0"}],
                    "resources": {"limits": {"amd.com/gpu": gpus}} if gpus else {}}]}}))
            assert kc("apply", "-f", str(tmp_path / f"{name}.json")).returncode == 0
        deadline = time.monotonic() + 90
        phases = {}
        while time.monotonic() < deadline:
            phases = {p["metadata"]["name"]: p["status"].get("phase") for p in json.loads(kc("get", "pods", "-o", "json").stdout)["items"]}
            if all(phases.get(n) in ("Succeeded", "Failed") for n in ("no-gpu", "one-gpu")):
                break
            time.sleep(0.2)
        logs = {n: kc("logs", n).stdout for n in ("no-gpu", "one-gpu")}
        outs = {n: json.loads(t.strip().splitlines()[-1]) for n, t in logs.items()}
        assert outs["no-gpu"]["device_count"] == 0, outs
        assert outs["one-gpu"]["device_count"] == 1 and phases["one-gpu"] == "Succeeded", (outs, phases)
        for n, t in logs.items():
            for f in secrets:
                assert f"denied {f}" in t, (n, t)
        d = kc("describe", "pod", "no-gpu").stdout
        assert "Isolation:" in d and "landlock" in d and "may open no GPU" in d, d
        # no user namespaces on this tier: the CPU pod shares the host's PIDs, its signals are scoped
        assert "signals scoped to the pod" in d or "user,pid,mount" in d, d
        d = kc("describe", "pod", "one-gpu").stdout
        assert "node state denied" in d and "signals scoped to the pod" in d, d
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


@pytest.mark.parametrize("knob", [{"TK8S_HSA_CPU_CACHES": "1"}, {"TK8S_HOST_BURNIN": "0"}],
                         ids=["cpu-cache-walk-kept", "no-early-burnin"])
def test_setup_without_a_startup_shortcut_on_a_real_gpu(tmp_path, knob):
    """with the CPU-cache-walk skip switched off, or without the early host
    burn-in, the bring-up takes the plain path and still validates."""
    import subprocess

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = _real_ws(tmp_path)
    env.update(knob)
    (tmp_path / "answers.json").write_text(json.dumps({"nodes": 1, "package": "mi355x-1gpu", "confirm": "yes"}))
    try:
        r = subprocess.run(["./setup.sh", "--answers", "answers.json", "--yes", "--json", "--port", "0", "--timeout",
                            "120"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["gpus_allocatable"] == 1 and s["nodes_validated"] == 1, s
        if knob.get("TK8S_HOST_BURNIN") == "0":  # the validation pod probed the GPU itself
            assert not s.get("host_burnin"), s.get("host_burnin")
        else:
            assert (s.get("host_burnin") or {}).get("ok"), s.get("host_burnin")
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_setup_on_the_plain_path_on_a_real_gpu(tmp_path):
    """TK8S_SHORTCUTS=0 turns every start-up shortcut off at once (no preloaded
    or early burn-in, no zygotes, no caches, interpreters with site processing): the validation
    DaemonSet then probes the GPU itself, and the bring-up still reaches Ready, validated."""
    import subprocess

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = _real_ws(tmp_path)
    env["TK8S_SHORTCUTS"] = "0"
    (tmp_path / "answers.json").write_text(json.dumps({"nodes": 1, "package": "mi355x-1gpu", "confirm": "yes"}))
    try:
        r = subprocess.run(["./setup.sh", "--answers", "answers.json", "--yes", "--json", "--port", "0", "--timeout",
                            "120"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["gpus_allocatable"] == 1 and s["nodes_validated"] == 1, s
        assert not s.get("host_burnin"), s.get("host_burnin")  # the plain path: no early burn-in
        v = next(iter(s["validation"].values()))
        assert float(v["hbm-write-gbps"]) > 1000.0 and float(v["md5-mbps"]) > 1000.0, v
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_multi_gpu_burnin_command_runs_on_one_gpu(tmp_path):
    """The host burn-in command a >= 2-GPU bring-up runs (the HSA payload by default, VERDICT r5
    #5, --peers with the Ready path's 16 MiB pulls, earlyburn.host_burnin_command) parses and
    passes on the one GPU here, and its JSON is what the burn-in split and the xGMI judge read;
    its HIP fallback command too."""
    import os
    import subprocess

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tritonk8ssupervisor_amd import earlyburn, xgmi

    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    cmd = earlyburn.host_burnin_command(earlyburn.default_validation_command(peers=False), [0, 1])
    assert os.path.basename(cmd[0]) == "tk8s-hsaprobe" and cmd[cmd.index("--peer-bytes") + 1] == str(16 << 20), cmd
    for c in (cmd, earlyburn.hip_peer_command(cmd)):
        r = subprocess.run(c + ["--out", str(tmp_path / "r.json")], capture_output=True, text=True, timeout=120,
                           env={**env, "ROCR_VISIBLE_DEVICES": "0"})
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        res = json.loads((tmp_path / "r.json").read_text())
        assert res["ok"] and res["device_count"] == 1, res
        if c is cmd:
            assert res["md5"]["digest"] == res["md5_expected"], res
        rep = xgmi.link_report(res, [0])
        assert rep["pulls"] == 0 and not rep["degraded"]


def test_gpu_busy_metric_and_hpa_on_a_real_gpu(tmp_path):
    """A pod keeping its MI355X busy shows up in the metrics API as amd.com/gpu-utilization (AMD SMI
    gfx activity, sampled by the node agent), and an HPA on resource amd.com/gpu scales its
    Deployment up from it."""
    import subprocess
    import sys as _sys
    import time

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tritonk8ssupervisor_amd.controlplane.client import client_from_kubeconfig

    env = _real_ws(tmp_path)
    env.update(TK8S_SMI_INTERVAL="1", TK8S_SMI_DELAY="0.5", TK8S_METRICS_PERIOD="1", TK8S_HPA_PERIOD="2")
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=60)
    busy = ("import time, torch\n"
            "a = torch.randn(8192, 8192, device='cuda', dtype=torch.bfloat16)\n"
            "print('busy', flush=True)\n"
            "t = time.time()\n"
            "while time.time() - t < 40:\n"
            "    for _ in range(20):\n"
            "        a = (a @ a) * 1e-4\n"
            "    torch.cuda.synchronize()\n")
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "120"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        (tmp_path / "busy.json").write_text(json.dumps({"apiVersion": "v1", "kind": "List", "items": [
            {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "busy"},
             "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "busy"}},
                      "template": {"metadata": {"labels": {"app": "busy"}}, "spec": {"containers": [{
                          "name": "c", "command": [_sys.executable, "-c", busy],
                          "resources": {"limits": {"amd.com/gpu": 1}}}]}}}},
            {"apiVersion": "autoscaling/v2", "kind": "HorizontalPodAutoscaler", "metadata": {"name": "busy"},
             "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "busy"},
                      "minReplicas": 1, "maxReplicas": 2,
                      "metrics": [{"type": "Resource", "resource": {"name": "amd.com/gpu", "target": {
                          "type": "Utilization", "averageUtilization": 20}}}]}}]}))
        assert kc("apply", "-f", "busy.json").returncode == 0
        k = client_from_kubeconfig(json.loads((tmp_path / ".tk8s" / "kubeconfig.json").read_text()))
        deadline = time.monotonic() + 100
        seen, replicas = 0.0, 1
        while time.monotonic() < deadline:
            for m in k.get(k.k8s("/apis/metrics.k8s.io/v1beta1/namespaces/default/pods"))["items"]:
                for c in m["containers"]:
                    seen = max(seen, float(c["usage"].get("amd.com/gpu-utilization", 0)))
            replicas = json.loads(kc("get", "deploy", "busy", "-o", "json").stdout)["spec"]["replicas"]
            if seen >= 20 and replicas == 2:
                break
            time.sleep(1)
        hpa = json.loads(kc("get", "hpa", "busy", "-o", "json").stdout)
        assert seen >= 20, (seen, hpa.get("status"), kc("logs", json.loads(kc("get", "pods", "-o", "json").stdout)[
            "items"][-1]["metadata"]["name"]).stdout[-500:])
        assert replicas == 2, hpa.get("status")
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def _allreduce_job(completions: int, max_bytes: int) -> dict:
    """manifests/examples/torch-allreduce-job.yaml with ``completions`` ranks and RCCL's INFO log on."""
    from pathlib import Path

    import yaml

    job = yaml.safe_load((Path(__file__).resolve().parents[1] / "manifests" / "examples" /
                          "torch-allreduce-job.yaml").read_text())
    job["spec"].update(completions=completions, parallelism=completions)
    c = job["spec"]["template"]["spec"]["containers"][0]
    c["command"][c["command"].index("--max-bytes") + 1] = str(max_bytes)
    c.setdefault("env", []).extend([{"name": "NCCL_DEBUG", "value": "INFO"},
                                    {"name": "NCCL_DEBUG_SUBSYS", "value": "INIT,P2P,SHM,NET"}])
    return job


def _rank_results(kc, n: int, timeout: float) -> dict:
    import time

    deadline = time.monotonic() + timeout
    pods = {}
    while time.monotonic() < deadline:
        pods = {p["metadata"]["name"]: p for p in json.loads(kc("get", "pods", "-o", "json").stdout)["items"]
                if (p["metadata"].get("labels") or {}).get("job-name") == "torch-allreduce"}
        if len(pods) == n and all(p["status"].get("phase") in ("Succeeded", "Failed") for p in pods.values()):
            break
        time.sleep(0.5)
    out = {}
    for name, p in pods.items():
        log = kc("logs", name).stdout
        lines = [x for x in log.strip().splitlines() if x.startswith("{") and '"nranks"' in x]
        assert p["status"].get("phase") == "Succeeded" and lines, (name, p.get("status"), log[-3000:])
        out[name] = (p, json.loads(lines[-1]), log)
    assert len(out) == n, pods.keys()
    return out


def test_torch_allreduce_job_manifest_on_one_gpu(tmp_path):
    """VERDICT r3 next-4, the 1-GPU variant: the example Job (one rank, its gpu-peers opt-in on,
    NCCL_DEBUG=INFO) runs in the jail on the MI355X, RCCL's init completes and the rank reports
    what its log says about transports. Also VERDICT r3 next-2 on the box: the rank runs on its
    GPU's NUMA-local CPUs."""
    import os
    import subprocess

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = _real_ws(tmp_path)
    kc = lambda *a, stdin=None: subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True, text=True,
                                               timeout=60, input=stdin)
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--timeout", "120"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        job = _allreduce_job(1, 16 << 20)
        job["spec"]["template"]["spec"]["containers"][0]["command"] = [
            "sh", "-c", 'grep Cpus_allowed_list /proc/self/status >&2; exec "$0" "$@"',
            *job["spec"]["template"]["spec"]["containers"][0]["command"]]
        assert kc("apply", "-f", "-", stdin=json.dumps(job)).returncode == 0
        (name, (p, res, log)), = _rank_results(kc, 1, 180).items()
        assert res["ok"] and res["backend"] == "nccl" and res["nranks"] == 1, res
        assert all(x["bad"] == 0 for x in res["results"])
        assert res["transport"]["init_complete"], (res["transport"], log[-3000:])
        assert "NCCL INFO" in log  # the rank's RCCL log is in the pod log
        d = kc("describe", "pod", name).stdout
        assert "no Job peer on this host" in d and "may open gpu" in d, d
        node = json.loads(kc("get", "node", p["spec"]["nodeName"], "-o", "json").stdout)
        minor = node["status"]["devices"][0].get("renderMinor", -1)
        local_f = f"/sys/class/drm/renderD{minor}/device/local_cpulist"
        if minor >= 0 and os.path.exists(local_f):
            from tritonk8ssupervisor_amd.agent.resources import parse_cpulist

            local = set(parse_cpulist(open(local_f).read().strip()))
            got = set(parse_cpulist(next(x for x in log.splitlines() if x.startswith("Cpus_allowed_list")).split()[-1]))
            want = local & os.sched_getaffinity(0) or os.sched_getaffinity(0)
            assert got == want, (sorted(got)[:8], len(got), sorted(local)[:8], len(local))
        if os.environ.get("GRAFT_REPO_ROOT"):  # evidence for profiles/: what the rank saw
            from pathlib import Path

            ev = Path(os.environ["GRAFT_REPO_ROOT"]) / "gpurun_out" / "torch_job_1gpu.json"
            ev.parent.mkdir(parents=True, exist_ok=True)
            ev.write_text(json.dumps({"result": res, "describe": d, "render_minor": minor,
                                      "cpus_allowed": next((x for x in log.splitlines()
                                                            if x.startswith("Cpus_allowed_list")), ""),
                                      "local_cpulist": open(local_f).read().strip() if os.path.exists(local_f) else None,
                                      "rccl_log_tail": [x for x in log.splitlines() if "NCCL INFO" in x][-40:]}, indent=1))
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X (xGMI)")
def test_torch_allreduce_job_two_pods_goes_p2p_over_xgmi(tmp_path):
    """the example Job with 2 one-GPU pods (two workers of one host). With the
    Job's gpu-peers opt-in each rank can open its peer's GPU, and every RCCL channel is P2P --
    no SHM, no NET -- at a bus bandwidth above the 2-GPU xGMI floor."""
    import subprocess

    from tritonk8ssupervisor_amd.xgmi import fabric_floors

    env = _real_ws(tmp_path)
    kc = lambda *a, stdin=None: subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True, text=True,
                                               timeout=60, input=stdin)
    try:
        r = subprocess.run(["./setup.sh", "--nodes", "2", "--yes", "--json", "--port", "0", "--timeout", "240",
                            "--rccl", "off"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=400)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
        assert kc("apply", "-f", "-", stdin=json.dumps(_allreduce_job(2, 64 << 20))).returncode == 0
        ranks = _rank_results(kc, 2, 300)
        for name, (p, res, log) in ranks.items():
            t = res["transport"]
            assert res["ok"] and res["nranks"] == 2 and t["init_complete"], (res, log[-3000:])
            assert t["counts"].get("P2P", 0) > 0, (t, log[-3000:])
            assert t["counts"].get("SHM", 0) == 0 and t["counts"].get("NET", 0) == 0, t  # no host fallback
            assert res["peak_busbw_gbps"] > fabric_floors(2)["allreduce_busbw_gbps"], res
            assert "Job peers on this host" in kc("describe", "pod", name).stdout
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def test_resource_limits_are_enforced_unprivileged_on_the_gpu_box(tmp_path):
    """VERDICT r4 next-3 on the target box itself (an ordinary user, no delegated cgroup): a real
    1-GPU bring-up picks the watchdog, a CPU pod with limits.cpu 250m spinning for 3 s of wall
    time gets at most ~0.35 CPU from the SIGSTOP/SIGCONT duty cycle, and a pod that grows past
    limits.memory 64Mi is OOMKilled."""
    import os
    import shutil
    import subprocess
    import sys
    import time
    from pathlib import Path

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parents[1]
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(repo / f, tmp_path / f)
    env = {k: v for k, v in os.environ.items() if k not in ("TK8S_FAKE_GPUS", "TK8S_POD_RESOURCES")}
    env.update(PYTHONPATH=str(repo), TK8S_PYTHON=sys.executable)

    def kc(*a, stdin=None):
        p = subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120,
                           input=stdin)
        assert p.returncode == 0, f"kubectl {' '.join(a)}: {p.stdout}{p.stderr}"
        return p

    def until_done(name, timeout=60.0):
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            pod = json.loads(kc("get", "pod", name, "-o", "json").stdout)
            if pod["status"].get("phase") in ("Succeeded", "Failed"):
                return pod
            time.sleep(0.2)
        raise AssertionError(f"pod {name} did not finish")

    try:
        r = subprocess.run(["./setup.sh", "--nodes", "1", "--yes", "--json", "--port", "0", "--rccl", "off"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        node = json.loads(kc("get", "node", "kubenode1", "-o", "json").stdout)
        enf = node["metadata"]["annotations"]["tk8s.amd.com/resource-enforcement"]
        if not enf.startswith("watchdog"):
            pytest.skip(f"this box delegates cgroups ({enf[:80]}): the kernel enforces, not the duty cycle")
        assert "duty cycle" in enf and "NOT enforced" not in enf, enf
        busy = ("import os, time\nt = time.time()\nwhile time.time() - t < 5:\n    pass\n"
                "u = os.times()\nprint('cpu', round(u.user + u.system, 3), flush=True)\n")
        kc("apply", "-f", "-", stdin=json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "spin"},
                                                  "spec": {"restartPolicy": "Never", "containers": [{
                                                      "name": "c", "command": [sys.executable, "-c", busy],
                                                      "resources": {"limits": {"cpu": "250m"}}}]}}))
        until_done("spin")
        out = kc("logs", "spin").stdout.split()
        used = float(out[out.index("cpu") + 1])
        assert used <= 0.35 * 5.0, out  # <= 0.35 CPU over 5 s (interpreter start included)
        # 8 MiB a tenth of a second, every page touched: the resident-set sampler (0.5 s) sees it
        # far below the RLIMIT_DATA backstop (2 x 64Mi + 256Mi), which would end it differently
        grow = ("import time\nb = []\nwhile True:\n    b.append(bytearray(8 << 20))\n"
                "    for i in range(0, len(b[-1]), 4096):\n        b[-1][i] = 1\n    time.sleep(0.1)\n")
        kc("apply", "-f", "-", stdin=json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "grow"},
                                                  "spec": {"restartPolicy": "Never", "containers": [{
                                                      "name": "c", "command": [sys.executable, "-c", grow],
                                                      "resources": {"limits": {"memory": "64Mi"}}}]}}))
        pod = until_done("grow")
        term = (pod["status"].get("containerStatuses") or [{}])[0].get("state", {}).get("terminated", {})
        assert pod["status"]["phase"] == "Failed" and term.get("reason") == "OOMKilled", pod["status"]
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)
