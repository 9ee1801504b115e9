"""Native layer on the CPU box: the gfx950 build (hipcc cross-compiles without a GPU), the
restart-policy supervisor (tk8s-supervise, the `docker --restart` of the reference's
rancher/server and rancher/agent, ranchermaster/tasks/main.yml:11) and the tools' no-GPU
failure mode (fail loudly, never a silent fallback)."""
import json
import os
import signal
import subprocess
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
BIN = REPO / "tritonk8ssupervisor_amd" / "bin"


def test_build_produces_gfx950_code_objects(native_build):
    for name in ("libtk8s", "libtk8s_rccl", "native_module", "topo_module", "tk8s-supervise", "tk8s-smi",
                 "tk8s-gpuinfo", "tk8s-probe", "tk8s-rccl"):
        assert Path(native_build[name]).exists(), name
    lib = Path(native_build["libtk8s"]).read_bytes()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in lib  # device code is built for MI355X only
    assert b"gfx942" not in lib and b"gfx90a" not in lib


def _needed(path) -> list[str]:
    out = subprocess.run(["readelf", "-d", str(path)], capture_output=True, text=True, check=True).stdout
    return [line.split("[", 1)[1].split("]", 1)[0] for line in out.splitlines() if "(NEEDED)" in line]


def test_only_rccl_artefacts_link_librccl(native_build):
    # librccl is ~0.5 GB: the probe and gpuinfo payloads on the bring-up critical path must not map it
    for name in ("libtk8s", "tk8s-probe", "tk8s-gpuinfo"):
        assert not any(n.startswith("librccl") for n in _needed(native_build[name])), name
    for name in ("libtk8s_rccl", "tk8s-rccl", "native_module"):
        assert any(n.startswith("librccl") for n in _needed(native_build[name])), name


@pytest.mark.parametrize("tool", ["tk8s-hsaprobe", "tk8s-probe", "tk8s-gpuinfo", "tk8s-rccl"])
def test_gpu_tools_export_their_opendir_for_the_thunk(native_build, tool):
    # the per-CPU cache walk of the runtime start is skipped by the tool's own opendir
    # (native/tools/cachewalk.h, profiles/r2_hsainit/): it only takes effect if the dynamic symbol
    # table carries it ahead of libc's
    out = subprocess.run(["nm", "-D", "--defined-only", str(native_build[tool])],
                         capture_output=True, text=True, check=True).stdout
    assert any(line.split()[-1] == "opendir" and line.split()[-2] == "T" for line in out.splitlines() if line.strip())


def test_smi_tool_is_hip_free_and_fails_loudly_without_a_gpu(native_build):
    smi = native_build["tk8s-smi"]
    needed = _needed(smi)
    assert any(n.startswith("libamd_smi") for n in needed)
    assert not any(n.startswith(("libamdhip64", "librccl", "libhsa")) for n in needed)  # agent-safe: no KFD process
    if Path("/dev/kfd").exists():
        pytest.skip("a GPU host: covered by the GPU suite")
    r = subprocess.run([str(smi), "--no-links"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3
    out = json.loads(r.stdout)
    assert out["ok"] is False and out["error"]


def test_build_is_incremental(native_build):
    from tritonk8ssupervisor_amd.utils.build_native import build

    before = {k: Path(v).stat().st_mtime for k, v in native_build.items()}
    t = time.monotonic()
    out = build()
    assert {k: Path(v).stat().st_mtime for k, v in out.items()} == before  # nothing rebuilt
    assert time.monotonic() - t < 20  # a rebuild of the HIP layer takes minutes; the checks, seconds


def test_native_module_imports_without_a_gpu(native_build):
    from tritonk8ssupervisor_amd.ops import native

    nat = native()
    info = json.loads(nat.gpuinfo_json(False))
    if info.get("ok"):
        pytest.skip("a GPU is visible here")
    assert info["device_count"] == 0 and "error" in info


def test_busbw_is_the_n3_formula_at_every_n(native_build):
    """busbw = algbw * 2(n-1)/n -- 0 at one rank, where the
    all-reduce is a local copy (the fabric line then says "1 GPU: no fabric", busbw null) -- in
    the native validator, its gloo twin and the fabric report alike."""
    from tritonk8ssupervisor_amd.fabric import bandwidth_summary, fabric_line
    from tritonk8ssupervisor_amd.ops import native

    nat = native()
    for n, want in ((1, 0.0), (2, 100.0), (4, 150.0), (8, 175.0)):
        assert nat.allreduce_busbw(100.0, n) == pytest.approx(want)
    one = bandwidth_summary([{"ok": True, "peak_algbw_gbps": 3381.0, "peak_busbw_gbps": None}], 1)
    assert one == {"peak_busbw_gbps": None, "peak_algbw_gbps": 3381.0, "fabric": "1 GPU: no fabric"}
    assert "no fabric" in fabric_line({**one, "nranks": 1})
    eight = bandwidth_summary([{"peak_algbw_gbps": 100.0, "peak_busbw_gbps": 175.0},
                               {"peak_algbw_gbps": 90.0, "peak_busbw_gbps": 157.5}], 8)
    assert eight == {"peak_busbw_gbps": 175.0, "peak_algbw_gbps": 100.0}
    assert fabric_line({**eight, "nranks": 8}) == "RCCL all-reduce peak busbw 175.0 GB/s over 8 GPU(s)"


def test_the_validator_defaults_are_the_rccl_tests_sweep():
    """8 B x2 to >= 1 GiB, fp32 and bf16 -- tk8s-rccl's defaults (the fabric check on
    the Ready path asks for its shorter sweep explicitly and says so)."""
    src = (REPO / "native" / "tools" / "tk8s_rccl.cpp").read_text()
    assert 'a.num("min-bytes", 8)' in src and 'a.num("max-bytes", 1LL << 30)' in src
    assert 'a.num("factor", 2)' in src and 'a.str("dtype", "both")' in src


@pytest.mark.parametrize("tool", ["tk8s-gpuinfo", "tk8s-probe"])
def test_tools_fail_loudly_without_a_gpu(native_build, tool):
    if Path("/dev/kfd").exists():
        pytest.skip("GPU host")
    r = subprocess.run([str(BIN / tool)], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert json.loads(r.stdout)["ok"] is False


def _pidfile(p):
    deadline = time.monotonic() + 5
    while time.monotonic() < deadline:
        try:
            return json.loads(Path(p).read_text())
        except (OSError, ValueError):
            time.sleep(0.01)
    raise AssertionError("no pidfile")


def test_supervise_restarts_on_failure_then_gives_up(native_build, tmp_path):
    pf, log, cnt = tmp_path / "x.pid", tmp_path / "x.log", tmp_path / "count"
    r = subprocess.run([str(BIN / "tk8s-supervise"), "--pidfile", str(pf), "--log", str(log), "--restart", "on-failure",
                        "--max-restarts", "2", "--backoff-ms", "10", "--", "sh", "-c", f"echo run >> {cnt}; exit 3"],
                       timeout=30)
    assert r.returncode == 3
    assert cnt.read_text().count("run") == 3  # first run + 2 restarts
    assert "not restarting" in log.read_text()
    assert not pf.exists()


def test_supervise_on_failure_does_not_restart_success(native_build, tmp_path):
    cnt = tmp_path / "count"
    r = subprocess.run([str(BIN / "tk8s-supervise"), "--pidfile", str(tmp_path / "p"), "--restart", "on-failure", "--",
                        "sh", "-c", f"echo run >> {cnt}"], timeout=30, capture_output=True)
    assert r.returncode == 0 and cnt.read_text().count("run") == 1


def test_supervise_sigterm_stops_child_and_group(native_build, tmp_path):
    pf = tmp_path / "s.pid"
    p = subprocess.Popen([str(BIN / "tk8s-supervise"), "--pidfile", str(pf), "--restart", "unless-stopped", "--",
                          "sleep", "600"], start_new_session=True)
    info = _pidfile(pf)
    assert info["pid"] == p.pid and info["pgid"] == p.pid and info["restarts"] == 0
    child = info["child"]
    os.kill(child, signal.SIGKILL)  # crash the child: it comes back
    deadline = time.monotonic() + 5
    while time.monotonic() < deadline and _pidfile(pf)["child"] == child:
        time.sleep(0.01)
    info2 = _pidfile(pf)
    assert info2["child"] != child and info2["restarts"] == 1
    p.send_signal(signal.SIGTERM)
    assert p.wait(10) is not None
    assert not pf.exists()
    with pytest.raises(ProcessLookupError):
        os.kill(info2["child"], 0)


def test_supervise_usage_errors(native_build):
    r = subprocess.run([str(BIN / "tk8s-supervise"), "--restart", "sometimes", "--", "true"], capture_output=True)
    assert r.returncode == 2 and b"usage" in r.stderr


def test_summarize_rocprof_stats(tmp_path):
    from tritonk8ssupervisor_amd.orchestrator import summarize_rocprof

    d = tmp_path / "prof" / "host"
    d.mkdir(parents=True)
    (d / "rank0_kernel_stats.csv").write_text(
        '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
        '"small",2,100,50,1,40,60,1\n"ncclDevKernel_Generic",10,90000,9000,99,8000,10000,5\n')
    s = summarize_rocprof(tmp_path / "prof")
    assert list(s["ranks"]) == ["rank0"]
    assert s["ranks"]["rank0"][0] == {"kernel": "ncclDevKernel_Generic", "calls": 10, "total_us": 90.0, "avg_us": 9.0}


def test_supervise_spawn_list_starts_one_supervisor_per_line_each_in_its_own_session(native_build, tmp_path):
    """`tk8s-supervise --spawn-list FILE` (how the CLI hands over its node-agent zygotes): one
    supervisor per tab-separated line, each a session leader with its pidfile, the helper gone."""
    sup = native_build["tk8s-supervise"]
    import shutil

    sleep = shutil.which("sleep")
    lines = [f"--pidfile\t{tmp_path / f'{n}.pid'}\t--restart\tno\t--\t{sleep}\t30" for n in ("a", "b")]
    (tmp_path / "list").write_text("\n".join(lines) + "\n\n")
    # (stdio not captured: the supervisors inherit it, as the CLI's helper gives them /dev/null)
    r = subprocess.run([str(sup), "--spawn-list", str(tmp_path / "list")], stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL, timeout=10)
    assert r.returncode == 0
    pids = []
    deadline = time.monotonic() + 5
    for n in ("a", "b"):
        while not (tmp_path / f"{n}.pid").exists() and time.monotonic() < deadline:
            time.sleep(0.01)
        rec = json.loads((tmp_path / f"{n}.pid").read_text())
        assert rec["pid"] == rec["pgid"] == os.getsid(rec["pid"]) and rec["child"] > 0, rec
        pids.append(rec["pid"])
    assert len(set(pids)) == 2
    for pid in pids:
        os.killpg(pid, signal.SIGTERM)
    assert subprocess.run([str(sup), "--spawn-list", str(tmp_path / "missing")], capture_output=True, timeout=10).returncode == 2
