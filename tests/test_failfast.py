"""Fail fast on the fabric and link path, on the CPU.

* ``native/include/tk8s/failfast.h`` -- the deadlines, watchdog and TK8S_FAULTS points of
  tk8s-rccl / tk8s-probe / tk8s-hsaprobe -- under AddressSanitizer + UBSan (host code).
* The gloo twin of tk8s-rccl (parallel/dist_allreduce.py, the fabric check's payload when the
  GPUs are faked) at 2 and 8 ranks with one rank hung or dead: every rank must end within its
  deadline with a JSON line naming the phase -- never a hang (the reference's readiness loop has
  no bound at all: /root/reference/setup.sh:56-85).
"""
import json
import os
import shutil
import subprocess
import sys
import time
from pathlib import Path

import pytest

from test_controlplane import _start, _stop

REPO = Path(__file__).resolve().parents[1]
NATIVE = REPO / "native"
SAN = ["-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all",
       "-pthread"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def selftest(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = tmp_path_factory.mktemp("failfast") / "failfast_selftest"
    r = subprocess.run(["g++", *SAN, f"-I{NATIVE / 'include'}", str(NATIVE / "tests" / "failfast_selftest.cpp"),
                        "-o", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def _run(exe, *args, faults="", timeout=30):
    return subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, timeout=timeout,
                          env={**ENV, "TK8S_FAULTS": faults})


@pytest.mark.parametrize("faults,query,want", [
    ("rccl.hang@sweep", ("rccl", "hang", "sweep", 0, 1), "1"),
    ("rccl.hang@sweep", ("rccl", "hang", "check", 0, 1), "0"),
    ("rccl.exit@init:3", ("rccl", "exit", "init", 3, 1), "1"),
    ("rccl.exit@init:3", ("rccl", "exit", "init", 2, 1), "0"),
    ("rccl.exit@init:3", ("rccl", "exit", "init", 0, 8), "1"),     # a process holding ranks 0..7
    ("rccl.exit@init:3", ("rccl", "exit", "init", -1, 0), "0"),    # ranks not known yet: targeted points off
    ("rccl.exit@init:x", ("rccl", "exit", "init", 0, 8), "0"),     # malformed rank: matches nothing
    ("probe.hang_peers", ("probe", "hang", "peers", 0, 1), "1"),   # the VERDICT's shorthand names
    ("probe.crash", ("probe", "crash", "peers", 0, 1), "1"),
    (" xgmi.degrade@0-1:0.1 , rccl.hang@uid ", ("rccl", "hang", "uid", 5, 1), "1"),
])
def test_fault_points_parse_like_utils_faults(selftest, faults, query, want):
    r = _run(selftest, "armed", *query, faults=faults)
    assert r.returncode == 0 and r.stdout.strip() == want, r.stdout + r.stderr


def test_fault_point_kinds(selftest):
    assert _run(selftest, "point", "rccl", "init", faults="rccl.exit@init").returncode == 3
    r = _run(selftest, "point", "rccl", "init", faults="rccl.crash@init")
    assert r.returncode in (-6, 134) and "aborting" in r.stderr
    r = _run(selftest, "point", "rccl", "init", faults="rccl.exit@sweep")
    assert r.returncode == 0 and r.stdout.strip() == "passed"
    with pytest.raises(subprocess.TimeoutExpired):  # a host hang really hangs (the watchdog ends it)
        _run(selftest, "point", "rccl", "uid", faults="rccl.hang@uid", timeout=1.5)


def test_watchdog_ends_a_process_that_makes_no_progress(selftest):
    t0 = time.monotonic()
    r = _run(selftest, "watchdog", "0.3")
    dt = time.monotonic() - t0
    assert r.returncode == 4, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"ok": False, "phase": "sweep", "waited_s": pytest.approx(0.3, abs=0.2)}
    assert dt < 5.0


def test_poll_until_bounds_and_errors(selftest):
    r = _run(selftest, "poll")
    assert r.returncode == 0 and "poll ok" in r.stdout, r.stdout + r.stderr


# ---- the gloo twin: one rank of a job hung or dead ------------------------------------------
def _job(tmp_path, nranks, faults, op_timeout):
    p, c = _start(tmp_path)
    try:
        url = f"{c.base}/v1/kv/ff-{nranks}/uid"
        env = {**os.environ, "TK8S_KV_TOKEN": c.token, "TK8S_FAULTS": faults, "OMP_NUM_THREADS": "1"}
        t0 = time.monotonic()
        procs = [subprocess.Popen([sys.executable, "-m", "tritonk8ssupervisor_amd.parallel.dist_allreduce", "--rank", str(r),
                                   "--nranks", str(nranks), "--kv-url", url, "--max-bytes", str(64 << 10),
                                   "--op-timeout", str(op_timeout)],
                                  cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
                 for r in range(nranks)]
        res = []
        for pr in procs:
            out, err = pr.communicate(timeout=op_timeout * 4 + 60)
            lines = [x for x in out.strip().splitlines() if x.startswith("{")]  # (gloo logs on stdout too)
            res.append({"rc": pr.returncode, "out": json.loads(lines[-1]) if lines else {}, "err": err[-800:],
                        "t": time.monotonic() - t0})
    finally:
        _stop(p)
    return res


@pytest.mark.parametrize("nranks,faults,victim,kind", [
    (2, "rccl.hang@sweep:1", 1, "hang"),
    (2, "rccl.exit@sweep:1", 1, "exit"),
    (2, "rccl.hang@uid:0", 0, "hang"),        # rank 0 never publishes its address
    (8, "rccl.hang@sweep:5", 5, "hang"),
    (8, "rccl.exit@init:3", 3, "exit"),
])
def test_one_rank_hung_or_dead_every_rank_ends_within_its_deadline(tmp_path, nranks, faults, victim, kind):
    op = 6.0 if nranks == 8 else 4.0
    res = _job(tmp_path, nranks, faults, op)
    bound = op * 2 + 10 + 25  # a deadline, the watchdog's grace, and interpreter start-up under load
    for r, x in enumerate(res):
        assert x["t"] < bound, (r, x)
        if not (r == victim and kind == "exit"):  # (a rank that died says nothing)
            assert x["out"].get("ok") is False, (r, x)  # nobody claims a pass for a broken job
        if r == victim:
            assert x["rc"] == (4 if kind == "hang" else 3), (r, x)
            if kind == "hang":
                assert x["out"]["watchdog"] and x["out"]["phase"] == faults.split("@")[1].split(":")[0], x
        else:
            assert x["rc"] in (2, 4), (r, x)
            assert x["out"]["phase"] in ("uid", "init", "sweep", "check"), (r, x)


# ---- the HSA payload's peer phase falls back to the HIP probe --------------
def _pull(src, dst, ok=True, error=None, gbps=60.0):
    p = {"ok": ok, "probe": "xgmi_peer_pull", "src_device": src, "dst_device": dst, "bytes": 16 << 20}
    if error:
        p["error"] = error
    else:
        p.update(kernel_gbps=gbps, bad_words=0)
    return p


def _result(runtime, pulls_ok=True, error=None):
    devs = []
    for d in (0, 1):
        pulls = [_pull(1 - d, d, ok=pulls_ok, error=None if pulls_ok else error)]
        devs.append({"device": d, "ok": True, "hbm": {"ok": True}, "md5": {"ok": True}, "copy": {"ok": True},
                     "digest_ok": True, "peers": pulls, "peers_ok": pulls_ok})
    return {"ok": True, "runtime": runtime, "device": 0, "device_count": 2, "probed": 2, "devices": devs,
            "timings_ms": {"total": 1.0}}


def _fake_tools(tmp_path, hsa_mode):
    """tk8s-hsaprobe / tk8s-probe stand-ins: the HSA one writes a result whose pulls timed out, or
    aborts without one; the HIP one prints passing pulls (and records that it ran)."""
    bindir = tmp_path / "bin"
    bindir.mkdir()
    bad = json.dumps(_result("hsa", pulls_ok=False, error="GPU dispatch did not complete within 3 s"))
    good = json.dumps(_result("hip"))
    hsa = bindir / "tk8s-hsaprobe"
    body = {"timeout": f"printf '%s\\n' '{bad}' > \"$out.tmp\" && mv \"$out.tmp\" \"$out\"",
            "crash": "kill -ABRT $$"}[hsa_mode]
    hsa.write_text("#!/bin/sh\nout=''\nwhile [ $# -gt 0 ]; do [ \"$1\" = --out ] && out=\"$2\"; shift; done\n"
                   f"{body}\n")
    hip = bindir / "tk8s-probe"
    hip.write_text(f"#!/bin/sh\necho \"$@\" > {tmp_path}/hip-args\nprintf '%s\\n' '{good}'\n")
    for f in (hsa, hip):
        f.chmod(0o755)
    return hsa


@pytest.mark.parametrize("hsa_mode", ["timeout", "crash"])
def test_hsa_peer_phase_failure_falls_back_to_the_hip_probe(tmp_path, monkeypatch, hsa_mode):
    from tritonk8ssupervisor_amd.burnin import HostBurnin, split_host_result
    from tritonk8ssupervisor_amd.xgmi import annotations

    monkeypatch.setenv("TK8S_FAKE_GPUS", "2")  # (visibility env only; the tools above are what runs)
    monkeypatch.setenv("TK8S_HOST_REGISTRY", str(tmp_path / "hostreg"))
    monkeypatch.delenv("TK8S_PEERS_RUNTIME", raising=False)
    hsa = _fake_tools(tmp_path, hsa_mode)
    events = []
    cmd = [str(hsa), "--all-devices", "--gpuinfo", "--peers", "--peer-bytes", str(16 << 20), "--iters", "2"]
    hb = HostBurnin(cmd, [0, 1], tmp_path / "state", log=lambda ev, **kw: events.append((ev, kw)))
    assert hb.start()
    assert hb.finished.wait(60)
    r = hb.result
    assert r is not None and r["peers_runtime"] == "hip-fallback", r
    assert all(p["ok"] and p["runtime"] == "hip" for d in r["devices"] for p in d["peers"]), r
    hip_args = (tmp_path / "hip-args").read_text().split()
    if hsa_mode == "timeout":  # pulls only: the HSA payload's own probes stand
        assert hip_args[hip_args.index("--hbm-bytes") + 1] == "0" and "--skip-md5" in hip_args
        assert r["devices"][0]["hsa_peer_errors"] and r["runtime"] == "hsa"
    else:  # no HSA result at all: the HIP probe ran the whole validation
        assert "--hbm-bytes" not in hip_args and r["runtime"] == "hip"
    assert [e for e, _ in events].count("gpu_burnin_peer_fallback") == 1
    share = split_host_result(r, [0, 1], [0], hb.xgmi)
    assert share["ok"] and share["xgmi"]["healthy"] and share["xgmi"]["runtimes"] == ["hip-fallback"]
    assert annotations(share["xgmi"])["tk8s.amd.com/xgmi-runtime"] == "hip-fallback"
    # learned: the next bring-ups on this host pull through the HIP probe directly
    from tritonk8ssupervisor_amd import earlyburn

    assert earlyburn.hsa_peers_failed()
    assert os.path.basename(earlyburn.probe_tool(peers=True)) == "tk8s-probe"
    monkeypatch.setenv("TK8S_PEERS_RUNTIME", "hsa")
    assert not earlyburn.hsa_peers_failed()


def test_no_fallback_for_a_passing_hsa_run_or_a_bad_word_verdict():
    from tritonk8ssupervisor_amd.burnin import peer_fallback_reason

    cmd = ["/x/tk8s-hsaprobe", "--all-devices", "--peers"]
    assert peer_fallback_reason(cmd, _result("hsa"), 0, 2) is None
    wrong = _result("hsa")
    wrong["devices"][0]["peers"][0].update(ok=False, bad_words=12)  # the link moved wrong bytes: a verdict
    assert peer_fallback_reason(cmd, wrong, 0, 2) is None
    assert peer_fallback_reason(cmd, None, 134, 2).startswith("the HSA payload ended without a result")
    assert peer_fallback_reason(["/x/tk8s-probe", "--peers"], None, 134, 2) is None  # HIP: nothing to fall back to
    assert peer_fallback_reason(cmd, None, 134, 1) is None  # one GPU: no pulls


# ---- tk8s-rccl's own host-side bounds (no GPU needed before the communicator) -----------------
def _rccl_tool():
    p = REPO / "tritonk8ssupervisor_amd" / "bin" / "tk8s-rccl"
    if not p.exists():
        pytest.skip("native tools not built")
    return p


def test_native_rank_without_a_uid_gives_up_at_its_deadline(tmp_path):
    t0 = time.monotonic()
    r = subprocess.run([str(_rccl_tool()), "--rank", "1", "--nranks", "2", "--device", "0", "--uid-file",
                        str(tmp_path / "uid"), "--op-timeout", "2"], capture_output=True, text=True, timeout=60,
                       env={**os.environ, "TK8S_FAULTS": ""})
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 1 and out == {"ok": False, "phase": "uid", "error": "no unique id from rank 0 within 2 s",
                                          "timed_out": True, "nranks": 2, "first_rank": 1}
    assert time.monotonic() - t0 < 10


def test_native_rank_hung_in_the_uid_phase_is_ended_by_its_watchdog(tmp_path):
    t0 = time.monotonic()
    r = subprocess.run([str(_rccl_tool()), "--rank", "1", "--nranks", "2", "--device", "0", "--uid-file",
                        str(tmp_path / "uid"), "--op-timeout", "1"], capture_output=True, text=True, timeout=60,
                       env={**os.environ, "TK8S_FAULTS": "rccl.hang@uid:1"})
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 4 and out["watchdog"] and out["phase"] == "uid" and out["first_rank"] == 1, out
    assert 1 + 10 <= time.monotonic() - t0 < 20
    # the same point aimed at another rank leaves this one alone (it times out on its own bound)
    r = subprocess.run([str(_rccl_tool()), "--rank", "1", "--nranks", "2", "--device", "0", "--uid-file",
                        str(tmp_path / "uid"), "--op-timeout", "1"], capture_output=True, text=True, timeout=60,
                       env={**os.environ, "TK8S_FAULTS": "rccl.hang@uid:0"})
    assert r.returncode == 1 and json.loads(r.stdout.strip().splitlines()[-1])["phase"] == "uid"
