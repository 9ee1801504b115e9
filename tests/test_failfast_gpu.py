"""Fail fast on the fabric and link path, on the MI355X (VERDICT r5 #1 "done when", GPU part).

Every case injects a fault into a real payload on the one GPU and checks that it ends within its
deadline + a few seconds, names the phase, leaves no process holding the GPU, and that the GPU
still runs the next payload normally:

* tk8s-rccl: a stalled queue in the sweep (GPU-side stall kernel, released at the deadline), a
  dead peer at init (rank 0 of a 2-rank communicator whose rank 1 never comes), a host hang in
  the init (the watchdog's backstop), a rank that exits before the uid is published;
* tk8s-probe (HIP): a stalled xGMI pull (the peer path forced onto the one GPU);
* tk8s-hsaprobe: a stalled pull, and a payload that dies in its peer phase (then the HIP fallback).
"""
import json
import os
import subprocess
import time
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
BIN = Path(__file__).resolve().parents[1] / "tritonk8ssupervisor_amd" / "bin"


@pytest.fixture(scope="module", autouse=True)
def gpu(native_build):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(args, faults="", timeout=90, **env):
    e = {**os.environ, "TK8S_FAULTS": faults, **{k: str(v) for k, v in env.items()}}
    t0 = time.monotonic()
    p = subprocess.Popen([str(a) for a in args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, 9)
        out, err = p.communicate()
        pytest.fail(f"{args[0]} did not end within {timeout}s: {err[-1500:]}")
    dt = time.monotonic() - t0
    lines = [x for x in out.strip().splitlines() if x.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else {}), dt, p.pid, err


def _no_gpu_holder(pid):
    """Nothing the payload started is still running: no process of its session (it was started
    in a session of its own) is left in this pid namespace -- no helper or child still holding
    the GPU. (The KFD's own process list names host pids and, on the shared box, other
    processes' entries come and go, so it cannot be diffed.)"""
    deadline = time.monotonic() + 10
    while True:
        left = []
        for d in os.listdir("/proc"):
            if not d.isdigit():
                continue
            try:
                with open(f"/proc/{d}/stat") as f:
                    fields = f.read().rsplit(")", 1)[1].split()
            except OSError:
                continue
            if int(fields[3]) == pid and fields[0] != "Z":  # session id
                left.append(int(d))
        if not left or time.monotonic() > deadline:
            break
        time.sleep(0.05)
    assert not left, {"session": pid, "left": left}
    return True


def _healthy_rccl():
    rc, out, _, _, err = _run([BIN / "tk8s-rccl", "--ngpus", "1", "--max-bytes", 1 << 20, "--iters", 2, "--warmup", 1,
                               "--dtype", "float32"])
    assert rc == 0 and out["ok"], (out, err[-1500:])


def test_rccl_stalled_sweep_aborts_within_the_deadline():
    _healthy_rccl()  # a cold box's first communicator init can itself take longer than 3 s
    rc, out, dt, pid, err = _run([BIN / "tk8s-rccl", "--ngpus", "1", "--max-bytes", 1 << 20, "--iters", 2,
                                  "--warmup", 1, "--op-timeout", 3], faults="rccl.hang@sweep")
    assert rc == 1 and out["ok"] is False and out["phase"] == "sweep", (out, err[-1500:])
    assert out["timed_out"] and out["aborted"], out
    assert dt < 3 + 5 + 15, dt  # deadline + 5 s, plus the runtime's start
    assert _no_gpu_holder(pid)
    _healthy_rccl()


def test_rccl_dead_peer_at_init_aborts_within_the_deadline(tmp_path):
    """Rank 0 of a 2-rank communicator publishes its unique id; rank 1 never comes. The
    non-blocking init is polled under the deadline, then aborted; an abort that itself blocks in
    RCCL's bootstrap is given 2 s (abort_returned says which), so the report is never held."""
    rc, out, dt, pid, err = _run([BIN / "tk8s-rccl", "--rank", 0, "--nranks", 2, "--device", 0,
                                  "--uid-file", tmp_path / "uid", "--max-bytes", 1 << 20, "--op-timeout", 3])
    assert rc == 1 and out["phase"] == "init" and out["timed_out"] and not out.get("watchdog"), (out, err[-1500:])
    assert "abort_returned" in out
    assert dt < 3 + 2 + 5 + 15, dt
    assert _no_gpu_holder(pid)
    _healthy_rccl()


def test_rccl_host_hang_in_init_is_ended_by_the_watchdog():
    rc, out, dt, pid, err = _run([BIN / "tk8s-rccl", "--ngpus", "1", "--max-bytes", 1 << 20, "--op-timeout", 1],
                                 faults="rccl.hang@init")
    assert rc == 4 and out["watchdog"] and out["phase"] == "init", (out, err[-1500:])
    assert dt < 1 + 10 + 5 + 15, dt
    assert _no_gpu_holder(pid)


def test_rccl_rank_that_dies_before_the_uid(tmp_path):
    rc, _, dt, _, _ = _run([BIN / "tk8s-rccl", "--rank", 0, "--nranks", 2, "--device", 0,
                            "--uid-file", tmp_path / "uid", "--op-timeout", 3], faults="rccl.exit@uid")
    assert rc == 3 and dt < 20
    rc, out, dt, _, _ = _run([BIN / "tk8s-rccl", "--rank", 1, "--nranks", 2, "--device", 0,
                              "--uid-file", tmp_path / "uid", "--op-timeout", 2])
    assert rc == 1 and out["phase"] == "uid" and out["timed_out"] and dt < 2 + 5 + 15, out


def test_hip_probe_stalled_pull_is_bounded_and_names_the_link():
    rc, out, dt, pid, err = _run([BIN / "tk8s-probe", "--hbm-bytes", 64 << 20, "--md5-bytes", 1 << 20, "--copy-bytes",
                                  16 << 20, "--iters", 1],
                                 faults="probe.hang@peers", TK8S_PROBE_PEER_PATH=1, TK8S_GPU_SYNC_TIMEOUT_S=3)
    assert rc == 1 and not out["ok"], (out, err[-1500:])
    c = out["devices"][0]["copy"]
    assert not c["ok"] and "timed out" in c["error"] and c["src_device"] == c["dst_device"] == 0, c
    assert out["devices"][0]["hbm"]["ok"] and out["devices"][0]["md5"]["ok"]  # the rest of the node stands
    assert dt < 3 + 5 + 15, dt
    assert _no_gpu_holder(pid)
    rc, out, _, _, _ = _run([BIN / "tk8s-probe", "--hbm-bytes", 64 << 20, "--md5-bytes", 1 << 20, "--copy-bytes", 16 << 20,
                             "--iters", 1], TK8S_PROBE_PEER_PATH=1)
    assert rc == 0 and out["ok"], out


def test_hsaprobe_stalled_pull_is_bounded():
    args = [BIN / "tk8s-hsaprobe", "--devices", "0,0", "--peers", "--peer-bytes", 16 << 20, "--hbm-bytes", 64 << 20,
            "--md5-bytes", 1 << 20, "--copy-bytes", 16 << 20, "--iters", 1]
    rc, out, dt, pid, err = _run(args, faults="probe.hang@peers", TK8S_GPU_SYNC_TIMEOUT_S=3)
    pulls = [p for d in out["devices"] for p in d["peers"]]
    # (one stall flag per process: the first pull to give up releases the others' stalls too)
    bad = [p for p in pulls if not p["ok"]]
    assert len(pulls) == 2 and bad and all("did not complete within 3 s" in p["error"] for p in bad), out
    assert all(d["hbm"]["ok"] for d in out["devices"])
    assert dt < 2 * (3 + 5) + 15, dt  # two rounds of pulls, each bounded
    assert _no_gpu_holder(pid)
    rc, out, _, _, _ = _run(args)
    assert rc == 0 and all(p["ok"] for d in out["devices"] for p in d["peers"]), out


def test_hsaprobe_dies_in_the_peer_phase_then_the_hip_fallback():
    """The HSA payload dies in its peer phase (probe.exit@peers: it exits without a result -- a
    clean exit standing for the crash, which is not provoked on the shared box); the host
    burn-in's fallback then re-runs the whole validation through the HIP probe in a fresh child
    process and the record says so (burnin.peer_fallback_reason / run_hip_peer_fallback)."""
    from tritonk8ssupervisor_amd.burnin import merge_peer_fallback, peer_fallback_reason, run_hip_peer_fallback

    cmd = [str(BIN / "tk8s-hsaprobe"), "--devices", "0,0", "--peers", "--peer-bytes", str(16 << 20),
           "--hbm-bytes", str(64 << 20), "--md5-bytes", str(1 << 20), "--copy-bytes", str(16 << 20), "--iters", "1"]
    rc, out, dt, pid, err = _run(cmd, faults="probe.exit@peers")
    assert rc == 3 and not out and dt < 20, (rc, out, err[-1000:])
    assert _no_gpu_holder(pid)
    reason = peer_fallback_reason(cmd, None, rc, 2)
    assert reason and "without a result" in reason
    env = {**os.environ, "TK8S_PROBE_PEER_PATH": "1", "TK8S_FAULTS": ""}
    t0 = time.monotonic()
    hip, hrc = run_hip_peer_fallback(cmd, env, full=True)
    assert hrc == 0 and hip and hip["ok"] and hip["runtime"] == "hip", hip
    assert time.monotonic() - t0 < 60
    merged = merge_peer_fallback(None, hip, reason)
    assert merged["peers_runtime"] == "hip-fallback" and merged["hsa_fallback_reason"] == reason
