"""The early host burn-in (earlyburn.py): started by ``cli/__main__.py`` before the CLI imports
anything, then adopted by the orchestrator -- or discarded when its plan is not exactly the run's."""
import json
import os

import pytest

from tritonk8ssupervisor_amd import earlyburn
from tritonk8ssupervisor_amd.models.hostinfo import discover


def _ws(tmp_path, answers=None):
    (tmp_path / "answers.json").write_text(json.dumps(answers or {"nodes": 2, "package": "mi355x-1gpu"}))
    return str(tmp_path)


def test_plan_for_a_plain_non_interactive_bring_up(tmp_path):
    env = {"TK8S_FAKE_GPUS": "8"}
    ws = _ws(tmp_path)
    p = earlyburn.plan(["--answers", "answers.json", "--yes", "--json", "--port", "0"], env, ws)
    assert p["gpus"] == [0, 1] and p["result"] == os.path.join(ws, ".tk8s", "run", "host-burnin.json")
    assert earlyburn.plan(["--answers=answers.json", "--nodes", "3"], env, ws)["gpus"] == [0, 1, 2]
    four = earlyburn.plan(["--answers", "answers.json", "--package", "mi355x-4gpu"], env, ws)
    assert four["gpus"] == list(range(8))
    assert earlyburn.plan(["--answers", "answers.json", "--nodes", "3", "--package", "mi355x-4gpu"], env, ws) is None
    # cpu-only workers: nothing to burn in, but the control-plane and agent zygotes are planned
    cpu = earlyburn.plan(["--answers", "answers.json", "--package", "cpu-only"], env, ws)
    assert cpu["gpus"] == [] and cpu["command"] is None
    assert cpu["workers"] == ["kubenode1", "kubenode2"] and cpu["master"] == "kubemaster"


def test_anything_unusual_is_left_to_the_orchestrator(tmp_path):
    env = {"TK8S_FAKE_GPUS": "8"}
    ws = _ws(tmp_path)
    for argv in (["--yes"],                                          # interactive: no answers file
                 ["--answers", "answers.json", "--resume"],
                 ["--answers", "answers.json", "--no-validate"],
                 ["--answers", "answers.json", "--hbm-bytes", "1024"],
                 ["--answers", "answers.json", "--rocprof"],
                 ["--answers", "answers.json", "--package", "2"]):  # a menu index: the wizard maps it
        assert earlyburn.plan(argv, env, ws) is None, argv
    assert earlyburn.plan(["--answers", "answers.json"], dict(env, TK8S_HOST_BURNIN="0"), ws) is None
    assert earlyburn.plan(["--answers", "answers.json"], dict(env, TK8S_BACKEND="triton"), ws) is None
    (tmp_path / "config").write_text("KUBERNETES_NAME=x\n")  # the wizard refuses an old configuration
    assert earlyburn.plan(["--answers", "answers.json"], env, ws) is None


def test_real_host_view_skips_claimed_gpus_and_matches_hostinfo(tmp_path, monkeypatch):
    root = tmp_path / "kfd"
    for node, gfx in ((0, 0), (1, 90500), (2, 90500), (3, 90500)):  # node 0: the CPU
        d = root / str(node)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"gfx_target_version {gfx}\nsimd_count {1024 if gfx else 0}\n")
    monkeypatch.delenv("TK8S_FAKE_GPUS", raising=False)
    assert len(earlyburn.kfd_gpu_nodes(str(root))) == discover(root, cache=False).count == 3
    reg = tmp_path / "reg"
    reg.mkdir()
    (reg / "claims.json").write_text(json.dumps({"gpus": {"0": {}}, "ips": {}}))
    env = {"TK8S_HOST_REGISTRY": str(reg)}
    ws = _ws(tmp_path)
    assert earlyburn.plan(["--answers", "answers.json"], env, ws, kfd_root=str(root))["gpus"] == [1, 2]
    assert earlyburn.plan(["--answers", "answers.json", "--nodes", "3"], env, ws, kfd_root=str(root)) is None


def _setup_obj(tmp_path, events):
    import types

    from tritonk8ssupervisor_amd import orchestrator
    from tritonk8ssupervisor_amd.config import ClusterConfig
    from tritonk8ssupervisor_amd.provider.local import LocalProvider

    s = orchestrator.Setup.__new__(orchestrator.Setup)
    s.ws, s.validate = orchestrator.Workspace(tmp_path), True
    s.hbm_bytes, s.md5_bytes, s.probe_iters = 1 << 30, 256 << 20, 3
    s.provider = LocalProvider(tmp_path / ".tk8s")
    s.cfg = ClusterConfig(HOST_PACKAGE="mi355x-1gpu", KUBERNETES_NUMBER_OF_NODES=2)
    s.events = types.SimpleNamespace(emit=lambda ev, **kw: events.append((ev, kw)))
    s.host_burnin = None
    return s


def _spawn_early(tmp_path, gpus, cmd):
    import sys

    result = tmp_path / ".tk8s" / "run" / "host-burnin.json"
    result.parent.mkdir(parents=True, exist_ok=True)
    env = dict(os.environ, **earlyburn.compose_visible_devices(gpus), NODE_NAME="host")
    argv = cmd + ["--out", str(result)]
    pid = os.posix_spawn(sys.executable if cmd[0] == sys.executable else cmd[0], argv, env, setsid=True)
    earlyburn._LAUNCHED = earlyburn.Early(earlyburn.Spawned(pid), gpus, cmd, str(result))
    return earlyburn._LAUNCHED


def test_orchestrator_adopts_a_matching_early_burnin(tmp_path, monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")
    # the host burn-in of two 1-GPU workers: the per-machine command plus the xGMI pulls
    cmd = earlyburn.host_burnin_command(earlyburn.default_validation_command(peers=False), [5, 6])
    early = _spawn_early(tmp_path, [5, 6], cmd)  # not the allocator's own first choice
    events = []
    s = _setup_obj(tmp_path, events)
    s._start_host_burnin()
    hb = s.host_burnin
    assert hb is not None and hb.proc is early.proc and hb.gpus == [5, 6]
    assert ("gpu_burnin_host_started", {"gpus": [5, 6], "pid": early.proc.pid, "early": True}) in events
    assert hb.finished.wait(30) and hb.result["ok"]
    # the workers then get exactly the GPUs the early run validated
    m1 = s.provider.create_machine("kubenode1", "mi355x-1gpu", ["local-public"])
    m2 = s.provider.create_machine("kubenode2", "mi355x-1gpu", ["local-public"])
    assert sorted(m1.gpus + m2.gpus) == [5, 6]
    assert earlyburn.take() is None


def test_orchestrator_discards_an_early_burnin_planned_differently(tmp_path, monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")
    cmd = [a for a in earlyburn.default_validation_command() if a != "--peers"] + ["--iters", "9"]
    early = _spawn_early(tmp_path, [5, 6], ["/bin/sleep", "30"])
    early.command = cmd
    events = []
    s = _setup_obj(tmp_path, events)
    s._start_host_burnin()
    assert early.proc.returncode is not None  # killed and reaped before the right one started
    assert any(ev == "gpu_burnin_early_discarded" for ev, _ in events)
    hb = s.host_burnin
    assert hb is not None and hb.proc is not early.proc and hb.gpus == [0, 1]
    assert hb.finished.wait(30) and hb.result["ok"]


def test_controlplane_zygote_nobody_hands_arguments_to_stops_with_its_supervisor(tmp_path, native_build):
    """A bring-up that dies before its master exists must not leave a control plane (or a
    supervisor restarting it) behind."""
    import subprocess
    import sys
    import time

    from tritonk8ssupervisor_amd.ops import BIN

    pidfile = tmp_path / "cp.pid"
    env = dict(os.environ, TK8S_ZYGOTE_TIMEOUT="0.3", PYTHONPATH=str(earlyburn.PKG.rsplit(os.sep, 1)[0]))
    p = subprocess.Popen([str(BIN / "tk8s-supervise"), "--pidfile", str(pidfile), "--restart", "unless-stopped", "--",
                          sys.executable, "-S", "-m", "tritonk8ssupervisor_amd.controlplane", "--await-args",
                          str(tmp_path / "never.args")], env=env, start_new_session=True)
    assert p.wait(30) in (0, 143, -15)
    time.sleep(0.05)
    assert not pidfile.exists()


def test_controlplane_zygote_serves_once_its_arguments_arrive(tmp_path):
    import socket
    import subprocess
    import sys
    import urllib.request

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    args = tmp_path / "cp.args"
    env = dict(os.environ, PYTHONPATH=str(earlyburn.PKG.rsplit(os.sep, 1)[0]))
    p = subprocess.Popen([sys.executable, "-S", "-m", "tritonk8ssupervisor_amd.controlplane", "--await-args", str(args)],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        args.write_text(json.dumps(["--host", "127.0.0.1", "--port", str(port), "--dns-port", "0", "--ingress-port", "0"]))
        line = p.stdout.readline()
        assert "Listening on" in line, line
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/v2-beta/projectTemplates?name=kubernetes", timeout=5) as r:
            assert r.status == 200
    finally:
        p.terminate()
        p.wait(10)


def _hsaprobe():
    from tritonk8ssupervisor_amd.ops import BIN

    p = BIN / "tk8s-hsaprobe"
    if not p.exists():
        pytest.skip("native tools not built")
    return p


    del ws


def test_multi_gpu_pulls_take_the_hsa_payload_unless_asked(monkeypatch):
    """one burn-in runtime at every N -- the HSA payload pulls the xGMI links too
    (its peer phase falls back to the HIP probe when it fails, burnin.HostBurnin), unless
    TK8S_PEERS_RUNTIME=hip; the Ready path pulls 16 MiB per link."""
    monkeypatch.delenv("TK8S_FAKE_GPUS", raising=False)
    monkeypatch.delenv("TK8S_PEERS_RUNTIME", raising=False)
    monkeypatch.delenv("TK8S_PROBE_RUNTIME", raising=False)
    base = earlyburn.default_validation_command(peers=False)
    one = earlyburn.host_burnin_command(base, [0])
    many = earlyburn.host_burnin_command(base, [0, 1])
    assert "--peers" not in one and "--peers" in many
    assert many[many.index("--peer-bytes") + 1] == str(16 << 20)
    assert os.path.basename(many[0]) == os.path.basename(base[0])  # the same runtime as the local probes
    if os.path.basename(many[0]) == "tk8s-hsaprobe":
        assert "--no-peer-dma" not in many
    monkeypatch.setenv("TK8S_PEERS_RUNTIME", "hip")
    hip = earlyburn.host_burnin_command(base, [0, 1])
    assert os.path.basename(hip[0]) == "tk8s-probe" and "--no-peer-dma" in hip
    fb = earlyburn.hip_peer_command(many)
    assert os.path.basename(fb[0]) == "tk8s-probe" and fb[fb.index("--peer-bytes") + 1] == str(16 << 20)
    assert fb[fb.index("--hbm-bytes") + 1] == "0" and "--skip-md5" in fb and fb[fb.index("--copy-bytes") + 1] == "0"