"""Ranks of one Job in separate one-GPU pods (RCCL over xGMI on
one node). The GPU jail lets a pod open only its own render node, and RCCL's P2P transport over
xGMI connects only GPUs every rank's runtime can see -- so ranks in separate pods would fall back
to SHM. ``tk8s.amd.com/gpu-peers: job`` in an Indexed Job's pod template is the opt-in: the pods
of that Job on one host open each other's GPUs (own GPU first, as device 0) and nothing else;
``kubectl describe pod`` names the peers. Here on fake GPUs; tests/test_kernels_gpu.py runs the
torch all-reduce Job on the MI355X (1 GPU: transport logged; >= 2 GPUs: P2P asserted)."""
import json
import subprocess
import time

import pytest

from test_bringup import _env, _fake_gpu_tree, _setup, _summary, ws  # noqa: F401 - fixture

PROBE = ("for m in 128 129; do cat {dri}/renderD$m >/dev/null 2>&1 && echo render$m=open || echo render$m=denied; done; "
         "echo rocr=$ROCR_VISIBLE_DEVICES; echo own=$TK8S_GPU_DEVICES; echo peers=$TK8S_GPU_PEER_DEVICES; "
         "echo ids=$TK8S_GPU_IDS; sleep 1")  # (alive a while, as ranks are: a peer that already finished is no peer)


def _job(name: str, dri, peers: bool, indexed: bool = True) -> dict:
    tmpl_md = {"annotations": {"tk8s.amd.com/gpu-peers": "job"}} if peers else {}
    return {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": name}, "spec": {
        "completions": 2, "parallelism": 2, **({"completionMode": "Indexed"} if indexed else {}), "backoffLimit": 0,
        "template": {"metadata": tmpl_md, "spec": {"restartPolicy": "Never", "containers": [{
            "name": "rank", "command": ["sh", "-c", PROBE.format(dri=dri)],
            "resources": {"limits": {"amd.com/gpu": 1}}}]}}}}


def _kc(ws, env):
    return lambda *a, stdin=None: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True,
                                                 timeout=60, input=stdin)


def _finished(kc, job: str, timeout: float = 60.0) -> dict:
    deadline = time.monotonic() + timeout
    pods = {}
    while time.monotonic() < deadline:
        pods = {p["metadata"]["name"]: p for p in json.loads(kc("get", "pods", "-o", "json").stdout)["items"]
                if (p["metadata"].get("labels") or {}).get("job-name") == job}
        if len(pods) == 2 and all(p["status"].get("phase") in ("Succeeded", "Failed") for p in pods.values()):
            return pods
        time.sleep(0.2)
    raise AssertionError(f"job {job} did not finish: {json.dumps({n: p.get('status') for n, p in pods.items()})[:2000]}")


def _out(kc, pod: str) -> dict:
    return dict(x.split("=", 1) for x in kc("logs", pod).stdout.split() if "=" in x)


def test_indexed_job_pods_open_their_peers_gpus_and_nothing_more(ws, tmp_path_factory):
    from tritonk8ssupervisor_amd.agent.runtime import gpu_jail

    if not gpu_jail()[0]:
        pytest.skip(f"GPU jail unavailable here: {gpu_jail()[1]}")
    d = tmp_path_factory.mktemp("peers")
    kfd, dri = _fake_gpu_tree(d, 2)
    env = _env(TK8S_FAKE_GPUS="2", TK8S_GPU_JAIL_KFD_ROOT=str(kfd), TK8S_GPU_JAIL_DRI_ROOT=str(dri))
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=env))
    kc = _kc(ws, env)
    assert kc("apply", "-f", "-", stdin=json.dumps(_job("ring", dri, peers=True))).returncode == 0
    pods = _finished(kc, "ring")
    nodes = sorted(p["spec"]["nodeName"] for p in pods.values())
    assert nodes == ["kubenode1", "kubenode2"], nodes  # one GPU per worker: the ranks are on two nodes
    why = json.dumps({n: (p["metadata"].get("annotations"), p["status"]) for n, p in pods.items()})[:3000]
    for name, p in pods.items():
        assert p["status"]["phase"] == "Succeeded", why
        o = _out(kc, name)
        own = int(p["metadata"]["annotations"]["amd.com/gpu-ids"].replace("gpu", ""))
        peer = 1 - own
        # both render nodes: its own and its peer's (the other node's GPU)
        assert o["render128"] == "open" and o["render129"] == "open", (o, why)
        assert o["rocr"] == f"{own},{peer}" and o["own"] == "0" and o["peers"] == "1", o  # own GPU is device 0
        other = next(q for q in pods.values() if q is not p)
        assert o["ids"] == f"gpu{own},{other['spec']['nodeName']}/gpu{peer}", o
        devs = json.loads(p["metadata"]["annotations"]["tk8s.amd.com/gpu-devices"])
        assert [(x["node"], x["id"], x["renderMinor"]) for x in devs] == [(p["spec"]["nodeName"], f"gpu{own}", 128 + own)]
        desc = kc("describe", "pod", name).stdout
        assert f"Job peers on this host: {other['spec']['nodeName']}/gpu{peer}" in desc, desc
    # the same Job without the opt-in: each rank opens its own GPU only
    assert kc("apply", "-f", "-", stdin=json.dumps(_job("plain", dri, peers=False))).returncode == 0
    for name, p in _finished(kc, "plain").items():
        o = _out(kc, name)
        own = int(p["metadata"]["annotations"]["amd.com/gpu-ids"].replace("gpu", ""))
        assert o[f"render{128 + own}"] == "open" and o[f"render{128 + 1 - own}"] == "denied", o
        assert o["peers"] == "" and "Job peers" not in kc("describe", "pod", name).stdout


def test_gpu_peers_is_admitted_for_indexed_jobs_only(ws):
    """The opt-in widens what a pod may open, so only the Job controller gives it to pods: a pod
    cannot carry it (or forge the agent's gpu-devices record), a NonIndexed Job or a Deployment
    cannot ask for it."""
    env = _env(TK8S_FAKE_GPUS="2")
    _summary(_setup(ws, "--nodes", "1", "--rccl", "off", env=env))
    kc = _kc(ws, env)
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "annotations": {"tk8s.amd.com/gpu-peers": "job"}},
           "spec": {"containers": [{"name": "c", "command": ["true"]}]}}
    r = kc("apply", "-f", "-", stdin=json.dumps(pod))
    assert r.returncode != 0 and "gpu-peers" in r.stderr + r.stdout, r.stdout + r.stderr
    pod["metadata"]["annotations"] = {"tk8s.amd.com/gpu-devices": "[]"}
    r = kc("apply", "-f", "-", stdin=json.dumps(pod))
    assert r.returncode != 0 and "set by the pod's node" in r.stderr + r.stdout, r.stdout + r.stderr
    r = kc("apply", "-f", "-", stdin=json.dumps(_job("flat", "/nonexistent", peers=True, indexed=False)))
    assert r.returncode != 0 and "Indexed" in r.stderr + r.stdout, r.stdout + r.stderr
    dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"}, "spec": {
        "replicas": 1, "selector": {"matchLabels": {"a": "d"}}, "template": {
            "metadata": {"labels": {"a": "d"}, "annotations": {"tk8s.amd.com/gpu-peers": "job"}},
            "spec": {"containers": [{"name": "c", "command": ["true"]}]}}}}
    r = kc("apply", "-f", "-", stdin=json.dumps(dep))
    assert r.returncode != 0 and "Indexed Job" in r.stderr + r.stdout, r.stdout + r.stderr


def test_peers_on_another_host_are_not_opened(ws, tmp_path_factory):
    """Two one-GPU workers on two (fake) hosts: a rank's peer is on the other host, so there is
    nothing to open -- RCCL goes over the network there -- and describe pod says so."""
    from tritonk8ssupervisor_amd.agent.runtime import gpu_jail

    if not gpu_jail()[0]:
        pytest.skip(f"GPU jail unavailable here: {gpu_jail()[1]}")
    d = tmp_path_factory.mktemp("peers2")
    kfd, dri = _fake_gpu_tree(d, 2)
    env = _env(TK8S_FAKE_GPUS="2", TK8S_FAKE_HOSTS="2", TK8S_GPU_JAIL_KFD_ROOT=str(kfd), TK8S_GPU_JAIL_DRI_ROOT=str(dri))
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=env))
    kc = _kc(ws, env)
    assert kc("apply", "-f", "-", stdin=json.dumps(_job("ring", dri, peers=True))).returncode == 0
    for name, p in _finished(kc, "ring").items():
        assert p["status"]["phase"] == "Succeeded", p["status"]
        o = _out(kc, name)
        own = int(p["metadata"]["annotations"]["amd.com/gpu-ids"].replace("gpu", ""))
        assert o[f"render{128 + 1 - own}"] == "denied" and o["peers"] == "", o
        assert "no Job peer on this host" in kc("describe", "pod", name).stdout


def test_the_example_torch_allreduce_job_runs_across_two_pods(ws):
    """manifests/examples/torch-allreduce-job.yaml itself (gloo instead of RCCL on the fake GPUs):
    two ranks in two jailed pods on two workers rendezvous through the control plane's KV and
    all-reduce; each knows its peer GPU from the opt-in."""
    from pathlib import Path

    import yaml

    job = yaml.safe_load((Path(__file__).resolve().parents[1] / "manifests" / "examples" /
                          "torch-allreduce-job.yaml").read_text())
    assert job["spec"]["template"]["metadata"]["annotations"]["tk8s.amd.com/gpu-peers"] == "job"
    cmd = job["spec"]["template"]["spec"]["containers"][0]["command"]
    cmd[cmd.index("nccl")] = "gloo"
    cmd[cmd.index("--max-bytes") + 1] = "65536"
    env = _env(TK8S_FAKE_GPUS="2")
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=env))
    kc = _kc(ws, env)
    assert kc("apply", "-f", "-", stdin=json.dumps(job)).returncode == 0
    pods = _finished(kc, "torch-allreduce", timeout=120)
    for name, p in pods.items():
        log = kc("logs", name).stdout
        assert p["status"]["phase"] == "Succeeded", (p["status"], log[-2000:])
        res = json.loads([x for x in log.splitlines() if x.startswith("{")][-1])
        assert res["ok"] and res["nranks"] == 2 and res["backend"] == "gloo", res
    assert sorted(json.loads(kc("get", "pods", "-o", "json").stdout)["items"][i]["spec"]["nodeName"]
                  for i in range(2)) == ["kubenode1", "kubenode2"]


def test_a_forged_peer_record_is_not_opened():
    """the agent cross-checks every entry of a peer pod's gpu-devices record before
    its pod may open that GPU -- the GPU must be one the peer's node allocated to that pod
    (amd.com/gpu-ids, node-written) and registered as its own; ordinal and render minor come from
    the node's registration and the host inventory, not from the record."""
    import types

    from tritonk8ssupervisor_amd.agent.agent import Agent

    gpus = [types.SimpleNamespace(ordinal=i, render_minor=128 + i) for i in range(4)]
    fake = types.SimpleNamespace(
        name="kubenode1", plugin=types.SimpleNamespace(inventory=types.SimpleNamespace(gpus=gpus)),
        _node_devices=lambda node: {"kubenode2": {"gpu1": 1}, "kubenode3": {"gpu2": 2}}[node])
    peer = {"metadata": {"name": "rank1", "annotations": {"amd.com/gpu-ids": "gpu1"}}}
    honest = json.dumps([{"node": "kubenode2", "id": "gpu1", "ordinal": 1, "renderMinor": 129}])
    got = Agent._peer_record(fake, peer, "kubenode2", honest, "host0")
    assert got == [{"node": "kubenode2", "id": "gpu1", "ordinal": 1, "host": "host0", "renderMinor": 129}]
    # naming another node's GPU (gpu2 is kubenode3's), a GPU not allocated to the pod, or a lying
    # ordinal / render minor: the first two are dropped, the last is re-derived
    forged = json.dumps([{"node": "kubenode2", "id": "gpu2", "ordinal": 2, "renderMinor": 130},
                         {"node": "kubenode2", "id": "gpu3", "ordinal": 3, "renderMinor": 131},
                         {"node": "kubenode2", "id": "gpu1", "ordinal": 3, "renderMinor": 131}])
    got = Agent._peer_record(fake, peer, "kubenode2", forged, "host0")
    assert got == [{"node": "kubenode2", "id": "gpu1", "ordinal": 1, "host": "host0", "renderMinor": 129}]
    peer["metadata"]["annotations"]["amd.com/gpu-ids"] = "gpu2"  # kubenode2 never had gpu2
    assert Agent._peer_record(fake, peer, "kubenode2", forged, "host0") == []


def test_a_deleted_waiting_pod_is_not_started_from_a_stale_snapshot():
    """the peer poller and the config-retry tick work from a snapshot of the waiting
    pods; one deleted meanwhile (DELETED, bookkept under the start lock) must not start -- nor
    get its GPUs reserved again -- and a successor of the same name is not started from the old
    pod's snapshot entry."""
    import threading
    import types

    from tritonk8ssupervisor_amd.agent.agent import Agent

    started = []
    fake = types.SimpleNamespace(_config_wait={}, _reserved={}, _pods_meta={}, _start_lock=threading.RLock(),
                                 runtime=types.SimpleNamespace(stop=lambda *a, **k: None),
                                 _terminated=lambda key: None)
    fake._start_pod_locked = lambda p: started.append(p["metadata"]["uid"])
    old = {"metadata": {"namespace": "default", "name": "rank0", "uid": "u1"}, "spec": {}}
    fake._config_wait["default/rank0"] = old
    fake._reserved["default/rank0"] = (["gpu0"], {}, 0.0)
    snapshot = list(fake._config_wait.values())     # what _poll_peers iterates over
    Agent._handle(fake, "DELETED", old)             # the delete lands in between
    assert fake._config_wait == {} and fake._reserved == {}
    Agent._start_if_waiting(fake, snapshot[0])
    assert started == []
    new = {"metadata": {"namespace": "default", "name": "rank0", "uid": "u2"}, "spec": {}}
    fake._config_wait["default/rank0"] = new        # a successor with the same name waits
    Agent._start_if_waiting(fake, snapshot[0])      # the stale entry does not start it
    assert started == []
    Agent._start_if_waiting(fake, new)
    assert started == ["u2"]
