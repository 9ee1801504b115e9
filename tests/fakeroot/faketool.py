#!/usr/bin/env python3
"""Stand-ins for the system tools the kubeadm platform's roles drive, for a fake host of
tests/fakessh.py (a host directory whose PATH holds only these and safe coreutils).

apt-get, apt-mark, dpkg-query, modprobe, sysctl, swapoff, systemctl, containerd, curl, kubeadm,
kubectl -- dispatched on the name this file is invoked as. State lives under $TK8S_SYSROOT (the
host's staging root: installed packages, /etc/kubernetes/*.conf, /dev/kfd) and in one cluster
file shared by the hosts ($FAKE_K8S_STATE: nodes, their GPUs, labels and taints, applied objects,
Jobs and pods). Every call is appended to $TK8S_SYSROOT/var/log/fake-tools.log. Nothing here
touches the real system.

The RCCL-tests Jobs follow a scenario a test may put into the state file (``rccl_scenario``):
``pending_polls`` (default 1: the first poll sees the pod Pending), ``fail`` (nodes whose pod
fails), ``never`` (nodes whose pod is never scheduled). A pod takes its node's GPUs while Running
and frees them when it terminates; a plain Pod is scheduled on apply (taints, nodeSelector, free
amd.com/gpu) -- so a test can show the GPUs are usable after the check.
"""
import fcntl
import json
import os
import sys
from pathlib import Path

ROOT = Path(os.environ.get("TK8S_SYSROOT") or "/nonexistent-sysroot")
STATE = Path(os.environ.get("FAKE_K8S_STATE", "/nonexistent-state"))


def log(tool, args):
    p = ROOT / "var" / "log" / "fake-tools.log"
    p.parent.mkdir(parents=True, exist_ok=True)
    with open(p, "a") as f:
        f.write(" ".join([tool, *args]) + "\n")


class Cluster:
    def __enter__(self):
        STATE.parent.mkdir(parents=True, exist_ok=True)
        self.f = open(STATE, "a+")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        self.f.seek(0)
        text = self.f.read()
        self.d = json.loads(text) if text.strip() else {"nodes": {}, "objects": [], "uid": "", "master": ""}
        return self.d

    def __exit__(self, *exc):
        self.f.seek(0)
        self.f.truncate()
        self.f.write(json.dumps(self.d))
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def opt(args, name, default=None):
    return args[args.index(name) + 1] if name in args and args.index(name) + 1 < len(args) else default


def installed() -> Path:
    return ROOT / "var" / "lib" / "dpkg" / "fake-installed"


def apt_get(args):
    if "install" in args:
        pkgs = [a for a in args[args.index("install") + 1:] if not a.startswith("-")]
        p = installed()
        p.parent.mkdir(parents=True, exist_ok=True)
        have = set(p.read_text().split()) if p.exists() else set()
        p.write_text("\n".join(sorted(have | set(pkgs))) + "\n")
        for x in pkgs:
            print(f"Setting up {x} (fake) ...")
        print(f"{len(pkgs)} newly installed")
    return 0


def dpkg_query(args):
    pkg = args[-1]
    p = installed()
    if p.exists() and pkg in p.read_text().split():
        print("install ok installed", end="")
        return 0
    return 1


def modprobe(args):
    if "amdgpu" in args:
        if not (installed().exists() and "amdgpu-dkms" in installed().read_text().split()):
            print("modprobe: FATAL: Module amdgpu not found", file=sys.stderr)
            return 1
        (ROOT / "dev").mkdir(parents=True, exist_ok=True)
        (ROOT / "dev" / "kfd").touch()
    return 0


def containerd(args):
    if args[:2] == ["config", "default"]:
        print('version = 2\n[plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options]\n'
              "  SystemdCgroup = false")
    return 0


def curl(args):
    dest = opt(args, "-o")
    if dest:
        Path(dest).parent.mkdir(parents=True, exist_ok=True)
        Path(dest).write_text(f"-----BEGIN PGP PUBLIC KEY BLOCK----- (fake key of {args[-1]})\n")
    return 0


def host_gpus() -> int:
    if os.environ.get("FAKE_HOST_GPUS"):
        return int(os.environ["FAKE_HOST_GPUS"])
    return len([g for g in os.environ.get("TK8S_MACHINE_GPUS", "").split(",") if g])


def kubeadm(args):
    kube = ROOT / "etc" / "kubernetes"
    if args[:1] == ["init"]:
        kube.mkdir(parents=True, exist_ok=True)
        (kube / "admin.conf").write_text("apiVersion: v1\nkind: Config\nclusters: [{name: fake}]\n")
        with Cluster() as d:
            name = opt(args, "--node-name")
            d["master"] = opt(args, "--apiserver-advertise-address", "")
            d["uid"] = d["uid"] or "5f0c1c8e-fake-4c1d-9e7a-kube-system"
            # a kubelet sees every GPU of its host (FAKE_HOST_GPUS, the host's .env)
            d["nodes"][name] = {"gpus": host_gpus(), "labels": {}, "control_plane": True,
                                "taints": ["node-role.kubernetes.io/control-plane:NoSchedule"]}
        print("Your Kubernetes control-plane has initialized successfully!")
        return 0
    if args[:2] == ["token", "create"]:
        with Cluster() as d:
            print(f"kubeadm join {d['master']}:6443 --token abcdef.0123456789abcdef "
                  "--discovery-token-ca-cert-hash sha256:" + "ab" * 32)
        return 0
    if args[:1] == ["join"]:
        if "--token" not in args or "--discovery-token-ca-cert-hash" not in args:
            print("error: a join needs the token and the CA cert hash", file=sys.stderr)
            return 1
        kube.mkdir(parents=True, exist_ok=True)
        (kube / "kubelet.conf").write_text("apiVersion: v1\nkind: Config\n")
        with Cluster() as d:
            d["nodes"][opt(args, "--node-name")] = {"gpus": host_gpus(), "labels": {}, "taints": []}
        print("This node has joined the cluster")
        return 0
    if args[:1] == ["reset"]:
        for f in ("admin.conf", "kubelet.conf"):
            (kube / f).unlink(missing_ok=True)
        return 0
    return 0


RCCL_RESULT = {"ok": True, "mode": "single_process", "nranks": 0, "peak_busbw_gbps": 0.0, "comm_init_ms": 310.0}


def load_docs(path):
    import yaml

    docs = []
    text = Path(path).read_text()
    for doc in yaml.safe_load_all(text):
        if doc:
            docs += doc.get("items", []) if doc.get("kind") == "List" else [doc]
    return docs


def gpu_request(spec):
    return sum(int(((c.get("resources") or {}).get("limits") or {}).get("amd.com/gpu", 0) or 0)
               for c in spec.get("containers", []))


def schedulable(d, node, spec):
    """Can a pod with this spec go to node (taints, nodeSelector, free amd.com/gpu)?"""
    v = d["nodes"][node]
    tol = {t.get("key") for t in spec.get("tolerations") or []}
    if any(t.split(":")[0].split("=")[0] not in tol for t in v.get("taints", [])):
        return False, f"node {node} has an untolerated taint"
    sel = spec.get("nodeSelector") or {}
    labels = dict(v["labels"], **{"kubernetes.io/hostname": node})
    if any(labels.get(k) != str(x) for k, x in sel.items()):
        return False, f"node {node} does not match the nodeSelector"
    need = gpu_request(spec)
    if need > v["gpus"] - used_gpus(d, node):
        return False, f"Insufficient amd.com/gpu on {node}"
    return True, ""


def used_gpus(d, node):
    n = sum(p["gpus"] for p in d.get("pods", {}).values() if p.get("node") == node and p["phase"] == "Running")
    for j in d.get("jobs", {}).values():
        if j.get("node") == node and j.get("phase") == "Running":
            n += j["gpus"]
    return n


def step_job(d, name, j):
    """One poll of an RCCL-tests Job's pod: Pending (not placeable, or the scenario's first polls),
    Running, then Succeeded -- or Failed for the nodes the scenario names."""
    sc = d.get("rccl_scenario") or {}
    if j["phase"] in ("Succeeded", "Failed"):
        return
    node = j["spec"].get("nodeSelector", {}).get("kubernetes.io/hostname")
    j["polls"] += 1
    if j["phase"] == "Running":  # placed: it holds its GPUs until it terminates
        j["phase"] = "Failed" if node in sc.get("fail", []) else "Succeeded"
        return
    ok, why = schedulable(d, node, j["spec"]) if node in d["nodes"] else (False, f"no node {node}")
    if not ok or node in sc.get("never", []):
        j["phase"], j["why"] = "Pending", why or "scenario: never scheduled"
        return
    j["node"] = node
    if j["polls"] <= int(sc.get("pending_polls", 1)):
        j["phase"], j["why"] = "Pending", "ContainerCreating"
    else:
        j["phase"] = "Running"


def job_pod(name, j):
    st = {"phase": j["phase"]}
    if j["phase"] in ("Succeeded", "Failed"):
        code = 0 if j["phase"] == "Succeeded" else 1
        st["containerStatuses"] = [{"name": "rccl", "ready": False, "state": {"terminated": {
            "exitCode": code, "reason": "Completed" if code == 0 else "Error",
            "message": "" if code == 0 else "ncclCommInitAll failed: unhandled system error"}}}]
    elif j["phase"] == "Running":
        st["containerStatuses"] = [{"name": "rccl", "ready": True, "state": {"running": {}}}]
    elif j.get("why"):
        st["conditions"] = [{"type": "PodScheduled", "status": "False", "message": j["why"]}]
    return {"metadata": {"name": f"{name}-pod", "labels": dict(j["labels"], **{"job-name": name})},
            "spec": {"nodeName": j.get("node")}, "status": st}


def kubectl(args):
    a = [x for i, x in enumerate(args) if not (x == "--kubeconfig" or (i and args[i - 1] == "--kubeconfig"))]
    if "-n" in a:  # the namespace plays no part in this simulation
        k = a.index("-n")
        a = a[:k] + a[k + 2:]
    with Cluster() as d:
        d.setdefault("jobs", {})
        d.setdefault("pods", {})
        dp = any("device-plugin" in o for o in d["objects"])
        if a[:1] == ["apply"]:
            src = opt(a, "-f")
            if "://" in src:
                name = "kubernetes-dashboard" if "dashboard" in src else "kube-flannel-ds"
                d["objects"].append(name)
                print(f"daemonset.apps/{name} created")
                return 0
            docs = load_docs(src) if src.endswith((".json", ".yaml", ".yml")) else []
            for o in docs:
                kind, name = o.get("kind"), o["metadata"]["name"]
                if kind == "Job":
                    spec = o["spec"]["template"]["spec"]
                    d["jobs"][name] = {"spec": spec, "gpus": gpu_request(spec), "phase": "New", "polls": 0,
                                       "labels": o["spec"]["template"]["metadata"].get("labels", {})}
                    print(f"job.batch/{name} created")
                elif kind == "Pod":
                    spec = o["spec"]
                    node = next((n for n in sorted(d["nodes"]) if schedulable(d, n, spec)[0]), None)
                    d["pods"][name] = {"node": node, "gpus": gpu_request(spec),
                                       "phase": "Running" if node else "Pending"}
                    print(f"pod/{name} created")
            name = Path(src).stem
            d["objects"].append(name)
            if not docs:
                print(f"daemonset.apps/{name} created")
            return 0
        if a[:3] == ["get", "namespace", "kube-system"]:
            print(d["uid"], end="")
            return 0
        if a[:2] == ["label", "node"]:
            k, _, v = a[3].partition("=")
            d["nodes"][a[2]]["labels"][k] = v
            print(f"node/{a[2]} labeled")
            return 0
        if a[:2] == ["taint", "nodes"]:
            if a[2] not in d["nodes"]:
                print(f'Error from server (NotFound): nodes "{a[2]}" not found', file=sys.stderr)
                return 1
            t = a[3].rstrip("-")
            taints = d["nodes"][a[2]].setdefault("taints", [])
            if t in taints:
                taints.remove(t)
                print(f"node/{a[2]} untainted")
                return 0
            print(f"error: taint {t!r} not found", file=sys.stderr)
            return 1
        if a[:3] == ["create", "token", "admin-user"]:
            print("eyJhbGciOiJSUzI1NiJ9.fake-dashboard-token")
            return 0
        if a[:1] == ["drain"]:
            print(f"node/{a[1]} drained")
            return 0
        if a[:2] == ["delete", "node"]:
            d["nodes"].pop(a[2], None)
            print(f'node "{a[2]}" deleted')
            return 0
        if a[:1] == ["wait"]:
            for n in d["nodes"]:
                print(f"node/{n} condition met")
            return 0
        if a[:2] == ["get", "nodes"]:
            items = [{"metadata": {"name": n, "labels": v["labels"]},
                      "spec": {"taints": [{"key": t.split(":")[0], "effect": t.split(":")[1]} for t in v.get("taints", [])]},
                      "status": {"allocatable": {"amd.com/gpu": str(v["gpus"] if dp else 0), "cpu": "8"},
                                 "conditions": [{"type": "Ready", "status": "True"}]}} for n, v in d["nodes"].items()]
            print(json.dumps({"items": items}))
            return 0
        if a[:2] == ["get", "pods"] and opt(a, "-l", "").startswith("tk8s.amd.com/rccl-run="):
            run = opt(a, "-l").split("=", 1)[1]
            items = []
            for name, j in sorted(d["jobs"].items()):
                if j["labels"].get("tk8s.amd.com/rccl-run") == run:
                    step_job(d, name, j)
                    if j["phase"] != "New":
                        items.append(job_pod(name, j))
            print(json.dumps({"items": items}, indent=1))
            return 0
        if a[:2] == ["get", "pod"]:
            p = d["pods"].get(a[2])
            if p is None:
                print(f'Error from server (NotFound): pods "{a[2]}" not found', file=sys.stderr)
                return 1
            print(json.dumps({"metadata": {"name": a[2]}, "spec": {"nodeName": p["node"]},
                              "status": {"phase": p["phase"]}}))
            return 0
        if a[:1] == ["logs"]:
            job = a[1][:-len("-pod")] if a[1].endswith("-pod") else a[1]
            j = d["jobs"].get(job)
            if j is None:
                print(f'Error from server (NotFound): pods "{a[1]}" not found', file=sys.stderr)
                return 1
            print("RCCL version : 2.27.7 (fake)")
            print(json.dumps(dict(RCCL_RESULT, nranks=j["gpus"], peak_busbw_gbps=40.0 * j["gpus"],
                                  ok=j["phase"] == "Succeeded")))
            return 0
    print(f"fake kubectl: unsupported {' '.join(a)}", file=sys.stderr)
    return 1


TOOLS = {"apt-get": apt_get, "dpkg-query": dpkg_query, "modprobe": modprobe, "containerd": containerd,
         "curl": curl, "kubeadm": kubeadm, "kubectl": kubectl}


def main():
    tool = os.environ.pop("FAKETOOL_NAME", "") or os.path.basename(sys.argv[0])
    args = sys.argv[1:]
    log(tool, args)
    return TOOLS.get(tool, lambda _a: 0)(args)  # apt-mark, sysctl, swapoff, systemctl: record only


if __name__ == "__main__":
    sys.exit(main())
