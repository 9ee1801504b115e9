#!/usr/bin/env python3
"""Stand-ins for the system tools the kubeadm platform's roles drive, for a fake host of
tests/fakessh.py (a host directory whose PATH holds only these and safe coreutils).

apt-get, apt-mark, dpkg-query, modprobe, sysctl, swapoff, systemctl, containerd, curl, kubeadm,
kubectl -- dispatched on the name this file is invoked as. State lives under $TK8S_SYSROOT (the
host's staging root: installed packages, /etc/kubernetes/*.conf, /dev/kfd) and in one cluster
file shared by the hosts ($FAKE_K8S_STATE: nodes, their GPUs and labels, applied objects). Every
call is appended to $TK8S_SYSROOT/var/log/fake-tools.log. Nothing here touches the real system.
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


def kubeadm(args):
    kube = ROOT / "etc" / "kubernetes"
    if args[:1] == ["init"]:
        kube.mkdir(parents=True, exist_ok=True)
        (kube / "admin.conf").write_text("apiVersion: v1\nkind: Config\nclusters: [{name: fake}]\n")
        with Cluster() as d:
            name = opt(args, "--node-name")
            d["master"] = opt(args, "--apiserver-advertise-address", "")
            d["uid"] = d["uid"] or "5f0c1c8e-fake-4c1d-9e7a-kube-system"
            d["nodes"][name] = {"gpus": 0, "labels": {}, "control_plane": True}
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
        gpus = [g for g in os.environ.get("TK8S_MACHINE_GPUS", "").split(",") if g]
        with Cluster() as d:
            d["nodes"][opt(args, "--node-name")] = {"gpus": len(gpus), "labels": {}}
        print("This node has joined the cluster")
        return 0
    if args[:1] == ["reset"]:
        for f in ("admin.conf", "kubelet.conf"):
            (kube / f).unlink(missing_ok=True)
        return 0
    return 0


def kubectl(args):
    a = [x for i, x in enumerate(args) if not (x == "--kubeconfig" or (i and args[i - 1] == "--kubeconfig"))]
    with Cluster() as d:
        dp = any("device-plugin" in o for o in d["objects"])
        if a[:1] == ["apply"]:
            src = opt(a, "-f")
            name = Path(src).stem if "://" not in src else "kube-flannel-ds"
            d["objects"].append(name)
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
                      "status": {"allocatable": {"amd.com/gpu": str(v["gpus"] if dp else 0), "cpu": "8"},
                                 "conditions": [{"type": "Ready", "status": "True"}]}} for n, v in d["nodes"].items()]
            print(json.dumps({"items": items}))
            return 0
        if "pods" in a and "app=tk8s-rccl-tests" in a:
            rccl = any("rccl-tests" in o for o in d["objects"])
            for n, v in d["nodes"].items():
                if rccl and v["labels"].get("amd.com/gpu.family") == "gfx950":
                    print(f"tk8s-rccl-tests-{n} true")
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
