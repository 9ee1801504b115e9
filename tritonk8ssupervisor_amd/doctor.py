"""``./tk8s doctor``: preflight checks of what a bring-up on this backend/platform will need.

The reference lists its prerequisites in prose (README.md:17-96: the triton CLI, Terraform,
Ansible, kubectl, an SSH key registered with the account) and only finds out they are missing
half way through ``./setup.sh``. This runs the same questions as checks, before anything is
created, for the backend and platform the next ``./setup.sh`` would use:

* every backend: Python >= 3.8, PyYAML, the in-tree native build (probe, RCCL validator,
  supervisor);
* local: ROCm userspace and version, ``/dev/kfd`` and the render nodes, the MI355X GPUs the KFD
  exposes (gfx950) and how many are not held by another cluster on this host, the loopback
  addresses machines get, user/PID/mount namespaces for CPU pods, free disk for the workspace;
* baremetal: the inventory parses, every host answers over SSH with the inventory key (batch
  mode, the per-cluster known-hosts file), and reports its Python, ROCm, KFD and GPU count;
* triton: the ``triton`` CLI and its profile (``triton env``), an SSH key whose MD5
  fingerprint matches SDC_KEY_ID;
* kubeadm platform: machines the backend owns, reached as root, with apt (the k8sruntime
  role installs packages).

Each check is OK, WARN (the bring-up can run but something is degraded) or FAIL (it cannot);
the exit status is 1 when anything FAILs. ``--json`` prints the checks as one JSON list.
"""
from __future__ import annotations

import json
import os
import shutil
import socket
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
OK, WARN, FAIL = "OK", "WARN", "FAIL"


def _check(name: str, status: str, detail: str) -> dict:
    return {"check": name, "status": status, "detail": detail}


def common_checks() -> list[dict]:
    out = []
    v = sys.version_info
    out.append(_check("python", OK if v >= (3, 8) else FAIL, sys.version.split()[0]))
    try:
        import yaml  # noqa: F401

        out.append(_check("pyyaml", OK, getattr(yaml, "__version__", "present")
                          + (" (libyaml)" if hasattr(yaml, "CSafeLoader") else " (pure Python loader: slower)")))
    except ImportError:
        out.append(_check("pyyaml", FAIL, "PyYAML is not importable (pip install pyyaml)"))
    tools = ["tk8s-probe", "tk8s-hsaprobe", "tk8s-rccl", "tk8s-supervise", "tk8s-reuse", "tk8s-smi"]
    missing = [t for t in tools if not os.access(PKG / "bin" / t, os.X_OK)]
    out.append(_check("native build", FAIL if "tk8s-supervise" in missing or "tk8s-probe" in missing
                      else (WARN if missing else OK),
                      "all tools built" if not missing else f"missing {', '.join(missing)} (python3 __graft_entry__.py build)"))
    from .utils.rccl_unpack import OUT, installed_library, library_dir

    src = installed_library()
    if src is not None:  # the fabric check's communicator start: 0.4 s unpacked, 1.8 s installed
        out.append(_check("rccl device code", OK if library_dir() else WARN,
                          f"gfx950 code unpacked once ({OUT})" if library_dir() else
                          f"{src} inflates its 5.3 GB bundle in every rank (~1.7 s): python3 __graft_entry__.py build"))
        out.append(transparent_huge_pages())
    return out


def transparent_huge_pages(path: str = "/sys/kernel/mm/transparent_hugepage/enabled") -> dict:
    """The fabric rank's malloc goes on huge pages when the kernel allows it (madvise or always:
    HIP's copies of RCCL's 108 MB code object, 318 -> 202 ms of the communicator start,
    profiles/r5_thp/); with ``never`` the advice is ignored and the rank runs as before."""
    try:
        text = Path(path).read_text()
    except OSError as e:
        return _check("huge pages", WARN, f"{path} unreadable ({e}): the fabric rank's huge-page malloc may not apply")
    mode = text[text.find("[") + 1:text.find("]")] if "[" in text else text.strip()
    if mode in ("madvise", "always"):
        return _check("huge pages", OK, f"transparent huge pages: {mode} (the fabric rank's malloc uses them)")
    return _check("huge pages", WARN, f"transparent huge pages: {mode}: the fabric rank's communicator start "
                                      "is ~0.1 s slower (profiles/r5_thp/)")


def _kfd_gpus() -> list[dict]:
    from .earlyburn import kfd_gpu_nodes

    gpus = []
    for node, props, _d in kfd_gpu_nodes():
        ver = int(props.get("gfx_target_version", 0))
        gpus.append({"node": node, "gfx": f"gfx{ver // 10000}{(ver // 100) % 100:x}{ver % 100:x}" if ver else "?",
                     "simd": props.get("simd_count", 0)})
    return gpus


def local_checks(workdir: str) -> list[dict]:
    out = []
    ver = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / ".info" / "version"
    try:
        rocm = ver.read_text().strip()
        major = int(rocm.split(".")[0])
        out.append(_check("rocm", OK if major >= 7 else WARN, f"{rocm} at {ver.parents[1]}"
                          + ("" if major >= 7 else " (tested with ROCm >= 7.0)")))
    except (OSError, ValueError):
        out.append(_check("rocm", FAIL, f"no ROCm userspace at {ver.parents[1]} (ROCM_PATH)"))
    fake = os.environ.get("TK8S_FAKE_GPUS")
    kfd = os.path.exists("/dev/kfd")
    kfd_ok = kfd and os.access("/dev/kfd", os.R_OK | os.W_OK)
    out.append(_check("/dev/kfd", OK if kfd_ok else (WARN if fake else FAIL),
                      "read/write" if kfd_ok
                      else ("not accessible: add the user to the render/video groups" if kfd else "missing (amdgpu driver)")
                      + ("" if kfd_ok or not fake else " -- not needed with TK8S_FAKE_GPUS")))
    if fake and out[-2]["check"] == "rocm" and out[-2]["status"] == FAIL:
        out[-2]["status"] = WARN
    if fake:
        out.append(_check("gpus", WARN, f"TK8S_FAKE_GPUS={fake}: fake gfx950 devices (CPU rehearsal, no GPU validation)"))
    else:
        gpus = _kfd_gpus()
        archs = sorted({g["gfx"] for g in gpus})
        if not gpus:
            out.append(_check("gpus", FAIL, "the KFD exposes no GPU this user can open"))
        else:
            out.append(_check("gpus", OK if archs == ["gfx950"] else WARN,
                              f"{len(gpus)} x {'/'.join(archs)}" + ("" if archs == ["gfx950"] else " (built for gfx950)")))
            try:
                from .provider.hostreg import HostRegistry

                with HostRegistry().locked() as table:
                    held = set(table.get("gpus", {}))
                free = len(gpus) - len([g for g in held if str(g).isdigit() and int(g) < len(gpus)])
                out.append(_check("free gpus", OK if free else FAIL,
                                  f"{free} of {len(gpus)} not held by another cluster on this host"))
            except Exception as e:  # noqa: BLE001 - the registry is advisory here
                out.append(_check("free gpus", WARN, f"host registry unreadable: {e}"))
    try:
        with socket.socket() as s:
            s.bind(("127.0.1.250", 0))
        out.append(_check("loopback addresses", OK, "127.0.1.0/24 bindable (machine addresses)"))
    except OSError as e:
        out.append(_check("loopback addresses", WARN, f"127.0.1.x not bindable ({e}): machines share 127.0.0.1"))
    from .agent.runtime import container_runtime, gpu_jail, namespace_isolation

    iso, why = namespace_isolation()
    out.append(_check("pod isolation", OK if iso else WARN, "user/PID/mount namespaces for CPU pods" if iso else why))
    jail, jhow = gpu_jail()
    out.append(_check("gpu jail", OK if jail else WARN,
                      f"{jhow}: a pod can open only its own GPUs' render nodes" if jail else
                      f"{jhow}: a pod's GPU view is its *_VISIBLE_DEVICES only"))
    from .agent.resources import detect_mode
    from .agent.runtime import jail_signal_scoping

    out.append(_check("pod signals", OK if jail_signal_scoping() else WARN,
                      "Landlock scopes a pod's signals: GPU pods (host PID namespace) cannot signal the agent"
                      if jail_signal_scoping() else "Landlock ABI < 6: pods sharing the host PID namespace may "
                                                   "signal other processes of the operator"))
    mode, mwhy = detect_mode()
    out.append(_check("resource limits", OK if mode in ("cgroup2", "cgroup1") else WARN, {
        "cgroup2": f"cgroup v2 ({mwhy}): memory, cpu and cpuset limits per pod and per machine",
        "cgroup1": f"cgroup v1 ({mwhy}): memory, cpu and cpuset limits per pod and per machine",
        "watchdog": f"unprivileged watchdog: limits.memory by resident-set sampling (OOMKilled), limits.cpu by a "
                    f"SIGSTOP/SIGCONT duty cycle, NUMA pinning ({mwhy})",
    }.get(mode, f"none: {mwhy}")))
    cont, chow = container_runtime()
    out.append(_check("image pods", OK if cont else WARN,
                      f"{chow}: pods can run loaded images (./tk8s image load)" if cont else
                      f"{chow}: pods run as processes; images not in the app catalogue fail"))
    try:
        free_gb = shutil.disk_usage(workdir).free / 2**30
        out.append(_check("disk", OK if free_gb >= 1 else WARN, f"{free_gb:.1f} GiB free in {workdir}"))
    except OSError as e:
        out.append(_check("disk", WARN, str(e)))
    return out


_REMOTE_PROBE = ("python3 -c 'import sys; print(sys.version.split()[0])'; "
                 "cat /opt/rocm/.info/version 2>/dev/null || echo none; "
                 "test -r /dev/kfd -a -w /dev/kfd && echo kfd || echo nokfd; id -u; "
                 "test -x /usr/bin/apt && echo apt || echo noapt; echo \"fake=${TK8S_FAKE_GPUS:-}\"")


def baremetal_checks(workdir: str, platform: str = "tk8s") -> list[dict]:
    out = []
    try:
        from .provider.baremetal import BareMetalProvider

        prov = BareMetalProvider(str(Path(workdir) / ".tk8s"))
        hosts = prov.inventory()["hosts"]
    except Exception as e:  # noqa: BLE001 - reported as the check
        return [_check("inventory", FAIL, str(e))]
    out.append(_check("inventory", OK, f"{len(hosts)} host(s): " + ", ".join(h['name'] for h in hosts)))
    from .utils import ssh as sshu

    for h in hosts:
        target = prov.target(h)
        try:
            rc, text = sshu.run(target, _REMOTE_PROBE, timeout=20)
        except Exception as e:  # noqa: BLE001
            rc, text = 255, str(e)
        if rc != 0:
            out.append(_check(f"ssh {h['name']}", FAIL, (text.strip().splitlines() or ["unreachable"])[-1][:200]))
            continue
        lines = text.strip().splitlines()
        pyv, rocm, kfd, uid, apt, fake = (lines + ["?"] * 6)[:6]
        fake = fake.partition("=")[2]
        g = h.get("gpus") or 0
        gpu_host = bool(g) if isinstance(g, (list, tuple)) else int(g) > 0  # normalised: a list of ordinals
        if kfd == "kfd" and rocm != "none":
            status, note = OK, ""
        elif fake:
            status, note = WARN, f" (fake GPUs: TK8S_FAKE_GPUS={fake})"
        else:
            status, note = (FAIL if gpu_host else WARN), " (no usable ROCm/KFD)" if gpu_host else ""
        if platform == "kubeadm" and (uid != "0" or apt != "apt"):
            status, note = FAIL, note + " (the kubeadm platform needs root and apt)"
        out.append(_check(f"ssh {h['name']}", status, f"python {pyv}, ROCm {rocm}, {kfd}, uid {uid}, {apt}{note}"))
    return out


def triton_checks() -> list[dict]:
    out = []
    tri = shutil.which("triton")
    if not tri:
        return [_check("triton cli", FAIL, "the triton CLI is not on PATH (npm install -g triton)")]
    out.append(_check("triton cli", OK, tri))
    try:
        r = subprocess.run([tri, "env"], capture_output=True, text=True, timeout=30)
        out.append(_check("triton profile", OK if r.returncode == 0 else FAIL,
                          "triton env works" if r.returncode == 0 else (r.stderr.strip() or "triton env failed")[:200]))
    except (OSError, subprocess.TimeoutExpired) as e:
        out.append(_check("triton profile", FAIL, str(e)))
    key_id = os.environ.get("SDC_KEY_ID", "")
    if key_id:
        from .provider.keys import find_key

        key = find_key(key_id, ["~/.ssh"])
        out.append(_check("ssh key", OK if key else FAIL, key or f"no key in ~/.ssh has the fingerprint {key_id}"))
    else:
        out.append(_check("ssh key", WARN, "SDC_KEY_ID not set (eval \"$(triton env)\" first)"))
    return out


def kubeadm_checks(backend: str, workdir: str = ".") -> list[dict]:
    if backend == "local":
        from .orchestrator import local_kubeadm_allowed

        if local_kubeadm_allowed():
            return [_check("kubeadm platform", OK, "single-node on this host (as root, no ssh): installs ROCm, "
                                                   "amdgpu-dkms, containerd and kubeadm here (needs apt and network "
                                                   "access)")]
        return [_check("kubeadm platform", FAIL, "installs a node runtime: as root on this host (single-node), or "
                                                 "--backend baremetal / triton with machines it owns")]
    layout = ""
    if backend == "baremetal":
        try:
            from .provider.baremetal import BareMetalProvider

            p = BareMetalProvider(Path(workdir) / ".tk8s")
            layout = (" -- single-node: control plane and every GPU on the one host" if p.single_host()
                      else " -- a kubelet per host")
        except Exception:  # noqa: BLE001 - the inventory check reports it
            pass
    return [_check("kubeadm platform", OK, "installs ROCm, amdgpu-dkms, containerd and kubeadm as root over ssh "
                                          "(the machines need apt and network access)" + layout)]


def run_checks(workdir: str, backend: str | None = None, platform: str | None = None) -> list[dict]:
    backend = backend or os.environ.get("TK8S_BACKEND", "local")
    platform = platform or os.environ.get("TK8S_PLATFORM", "tk8s")
    out = common_checks()
    if backend == "local":
        out += local_checks(workdir)
    elif backend == "baremetal":
        out += baremetal_checks(workdir, platform)
    elif backend == "triton":
        out += triton_checks()
    else:
        out.append(_check("backend", FAIL, f"unknown backend {backend!r}"))
    if platform == "kubeadm":
        out += kubeadm_checks(backend, workdir)
    return out


def render(checks: list[dict]) -> str:
    w = max(len(c["check"]) for c in checks)
    return "\n".join(f"{c['status']:<4}  {c['check']:<{w}}  {c['detail']}" for c in checks)


def main(workdir: str, backend: str | None, platform: str | None, as_json: bool) -> int:
    checks = run_checks(workdir, backend, platform)
    print(json.dumps(checks) if as_json else render(checks))
    return 1 if any(c["status"] == FAIL for c in checks) else 0
