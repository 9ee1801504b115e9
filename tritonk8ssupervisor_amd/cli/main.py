"""`tk8s` command line: setup / clean / status / provider listings / engines / kubectl.

  ./setup.sh [--answers FILE] [--yes] [--resume] [--timeout S] ...   -> tk8s setup
  ./setup.sh -c [--yes]                                               -> tk8s clean
  ./tk8s networks|packages [-l]     (triton networks / triton packages)
  ./tk8s env                        (triton env)
  ./tk8s doctor [--platform P] [--json]   (preflight checks for the backend / platform)
  ./tk8s debug-vars                 (debugVars: the exported ./config)
  ./tk8s terraform get|plan|apply|destroy     (provisioning engine, in terraform/)
  ./tk8s ansible-playbook [--check] [-i hosts] clusterUp.yml           (playbook engine)
  ./tk8s status [--json]            (phases, nodes, GPUs, last RCCL busbw)
  ./tk8s scale N [--json]           (add / drain and remove workers of the running cluster)
  ./tk8s image load FILE | ls | rm REF   (this host's container images, loaded from files)
  ./kubectl ...                     (see cli/kubectl.py)
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path


def _ws(args):
    from ..orchestrator import Workspace

    return Workspace(Path(args.workdir).resolve())


def cmd_setup(args) -> int:
    from ..orchestrator import Setup, SetupError
    from ..provider.base import ProvisionError
    from ..wizard import WizardAbort, load_answers

    answers = load_answers(args.answers) if args.answers else None
    if answers is None and args.nodes:
        answers = {}
    if answers is not None:
        for k in ("nodes", "package", "name", "master_hostname", "node_prefix"):
            v = getattr(args, k, None)
            if v is not None:
                answers[k] = v
    s = Setup(_ws(args), answers=answers, assume_yes=args.yes, resume=args.resume, timeout=args.timeout,
              validate=not args.no_validate, rccl=(None if args.rccl is None else args.rccl == "on"),
              quiet_ansible=not args.verbose, backend=args.backend, master_port=args.port,
              hbm_bytes=args.hbm_bytes, md5_bytes=args.md5_bytes, probe_iters=args.probe_iters,
              node_grace=args.node_grace, rocprof=args.rocprof, rocprof_counters=args.rocprof_counters,
              rccl_max_bytes=args.rccl_max_bytes,
              rccl_timeout=args.rccl_timeout, rccl_op_timeout=args.rccl_op_timeout, platform=args.platform)
    try:
        summary = s.dry_run() if args.dry_run else s.run()
    except WizardAbort:
        return 0
    except SetupError as e:
        print(str(e), file=sys.stderr)
        return e.code
    except ProvisionError as e:  # a provider refusing before any phase could (inventory, credentials)
        print(f"error: {e}", file=sys.stderr)
        return 1
    if args.json:
        print(json.dumps(summary))
    if args.dry_run and not summary.get("check_ok"):
        print(f"dry run: the --check playbook failed on {', '.join(summary.get('check_failures') or ['?'])}",
              file=sys.stderr)
        return 2
    return 0


def cmd_doctor(args) -> int:
    from ..doctor import main as doctor

    return doctor(args.workdir, getattr(args, "backend", None), args.platform, args.json)


def cmd_scale(args) -> int:
    from ..orchestrator import Setup, SetupError

    s = Setup(_ws(args), resume=False, timeout=args.timeout, rccl=(None if args.rccl is None else args.rccl == "on"),
              quiet_ansible=not args.verbose, backend=args.backend)
    try:
        out = s.scale(args.nodes)
    except SetupError as e:
        print(str(e), file=sys.stderr)
        return e.code
    if args.json:
        print(json.dumps(out))
    return 0


def cmd_clean(args) -> int:
    from ..orchestrator import clean

    return clean(_ws(args), assume_yes=args.yes, backend=args.backend)


def cmd_status(args) -> int:
    ws = _ws(args)
    st = ws.state()
    out = {"completed": st.get("completed", []), "timings": st.get("timings", {}), "summary": st.get("summary")}
    summ = st.get("summary") or {}
    if summ.get("platform") == "kubeadm":  # a real Kubernetes: ask its API server through the master
        from ..config import read_config
        from ..orchestrator import MachineExecutor
        from ..provision import Engine

        try:
            cfg = read_config(ws.config)
            prov = _provider(args)
            machines = Engine(ws.tf, prov).machines()
            rc, text = MachineExecutor(prov, machines).exec(
                cfg.RANCHER_MASTER_HOSTNAME, "kubectl --kubeconfig ${TK8S_SYSROOT:-}/etc/kubernetes/admin.conf get nodes -o json",
                timeout=60)
            items = json.loads(text)["items"] if rc == 0 else []
            ready = [n for n in items if any(c.get("type") == "Ready" and c.get("status") == "True"
                                             for c in n["status"].get("conditions", []))]
            out["cluster"] = {"nodes": len(items), "nodes_ready": len(ready), "nodes_validated": len(ready),
                              "gpus_allocatable": sum(int(n["status"].get("allocatable", {}).get("amd.com/gpu", 0) or 0)
                                                      for n in ready), "gpus_in_use": None}
        except Exception as e:  # noqa: BLE001 - reporting only
            out["cluster"] = {"error": str(e)}
    elif summ.get("api"):
        from ..controlplane.client import Client

        try:
            out["cluster"] = Client(summ["api"], token=ws.admin_token(), timeout=5).get(
                "/v1/cluster/status", query={"project": summ.get("project")})
        except Exception as e:  # noqa: BLE001
            out["cluster"] = {"error": str(e)}
    if args.json:
        print(json.dumps(out, indent=1))
    else:
        print(f"completed phases: {', '.join(out['completed']) or '-'}")
        for k, v in out["timings"].items():
            print(f"  {k:<16} {v:8.3f}s")
        c = out.get("cluster") or {}
        if c and "error" not in c:
            print(f"nodes: {c['nodes_ready']}/{c['nodes']} Ready, {c['nodes_validated']} validated; "
                  f"amd.com/gpu allocatable {c['gpus_allocatable']} (in use {c['gpus_in_use']})")
        r = summ.get("rccl") or {}
        if r.get("ok") and r.get("nranks"):
            from ..fabric import fabric_line

            print(f"last {fabric_line(r)}")
        elif r:
            print(f"RCCL all-reduce: {'ok' if r.get('ok') else 'FAILED'} on {r.get('pods')} pod(s)")
    return 0


def cmd_image(args) -> int:
    """``./tk8s image load FILE | ls | rm REF``: the node's image store (agent/images.py), the
    reference's ``docker pull`` for an offline host: pods naming a loaded image run in it."""
    from ..agent.images import ImageError, ImageStore

    store = ImageStore()
    try:
        if args.action == "load":
            if not args.source:
                raise ImageError("image load needs a file or directory")
            out = {"loaded": store.load(args.source, tag=args.tag)}
            text = "\n".join(f"Loaded image: {r}" for r in out["loaded"])
        elif args.action == "ls":
            out = {"images": store.list()}
            text = "\n".join([f"{'IMAGE':<60} {'LAYERS':>6} {'SIZE':>12}"] +
                              [f"{i['ref']:<60} {i['layers']:>6} {i['size']:>12}" for i in out["images"]])
        else:
            if not args.source:
                raise ImageError("image rm needs a reference")
            if not store.remove(args.source):
                raise ImageError(f"no such image: {args.source}")
            out = {"removed": args.source}
            text = f"Untagged: {args.source}"
    except (ImageError, OSError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    print(json.dumps(out) if args.json else text)
    return 0


def cmd_debug_vars(args) -> int:
    """debugVars (setup.sh:522-531, never called there): the exported configuration."""
    from ..config import read_config

    ws = _ws(args)
    if not ws.config.exists():
        print("no ./config yet (run ./setup.sh first)", file=sys.stderr)
        return 1
    env = read_config(ws.config).as_env()
    for k in ("KUBERNETES_NAME", "KUBERNETES_DESCRIPTION", "RANCHER_MASTER_HOSTNAME",
              "KUBERNETES_NODE_HOSTNAME_BEGINSWITH", "KUBERNETES_NUMBER_OF_NODES", "RANCHER_MASTER_NETWORKS",
              "KUBERNETES_NODE_NETWORKS", "HOST_PACKAGE"):
        print(f"{k}={env.get(k, '')}")
    return 0


def _provider(args):
    from ..provider import get_provider

    ws = _ws(args)
    return get_provider(args.backend or os.environ.get("TK8S_BACKEND", "local"), ws.state_dir)


def cmd_networks(args) -> int:
    for n in _provider(args).networks():
        print(f"{n.name:<20} {n.id}" + (f"  {n.subnet}{'  public' if n.public else ''}" if args.l else ""))
    return 0


def cmd_packages(args) -> int:
    for p in _provider(args).packages():
        extra = f"  gpus={p.gpus} cpus={p.cpus} memory={p.memory_mb}M  {p.description}" if args.l else ""
        print(f"{p.name:<16} {p.id}{extra}")
    return 0


def cmd_env(args) -> int:
    for k, v in _provider(args).env().items():
        print(f'export {k}="{v}"')
    return 0


def cmd_gpu_health(args) -> int:
    """AMD SMI health of every GPU of this host (what the node agents sample)."""
    from ..agent.agent import read_smi

    r = read_smi()
    if r is None:
        print("tk8s-smi is not available (build the native layer first)", file=sys.stderr)
        return 3
    if args.json:
        print(json.dumps(r, indent=1))
    else:
        print(f"{'GPU':<4} {'PCI':<13} {'HEALTHY':<8} {'HOTSPOT':>7} {'POWER':>6} {'VRAM USED':>10} {'ECC UE/CE':>10}")
        for g in r.get("gpus", []):
            ecc = g.get("ecc", {})
            used = g.get("vram_used_bytes")
            print(f"{g.get('index', '?'):<4} {g.get('pci_bus_id', '?'):<13} {str(g.get('healthy')):<8} "
                  f"{str(g.get('temp_c', {}).get('hotspot', '-')) + 'C':>7} "
                  f"{str(g.get('power', {}).get('current_w', '-')) + 'W':>6} "
                  f"{(f'{used / 2**30:.1f}GiB' if used is not None else '-'):>10} "
                  f"{str(ecc.get('uncorrectable', '-')) + '/' + str(ecc.get('correctable', '-')):>10}")
        if not r.get("ok"):
            print(r.get("error", "no GPU"), file=sys.stderr)
    return 0 if r.get("ok") and r.get("healthy") else (3 if not r.get("ok") else 1)


def cmd_machine(args) -> int:
    """``./tk8s machine create|delete|list``: the provider's machine lifecycle as a CLI -- what the
    stock-Terraform modules' local-exec provisioners call (terraform/compat/*/main.tf)."""
    import fcntl

    from ..provider.base import ProvisionError
    from ..provision import BOOTSTRAP

    ws = _ws(args)
    prov = _provider(args)
    if args.action == "list":
        for m in getattr(prov, "list_machines", lambda: [])():
            print(json.dumps(m.to_dict()))
        return 0
    if args.action == "create":
        key = ""
        if args.authorized_keys and Path(args.authorized_keys).exists():
            key = Path(args.authorized_keys).read_text()
        try:
            m = prov.create_machine(args.name, args.package, [n for n in args.networks.split(",") if n],
                                    image=args.image or "", root_authorized_keys=key,
                                    tags={"name": args.name, "role": args.role})
        except ProvisionError as e:
            print(f"Error: {e}", file=sys.stderr)
            return 1
        rc, out = prov.exec(m, "set -e\n" + "\n".join(BOOTSTRAP))
        if rc != 0:
            prov.delete_machine(m)
            print(f"Error: {args.name}: bootstrap failed: {out.strip()[-400:]}", file=sys.stderr)
            return 1
        if args.ip_file:  # the masters.ip / hosts.ip hand-off, appended under a lock
            with open(ws.tf / args.ip_file if not Path(args.ip_file).is_absolute() else args.ip_file, "a") as f:
                fcntl.flock(f, fcntl.LOCK_EX)
                f.write(m.primaryip + "\n")
        print(json.dumps(m.to_dict()))
        return 0
    m = prov.get_machine(args.name)
    if m is None:
        print(f"machine {args.name} not found (already deleted)")
        return 0
    prov.delete_machine(m)
    print(f"machine {args.name} deleted")
    return 0


def cmd_terraform(args) -> int:
    from ..provision import Engine

    ws = _ws(args)
    eng = Engine(ws.tf, _provider(args))
    if args.action == "get":
        print("\n".join(f"- module.{m}" for m in eng.get()))
    elif args.action == "plan":
        print(Engine.plan_summary(eng.plan()))
    elif args.action == "apply":
        r = eng.apply()
        print(f"Apply complete! Resources: {len(r.created)} added, 0 changed, 0 destroyed ({r.seconds:.3f}s)")
        for a, e in r.failed.items():
            print(f"Error: {a}: {e}", file=sys.stderr)
        return 0 if r.ok else 1
    elif args.action == "destroy":
        print(f"Destroy complete! Resources: {len(eng.destroy())} destroyed.")
    return 0


def cmd_playbook(args) -> int:
    from ..orchestrator import MachineExecutor
    from ..playbook import Playbook
    from ..provision import Engine

    ws = _ws(args)
    prov = _provider(args)
    machines = {}
    if (ws.tf / "terraform.tfstate").exists():
        machines = Engine(ws.tf, prov).machines()
    elif hasattr(prov, "list_machines"):  # machines made by stock Terraform (terraform/compat)
        machines = {m.name: m for m in prov.list_machines()}
    pb = Path(args.playbook)
    if not pb.is_absolute():
        pb = ws.ansible / pb
    inv = Path(args.inventory) if args.inventory else ws.ansible / "hosts"
    if not inv.is_absolute() and not inv.exists():
        inv = ws.ansible / inv
    extra = {}
    if machines and ws.config.exists():
        from ..config import read_config
        from ..orchestrator import playbook_extra_vars

        cfg = read_config(ws.config)
        if cfg.RANCHER_MASTER_HOSTNAME in machines:
            extra = playbook_extra_vars(ws, cfg, machines)
    if args.extra_vars:
        extra.update(dict(kv.split("=", 1) for kv in args.extra_vars))
    res = Playbook(pb, inv, executor=MachineExecutor(prov, machines) if machines else None, extra_vars=extra,
                   check=args.check).run()
    return 0 if res.ok else 2


# `tk8s setup` options: argparse builds the parser from this table, and _fast_setup_args parses
# the same table by hand on the bring-up path (argparse + gettext + locale cost ~5 ms there).
SETUP_OPTIONS: list[tuple[tuple[str, ...], dict]] = [
    (("--answers",), {"help": "YAML/JSON answers file (non-interactive)"}),
    (("--yes",), {"action": "store_true", "help": "answer yes to the confirmation"}),
    (("--resume",), {"action": "store_true", "help": "continue a partial run"}),
    (("--timeout",), {"type": float, "default": 600.0, "help": "bound on the readiness wait (s)"}),
    (("--nodes",), {"type": int}),
    (("--package",), {}),
    (("--name",), {}),
    (("--master-hostname",), {}),
    (("--node-prefix",), {}),
    (("--port",), {"type": int, "default": None}),
    (("--no-validate",), {"action": "store_true", "help": "skip the GPU validation DaemonSet"}),
    (("--rccl",), {"choices": ["on", "off"], "default": None,
                   "help": "cluster RCCL all-reduce (default: on if >= 2 GPUs)"}),
    (("--hbm-bytes",), {"type": int, "default": 1 << 30}),
    (("--md5-bytes",), {"type": int, "default": 256 << 20}),
    (("--probe-iters",), {"type": int, "default": 3}),
    (("--node-grace",), {"type": float, "default": 5.0}),
    (("--rocprof",), {"action": "store_true",
                      "help": "run the RCCL Job's ranks under rocprofv3 --kernel-trace --stats (rocprof/<job>/)"}),
    (("--rocprof-counters",), {"default": None, "metavar": "C1,C2,...",
                               "help": "with --rocprof: also collect these PMC counters per kernel (their own --pmc "
                                       "pass with --kernel-trace/--stats only; at most 8 SQ_ and 2 GRBM_ counters), "
                                       "e.g. SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE"}),
    (("--rccl-max-bytes",), {"type": int, "default": 64 << 20}),
    (("--rccl-timeout",), {"type": float, "default": None, "help": "bound on the RCCL Job (default: --timeout)"}),
    (("--rccl-op-timeout",), {"type": float, "default": 20.0,
                              "help": "bound on each wait of an RCCL rank (unique id, communicator init, each "
                                      "sweep point): a dead or hung peer aborts the Job within it (default 20 s)"}),
    (("--dry-run",), {"action": "store_true",
                      "help": "terraform plan + ansible-playbook --check of what setup would do; changes nothing "
                              "(BASELINE.json config 1)"}),
    (("--platform",), {"choices": ["tk8s", "kubeadm"], "default": None,
                       "help": "tk8s (default): the in-repo control plane and node agents; kubeadm: install ROCm, "
                               "amdgpu-dkms, containerd and a real Kubernetes on the machines (needs root + network)"}),
    (("--json",), {"action": "store_true"}),
    (("-v", "--verbose"), {"action": "store_true"}),
]


def _fast_setup_args(argv: list[str]):
    """``setup`` arguments parsed from SETUP_OPTIONS without argparse -- the same Namespace
    argparse would build -- or None for anything it does not handle exactly like argparse (help,
    an unknown or abbreviated option, a bad value), which then goes to argparse."""
    if not argv or argv[0] != "setup":
        return None
    from types import SimpleNamespace

    opts = {}
    ns = {"workdir": os.environ.get("TK8S_WORKDIR", os.getcwd()), "backend": None, "inventory": None,
          "cmd": "setup", "fn": cmd_setup}
    for flags, kw in SETUP_OPTIONS:
        dest = flags[-1].lstrip("-").replace("-", "_")
        ns[dest] = False if kw.get("action") == "store_true" else kw.get("default")
        for f in flags:
            opts[f] = (dest, kw)
    for f in ("--backend", "--inventory"):
        opts[f] = (f[2:], {})
    i, rest = 0, argv[1:]
    while i < len(rest):
        a = rest[i]
        name, eq, val = a.partition("=") if a.startswith("--") else (a, "", "")
        if name not in opts:
            return None
        dest, kw = opts[name]
        if kw.get("action") == "store_true":
            if eq:
                return None
            ns[dest] = True
            i += 1
            continue
        if not eq:
            if i + 1 >= len(rest) or rest[i + 1].startswith("-"):
                return None
            val = rest[i + 1]
            i += 1
        i += 1
        try:
            val = kw.get("type", str)(val)
        except ValueError:
            return None
        if "choices" in kw and val not in kw["choices"]:
            return None
        ns[dest] = val
    return SimpleNamespace(**ns)


def _backend_flags(p: argparse.ArgumentParser) -> None:
    """--backend/--inventory also after the subcommand (``./setup.sh --backend baremetal ...``)."""
    import argparse
    p.add_argument("--backend", default=argparse.SUPPRESS, help="local (default), baremetal or triton")
    p.add_argument("--inventory", default=argparse.SUPPRESS, help="baremetal: the SSH inventory file")


def build_parser() -> argparse.ArgumentParser:
    import argparse
    ap = argparse.ArgumentParser(prog="tk8s", description="MI355X-native cluster bring-up")
    ap.add_argument("--workdir", default=os.environ.get("TK8S_WORKDIR", os.getcwd()))
    ap.add_argument("--backend", default=None, help="local (default), baremetal (ssh inventory) or triton")
    ap.add_argument("--inventory", default=None, help="baremetal: the SSH inventory file (TK8S_INVENTORY)")
    sub = ap.add_subparsers(dest="cmd", required=True)

    s = sub.add_parser("setup", help="create the cluster (./setup.sh)")
    for flags, kw in SETUP_OPTIONS:
        s.add_argument(*flags, **kw)
    _backend_flags(s)
    s.set_defaults(fn=cmd_setup)

    sc = sub.add_parser("scale", help="change the number of workers of the running cluster (1-9)")
    sc.add_argument("nodes", type=int)
    sc.add_argument("--timeout", type=float, default=600.0, help="bound on the readiness wait (s)")
    sc.add_argument("--rccl", choices=["on", "off"], default=None, help="re-run the RCCL all-reduce Job afterwards")
    sc.add_argument("--json", action="store_true")
    sc.add_argument("-v", "--verbose", action="store_true")
    _backend_flags(sc)
    sc.set_defaults(fn=cmd_scale)

    c = sub.add_parser("clean", help="destroy machines and reset configuration (./setup.sh -c)")
    c.add_argument("--yes", action="store_true")
    _backend_flags(c)
    c.set_defaults(fn=cmd_clean)

    st = sub.add_parser("status")
    st.add_argument("--json", action="store_true")
    st.set_defaults(fn=cmd_status)

    for name, fn in (("networks", cmd_networks), ("packages", cmd_packages)):
        p = sub.add_parser(name)
        p.add_argument("-l", action="store_true")
        p.set_defaults(fn=fn)
    sub.add_parser("env").set_defaults(fn=cmd_env)
    dr = sub.add_parser("doctor", help="preflight: check what a bring-up on this backend/platform needs")
    dr.add_argument("--platform", choices=["tk8s", "kubeadm"], default=None)
    dr.add_argument("--json", action="store_true")
    _backend_flags(dr)
    dr.set_defaults(fn=cmd_doctor)
    gh = sub.add_parser("gpu-health", help="AMD SMI health/telemetry of this host's GPUs (tk8s-smi)")
    gh.add_argument("--json", action="store_true")
    gh.set_defaults(fn=cmd_gpu_health)
    sub.add_parser("debug-vars", help="print the exported configuration (debugVars)").set_defaults(fn=cmd_debug_vars)

    mc = sub.add_parser("machine", help="create/delete/list machines (what the stock-Terraform modules call)")
    mc.add_argument("action", choices=["create", "delete", "list"])
    mc.add_argument("--name")
    mc.add_argument("--package", default="")
    mc.add_argument("--networks", default="")
    mc.add_argument("--role", default="host", choices=["master", "host"])
    mc.add_argument("--image", default="")
    mc.add_argument("--authorized-keys", default=None, help="public key file to authorise on the machine")
    mc.add_argument("--ip-file", default=None, help="append the machine's IP here (relative to terraform/)")
    mc.set_defaults(fn=cmd_machine)

    t = sub.add_parser("terraform")
    t.add_argument("action", choices=["get", "plan", "apply", "destroy"])
    t.set_defaults(fn=cmd_terraform)

    pb = sub.add_parser("ansible-playbook")
    pb.add_argument("playbook", nargs="?", default="clusterUp.yml")
    pb.add_argument("-i", "--inventory", default=None)
    pb.add_argument("--check", "-C", action="store_true")
    pb.add_argument("-e", "--extra-vars", action="append")
    pb.set_defaults(fn=cmd_playbook)

    im = sub.add_parser("image", help="this host's container images (air-gapped: loaded from files)")
    im.add_argument("action", choices=["load", "ls", "rm"])
    im.add_argument("source", nargs="?", help="load: a docker save archive or an OCI layout; rm: a reference")
    im.add_argument("--tag", default=None, help="load: the name for an image the file does not name")
    im.add_argument("--json", action="store_true")
    im.set_defaults(fn=cmd_image)

    k = sub.add_parser("kubectl", add_help=False)
    k.add_argument("rest", nargs=argparse.REMAINDER)
    k.set_defaults(fn=lambda a: __import__("tritonk8ssupervisor_amd.cli.kubectl", fromlist=["main"]).main(a.rest, workdir=a.workdir))
    return ap


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    from .. import shortcut_on

    args = (_fast_setup_args(argv) if shortcut_on("TK8S_FAST_ARGS") else None) or build_parser().parse_args(argv)
    if getattr(args, "inventory", None):
        os.environ["TK8S_INVENTORY"] = str(Path(args.inventory).resolve())
    if getattr(args, "backend", None):
        os.environ["TK8S_BACKEND"] = args.backend  # the same backend for every later step of this run
    prof = os.environ.get("TK8S_PROFILE")
    if not prof:
        return args.fn(args)
    import cProfile  # TK8S_PROFILE=<file>: where does a bring-up spend its host time?

    pr = cProfile.Profile()
    try:
        return pr.runcall(args.fn, args)
    finally:
        pr.dump_stats(prof)


if __name__ == "__main__":
    sys.exit(main())
