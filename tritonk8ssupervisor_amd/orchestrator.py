"""Bring-up orchestrator: ``./setup.sh`` (create) and ``./setup.sh -c`` (teardown).

Reference: main setup.sh:8-92 (W1), runTerraformTasks/updateTerraformConfig :138-198 (W9/W10),
createAnsibleConfigs :116-137 (W12), runAnsible :111-115 (W16), cleanRunner :484-521 (W13),
readiness loop :56-85 (W14). Phase order is the same; what changed:

  * no fixed sleeps (the reference sleeps 2 s x3 between phases, 30 s per VM, 15 s pause);
  * readiness is event-driven (control-plane long-poll) and BOUNDED (--timeout), instead of a
    1 s tick / 15 s curl loop that can run forever; "Ready" means every worker heartbeating,
    every GPU worker validated by tk8s-probe, amd.com/gpu allocatable == expected, and (with
    >= 2 GPUs) an RCCL all-reduce across all of them reduced exactly;
  * every phase is timed into .tk8s/events.jsonl and .tk8s/state.json (``--resume`` skips
    completed phases; the reference can only be cleaned and restarted);
  * teardown also removes ansible/tmp/kubernetes_environment.id and vars.yml (W13 bug).
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from pathlib import Path

from . import hcl
from .config import ClusterConfig, export_vars, read_config, write_config
from .earlyburn import default_validation_command  # noqa: F401 - shared with the early burn-in
from .fabric import FabricCheck, check_pmc_counters, fabric_line, rccl_transports, summarize_rocprof  # noqa: F401
from .kubeadm_platform import KUBEADM_RESET, KubeadmPlatform, kubeadm_extra_vars
from .provider import get_provider
from .provider.base import Machine, ProvisionError
from .provision import Engine
from .utils.events import EventLog
from .utils.faults import fault
from .utils.fsutil import atomic_write, atomic_write_json, read_json
from .utils.procs import kill_pidfile, pid_alive
from .workspace import (  # noqa: F401 - the orchestrator's public names, re-exported
    PHASES, PLATFORMS, PLAYBOOKS, REPO, TEMPLATE_DIRS, TEMPLATE_FILES, SetupError, Workspace, agent_standby_argv,
    controlplane_argv, init_workspace, pod_portable, validation_pod_command,
)


def local_kubeadm_allowed() -> bool:
    """May ``--platform kubeadm`` run on this host itself (the local backend)? As root -- it installs
    the node runtime -- or against a simulated root (TK8S_LOCAL_HOST_ROOT, the CPU tests)."""
    return os.geteuid() == 0 or bool(os.environ.get("TK8S_LOCAL_HOST_ROOT"))


# ---- machine executor for the playbook engine ---------------------------------------------
# executor.py: LocalExecutor for colocated sandboxes, RemoteExecutor (ssh) for everything else.
from .executor import MachineExecutor  # noqa: E402,F401 - re-exported (./tk8s ansible-playbook)


def playbook_extra_vars(ws: Workspace, cfg: ClusterConfig, machines: dict[str, Machine], *, node_grace: float = 5.0,
                        validate: bool = True, validation_command: list[str] | None = None) -> dict:
    """Variables the roles need beyond inventory + vars.yml (shared by setup and
    `./tk8s ansible-playbook`, so a by-hand run of clusterUp.yml behaves like setup's)."""
    m = machines[cfg.RANCHER_MASTER_HOSTNAME]
    vcmd = validation_command or default_validation_command()
    return {
        "tk8s_python": sys.executable,
        "tk8s_pythonpath": os.pathsep.join([str(REPO)] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p]),
        "tk8s_master_port": int(cfg.TK8S_MASTER_PORT),
        "tk8s_bind_host": m.primaryip,
        "tk8s_cp_state_dir": str(Path(m.sandbox) / "controlplane"),
        "tk8s_admin_token_file": str(ws.admin_token_file),
        "tk8s_node_grace": node_grace,
        "tk8s_controlplane_argv": controlplane_argv(m.primaryip, int(cfg.TK8S_MASTER_PORT), m.primaryip,
                                                    str(Path(m.sandbox) / "controlplane"), node_grace),
        "tk8s_manifests": str(ws.manifests),
        "tk8s_validation_command": vcmd,
        "tk8s_validation_pod_command": validation_pod_command(vcmd),
        "tk8s_validate": validate,
        "tk8s_fake_gpus": os.environ.get("TK8S_FAKE_GPUS", ""),
    }


# ---- setup ---------------------------------------------------------------------------------
class Setup(KubeadmPlatform, FabricCheck):
    def __init__(self, ws: Workspace, *, answers: dict | None = None, assume_yes: bool = False,
                 resume: bool = False, timeout: float = 600.0, validate: bool = True, rccl: bool | None = None,
                 out: Callable[[str], None] = None, quiet_ansible: bool = True, hbm_bytes: int = 1 << 30,
                 md5_bytes: int = 256 << 20, probe_iters: int = 3, rccl_max_bytes: int = 64 << 20,
                 node_grace: float = 5.0, backend: str | None = None, master_port: int | None = None,
                 rocprof: bool = False, rccl_timeout: float | None = None, rocprof_counters: str | None = None,
                 platform: str | None = None, rccl_op_timeout: float = 20.0):
        self.ws = ws
        self.answers = answers
        self.assume_yes = assume_yes
        self.resume = resume
        self.timeout = timeout
        self.validate = validate
        self.rccl = rccl
        self.out = out or _flush_print
        self.quiet_ansible = quiet_ansible
        self.hbm_bytes, self.md5_bytes, self.probe_iters = hbm_bytes, md5_bytes, probe_iters
        self.rccl_max_bytes = rccl_max_bytes
        self.node_grace = node_grace
        self.backend = backend or os.environ.get("TK8S_BACKEND", "local")
        self.platform = platform or os.environ.get("TK8S_PLATFORM", "tk8s")
        if self.platform not in PLATFORMS:
            raise SetupError(f"error: unknown platform {self.platform!r} (expected one of {', '.join(PLATFORMS)})")
        self.master_port = master_port
        self.rocprof = rocprof
        self.rocprof_counters = [c for c in (rocprof_counters or "").replace(" ", ",").split(",") if c]
        self.rccl_timeout = rccl_timeout
        self.rccl_op_timeout = rccl_op_timeout
        ws.state_dir.mkdir(parents=True, exist_ok=True)
        self.events = EventLog(ws.events, echo=False)
        if self.platform == "kubeadm" and self.backend == "local" and local_kubeadm_allowed():
            # one command on one box (the reference's setup.sh:8-92): kubeadm single-node on THIS host,
            # as root, through the bare-metal path with a one-host inventory reached without ssh
            from .provider.baremetal import BareMetalProvider, local_host_inventory

            self.backend = "baremetal"
            self.provider = BareMetalProvider(ws.state_dir, inventory=local_host_inventory(ws.state_dir))
        else:
            self.provider = get_provider(self.backend, ws.state_dir)
        self.engine = Engine(ws.tf, self.provider, self.events, on_created=self._machine_booted)
        self.cfg: ClusterConfig | None = None
        self.summary: dict = {}
        self.host_burnin = None

    def banner(self, text: str) -> None:
        self.out("#" * 80)
        self.out(f"### {text}")
        self.out("#" * 80)

    def done(self, phase: str) -> bool:
        return self.resume and phase in self.ws.state().get("completed", [])

    def mark(self, phase: str) -> None:
        st = self.ws.state()
        comp = [p for p in st.get("completed", []) if p != phase] + [phase]
        timings = st.get("timings", {})
        timings[phase] = round(self.events.phases.get(phase, 0.0), 6)
        self.ws.save_state(completed=comp, timings=timings)

    # -- phases --------------------------------------------------------------------------
    def configure(self) -> ClusterConfig:
        from .wizard import run_wizard

        ws = self.ws
        if self.resume and ws.config.exists():
            cfg = read_config(ws.config)
        else:
            if ws.config.exists():
                raise SetupError("error: old configuration found\n    clean the configuration (./setup.sh -c)")
            cfg = ClusterConfig(TK8S_BACKEND=self.backend, TK8S_PLATFORM=self.platform)
            if self.master_port == 0:  # a free port outside the ephemeral and NodePort ranges (utils/net.pick_port; clusters side by side)
                cfg.TK8S_MASTER_PORT = _free_port()
            elif self.master_port:
                cfg.TK8S_MASTER_PORT = self.master_port
            env = self.provider.env()
            cfg.SDC_URL, cfg.SDC_ACCOUNT, cfg.SDC_KEY_ID = env["SDC_URL"], env["SDC_ACCOUNT"], env["SDC_KEY_ID"]
            key = self.provider.find_key(cfg.SDC_KEY_ID)
            if not key:
                raise SetupError(f"error: couldn't find the key associated with fingerprint {cfg.SDC_KEY_ID}\n"
                                 "    Clean the setup and make sure your provider profile is set up.")
            cfg.SDC_KEY = key
            answers = self.answers
            if answers is not None and self.assume_yes:
                answers = dict(answers)
                answers.setdefault("confirm", "yes")
            run_wizard(cfg, self.provider, answers=answers, out=None if answers is None else _Sink(self.out))
            write_config(ws.config, cfg)
        export_vars(cfg)
        self.cfg = cfg
        self.platform = cfg.TK8S_PLATFORM or "tk8s"
        if self.platform == "kubeadm" and self.provider.colocated:
            raise SetupError("error: the kubeadm platform installs ROCm, amdgpu-dkms, containerd and Kubernetes as root: "
                             "run ./setup.sh --platform kubeadm as root for a single-node cluster on this host, or use "
                             "machines you own (--backend baremetal with an SSH inventory, or triton)")
        if self.platform == "kubeadm" and hasattr(self.provider, "whole_hosts"):
            # a kubelet per host: machines are whole hosts, not slices -- except on a one-host
            # inventory (single-node mode), where the workers are GPU slots of the master's node
            self.provider.whole_hosts = not self.kubeadm_single_node
        return cfg

    def _machine_booted(self, address: str, m: Machine) -> None:
        """Boot hook: a GPU machine starts its GPU burn-in the moment it exists (like a node
        image's boot-time GPU health check), overlapping the other machines' creation and play 1.
        rocmsetup's burn-in task then finds it running and does nothing."""
        if not self.provider.colocated:  # remote machines: the playbook does everything, over ssh
            return
        if self.cfg is not None and m.name == self.cfg.RANCHER_MASTER_HOSTNAME:
            self._boot_controlplane(m)
        elif self.cfg is not None:
            self._boot_agent(m)
        if not (self.validate and m.gpus):
            return
        if self.host_burnin is not None and self.host_burnin.register(m.name, m.sandbox, list(m.gpus)):
            self.events.emit("gpu_burnin_shared_pending", name=m.name, gpus=list(m.gpus))
            return
        from .burnin import start_burnin

        ex = MachineExecutor(self.provider, {m.name: m})
        r = start_burnin(ex, m.name, self._validation_command(), "run/gpu-burnin.json")
        self.events.emit("gpu_burnin_started", name=m.name, **{k: v for k, v in r.items() if k in ("pid", "gpus", "msg")})

    def _boot_agent(self, m: Machine) -> None:
        """Worker boot hook: the node agent (kubelet role) starts in standby with its machine, the
        way a node image starts its kubelet at boot. Its interpreter start and imports (~30 ms on
        the MI355X box, profiles/r1_trace2) then overlap provisioning and play 1 instead of
        delaying the join after play 3 hands it the registration URL; rocmsetup's standby task
        finds it running (same argv: agent_standby_argv)."""
        if os.environ.get("TK8S_BOOT_AGENT", "1") == "0":
            return
        pythonpath = os.pathsep.join([str(REPO)] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
        argv = agent_standby_argv(m.name, m.primaryip)
        from . import earlyburn

        z = earlyburn.agent_zygote_for(m.sandbox)  # its interpreter started with the CLI: hand it the arguments
        if z is not None and fault("zygote.no_args", m.name) is not None:
            return  # fault injection: the zygote is never handed its arguments (rocmsetup recovers)
        if z is not None:
            if pid_alive(z["pid"]):
                env = {**getattr(self.provider, "machine_env", lambda _m: {})(m), "PYTHONPATH": pythonpath}
                atomic_write(z["args"], json.dumps({"argv": argv[4:], "env": env, "cwd": m.sandbox}))
                self.events.emit("agent_boot_started", name=m.name, pid=z["pid"], zygote=True)
                return
            try:
                os.killpg(z["pid"], 15)
            except OSError:
                pass
        ex = MachineExecutor(self.provider, {m.name: m})
        info = ex.start_daemon(m.name, "agent", argv, env={"PYTHONPATH": pythonpath},
                               restart="unless-stopped", wait_for_log=None, timeout=0)
        self.events.emit("agent_boot_started", name=m.name, pid=info.get("pid"))

    def _boot_controlplane(self, m: Machine) -> None:
        """Master boot hook: the control plane service starts with its machine (the way a master
        image would start rancher/server at boot), overlapping the workers' creation and play 1;
        the ranchermaster role then finds it running and waits for its "Listening on"."""
        if os.environ.get("TK8S_BOOT_CONTROLPLANE", "1") == "0":
            return
        argv = controlplane_argv(m.primaryip, int(self.cfg.TK8S_MASTER_PORT), m.primaryip,
                                 str(Path(m.sandbox) / "controlplane"), self.node_grace)
        from . import earlyburn

        z = earlyburn.zygote_for(m.sandbox)  # its interpreter started with the CLI: hand it the arguments
        if z is not None and fault("zygote.no_args", m.name) is not None:
            return  # fault injection: the zygote is never handed its arguments (ranchermaster recovers)
        if z is not None:
            if pid_alive(z["pid"]):  # its supervisor (a child of this process)
                atomic_write(z["args"], json.dumps(argv[4:]))
                self.events.emit("controlplane_boot_started", name=m.name, pid=z["pid"], zygote=True)
                return
            try:  # gone or going: make sure no part of it outlives the regular start below
                os.killpg(z["pid"], 15)
            except OSError:
                pass
        # The machine was just created: whatever still runs under its pidfile is a zygote an earlier,
        # failed start left waiting; stop it, or its exit would later remove this start's pidfile.
        stale = Path(m.sandbox) / "run" / "controlplane.pid"
        if stale.exists():
            kill_pidfile(stale, grace=1.0)
        pythonpath = os.pathsep.join([str(REPO)] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
        ex = MachineExecutor(self.provider, {m.name: m})
        info = ex.start_daemon(m.name, "controlplane", argv, env={"PYTHONPATH": pythonpath}, restart="unless-stopped",
                               wait_for_log=None, timeout=0)
        self.events.emit("controlplane_boot_started", name=m.name, pid=info.get("pid"))

    def provision(self) -> None:
        cfg = self.cfg
        ws = self.ws
        key = cfg.SDC_KEY
        pub = key + ".pub" if Path(key + ".pub").exists() else key
        text = hcl.render_root(self.provider.name, cfg.SDC_ACCOUNT, key, pub, cfg.SDC_KEY_ID, cfg.SDC_URL,
                               cfg.RANCHER_MASTER_HOSTNAME, cfg.master_networks(), cfg.node_names(),
                               cfg.node_networks(), cfg.HOST_PACKAGE,
                               form=os.environ.get("TK8S_TERRAFORM_FORM", "tk8s"))
        if not (ws.tf / "rancher.tf").exists() or not self.resume:
            atomic_write(ws.tf / "rancher.tf", text)
        self.out("Generating terraform configs for environment...")
        self.out(f"    Master hostname: {cfg.RANCHER_MASTER_HOSTNAME}")
        for i, n in enumerate(cfg.node_names(), 1):
            self.out(f"    Kubernetes node {i}: {n}")
        self.engine.get()
        res = self.engine.apply()
        self.out(f"    terraform tasks completed: {len(res.created)} created, {len(res.unchanged)} unchanged "
                 f"in {res.seconds:.3f}s")
        if not res.ok:
            for a, e in res.failed.items():
                self.out(f"    {a}: {e}")
            raise SetupError("Terraform had too many errors. Make sure you haven't reached your provisioning limit.")

    def _start_host_burnin(self) -> None:
        """One burn-in process for every GPU about to be handed out (burnin.HostBurnin: the runtime
        start is host-wide and serialised across processes, so N per-machine burn-ins would stack
        N starts on the critical path), started as soon as the configuration says which GPUs the
        workers will get -- before the machines exist. Machines not covered probe on their own."""
        from . import earlyburn

        early = earlyburn.take()  # started by cli/__main__.py before any import (earlyburn.py)
        if (not (self.validate and self.provider.colocated and hasattr(self.provider, "predict_gpus"))
                or os.environ.get("TK8S_HOST_BURNIN", "1") == "0"):
            if early is not None:
                early.kill()
            return
        from .earlyburn import host_burnin_command

        try:
            pkg = self.provider.package_by_id_or_name(self.cfg.HOST_PACKAGE)
            base = self._validation_command()
            if (early is not None and hasattr(self.provider, "prefer_gpus")
                    and early.command == host_burnin_command(base, early.gpus)):
                self.provider.prefer_gpus(early.gpus)
            gpus = self.provider.predict_gpus(int(pkg.gpus or 0), int(self.cfg.KUBERNETES_NUMBER_OF_NODES))
            cmd = host_burnin_command(base, gpus)
        except Exception:  # noqa: BLE001 - prediction is an optimisation only
            gpus, cmd = [], None
        import threading

        from .burnin import HostBurnin

        hb = HostBurnin(cmd, gpus, self.ws.state_dir, log=self.events.emit) if gpus else None
        if early is not None:
            if (hb is not None and early.command == cmd and sorted(early.gpus) == sorted(gpus)
                    and Path(early.result) == hb.result_path):
                hb.adopt(early.proc, early.spawned_unix)
                self.host_burnin = hb
                self.events.emit("gpu_burnin_host_started", gpus=gpus, pid=early.proc.pid, early=True)
                return
            early.kill()  # planned differently from what the run needs: start the right one,
            early.proc.wait()  # once this one can no longer write the shared result file
            self.events.emit("gpu_burnin_early_discarded", gpus=early.gpus, wanted=gpus)
        if hb is None:
            return
        self.host_burnin = hb  # machines register from now on; the process starts off this thread

        def launch():
            if hb.start():
                self.events.emit("gpu_burnin_host_started", gpus=gpus, pid=hb.proc.pid)

        threading.Thread(target=launch, name="host-burnin-start", daemon=True).start()

    def ansible_config(self) -> None:
        """createAnsibleConfigs (setup.sh:116-137)."""
        ws, cfg = self.ws, self.cfg
        masters = (ws.tf / "masters.ip").read_text().split() if (ws.tf / "masters.ip").exists() else []
        hosts_ = (ws.tf / "hosts.ip").read_text().split() if (ws.tf / "hosts.ip").exists() else []
        if not masters or not hosts_:
            raise SetupError("Terraform had too many errors. Make sure you haven't reached your provisioning limit.")
        machines = self.engine.machines()
        def host_line(name: str) -> str:
            m = machines[name]
            hv = {"ansible_host": m.primaryip}
            hv.update(getattr(self.provider, "ansible_host_vars", lambda _m: {})(m))
            return name + "".join(f" {k}={_ini_quote(v)}" for k, v in hv.items())

        lines = ["[MASTER]", host_line(cfg.RANCHER_MASTER_HOSTNAME), "[HOST]"]
        lines += [host_line(n) for n in cfg.node_names()]
        atomic_write(ws.ansible / "hosts", "\n".join(lines) + "\n")
        # the variables the in-repo engine passes, for a by-hand stock run:
        #   cd ansible && ansible-playbook -i hosts clusterUp.yml -e @tmp/tk8s_extra_vars.json
        extra = playbook_extra_vars(ws, cfg, machines, node_grace=self.node_grace, validate=self.validate,
                                    validation_command=self._validation_command())
        if self.platform == "kubeadm":
            extra.update(kubeadm_extra_vars(self, cfg))
        atomic_write_json(ws.ansible / "tmp" / "tk8s_extra_vars.json", extra)
        self.out("Creating ansible hosts file and variable files")
        self.out("    created: ansible/hosts")
        master = masters[-1]
        from .utils.yamlio import flat_mapping

        atomic_write(ws.vars_file, flat_mapping({"master": master, "kubernetes_name": cfg.KUBERNETES_NAME,
                                                 "kubernetes_description": cfg.KUBERNETES_DESCRIPTION}))
        _set_ini_value(ws.ansible / "ansible.cfg", "private_key_file", cfg.SDC_KEY)
        self.out("    created: ansible/roles/ranchermaster/vars/vars.yml")

    def _validation_command(self) -> list[str]:
        # xGMI pulls only inside multi-GPU machines (a 1-GPU machine has none; the RCCL Job checks
        # the fabric between machines)
        peers = True
        try:
            peers = int(self.provider.package_by_id_or_name(self.cfg.HOST_PACKAGE).gpus or 0) > 1
        except Exception:  # noqa: BLE001 - no configuration yet: the full check
            pass
        return default_validation_command(self.hbm_bytes, self.md5_bytes, self.probe_iters, peers=peers)

    def ansible(self) -> None:
        from .playbook import Playbook

        ws, cfg = self.ws, self.cfg
        machines = self.engine.machines()
        extra = playbook_extra_vars(ws, cfg, machines, node_grace=self.node_grace, validate=self.validate,
                                    validation_command=self._validation_command())
        if self.platform == "kubeadm":
            extra.update(kubeadm_extra_vars(self, cfg))
        lines: list[str] = []
        pb = Playbook(ws.ansible / PLAYBOOKS[self.platform], ws.ansible / "hosts",
                      executor=MachineExecutor(self.provider, machines), extra_vars=extra, events=self.events,
                      out=(lines.append if self.quiet_ansible else self.out))
        res = pb.run()
        self.playbook_result = res
        atomic_write(ws.state_dir / "ansible.log", "\n".join(lines) + "\n")
        if not res.ok:
            if self.quiet_ansible:
                for line in lines[-40:]:
                    self.out(line)
            raise SetupError("ansible-playbook failed: " + "; ".join(res.failures[:5]))

    def _client(self):
        from .controlplane.client import Client

        m = self.engine.machines()[self.cfg.RANCHER_MASTER_HOSTNAME]
        return Client(f"{m.primaryip}:{self.cfg.TK8S_MASTER_PORT}", token=self.ws.admin_token(), timeout=30.0)

    def project_id(self) -> str:
        return self.ws.env_id_file.read_text().strip()

    def expected_gpus(self) -> int:
        pkg = self.provider.package_by_id_or_name(self.cfg.HOST_PACKAGE)
        return int(self.cfg.KUBERNETES_NUMBER_OF_NODES) * int(getattr(pkg, "gpus", 0) or 0)
    def wait_ready(self) -> dict:
        """Event-driven, bounded replacement of the readiness loop (setup.sh:56-85)."""
        if self.platform == "kubeadm":
            return self._kubeadm_ready()
        c = self._client()
        pid = self.project_id()
        n = int(self.cfg.KUBERNETES_NUMBER_OF_NODES)
        g = self.expected_gpus()
        # kubectl works from here on, also when the wait below fails (its message points at it)
        kc = threading.Thread(target=self._write_kubeconfig, args=(c.base, pid), name="kubeconfig", daemon=True)
        kc.start()
        self.out("Waiting on the cluster: all nodes Ready" + (f", {g} x amd.com/gpu validated" if g else ""))
        deadline = time.monotonic() + self.timeout
        last = {}
        while True:
            left = deadline - time.monotonic()
            if left <= 0:
                kc.join(5.0)
                raise SetupError(f"cluster not ready after {self.timeout:.0f}s: {json.dumps(last)}", code=124)
            last = c.get("/v1/cluster/wait", query={"project": pid, "nodes": n, "gpus": g,
                                                    "validated": int(self.validate), "timeout": min(left, 30.0)},
                         timeout=min(left, 30.0) + 10)
            if last.get("ready"):
                return last
            if last.get("failed"):
                kc.join(5.0)
                why = "; ".join(f"{f['node']}: {f['reason']}" + (f" ({f['message']})" if f.get("message") else "")
                                for f in last.get("validation_failures") or [])
                raise SetupError(f"GPU validation failed on {last.get('nodes_validation_failed')} node(s)"
                                 + (f": {why}" if why else "")
                                 + "\n    see `./kubectl describe nodes` and `./kubectl get pods -n kube-system`", code=2)

    # -- dry run (BASELINE.json config 1: `terraform plan` + `ansible-playbook --check`) -------
    def dry_run(self) -> dict:
        """What ``./setup.sh`` would do, changing nothing: the wizard's answers, the Terraform plan
        of the rendered rancher.tf, and the playbook in check mode against the planned machines.
        Everything is rendered in a scratch copy of the workspace, which is removed afterwards;
        no machine is created, no process started, no file of this workspace written."""
        import shutil
        import tempfile

        from .playbook import Playbook

        scratch = Path(tempfile.mkdtemp(prefix="tk8s-dry-"))
        try:
            sws = init_workspace(scratch, self.ws.root if (self.ws.root / "ansible" / "roles").is_dir() else REPO)
            twin = Setup(sws, answers=self.answers, assume_yes=self.assume_yes, validate=self.validate,
                         out=self.out, backend=self.backend, master_port=self.master_port, platform=self.platform,
                         quiet_ansible=self.quiet_ansible)
            twin.provider = self.provider if not self.provider.colocated else get_provider(self.backend, sws.state_dir)
            twin.engine = Engine(sws.tf, twin.provider, twin.events)
            cfg = twin.configure()
            key = cfg.SDC_KEY
            pub = key + ".pub" if Path(key + ".pub").exists() else key
            atomic_write(sws.tf / "rancher.tf", hcl.render_root(
                twin.provider.name, cfg.SDC_ACCOUNT, key, pub, cfg.SDC_KEY_ID, cfg.SDC_URL, cfg.RANCHER_MASTER_HOSTNAME,
                cfg.master_networks(), cfg.node_names(), cfg.node_networks(), cfg.HOST_PACKAGE,
                form=os.environ.get("TK8S_TERRAFORM_FORM", "tk8s")))
            twin.engine.get()
            plan = twin.engine.plan()
            self.banner("terraform plan")
            self.out(Engine.plan_summary(plan))
            lines = ["[MASTER]", f"{cfg.RANCHER_MASTER_HOSTNAME} ansible_host=planned-{cfg.RANCHER_MASTER_HOSTNAME}", "[HOST]"]
            lines += [f"{n} ansible_host=planned-{n}" for n in cfg.node_names()]
            atomic_write(sws.ansible / "hosts", "\n".join(lines) + "\n")
            atomic_write(sws.vars_file, f"master: planned-{cfg.RANCHER_MASTER_HOSTNAME}\n"
                                        f"kubernetes_name: {json.dumps(cfg.KUBERNETES_NAME)}\n"
                                        f"kubernetes_description: {json.dumps(cfg.KUBERNETES_DESCRIPTION)}\n")
            self.banner(f"ansible-playbook --check {PLAYBOOKS[twin.platform]}")
            extra = {"tk8s_master_port": int(cfg.TK8S_MASTER_PORT), "tk8s_validate": self.validate,
                     "tk8s_manifests": str(sws.manifests), "tk8s_python": sys.executable,
                     "tk8s_pythonpath": str(REPO), "tk8s_fake_gpus": os.environ.get("TK8S_FAKE_GPUS", ""),
                     "tk8s_validation_command": [], "tk8s_validation_pod_command": [],
                     "tk8s_controlplane_argv": [], "tk8s_machine_dir": "(known after apply)", "tk8s_gpus": "",
                     "tk8s_home": str(REPO)}
            if twin.platform == "kubeadm":
                extra.update(kubeadm_extra_vars(twin, cfg))
            pb = Playbook(sws.ansible / PLAYBOOKS[twin.platform], sws.ansible / "hosts", check=True,
                          extra_vars=extra, out=self.out)
            res = pb.run()
            return {"dry_run": True, "platform": twin.platform, "backend": self.backend,
                    "plan": [{"address": a.address, "action": a.action} for a in plan],
                    # the playbook's plan, task by task ("host: task"), what a --check golden pins
                    "check_plan": [f"{t['host']}: {t['task']}" for t in pb.trace if t.get("module") != "setup"],
                    "check_ok": res.ok, "check_failures": res.failures, "check_stats": res.stats}
        finally:
            shutil.rmtree(scratch, ignore_errors=True)

    # -- main ------------------------------------------------------------------------------
    def run(self) -> dict:
        ws = self.ws
        t0 = time.monotonic()
        if (ws.tf / "rancher.tf").exists() and not self.resume:
            raise SetupError("error: configuration for a previous run has been found\n"
                             "    clean the configuration (./setup.sh -c) or continue it (./setup.sh --resume)")
        self.events.emit("setup_start", backend=self.backend, resume=self.resume)
        if not self.resume:
            ws.save_state(completed=[], timings={}, started=time.time())
        steps = [("configure", self.configure, None), ("provision", self.provision, "Starting terraform tasks..."),
                 ("ansible-config", self.ansible_config, "Creating ansible configs..."),
                 ("ansible", self.ansible, "Running ansible tasks...")]
        for name, fn, title in steps:
            if name == "configure" or not self.done(name):
                if title:
                    self.banner(title)
                with self.events.phase(name):
                    fn()
                self.mark(name)
            if name == "configure" and not self.done("provision"):
                self._start_host_burnin()  # the GPUs are known now: validate them while machines are made
        with self.events.phase("ready"):
            ready = self.wait_ready()
        self.mark("ready")
        t_ready = time.monotonic() - t0
        # One greppable line the moment every node is Ready (bench.py timestamps it): the RCCL
        # fabric check that follows is reported on its own, it is not part of "all nodes Ready".
        self.out(self.ready_line(ready, t_ready))
        rccl = None
        with self.events.phase("rccl"):
            rccl = self.run_rccl()
        self.mark("rccl")
        total = time.monotonic() - t0
        if self.platform == "kubeadm":
            return self._kubeadm_finish(ready, rccl, t_ready, total)
        m = self.engine.machines()[self.cfg.RANCHER_MASTER_HOSTNAME]
        base = f"http://{m.primaryip}:{self.cfg.TK8S_MASTER_PORT}"
        pid = self.project_id()
        self._write_kubeconfig(base, pid)
        validation = {}
        try:  # per-node GPU validation results (annotations set from the validation pods)
            for n in self._client().get(f"/r/projects/{pid}/kubernetes/api/v1/nodes")["items"]:
                ann = {k.split("/", 1)[1]: v for k, v in n["metadata"].get("annotations", {}).items()
                       if k.startswith("tk8s.amd.com/")}
                if ann:
                    validation[n["metadata"]["name"]] = ann
        except Exception:  # noqa: BLE001 - reporting only
            pass
        self.summary = {
            "platform": "tk8s", "ready_seconds": round(t_ready, 4), "total_seconds": round(total, 4),
            "rccl_check_s": round(self.events.phases.get("rccl", 0.0), 4), "validation": validation,
            "nodes": int(self.cfg.KUBERNETES_NUMBER_OF_NODES), "gpus_allocatable": ready.get("gpus_allocatable", 0),
            "nodes_validated": ready.get("nodes_validated", 0), "rccl": rccl,
            "phases": {k: round(v, 4) for k, v in self.events.phases.items()},
            "dashboard": f"{base}/r/projects/{pid}/kubernetes-dashboard:9090/",
            "kubectl_config": f"{base}/env/{pid}/kubernetes/kubectl", "project": pid, "api": base,
        }
        hb = self.host_burnin
        if hb is not None and hb.done:
            t = (hb.result or {}).get("timings_ms") or {}
            self.summary["host_burnin"] = {"gpus": hb.gpus, "ok": bool(hb.result and hb.result.get("ok")),
                                           "pid": getattr(getattr(hb, "proc", None), "pid", None),
                                           "runtime_init_ms": t.get("runtime_init", t.get("hip_init")),
                                           "peers_ms": t.get("peers"), "total_ms": t.get("total"),
                                           "spawned_unix": hb.spawned_unix or None,
                                           "main_unix_ms": t.get("main_unix_ms"),
                                           "seen_unix": getattr(hb, "seen_unix", 0.0) or None,
                                           # which payload ran (the HSA one on 1 GPU, the HIP one for
                                           # xGMI pulls) and each GPU's own time: where an N-GPU
                                           # bring-up's burn-in went (the driver's SCALE runs)
                                           "runtime": (hb.result or {}).get("runtime"),
                                           "device_wall_ms": [round(d.get("wall_ms") or 0.0, 2)
                                                              for d in (hb.result or {}).get("devices", [])]}
            if hb.xgmi is not None:
                self.summary["xgmi"] = {k: hb.xgmi[k] for k in ("pulls", "median_gbps", "min_gbps", "floor_gbps",
                                                                 "min_fraction")}
                self.summary["xgmi"]["degraded"] = [f"{e['src']}->{e['dst']}" for e in hb.xgmi["degraded"]]
        ws.save_state(summary=self.summary, finished=time.time())
        self.events.emit("setup_done", **{k: v for k, v in self.summary.items() if k != "phases"})
        self.out("")
        self.out("Congratulations, your Kubernetes cluster setup has been complete.")
        self.out(f"----> To check what processes/containers are running, go to {base}/env/{pid}/infra/containers")
        self.out(f"----> Kubernetes dashboard is at {self.summary['dashboard']}")
        self.out(f"----> Kubernetes CLI config is at {self.summary['kubectl_config']}")
        self.out(f"----> {self.summary['nodes']} node(s) Ready, {self.summary['gpus_allocatable']} x amd.com/gpu allocatable"
                 + (f", {fabric_line(rccl)}" if rccl else ""))
        self.out(f"----> bring-up: {t_ready:.3f}s to all nodes Ready ({total:.3f}s including fabric validation)")
        self.out("")
        self.out("    CONGRATULATIONS, YOU HAVE CONFIGURED YOUR KUBERNETES ENVIRONMENT!")
        return self.summary

    def scale(self, n: int) -> dict:
        """Change the number of workers of a running cluster (the reference fixes it at creation,
        setup.sh:297-307, and could only be torn down and rebuilt). Shrinking drains the removed
        workers (cordon, evict every non-DaemonSet pod so its controller re-creates it elsewhere)
        and deletes their nodes before their machines go; then the same phases as a bring-up run
        against the new configuration: Terraform apply (creates the new machines / destroys the
        removed ones; new machines boot their agent and GPU burn-in), the playbook (idempotent on
        the existing hosts, joins the new ones), and the bounded readiness wait for exactly n
        validated workers."""
        ws = self.ws
        if not ws.config.exists() or "ready" not in ws.state().get("completed", []):
            raise SetupError("error: no running cluster in this directory (./setup.sh first)")
        if not 1 <= int(n) <= 9:
            raise SetupError("error: the number of nodes must be 1-9 (the wizard's limit)")
        cfg = read_config(ws.config)
        export_vars(cfg)
        self.cfg = cfg
        self.platform = cfg.TK8S_PLATFORM or "tk8s"
        if self.platform == "kubeadm" and hasattr(self.provider, "whole_hosts"):
            self.provider.whole_hosts = not self.kubeadm_single_node
        old = int(cfg.KUBERNETES_NUMBER_OF_NODES)
        if int(n) == old:
            self.out(f"{old} node(s) already; nothing to do")
            return {"nodes": old, "changed": False}
        t0 = time.monotonic()
        self.events.emit("scale_start", nodes=int(n), previous=old)
        removed = cfg.node_names()[int(n):]
        if removed:
            self.banner(f"Draining {', '.join(removed)}...")
            with self.events.phase("drain"):
                self._drain_and_delete(removed)
        cfg.KUBERNETES_NUMBER_OF_NODES = int(n)
        write_config(ws.config, cfg)
        export_vars(cfg)
        for name, fn, title in (("provision", self.provision, "Starting terraform tasks..."),
                                ("ansible-config", self.ansible_config, "Creating ansible configs..."),
                                ("ansible", self.ansible, "Running ansible tasks...")):
            self.banner(title)
            with self.events.phase(name):
                fn()
        with self.events.phase("ready"):
            ready = self.wait_ready()
        self.out(self.ready_line(ready, time.monotonic() - t0))
        rccl = None
        if self.rccl:
            with self.events.phase("rccl"):
                rccl = self.run_rccl()
        summary = dict(ws.state().get("summary") or {})
        summary.update(nodes=int(n), gpus_allocatable=ready.get("gpus_allocatable", 0),
                       nodes_validated=ready.get("nodes_validated", 0))
        if rccl is not None:
            summary["rccl"] = rccl
        ws.save_state(summary=summary)
        out = {"nodes": int(n), "previous": old, "changed": True, "removed": removed,
               "seconds": round(time.monotonic() - t0, 4), "gpus_allocatable": ready.get("gpus_allocatable", 0),
               "nodes_validated": ready.get("nodes_validated", 0), "rccl": rccl}
        self.events.emit("scale_done", **out)
        return out

    def _drain_and_delete(self, names: list[str]) -> None:
        from .controlplane.client import ApiError, client_from_kubeconfig

        if self.kubeadm_single_node:  # GPU slots of the master's node: no Kubernetes node to drain
            for node in names:
                self.out(f"    slot {node} released (single-node: its GPUs stay on {self.cfg.RANCHER_MASTER_HOSTNAME})")
            return
        if self.platform == "kubeadm":  # a real Kubernetes: kubectl drain on the master, kubeadm reset on the node
            machines = self.engine.machines()
            for node in names:
                rc, text = self._master_exec(
                    f"kubectl --kubeconfig ${{TK8S_SYSROOT:-}}/etc/kubernetes/admin.conf drain {node} --ignore-daemonsets "
                    f"--delete-emptydir-data --force --timeout=120s && kubectl --kubeconfig "
                    f"${{TK8S_SYSROOT:-}}/etc/kubernetes/admin.conf delete node {node}", timeout=300)
                self.out(f"    node/{node} {'drained and deleted' if rc == 0 else 'drain failed: ' + text.strip()[-200:]}")
                if node in machines:
                    self.provider.exec(machines[node], KUBEADM_RESET, timeout=300)
            return

        c = self._client()
        pid = self.project_id()
        k = client_from_kubeconfig(c.get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"}))
        for node in names:
            try:
                k.request("PATCH", k.k8s(f"/api/v1/nodes/{node}"), body={"spec": {"unschedulable": True}})
            except ApiError as e:
                if e.status != 404:
                    raise
                continue
            for p in k.get(k.k8s("/api/v1/pods"), query={"fieldSelector": f"spec.nodeName={node}"})["items"]:
                md = p["metadata"]
                k.delete(k.k8s(f"/api/v1/namespaces/{md['namespace']}/pods/{md['name']}"))
                self.out(f"    evicted pod {md['namespace']}/{md['name']}")
            k.delete(k.k8s(f"/api/v1/nodes/{node}"))
            self.out(f"    node/{node} drained and deleted")

    def _write_kubeconfig(self, base: str, pid: str) -> None:
        from .controlplane.client import Client

        kc = Client(base, token=self.ws.admin_token()).get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"})
        atomic_write_json(self.ws.state_dir / "kubeconfig.json", kc)


def _free_port() -> int:
    from .utils.net import pick_port

    return pick_port("0.0.0.0")


def _flush_print(s: str) -> None:
    print(s, flush=True)


class _Sink:
    """File-like adapter so the wizard's prompt echo goes to an out() callback line by line."""

    def __init__(self, out):
        self.out = out
        self.buf = ""

    def write(self, s: str) -> None:
        self.buf += s
        while "\n" in self.buf:
            line, self.buf = self.buf.split("\n", 1)
            self.out(line)

    def flush(self) -> None:
        pass


def _ini_quote(v) -> str:
    v = str(v)
    return v if v and not any(c in v for c in " \t'\"#=") else "'" + v.replace("'", "'\"'\"'") + "'"


def _set_ini_value(path: Path, key: str, value: str) -> None:
    """Replace `key = ...` in an ini file without sed (the reference's sed uses `;` as the
    delimiter on a user path, setup.sh:133)."""
    lines = path.read_text().splitlines() if path.exists() else ["[defaults]"]
    out, done = [], False
    for line in lines:
        if line.split("=", 1)[0].strip() == key:
            out.append(f"{key} = {value}")
            done = True
        else:
            out.append(line)
    if not done:
        out.append(f"{key} = {value}")
    atomic_write(path, "\n".join(out) + "\n")


from .teardown import clean  # noqa: E402,F401 - ./setup.sh -c (re-exported)
