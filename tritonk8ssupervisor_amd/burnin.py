"""Early GPU burn-in launcher (shared by the provisioning boot hook and the rocmsetup role).

Import-light on purpose: the boot hook runs inside provisioning, on the bring-up's critical
path, and must not pull in the playbook engine's HTTP/YAML stack before the burn-in starts.
"""
from __future__ import annotations

import os
from pathlib import Path


def start_burnin(ex, host: str, command: list, out: str = "run/gpu-burnin.json", name: str = "gpu-burnin",
                 env: dict | None = None) -> dict:
    """Start `command --out <out>` on a machine's GPUs as a one-shot daemon; idempotent (a burn-in
    that is running or has finished is left alone)."""
    gpus = ex.machine_gpus(host)
    if not gpus:
        return {"changed": False, "skipped": True, "msg": "machine has no GPUs"}
    from .models.hostinfo import compose_visible_devices

    mdir = Path(ex.machine_dir(host))
    pending = mdir / (out + ".pending")
    if (mdir / out).exists() or ex.daemon_status(host, name).get("running"):
        return {"changed": False, "msg": "GPU burn-in already started", "gpus": gpus, "out": out}
    pending.parent.mkdir(parents=True, exist_ok=True)
    pending.touch()
    denv = dict(compose_visible_devices(gpus))
    denv["NODE_NAME"] = host
    denv.update({str(k): str(v) for k, v in (env or {}).items()})
    argv = [str(a) for a in command] + ["--out", out]
    if os.sep in argv[0] and not os.access(argv[0], os.X_OK):
        pending.unlink(missing_ok=True)  # not built yet: the validation pod will probe itself
        return {"changed": False, "skipped": True, "msg": f"{argv[0]} is not built yet"}
    info = ex.start_daemon(host, name, argv, env=denv, restart="no", wait_for_log=None, timeout=0)
    if not info.get("ok"):
        pending.unlink(missing_ok=True)
        return {"failed": True, "msg": info.get("msg", "burn-in failed to start")}
    if not (mdir / out).exists():
        # the pid lets `--reuse` stop waiting if the burn-in dies without a result
        pending.write_text(f"{info.get('pid', 0)}\n")
    return {"changed": True, "pid": info.get("pid"), "gpus": gpus, "out": out}
