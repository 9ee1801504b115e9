#!/usr/bin/env python3
"""A stand-in for ``ssh`` for CPU tests of the remote (ssh) execution path.

    TK8S_SSH="python3 tests/fakessh.py"  FAKESSH_ROOT=<dir>

``<FAKESSH_ROOT>/<host>/`` is the remote host: its login home and cwd. A command runs there under
``bash -c`` with a CLEAN login environment (PATH, HOME, USER, LANG, SSH_CONNECTION, plus the
host's own ``.env`` file, the analogue of /etc/environment) -- nothing of the caller's
environment leaks through, just as over real ssh. stdin/stdout/stderr and the exit status pass
through. What real ssh would refuse is refused with exit 255:

* an unknown host (no directory): "No route to host";
* ``StrictHostKeyChecking=no`` (tk8s must never disable host-key checking);
* a host with ``.ssh/authorized_keys`` and no ``-i`` key whose public half is listed there.

``UserKnownHostsFile`` gets the host's (fake) key on first contact (accept-new). Every call is
appended to ``<FAKESSH_ROOT>/calls.jsonl`` (host, user, options, whether a key was passed).
"""
import json
import os
import re
import subprocess
import sys
import zlib
from pathlib import Path

OPTS_WITH_ARG = set("bcDEeFIiJLlmOopQRSWw")


def main(argv: list[str]) -> int:
    opts: dict[str, str] = {}
    ident = None
    port = "22"
    user = None
    i = 0
    while i < len(argv) and argv[i].startswith("-"):
        a = argv[i]
        flag = a[1:2]
        if flag in OPTS_WITH_ARG:
            val = a[2:] if len(a) > 2 else argv[i + 1]
            i += 1 if len(a) > 2 else 2
            if flag == "o":
                k, _, v = val.partition("=")
                opts[k] = v
            elif flag == "i":
                ident = val
            elif flag == "p":
                port = val
            elif flag == "l":
                user = val
            continue
        i += 1
    if i >= len(argv):
        print("usage: ssh destination [command]", file=sys.stderr)
        return 255
    dest = argv[i]
    command = " ".join(argv[i + 1:])
    if "@" in dest:
        user, host = dest.split("@", 1)
    else:
        host = dest
    root = Path(os.environ["FAKESSH_ROOT"])
    hd = root / host
    with open(root / "calls.jsonl", "a") as f:
        f.write(json.dumps({"host": host, "user": user, "port": port, "key": ident, "opts": opts,
                            "command": command[:200], "ppid": os.getppid()}) + "\n")
    if not hd.is_dir():
        print(f"ssh: connect to host {host} port {port}: No route to host", file=sys.stderr)
        return 255
    if opts.get("StrictHostKeyChecking", "").lower() == "no":
        print("fakessh: StrictHostKeyChecking=no refused", file=sys.stderr)
        return 255
    auth = hd / ".ssh" / "authorized_keys"
    if auth.exists():
        allowed = {ln.split()[1] for ln in auth.read_text().splitlines() if len(ln.split()) >= 2}
        pub = Path(str(ident) + ".pub") if ident else None
        blob = pub.read_text().split()[1] if pub and pub.exists() else None
        if blob not in allowed:
            print(f"{user}@{host}: Permission denied (publickey).", file=sys.stderr)
            return 255
    kh = opts.get("UserKnownHostsFile")
    if kh:
        line = f"{host} ssh-ed25519 FAKEHOSTKEY{zlib.crc32(host.encode())}\n"
        p = Path(os.path.expanduser(kh))
        if not p.exists() or line not in p.read_text():
            p.parent.mkdir(parents=True, exist_ok=True)
            with open(p, "a") as f:
                f.write(line)
    env = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"), "HOME": str(hd), "USER": user or "root",
           "LOGNAME": user or "root", "LANG": "C.UTF-8", "SHELL": "/bin/bash",
           "SSH_CONNECTION": f"127.0.0.1 0 {host} {port}", "FAKESSH_HOST": host}
    envf = hd / ".env"
    if envf.exists():
        for ln in envf.read_text().splitlines():
            if "=" in ln and not ln.startswith("#"):
                k, v = ln.split("=", 1)
                env[k.strip()] = v.strip()
    if not command:
        print("fakessh: interactive sessions are not supported", file=sys.stderr)
        return 255
    # A "fake root" host (a .fakeroot file; tests/fakeroot/) runs with a PATH of ONLY its own bin/
    # -- stand-ins for apt-get, kubeadm, systemctl ... and safe coreutils -- and $TK8S_SYSROOT
    # pointing into the host directory: the kubeadm roles run for real against simulated tools.
    fakeroot = (hd / ".fakeroot").exists()
    if fakeroot:
        env["PATH"] = str(hd / "bin")
        env["TK8S_SYSROOT"] = str(hd / "sysroot")
        # paths under the staging root (literal, or through $TK8S_SYSROOT) are the fake host's own
        sysroot_free = re.sub(r"\$\{?TK8S_SYSROOT(:-)?\}?/[^\s'\"]*", "",
                              re.sub(re.escape(str(hd / "sysroot")) + r"/[^\s'\"]*", "", command))
    else:
        sysroot_free = command
    # The "hosts" are directories of THIS machine: anything that would change the machine itself
    # (package managers, kernel modules, services, kubeadm) is refused, never run -- on a fake
    # root only system PATHS are checked (the tools there are the stand-ins).
    for word in ("apt-get", "dpkg ", "modprobe", "systemctl", "kubeadm", "swapoff", "sysctl ", "apt-mark",
                 "/etc/apt", "/etc/kubernetes", "/etc/containerd", "/etc/modules-load.d", "/etc/sysctl.d",
                 "/etc/fstab", "/opt/tk8s", "/root/.kube"):
        if fakeroot and not word.startswith("/"):
            continue
        if word in sysroot_free:
            print(f"fakessh: refusing a system-changing command on a fake host ({word.strip()})", file=sys.stderr)
            return 126
    r = subprocess.run(["bash", "-c", command], cwd=hd, env=env)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
