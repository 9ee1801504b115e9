"""Modules for the playbook engine.

Ansible built-ins used by the reference roles: command, shell, uri, slurp, pause, debug
(ansible/roles/*/tasks/main.yml) plus set_fact, wait_for, fail, assert, copy, file, stat,
include_vars, meta, ping. tk8s modules replace the Docker ones:

  tk8s_daemon    — start/stop/query a supervised long-running process on a machine
                   (replaces docker_container rancher/server and docker rancher/agent)
  tk8s_gpu_facts — ROCm/KFD facts of a machine (replaces the docker --version probe)
  tk8s_build     — ensure the native validation stack is built (replaces apt docker-engine)
  tk8s_kube      — create/delete/wait Kubernetes objects on the control plane
"""
from __future__ import annotations

import json
import os
import re
import shlex
import subprocess
import time
from pathlib import Path


from . import templating


def _bool(v: Any, default: bool = False) -> bool:
    if v is None:
        return default
    if isinstance(v, bool):
        return v
    return str(v).lower() in ("1", "yes", "true", "on")


def run_module(mod: str, args: dict, *, ctx, host, target, local: bool, env: dict, check: bool,
               variables: dict) -> dict:
    fn = MODULES.get(module_name(mod))
    if fn is None:
        return {"failed": True, "msg": f"module {mod!r} is not supported by the tk8s playbook engine"}
    try:
        return fn(args, ctx=ctx, host=host, target=target, local=local, env=env, check=check, variables=variables)
    except templating.Undefined:
        raise
    except Exception as e:  # noqa: BLE001 - module failure becomes a task failure
        return {"failed": True, "msg": f"{mod}: {type(e).__name__}: {e}"}


# ---- command / shell ---------------------------------------------------------------------
def _run_cmd(cmd: str | list[str], *, ctx, target, local, env, shell: bool, timeout: float = 600,
             chdir: str | None = None) -> dict:
    t = time.monotonic()
    if local or ctx.executor is None:
        argv = ["bash", "-c", cmd] if shell else (cmd if isinstance(cmd, list) else shlex.split(cmd))
        cwd = ctx.dir / chdir if chdir else ctx.dir
        r = subprocess.run(argv, cwd=cwd, env={**os.environ, **env}, capture_output=True, text=True, timeout=timeout)
        rc, out, err = r.returncode, r.stdout, r.stderr
    else:
        line = cmd if shell else " ".join(shlex.quote(a) for a in (cmd if isinstance(cmd, list) else shlex.split(cmd)))
        if chdir:
            line = f"cd {shlex.quote(chdir)} && {line}"
        rc, out = ctx.executor.exec(target.name, line, env=env, timeout=timeout)
        err = ""
    out = out or ""
    return {"rc": rc, "stdout": out.rstrip("\n"), "stderr": err.rstrip("\n"), "stdout_lines": out.splitlines(),
            "changed": True, "failed": rc != 0, "delta": round(time.monotonic() - t, 6),
            "msg": "" if rc == 0 else f"non-zero return code {rc}: {(err or out).strip()[-300:]}"}


_CMD_KEYS = ("creates", "removes", "chdir")


def _cmd_args(args: dict) -> tuple[str | list, dict]:
    """The command and its ``creates``/``removes``/``chdir`` options, from args or free form."""
    opts = {k: args[k] for k in _CMD_KEYS if k in args}
    cmd = args.get("_raw_params") or args.get("cmd") or args.get("argv")
    if isinstance(cmd, str):
        words = shlex.split(cmd)
        keep = []
        for w in words:
            k, eq, v = w.partition("=")
            if eq and k in _CMD_KEYS:
                opts[k] = v
            else:
                keep.append(w)
        if len(keep) != len(words):
            cmd = " ".join(shlex.quote(w) for w in keep)
    return cmd, opts


def _command(args, *, ctx, target, local, env, check, shell: bool) -> dict:
    cmd, opts = _cmd_args(args)
    fs = _fs(ctx, target, local)
    if opts.get("creates") and fs.stat(opts["creates"])["exists"]:
        return {"changed": False, "cmd": cmd, "rc": 0, "stdout": f"skipped, since {opts['creates']} exists",
                "stdout_lines": []}
    if opts.get("removes") and not fs.stat(opts["removes"])["exists"]:
        return {"changed": False, "cmd": cmd, "rc": 0, "stdout": f"skipped, since {opts['removes']} does not exist",
                "stdout_lines": []}
    if check:
        return {"skipped": True, "changed": False, "cmd": cmd, "msg": f"{'shell' if shell else 'command'} "
                                                                      "skipped in check mode"}
    res = _run_cmd(cmd, ctx=ctx, target=target, local=local, env=env, shell=shell, chdir=opts.get("chdir"))
    res["cmd"] = cmd
    return res


def m_command(args, *, ctx, target, local, env, check, **_):
    return _command(args, ctx=ctx, target=target, local=local, env=env, check=check, shell=False)


def m_shell(args, *, ctx, target, local, env, check, **_):
    return _command(args, ctx=ctx, target=target, local=local, env=env, check=check, shell=True)


# ---- node runtime installation (ansible.builtin apt / apt_repository / get_url / systemd_service /
# replace / lineinfile / fetch / setup): what the kubeadm platform's roles use --------------------
def _sh(ctx, target, local, script: str, env: dict | None = None, timeout: float = 1800) -> tuple[int, str]:
    if local or ctx.executor is None:
        r = subprocess.run(["bash", "-c", script], cwd=ctx.dir, env={**os.environ, **(env or {})},
                           capture_output=True, text=True, timeout=timeout)
        return r.returncode, (r.stdout or "") + (r.stderr or "")
    return ctx.executor.exec(target.name, script, env=env, timeout=timeout)


def _as_list(v) -> list[str]:
    if v is None:
        return []
    if isinstance(v, str):
        return [x.strip() for x in v.split(",") if x.strip()]
    return [str(x) for x in v]


def apt_script(args: dict) -> str:
    """The shell the apt module runs (also what --check reports): idempotent via dpkg-query."""
    names = _as_list(args.get("name") or args.get("pkg"))
    state = str(args.get("state", "present"))
    parts = ["export DEBIAN_FRONTEND=noninteractive"]
    if _bool(args.get("update_cache")):
        valid = int(args.get("cache_valid_time", 0) or 0)
        if valid:
            parts.append(f"if [ -z \"$(find /var/lib/apt/lists -maxdepth 1 -newermt '-{valid} seconds' -name '*Packages' "
                         "2>/dev/null | head -n1)\" ]; then apt-get update -q; fi")
        else:
            parts.append("apt-get update -q")
    if _bool(args.get("upgrade")) or args.get("upgrade") == "dist":
        parts.append("apt-get dist-upgrade -y -q")
    if names:
        q = " ".join(shlex.quote(n) for n in names)
        if state == "absent":
            parts.append(f"pkgs=$(for p in {q}; do dpkg-query -W -f='${{Status}}' \"$p\" 2>/dev/null | grep -q 'ok installed' "
                         f"&& echo \"$p\"; done); [ -z \"$pkgs\" ] || {{ apt-get remove -y -q $pkgs && echo TK8S_CHANGED; }}")
        else:
            flag = " --only-upgrade" if state == "latest" else ""
            miss = (f"pkgs=$(for p in {q}; do dpkg-query -W -f='${{Status}}' \"$p\" 2>/dev/null | grep -q 'ok installed' "
                    f"|| echo \"$p\"; done)")
            parts.append(miss)
            if state == "latest":
                parts.append(f"apt-get install -y -q --no-install-recommends{flag} {q} | grep -q 'newly installed' "
                             "&& echo TK8S_CHANGED || true")
            parts.append("[ -z \"$pkgs\" ] || { apt-get install -y -q --no-install-recommends $pkgs && echo TK8S_CHANGED; }")
    return "\n".join(parts)


def m_apt(args, *, ctx, target, local, env, check, **_):
    script = apt_script(args)
    if check:
        return {"changed": True, "cmd": script, "msg": "check mode: apt not run"}
    rc, out = _sh(ctx, target, local, script, env)
    return {"changed": "TK8S_CHANGED" in out, "failed": rc != 0, "rc": rc, "stdout": out[-2000:],
            "msg": "" if rc == 0 else f"apt failed rc={rc}: {out.strip()[-500:]}"}


def m_apt_repository(args, *, ctx, target, local, env, check, **_):
    repo = str(args["repo"])
    name = str(args.get("filename") or re.sub(r"[^A-Za-z0-9]+", "_", repo.split("//", 1)[-1]).strip("_")[:60])
    # TK8S_SYSROOT (the plays' environment): the staging root the fake hosts of the tests use
    dest = f"{(env or {}).get('TK8S_SYSROOT', '')}/etc/apt/sources.list.d/{name}.list"
    fs = _fs(ctx, target, local)
    if str(args.get("state", "present")) == "absent":
        changed = fs.stat(dest)["exists"]
        if changed and not check:
            fs.remove(dest)
        return {"changed": changed, "dest": dest}
    changed = fs.write(dest, (repo + "\n").encode(), mode=0o644, check=check)
    if changed and not check and _bool(args.get("update_cache", True)):
        rc, out = _sh(ctx, target, local, "DEBIAN_FRONTEND=noninteractive apt-get update -q")
        if rc != 0:
            return {"failed": True, "msg": f"apt-get update failed: {out.strip()[-500:]}"}
    return {"changed": changed, "dest": dest, "repo": repo}


def m_get_url(args, *, ctx, target, local, check, **_):
    url, dest = str(args["url"]), str(args["dest"])
    fs = _fs(ctx, target, local)
    if fs.stat(dest)["exists"] and not _bool(args.get("force")):
        return {"changed": False, "dest": dest, "url": url}
    cmd = f"curl -fsSL --retry 3 -o {shlex.quote(dest)} {shlex.quote(url)}"
    if "mode" in args:
        cmd += f" && chmod {str(args['mode'])} {shlex.quote(dest)}"
    if check:
        return {"changed": True, "cmd": cmd, "dest": dest}
    rc, out = _sh(ctx, target, local, cmd, timeout=float(args.get("timeout", 120)) + 60)
    return {"changed": rc == 0, "failed": rc != 0, "dest": dest, "url": url,
            "msg": "" if rc == 0 else f"download of {url} failed: {out.strip()[-300:]}"}


def m_systemd_service(args, *, ctx, target, local, check, **_):
    name = args.get("name")
    cmds = []
    if _bool(args.get("daemon_reload")):
        cmds.append("systemctl daemon-reload")
    if name is not None and "enabled" in args:
        cmds.append(f"systemctl {'enable' if _bool(args['enabled']) else 'disable'} {shlex.quote(str(name))}")
    verb = {"started": "start", "stopped": "stop", "restarted": "restart", "reloaded": "reload"}.get(
        str(args.get("state", "")))
    if name is not None and verb:
        cmds.append(f"systemctl {verb} {shlex.quote(str(name))}")
    script = " && ".join(cmds) or "true"
    if check:
        return {"changed": bool(cmds), "cmd": script}
    rc, out = _sh(ctx, target, local, script)
    return {"changed": bool(cmds), "failed": rc != 0, "name": name,
            "msg": "" if rc == 0 else f"systemctl failed: {out.strip()[-300:]}"}


def m_replace(args, *, ctx, target, local, check, **_):
    fs = _fs(ctx, target, local)
    path = args.get("path") or args.get("dest")
    data = fs.read(path)
    if data is None:
        if check:
            return {"skipped": True, "changed": False, "msg": f"check mode: {path} does not exist yet"}
        return {"failed": True, "msg": f"Path {path} does not exist !"}
    text = data.decode()
    new, n = re.subn(str(args["regexp"]), str(args.get("replace", "")), text, flags=re.MULTILINE)
    changed = new != text
    if changed:
        fs.write(path, new.encode(), check=check)
    return {"changed": changed, "msg": f"{n} replacements made" if changed else ""}


def m_lineinfile(args, *, ctx, target, local, check, **_):
    fs = _fs(ctx, target, local)
    path = args.get("path") or args.get("dest")
    data = fs.read(path)
    if data is None and not _bool(args.get("create")):
        return {"failed": True, "msg": f"Destination {path} does not exist !"}
    lines = (data or b"").decode().splitlines()
    line, rx = args.get("line"), args.get("regexp")
    state = str(args.get("state", "present"))
    out = list(lines)
    if state == "absent":
        out = [ln for ln in lines if not ((rx and re.search(rx, ln)) or (line is not None and ln == line))]
    else:
        idx = [i for i, ln in enumerate(lines) if rx and re.search(rx, ln)]
        if idx:
            out[idx[-1]] = str(line)
        elif str(line) not in lines:
            out.append(str(line))
    changed = out != lines
    if changed:
        fs.write(path, ("\n".join(out) + "\n").encode(), check=check)
    return {"changed": changed}


def m_fetch(args, *, ctx, target, local, check, **_):
    """Copy a file FROM the machine to the controller (``flat: yes``: exactly ``dest``)."""
    src, dest = str(args["src"]), str(args["dest"])
    data = _fs(ctx, target, local).read(src)
    if data is None:
        if check or _bool(args.get("fail_on_missing", True)) is False:
            return {"skipped": True, "changed": False, "msg": f"{src} not found"}
        return {"failed": True, "msg": f"the remote file does not exist: {src}"}
    from .executor import LocalFS

    d = dest if _bool(args.get("flat")) else os.path.join(dest, target.name, src.lstrip("/"))
    changed = LocalFS(ctx.dir).write(d, data, check=check)
    return {"changed": changed, "dest": str(LocalFS(ctx.dir).path(d))}


FACTS_SCRIPT = r"""
. /etc/os-release 2>/dev/null
echo "distribution=${NAME%% *}"
echo "release=${VERSION_CODENAME:-$UBUNTU_CODENAME}"
echo "version=$VERSION_ID"
echo "kernel=$(uname -r)"
echo "arch=$(uname -m)"
echo "hostname=$(hostname -s 2>/dev/null || uname -n)"
echo "ipv4=$(ip -4 route get 1.1.1.1 2>/dev/null | sed -n 's/.* src \([0-9.]*\).*//p' | head -n1)"
echo "processor_vcpus=$(nproc 2>/dev/null)"
echo "memtotal_mb=$(awk '/MemTotal/ {print int($2/1024)}' /proc/meminfo 2>/dev/null)"
echo "env_HOME=$HOME"
echo "env_USER=${USER:-$(id -un 2>/dev/null)}"
echo "env_PATH=$PATH"
"""


def m_setup(args, *, ctx, target, local, **_):
    """Fact gathering (the subset the roles read), run ON the machine."""
    rc, out = _sh(ctx, target, local, FACTS_SCRIPT, timeout=60)
    kv = dict(line.split("=", 1) for line in out.splitlines() if "=" in line)
    facts = {"ansible_distribution": kv.get("distribution", ""), "ansible_distribution_release": kv.get("release", ""),
             "ansible_distribution_version": kv.get("version", ""), "ansible_kernel": kv.get("kernel", ""),
             "ansible_architecture": kv.get("arch", ""), "ansible_hostname": kv.get("hostname", ""),
             "ansible_processor_vcpus": int(kv.get("processor_vcpus") or 0),
             "ansible_memtotal_mb": int(kv.get("memtotal_mb") or 0)}
    ip = kv.get("ipv4") or target.address
    facts["ansible_default_ipv4"] = {"address": ip}
    facts["ansible_env"] = {k[4:]: v for k, v in kv.items() if k.startswith("env_")}
    return {"ansible_facts": facts, "changed": False, "failed": rc != 0 and not out.strip()}


# ---- uri ----------------------------------------------------------------------------------
def _http(method: str, url: str, data: bytes | None, headers: dict, timeout: float,
          redirects: int = 5) -> tuple[int, bytes]:
    """One HTTP(S) request: plain HTTP over utils/http1.py (the connection the control-plane
    client uses; urllib.request would add its import cost to the bring-up), HTTPS over
    http.client. Follows redirects for GET/HEAD like the uri module's ``follow_redirects: safe``."""
    from urllib.parse import urljoin, urlsplit

    for _ in range(redirects + 1):
        u = urlsplit(url)
        if u.scheme not in ("http", "https") or not u.hostname:
            raise ValueError(f"unsupported URL {url!r}")
        target = (u.path or "/") + (f"?{u.query}" if u.query else "")
        hdrs = {"Connection": "close", "User-Agent": "tk8s-uri", **headers}
        if u.scheme == "http":
            from .utils.http1 import Connection

            conn = Connection(u.hostname, u.port or 80, timeout=timeout)
            try:
                r = conn.request(method, target, body=data, headers=hdrs)
            finally:
                conn.close()
            status, content, loc = r.status, r.body, r.header("location")
        else:
            import http.client

            hc = http.client.HTTPSConnection(u.hostname, u.port, timeout=timeout)
            try:
                hc.request(method, target, body=data, headers=hdrs)
                hr = hc.getresponse()
                status, content, loc = hr.status, hr.read(), hr.getheader("Location")
            finally:
                hc.close()
        if status in (301, 302, 303, 307, 308) and loc and method in ("GET", "HEAD"):
            url = urljoin(url, loc)
            continue
        return status, content
    raise ValueError(f"too many redirects from {url}")


def m_uri(args, *, check, **_):
    method = str(args.get("method", "GET")).upper()
    if check and method != "GET":
        return {"skipped": True, "changed": False, "msg": f"{method} skipped in check mode"}
    url = str(args["url"])
    codes = args.get("status_code", 200)
    if isinstance(codes, str):
        codes = [int(c) for c in codes.split(",")]
    elif isinstance(codes, int):
        codes = [codes]
    else:
        codes = [int(c) for c in codes]
    headers = {k[len("HEADER_"):]: str(v) for k, v in args.items() if k.startswith("HEADER_")}
    headers.update({k: str(v) for k, v in (args.get("headers") or {}).items()})
    body = args.get("body")
    data = None
    if body is not None:
        if args.get("body_format") == "json":
            if isinstance(body, str):
                body = json.loads(body)
            data = json.dumps(body).encode()
            headers.setdefault("Content-Type", "application/json")
        else:
            data = body.encode() if isinstance(body, str) else json.dumps(body).encode()
    if method in ("POST", "PUT", "PATCH") and data is None:
        data = b""
    timeout = float(args.get("timeout", 30))
    try:
        status, content = _http(method, url, data, headers, timeout)
    except (OSError, ValueError) as e:
        if check:  # dry run: the service this GET targets is not up yet
            return {"skipped": True, "changed": False, "status": -1, "msg": f"check mode: {url} unreachable: {e}"}
        return {"failed": True, "status": -1, "msg": f"request to {url} failed: {e}", "url": url}
    res = {"status": status, "url": url, "changed": method != "GET", "failed": status not in codes}
    text = content.decode(errors="replace")
    try:
        res["json"] = json.loads(text) if text else {}
    except ValueError:
        pass
    if _bool(args.get("return_content")) or res["failed"]:
        res["content"] = text
    if res["failed"]:
        res["msg"] = f"Status code was {status} and not {codes}: {text[:300]}"
    return res


# ---- files ----------------------------------------------------------------------------------
def _fs(ctx, target, local):
    """Where a file task acts: the controller (local_action / delegate_to localhost / no
    machines; relative to the playbook dir) or the target machine through its executor (relative
    to the machine's work dir; over ssh for remote machines)."""
    if local or ctx.executor is None:
        from .executor import LocalFS

        return LocalFS(ctx.dir)
    return ctx.executor.fs(target.name)


def _path(p: str, ctx, target, local) -> Path:
    """Controller-side path (the task runs locally)."""
    from .executor import LocalFS

    return LocalFS(ctx.dir).path(p)


def m_slurp(args, *, ctx, target, local, check, **_):
    fs = _fs(ctx, target, local)
    src = args.get("src") or args.get("path")
    data = fs.read(src)
    if data is None:
        if check:  # produced by a task that check mode did not run
            return {"skipped": True, "changed": False, "msg": f"check mode: {src} does not exist yet"}
        return {"failed": True, "msg": f"file not found: {fs.path(src)}"}
    import base64

    return {"content": base64.b64encode(data).decode(), "encoding": "base64", "source": str(fs.path(src)), "changed": False}


def m_copy(args, *, ctx, target, local, check, **_):
    fs = _fs(ctx, target, local)
    if "content" in args:
        data = str(args["content"]).encode()
    else:
        data = _path(args["src"], ctx, target, True).read_bytes()
    mode = int(str(args["mode"]), 8) if "mode" in args else None
    changed = fs.write(args["dest"], data, mode=mode, check=check)
    return {"changed": changed, "dest": str(fs.path(args["dest"]))}


def m_file(args, *, ctx, target, local, check, **_):
    fs = _fs(ctx, target, local)
    p = args.get("path") or args.get("dest")
    state = args.get("state", "file")
    st = fs.stat(p)
    changed = False
    if state == "directory":
        changed = not (st["exists"] and st.get("isdir"))
        if changed and not check:
            fs.mkdir(p)
    elif state == "absent":
        changed = st["exists"]
        if changed and not check:
            fs.remove(p)
    elif state == "touch":
        changed = True
        if not check:
            fs.touch(p)
    elif state == "link":
        src = str(args["src"])
        q = shlex.quote(str(fs.path(p)))
        cmd = f'mkdir -p "$(dirname -- {q})" && ln -sfn {shlex.quote(src)} {q}'
        rc, cur = _sh(ctx, target, local, f"readlink -- {shlex.quote(str(fs.path(p)))}")
        changed = cur.strip() != src
        if changed and not check:
            rc, out = _sh(ctx, target, local, cmd)
            if rc != 0:
                return {"failed": True, "msg": f"{cmd}: {out.strip()[-300:]}"}
        return {"changed": changed, "path": str(fs.path(p)), "state": state, "src": src}
    elif not st["exists"]:
        return {"failed": True, "msg": f"file {fs.path(p)} does not exist"}
    return {"changed": changed, "path": str(fs.path(p)), "state": state}


def m_stat(args, *, ctx, target, local, **_):
    return {"stat": _fs(ctx, target, local).stat(args["path"]), "changed": False}


def m_include_vars(args, *, ctx, target, local, **_):
    p = _path(args.get("file") or args.get("_raw_params"), ctx, target, True)
    from .utils import yamlio

    return {"ansible_facts": yamlio.load(p.read_text()) or {}, "changed": False}


# ---- control flow ---------------------------------------------------------------------------
def m_pause(args, *, check, **_):
    secs = float(args.get("seconds", 0)) + 60 * float(args.get("minutes", 0))
    if not check:
        time.sleep(secs)
    return {"changed": False, "delta": secs, "msg_out": args.get("prompt", "")}


def m_debug(args, *, variables, **_):
    if "var" in args:
        msg = templating.evaluate(str(args["var"]), variables, strict=False)
        return {"changed": False, "msg_out": json.dumps({str(args["var"]): msg}, default=str)}
    return {"changed": False, "msg_out": str(args.get("msg", args.get("_raw_params", "Hello world!")))}


def m_set_fact(args, **_):
    facts = {k: v for k, v in args.items() if k != "_raw_params"}
    return {"ansible_facts": facts, "changed": False}


def m_fail(args, **_):
    return {"failed": True, "msg": str(args.get("msg", "Failed as requested from task"))}


def m_assert(args, *, variables, **_):
    that = args.get("that", [])
    for cond in that if isinstance(that, list) else [that]:
        if not templating.test(cond, variables):
            return {"failed": True, "msg": args.get("fail_msg") or args.get("msg") or f"Assertion failed: {cond}",
                    "assertion": cond}
    return {"changed": False, "msg_out": args.get("success_msg", "All assertions passed")}


def m_wait_for(args, *, ctx, target, local, check, **_):
    if check:
        return {"skipped": True, "changed": False}
    timeout = float(args.get("timeout", 300))
    time.sleep(float(args.get("delay", 0)))
    deadline = time.monotonic() + timeout
    state = args.get("state", "started")
    while time.monotonic() < deadline:
        if "port" in args:
            host = args.get("host", "127.0.0.1")
            import socket

            s = socket.socket()
            s.settimeout(1.0)
            try:
                s.connect((host, int(args["port"])))
                up = True
            except OSError:
                up = False
            finally:
                s.close()
            if up == (state in ("started", "present")):
                return {"changed": False, "elapsed": round(timeout - (deadline - time.monotonic()), 3)}
        elif "path" in args:
            fs = _fs(ctx, target, local)
            if state == "absent":
                if not fs.stat(args["path"])["exists"]:
                    return {"changed": False}
            elif fs.search(args["path"], args.get("search_regex")):
                return {"changed": False}
        else:
            return {"changed": False}
        time.sleep(0.02)
    return {"failed": True, "msg": f"Timeout when waiting for {args}"}


def m_meta(args, **_):
    return {"changed": False}


def m_ping(args, **_):
    return {"ping": "pong", "changed": False}


# ---- tk8s modules -------------------------------------------------------------------------------
def m_tk8s_daemon(args, *, ctx, target, local, env, check, **_):
    """name, argv|cmd, state started|stopped|query, env, restart_policy, wait_for_log, timeout."""
    ex = ctx.executor
    name = args["name"]
    state = args.get("state", "started")
    if ex is None:
        if check:  # dry run without provisioned machines (BASELINE.json config 1)
            return {"changed": state == "started", "running": False, "msg": "check mode: no machine executor"}
        return {"failed": True, "msg": "tk8s_daemon needs a machine executor"}
    status = ex.daemon_status(target.name, name)
    if state == "query":
        return {"changed": False, "running": status["running"], "pid": status.get("pid"), "stdout": name if status["running"] else ""}
    if state == "stopped":
        if check or not status["running"]:
            return {"changed": status["running"], "running": False}
        ex.stop_daemon(target.name, name)
        return {"changed": True, "running": False}
    if status["running"] and not check and _orphaned_zygote(ex, target.name, name):
        # an interpreter started early for this daemon (earlyburn zygote) that its boot hook never
        # handed its arguments: it would wait forever. Stop it and start the daemon the plain way
        # below -- slower by the zygote's head start, but correct.
        ex.stop_daemon(target.name, name)
        status = {"running": False}
    if status["running"]:
        if args.get("wait_for_log") and not check and hasattr(ex, "wait_log"):
            info = ex.wait_log(target.name, name, str(args["wait_for_log"]), float(args.get("timeout", 300)))
            if not info.get("ok"):
                return {"failed": True, **info}
            return {"changed": False, "running": True, "pid": status.get("pid"), **info}
        return {"changed": False, "running": True, "pid": status.get("pid")}
    if check:
        return {"changed": True, "running": False, "msg": "would start"}
    argv = args.get("argv") or shlex.split(str(args.get("cmd", "")))
    denv = {str(k): str(v) for k, v in (args.get("env") or {}).items()}
    denv.update(env or {})
    info = ex.start_daemon(target.name, name, [str(a) for a in argv], env=denv,
                           restart=str(args.get("restart_policy", "unless-stopped")),
                           wait_for_log=args.get("wait_for_log"), timeout=float(args.get("timeout", 300)))
    if not info.get("ok"):
        return {"failed": True, "msg": info.get("msg", "daemon failed to start"), **info}
    return {"changed": True, "running": True, **info}


def _orphaned_zygote(ex, host: str, name: str) -> bool:
    """The running ``name`` daemon is a zygote (earlyburn: ``run/<name>.zygote``) still waiting for
    the ``run/<name>.args`` its boot hook should have written."""
    fs = getattr(ex, "fs", None)
    if fs is None:
        return False
    f = fs(host)
    return f.read(f"run/{name}.zygote") is not None and f.read(f"run/{name}.args") is None


def m_tk8s_burnin(args, *, ctx, target, local, env, check, **_):
    """Start the early GPU burn-in on a machine's GPUs (no-op for GPU-less machines).

    command: the validation command (list); out: result file relative to the machine dir.
    Creates ``<out>.pending`` first (the validation pod's ``--reuse`` waits on it), then starts
    ``command --out <out>`` as a one-shot daemon (pidfile under run/, killed on teardown)
    with ROCR_VISIBLE_DEVICES = the machine's GPUs composed onto this process's view.
    """
    ex = ctx.executor
    if ex is None or local:
        return {"changed": False, "skipped": True, "msg": "no machine executor"}
    if check:
        return {"changed": bool(ex.machine_gpus(target.name)), "msg": "would start the GPU burn-in"}
    from .burnin import start_burnin

    return start_burnin(ex, target.name, args["command"], str(args.get("out", "run/gpu-burnin.json")),
                        str(args.get("name", "gpu-burnin")), env)


def m_tk8s_gpu_facts(args, *, ctx, target, local, **_):
    """Node runtime facts (nodefacts.py) of the target machine -- gathered ON it (over ssh for a
    remote machine) -- plus the GPU slice the provider gave it."""
    from .models.hostinfo import compose_visible_devices

    timing: dict = {}
    if ctx.executor is not None and not local:
        facts = dict(ctx.executor.facts(target.name, timing))
        facts["tk8s_machine_gpus"] = ctx.executor.machine_gpus(target.name)
    else:
        from .nodefacts import node_facts

        facts = dict(node_facts(timing))
        facts["tk8s_machine_gpus"] = []
    facts["tk8s_machine_visible_devices"] = compose_visible_devices(facts["tk8s_machine_gpus"])["ROCR_VISIBLE_DEVICES"]
    return {"ansible_facts": facts, "changed": False, "timing_ms": timing}


def m_tk8s_build(args, *, check, **_):
    from .utils import build_native

    if check:
        return {"changed": False, "msg": "build checked only"}
    t = time.monotonic()
    before = {k: (p.stat().st_mtime if p.exists() else 0) for k, p in _artefacts(build_native).items()}
    build_native.build()
    after = {k: p.stat().st_mtime for k, p in _artefacts(build_native).items()}
    return {"changed": before != after, "seconds": round(time.monotonic() - t, 3)}


def _artefacts(bn) -> dict:
    out = {"lib": bn.lib_path(), "rccl_lib": bn.rccl_lib_path(), "native": bn.native_module_path(), "topo": bn.topo_module_path()}
    out.update({n: bn.tool_path(n) for n in list(bn.TOOLS) + ["tk8s-supervise", "tk8s-smi"]})
    return out


def m_tk8s_kube(args, *, ctx, check, **_):
    """api, project, token (the control plane's admin token), state present|absent|wait,
    definition|src, timeout. The result's ``timing_ms`` says where the task's time went (the
    validation DaemonSet's deploy is on the bring-up's critical path)."""
    t0 = time.perf_counter()
    timing: dict[str, float] = {}

    def mark(part: str) -> None:
        nonlocal t0
        t = time.perf_counter()
        timing[part] = round((t - t0) * 1e3, 3)
        t0 = t

    from .controlplane.client import ApiError, Client, client_from_kubeconfig
    from .kube import apply_objects, delete_objects, load_manifests

    mark("import")
    if "definition" in args:
        objs = args["definition"] if isinstance(args["definition"], list) else [args["definition"]]
    else:
        objs = load_manifests(_path(args["src"], ctx, None, True), args.get("vars") or {})
    mark("manifests")
    state = args.get("state", "present")
    if check:
        return {"changed": state != "wait", "objects": len(objs), "msg": "check mode"}
    api = str(args["api"])
    pid = str(args["project"])
    kc = Client(api, token=str(args["token"]) if args.get("token") else None).get(
        f"/env/{pid}/kubernetes/kubectl", query={"format": "json"})
    k = client_from_kubeconfig(kc)
    mark("kubeconfig")
    try:
        if state == "absent":
            n = delete_objects(k, objs)
            mark("delete")
            return {"changed": n > 0, "deleted": n, "timing_ms": timing}
        res = apply_objects(k, objs)
        mark("apply")
        return {"changed": any(r["created"] for r in res), "objects": res, "timing_ms": timing}
    except ApiError as e:
        return {"failed": True, "msg": str(e)}


MODULES = {
    "command": m_command, "shell": m_shell, "uri": m_uri, "slurp": m_slurp, "copy": m_copy, "file": m_file,
    "stat": m_stat, "include_vars": m_include_vars, "pause": m_pause, "debug": m_debug, "set_fact": m_set_fact,
    "fail": m_fail, "assert": m_assert, "wait_for": m_wait_for, "meta": m_meta, "ping": m_ping,
    "tk8s_daemon": m_tk8s_daemon, "tk8s_gpu_facts": m_tk8s_gpu_facts, "tk8s_burnin": m_tk8s_burnin, "tk8s_build": m_tk8s_build,
    "tk8s_kube": m_tk8s_kube,
    "apt": m_apt, "apt_repository": m_apt_repository, "get_url": m_get_url, "systemd_service": m_systemd_service,
    "systemd": m_systemd_service, "service": m_systemd_service, "replace": m_replace, "lineinfile": m_lineinfile,
    "fetch": m_fetch, "setup": m_setup, "gather_facts": m_setup,
}


def module_name(mod: str) -> str:
    """``ansible.builtin.apt`` / ``ansible.legacy.apt`` -> ``apt`` (FQCNs as real Ansible writes them)."""
    for prefix in ("ansible.builtin.", "ansible.legacy."):
        if mod.startswith(prefix):
            return mod[len(prefix):]
    return mod
