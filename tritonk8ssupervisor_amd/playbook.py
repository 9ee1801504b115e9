"""Playbook engine: the Ansible subset that ``ansible/clusterUp.yml`` and its roles use (L3b).

``ansible-playbook`` is not available offline; this engine executes the same YAML files
(reference: ansible/clusterUp.yml:1-26 + roles/*/tasks/main.yml) against the machines the
provisioning engine created. Semantics kept from Ansible:

  * plays in order; a play's tasks run host-parallel (``forks`` from ansible.cfg — default ALL
    hosts, not Ansible's 5), task after task (a barrier per task);
  * task keywords: name, register, when, until/retries/delay, with_items/loop, run_once,
    delegate_to, local_action, action, ignore_errors, failed_when, changed_when, environment;
  * a failed host leaves the play; the run fails if any host failed;
  * ``--check``: nothing mutates (BASELINE.json config 1 dry-run); templating errors that come
    from results a skipped task would have produced are reported as skips.

Bugs of the reference not replicated: inverted ``when:`` truthiness (dockersetup main.yml:10;
our role uses explicit tests), ``playbook_dir: $(pwd)`` (clusterUp.yml:12 — the real
``playbook_dir`` magic variable is provided), env-id file never cleaned (teardown removes it).
"""
from __future__ import annotations

import os
import shlex
import threading
import time
from pathlib import Path

from . import templating
from .templating import TemplateError, Undefined
from .utils import yamlio
from .utils.events import EventLog
from .utils.pool import Pool
from .utils.record import field, record as dataclass

_HOME = str(Path(__file__).resolve().parents[1])  # this checkout: the tk8s install of colocated machines

TASK_KEYS = {"name", "register", "when", "until", "retries", "delay", "with_items", "loop", "run_once",
             "delegate_to", "local_action", "action", "ignore_errors", "failed_when", "changed_when",
             "environment", "no_log", "tags", "vars", "check_mode", "loop_control", "become", "become_user", "args",
             "notify", "delegate_facts", "any_errors_fatal", "timeout"}


class PlaybookError(RuntimeError):
    pass


@dataclass
class Host:
    name: str
    vars: dict = field(default_factory=dict)
    groups: list[str] = field(default_factory=list)

    @property
    def address(self) -> str:
        return str(self.vars.get("ansible_host", self.name))


def parse_inventory(text: str) -> dict[str, Host]:
    """INI inventory: ``[GROUP]`` sections, ``name [k=v ...]`` lines."""
    hosts: dict[str, Host] = {}
    group = "ungrouped"
    for raw in text.splitlines():
        line = raw.split("#", 1)[0].strip()
        if not line:
            continue
        if line.startswith("[") and line.endswith("]"):
            group = line[1:-1].strip()
            continue
        parts = shlex.split(line)
        name, kv = parts[0], dict(p.split("=", 1) for p in parts[1:] if "=" in p)
        h = hosts.setdefault(name, Host(name))
        h.vars.update(kv)
        if group not in h.groups:
            h.groups.append(group)
    return hosts


def _free_form(text: str) -> tuple[dict, str]:
    """Split ``k=v k2="v 2" rest`` into (kv-dict, free-form remainder)."""
    kv, free = {}, []
    lex = shlex.shlex(text, posix=True)
    lex.whitespace_split = True
    lex.commenters = ""
    for tok in lex:
        if "=" in tok and tok.split("=", 1)[0].replace("_", "").replace("-", "").isalnum() and not free:
            k, v = tok.split("=", 1)
            kv[k] = v
        else:
            free.append(tok)
    return kv, " ".join(free)


@dataclass
class TaskResult:
    host: str
    status: str            # ok | changed | failed | skipped
    result: dict
    seconds: float = 0.0


@dataclass
class PlaybookResult:
    ok: bool
    stats: dict[str, dict[str, int]]
    failures: list[str]
    seconds: float
    hostvars: dict[str, dict]


class Playbook:
    def __init__(self, playbook: str | os.PathLike, inventory: str | os.PathLike, *, executor=None,
                 extra_vars: dict | None = None, check: bool = False, events: EventLog | None = None,
                 out: Callable[[str], None] | None = print, forks: int | None = None):
        self.path = Path(playbook).resolve()
        self.dir = self.path.parent
        self.hosts = parse_inventory(Path(inventory).read_text())
        self.executor = executor           # provider-backed remote executor (see modules.Executor)
        self.extra_vars = extra_vars or {}
        self.check = check
        self.events = events or EventLog(None)
        self.out = out or (lambda s: None)
        self.cfg = self._read_cfg()
        self.forks = forks or int(self.cfg.get("forks", "0") or 0) or None
        self.hostvars: dict[str, dict] = {h: {} for h in self.hosts}
        self.stats = {h: {"ok": 0, "changed": 0, "failed": 0, "skipped": 0, "unreachable": 0} for h in self.hosts}
        self._print_lock = threading.Lock()
        self._pool: Pool | None = None
        # every module invocation as rendered (play, host, task, module, args): what --check
        # reports and the golden tests pin
        self.trace: list[dict] = []
        self._trace_lock = threading.Lock()
        self._play = ""
        self._defaults: dict = {}
        self._play_env: dict = {}
        self._gv_cache: dict[str, dict] = {}

    def _read_cfg(self) -> dict:
        try:
            text = (self.dir / "ansible.cfg").read_text()
        except OSError:
            return {}
        return read_ini_section(text, "defaults")

    def say(self, s: str) -> None:
        with self._print_lock:
            self.out(s)

    # ---- variables ---------------------------------------------------------------------
    def _groups(self) -> dict[str, list[str]]:
        g: dict[str, list[str]] = {"all": list(self.hosts)}
        for h in self.hosts.values():
            for grp in h.groups:
                g.setdefault(grp, []).append(h.name)
        return g

    def host_vars(self, host: Host, play_vars: dict) -> dict:
        v = {"inventory_hostname": host.name, "ansible_host": host.address, "playbook_dir": str(self.dir),
             "groups": self._groups(), "group_names": host.groups, "ansible_check_mode": self.check,
             "ansible_default_ipv4": {"address": host.address}, "hostvars": self.hostvars}
        v.update(self._defaults)  # role defaults: the lowest precedence of all
        v.update(self._group_vars(host))  # group_vars/ next to the playbook (all, then the host's groups)
        v.update(self._machine_vars(host))  # what the provider knows of the machine (a hand-written
        v.update(host.vars)                 # inventory need not repeat it; the inventory wins)
        v.update(play_vars)
        v.update(self.hostvars.get(host.name, {}))
        v.update(self.extra_vars)
        return v

    def select(self, pattern: str) -> list[Host]:
        names: list[str] = []
        groups = self._groups()
        for part in str(pattern).replace(";", ":").split(":"):
            part = part.strip()
            if part in groups:
                names += groups[part]
            elif part in self.hosts:
                names.append(part)
        seen = set()
        return [self.hosts[n] for n in names if not (n in seen or seen.add(n))]

    # ---- task normalisation ------------------------------------------------------------
    def _module_of(self, task: dict) -> tuple[str, Any, bool]:
        """Returns (module, args, is_local)."""
        if "local_action" in task:
            spec = task["local_action"]
            if isinstance(spec, dict):
                spec = dict(spec)
                mod = spec.pop("module")
                return mod, spec, True
            mod, _, rest = str(spec).strip().partition(" ")
            return mod, rest, True
        if "action" in task:
            spec = task["action"]
            if isinstance(spec, dict):
                spec = dict(spec)
                return spec.pop("module"), spec, False
            mod, _, rest = " ".join(str(spec).split()).partition(" ")
            return mod, rest, False
        for k, v in task.items():
            if k not in TASK_KEYS and not k.startswith("_"):
                return k, v, False
        raise PlaybookError(f"task {task.get('name')!r} has no module")

    @staticmethod
    def _args(mod: str, raw: Any, extra: dict | None = None) -> dict:
        from .playbook_modules import module_name

        mod = module_name(mod)
        if isinstance(raw, dict):
            args = dict(raw)
        elif raw is None:
            args = {}
        elif mod in ("command", "shell"):
            args = {"_raw_params": str(raw)}
        else:
            kv, free = _free_form(str(raw))
            args = kv
            if free:
                args["_raw_params"] = free
        if extra:
            args.update(extra)
        return args

    # ---- run -----------------------------------------------------------------------------
    def run(self) -> PlaybookResult:
        t0 = time.monotonic()
        plays = yamlio.load(self.path.read_text()) or []
        failures: list[str] = []
        try:
            for play in plays:
                failures += self.run_play(play)
                if failures and not self.check:
                    break
        finally:
            if self._pool is not None:
                self._pool.shutdown(wait=False)
                self._pool = None
        self.say("")
        self.say("PLAY RECAP " + "*" * 68)
        for h, s in self.stats.items():
            self.say(f"{h:<26}: ok={s['ok']:<4} changed={s['changed']:<4} unreachable={s['unreachable']:<4} "
                     f"failed={s['failed']:<4} skipped={s['skipped']}")
        return PlaybookResult(not failures, self.stats, failures, time.monotonic() - t0, self.hostvars)

    def _role_tasks(self, role: str) -> list[dict]:
        p = self.dir / "roles" / role / "tasks" / "main.yml"
        if not p.exists():
            raise PlaybookError(f"role {role!r} not found at {p}")
        tasks = yamlio.load(p.read_text()) or []
        for t in tasks:
            t.setdefault("_role", role)
        return tasks

    def run_play(self, play: dict) -> list[str]:
        name = play.get("name", play.get("hosts"))
        self.say("")
        self.say(f"PLAY [{name}] " + "*" * max(3, 72 - len(str(name))))
        hosts = self.select(play.get("hosts", "all"))
        with self.events.phase(f"play:{name}", hosts=[h.name for h in hosts]):
            play_vars = dict(play.get("vars") or {})
            play_vars.pop("playbook_dir", None)  # reference sets the literal "$(pwd)"; use the real one
            for vf in play.get("vars_files") or []:
                f = templating.render(vf, {"playbook_dir": str(self.dir), **self.extra_vars})
                fp = Path(f) if Path(f).is_absolute() else self.dir / f
                if fp.exists():
                    play_vars.update(yamlio.load(fp.read_text()) or {})
                elif not self.check:
                    raise PlaybookError(f"vars_files entry {fp} not found")
            tasks: list[dict] = []
            self._defaults = {}
            for role in play.get("roles") or []:
                rname = role if isinstance(role, str) else role["role"]
                dfile = self.dir / "roles" / rname / "defaults" / "main.yml"
                if dfile.exists():
                    self._defaults.update(yamlio.load(dfile.read_text()) or {})
                rtasks = self._role_tasks(rname)
                rwhen = None if isinstance(role, str) else role.get("when")
                if rwhen is not None:  # a role's `when:` applies to every task of it (and-ed with theirs)
                    for t in rtasks:
                        own = t.get("when")
                        t["when"] = [*(rwhen if isinstance(rwhen, list) else [rwhen]),
                                     *([] if own is None else own if isinstance(own, list) else [own])]
                tasks += rtasks
            tasks += play.get("tasks") or []
            self._play = str(name)
            self._play_env = play.get("environment") or {}
            if play.get("gather_facts", True) and not self._facts_done(hosts):
                tasks = [{"name": "Gathering Facts", "setup": {}, "_facts": True}] + tasks
            alive = list(hosts)
            failures: list[str] = []
            for task in tasks:
                if not alive:
                    break
                res = self.run_task(task, alive, play_vars)
                for r in res:
                    if r.status == "failed":
                        failures.append(f"{r.host}: {task.get('name', '?')}: {r.result.get('msg', '')}")
                alive = [h for h in alive if not any(r.host == h.name and r.status == "failed" for r in res)]
        return failures

    def run_task(self, task: dict, hosts: list[Host], play_vars: dict) -> list[TaskResult]:
        title = task.get("name") or next(iter(k for k in task if k not in TASK_KEYS and not k.startswith("_")), "task")
        prefix = f"{task['_role']} : " if task.get("_role") else ""
        self.say("")
        self.say(f"TASK [{prefix}{title}] " + "*" * max(3, 70 - len(prefix + str(title))))
        t = time.monotonic()
        if task.get("run_once"):
            res = [self._run_on_host(task, hosts[0], play_vars)]
            if res[0].status != "skipped":  # run_once results are shared by every host
                for h in hosts[1:]:
                    if task.get("register"):
                        self.hostvars[h.name][task["register"]] = res[0].result
        elif len(hosts) == 1 or self._inline(task, hosts):
            res = [self._run_on_host(task, h, play_vars) for h in hosts]
        else:
            start = len(self.trace)
            # `when:` first, here: a host it skips needs no thread, and when it leaves one host
            # (or only hosts whose work is a pidfile read) that runs inline too
            done: dict[str, TaskResult] = {}
            if "when" in task:
                for h in hosts:
                    r = self._when(task, h, play_vars)
                    if r is not None:
                        done[h.name] = r
            todo = [h for h in hosts if h.name not in done]
            if len(todo) <= 1 or (done and self._inline(task, todo)):
                ran = [self._run_on_host(task, h, play_vars, when_checked=True) for h in todo]
            else:
                ran = list(self._executor().map(lambda h: self._run_on_host(task, h, play_vars, when_checked=True), todo))
            by_host = {**done, **{r.host: r for r in ran}}
            res = [by_host[h.name] for h in hosts]
            # hosts ran in parallel: the trace of this task in host order (each host's own
            # entries keep their order), so --check plans read the same on every run
            order = {h.name: i for i, h in enumerate(hosts)}
            with self._trace_lock:
                self.trace[start:] = sorted(self.trace[start:], key=lambda e: order.get(e["host"], len(order)))
        timing = {r.host: r.result["timing_ms"] for r in res if isinstance(r.result, dict) and r.result.get("timing_ms")}
        self.events.emit("task", task=f"{prefix}{title}", seconds=round(time.monotonic() - t, 6),
                         results={r.host: r.status for r in res}, **({"timing_ms": timing} if timing else {}))
        return res

    def _when(self, task: dict, host: Host, play_vars: dict, v: dict | None = None) -> TaskResult | None:
        """The recorded result of a host that the task's ``when:`` skips (or fails on), else None."""
        if "when" not in task:
            return None
        if v is None:
            v = self.host_vars(host, {**play_vars, **(task.get("vars") or {})})
        try:
            if not templating.test(task["when"], v):
                return self._record(task, host, TaskResult(host.name, "skipped", {"skipped": True, "changed": False}))
        except Undefined as e:
            if self.check:
                return self._record(task, host, TaskResult(host.name, "skipped", {"skipped": True, "msg": f"check mode: {e}"}))
            return self._record(task, host, TaskResult(host.name, "failed", {"failed": True, "msg": f"when: {e}"}))
        return None

    def _run_on_host(self, task: dict, host: Host, play_vars: dict, when_checked: bool = False) -> TaskResult:
        t0 = time.monotonic()
        v = self.host_vars(host, {**play_vars, **(task.get("vars") or {})})
        if not when_checked:
            r = self._when(task, host, play_vars, v)
            if r is not None:
                return r
        mod, raw, local = self._module_of(task)
        if task.get("delegate_to"):
            target = templating.render(task["delegate_to"], v)
            local = local or target in ("localhost", "127.0.0.1")
            deleg = self._host_by_addr(target)
        else:
            deleg = None
        items = task.get("with_items", task.get("loop"))
        try:
            if items is not None:
                items = templating.render(items, v)
                results = []
                for item in items:
                    iv = dict(v, item=item)
                    results.append(self._exec(task, mod, raw, iv, host, deleg, local))
                failed = any(r.get("failed") for r in results)
                changed = any(r.get("changed") for r in results)
                result = {"results": results, "changed": changed, "failed": failed,
                          "msg": next((r.get("msg") for r in results if r.get("failed")), "")}
            else:
                result = self._exec(task, mod, raw, v, host, deleg, local)
        except Undefined as e:
            if self.check:
                result = {"skipped": True, "changed": False, "msg": f"check mode: {e}"}
            else:
                result = {"failed": True, "msg": f"template error: {e}"}
        except TemplateError as e:
            result = {"failed": True, "msg": f"template error: {e}"}
        status = "skipped" if result.get("skipped") else "failed" if result.get("failed") else \
            "changed" if result.get("changed") else "ok"
        if status == "failed" and task.get("ignore_errors"):
            status = "ok"
            result["ignored"] = True
        r = TaskResult(host.name, status, result, time.monotonic() - t0)
        return self._record(task, host, r)

    def _machine_vars(self, host: Host) -> dict:
        ex = self.executor
        m = getattr(ex, "machines", {}).get(host.name) if ex is not None else None
        if m is None:
            return {}
        return {"tk8s_machine_dir": m.sandbox, "tk8s_gpus": ",".join(map(str, m.gpus)), "tk8s_home": m.home or _HOME}

    def _group_vars(self, host: Host) -> dict:
        out: dict = {}
        with self._trace_lock:  # hosts run in parallel: load each group's file exactly once
            for g in ["all", *host.groups]:
                if g not in self._gv_cache:
                    data = {}
                    for f in (self.dir / "group_vars" / f"{g}.yml", self.dir / "group_vars" / f"{g}.yaml"):
                        if f.exists():
                            data = yamlio.load(f.read_text()) or {}
                            break
                    self._gv_cache[g] = data
                out.update(self._gv_cache[g])
        return out

    def _facts_done(self, hosts: list[Host]) -> bool:
        return all("ansible_kernel" in self.hostvars.get(h.name, {}) for h in hosts)

    # modules that only read or write a few local files when the machines are sandboxes of this
    # host: nothing to overlap, so one thread per host only adds interpreter-lock contention
    _INLINE_MODULES = frozenset({"set_fact", "debug", "stat", "file", "copy", "lineinfile", "slurp", "assert",
                                 "fail", "tk8s_gpu_facts"})

    def _inline(self, task: dict, hosts: list[Host] = ()) -> bool:
        """Run this task's hosts one after another in this thread (local machines, a module of
        _INLINE_MODULES, no retries/loops/delegation). ``TK8S_PLAY_INLINE=0``: always a thread
        per host. ``tk8s_daemon`` too when it only reads pidfiles: a query, or a start of a daemon
        that already runs on every host (the standby agent its machine's boot hook started) --
        8 threads for 8 pidfile reads cost ~1 ms per host in interpreter-lock hand-offs."""
        ex = self.executor
        if ex is None or getattr(ex, "remote", True) or os.environ.get("TK8S_PLAY_INLINE", "1") == "0":
            return False
        if task.get("delegate_to") or "until" in task or task.get("with_items", task.get("loop")) is not None:
            return False
        try:
            mod, raw, _ = self._module_of(task)
        except PlaybookError:
            return False
        from .playbook_modules import module_name

        name = module_name(mod)
        if name == "tk8s_daemon" and isinstance(raw, dict):
            state, dname = raw.get("state", "started"), raw.get("name")
            if state == "query":
                return True
            if state == "started" and isinstance(dname, str) and "{" not in dname and hosts:
                try:
                    return all(ex.daemon_status(h.name, dname).get("running") for h in hosts)
                except Exception:  # noqa: BLE001 - undecided: the threads decide
                    return False
            return False
        return name in self._INLINE_MODULES

    def _executor(self) -> Pool:
        """One pool for the whole run (``forks`` workers; 0 = every host): starting fresh threads
        for every task cost ~2.5 ms per thread start under GIL contention at 9 hosts."""
        if self._pool is None:
            self._pool = Pool(max(1, self.forks or len(self.hosts)), "play")
        return self._pool

    def _host_by_addr(self, target: str) -> Host | None:
        for h in self.hosts.values():
            if target in (h.name, h.address):
                return h
        return None

    def _exec(self, task, mod, raw, v, host, deleg, local) -> dict:
        from .playbook_modules import run_module

        extra = task.get("args")
        args = templating.render(self._args(mod, raw, extra), v)
        play_env = self._play_env if not task.get("_facts") else {}  # facts come first: nothing to render yet
        env = {**templating.render(play_env, v), **templating.render(task.get("environment") or {}, v)}
        with self._trace_lock:
            self.trace.append({"play": self._play, "host": host.name, "task": task.get("name", ""),
                               "module": mod, "args": args, "local": bool(local), "delegate": deleg.name if deleg else None})
        retries = int(task.get("retries", 3)) if "until" in task else 0
        delay = float(task.get("delay", 5))
        attempt = 0
        while True:
            attempt += 1
            result = run_module(mod, args, ctx=self, host=host, target=deleg or host, local=local, env=env,
                                check=self.check and task.get("check_mode", True) is not False, variables=v)
            if "until" in task and not result.get("skipped"):
                rv = dict(v)
                if task.get("register"):
                    rv[task["register"]] = result
                if not templating.test(task["until"], rv):
                    if attempt <= retries:
                        time.sleep(delay)
                        continue
                    result["failed"] = True
                    result["msg"] = f"until condition not met after {attempt} attempts"
                result["attempts"] = attempt
            break
        vv = dict(v)
        if task.get("register"):
            vv[task["register"]] = result
        if "failed_when" in task:
            result["failed"] = templating.test(task["failed_when"], vv)
        if "changed_when" in task:
            result["changed"] = templating.test(task["changed_when"], vv)
        return result

    def _record(self, task: dict, host: Host, r: TaskResult) -> TaskResult:
        if task.get("register"):
            self.hostvars[host.name][task["register"]] = r.result
        if r.status == "ok" and r.result.get("ansible_facts"):
            self.hostvars[host.name].update(r.result["ansible_facts"])
        self.stats[host.name][r.status] = self.stats[host.name].get(r.status, 0) + 1
        word = {"ok": "ok", "changed": "changed", "failed": "fatal", "skipped": "skipping"}[r.status]
        msg = ""
        if r.status == "failed":
            msg = f" => {{\"msg\": {r.result.get('msg', '')!r}}}"
        elif task.get("debug") is not None or "msg_out" in r.result:
            msg = f" => {r.result.get('msg_out', '')}"
        self.say(f"{word}: [{host.name}]{msg}")
        return r


def copy_vars(d: dict) -> dict:
    import copy

    return copy.deepcopy(d)


def read_ini_section(text: str, section: str) -> dict:
    """``dict(ConfigParser()[section])`` of an INI text (ansible.cfg) without importing configparser
    on the bring-up path: ``key = value`` / ``key: value`` lines, keys lower-cased, ``#``/``;``
    comment lines. Anything beyond that (continuation lines, ``%(..)s`` interpolation, a
    DEFAULT section) goes to configparser itself."""
    if "%(" in text or "[DEFAULT]" in text:
        return _configparser_section(text, section)
    out: dict = {}
    cur = None
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line[0] in "#;":
            continue
        if raw[:1] in " \t":
            return _configparser_section(text, section)  # a continuation line
        if line.startswith("[") and line.endswith("]"):
            cur = line[1:-1]
            continue
        if cur != section:
            continue
        k, sep, v = _split_ini(line)
        if not sep:
            return _configparser_section(text, section)
        out[k.strip().lower()] = v.strip()
    return out


def _split_ini(line: str):
    i = min([j for j in (line.find("="), line.find(":")) if j >= 0], default=-1)
    return (line, "", "") if i < 0 else (line[:i], line[i], line[i + 1:])


def _configparser_section(text: str, section: str) -> dict:
    import configparser

    cp = configparser.ConfigParser()
    cp.read_string(text)
    return dict(cp[section]) if cp.has_section(section) else {}
