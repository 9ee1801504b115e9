"""Interactive setup wizard — the 8 prompts + confirmation of setup.sh, with the same text,
defaults and validation rules, and a non-interactive answers mode for benchmarking.

Reference: getArgument setup.sh:94-110 (W2), getConfigFromUser setup.sh:255-451 (W5),
verifyConfig setup.sh:452-483 (W6). Differences, on purpose:
  * getArgument without a default re-prompts until non-empty (the reference never `break`s).
  * answers can be supplied up-front (dict / file / list); they are fed through the very same
    prompt+validation path, so a scripted run cannot bypass a rule an interactive one obeys.
"""
from __future__ import annotations

import io
import json
import re
import sys
from pathlib import Path

from .config import ClusterConfig
from .provider.base import Provider

HOSTNAME_RE = re.compile(r"^[a-zA-Z][0-9a-zA-Z]+$")   # setup.sh:276, 288
NODES_RE = re.compile(r"^[1-9]$")                      # setup.sh:301
INDEX_LIST_RE = re.compile(r"^[1-9][0-9]?(,[1-9][0-9]?)*$")  # setup.sh:337, 380
PACKAGE_RE = re.compile(r"^[1-9][0-9]*$")              # setup.sh:428
SEP = "---------------"


class WizardAbort(SystemExit):
    """User answered `no` at the confirmation (setup.sh:477-478 exits 0)."""


def valid_hostname(s: str) -> bool:
    return bool(HOSTNAME_RE.match(s))


def valid_node_count(s: str) -> bool:
    return bool(NODES_RE.match(s))


def normalize_list(s: str) -> str:
    """`tr ',' '\\n' | sort | uniq | tr '\\n' ','` minus the trailing comma (setup.sh:333-334)."""
    items = sorted(set(x for x in s.replace('"', "").split(",") if x != ""))
    return ",".join(items)


def parse_index_list(s: str, count: int) -> list[int] | None:
    """Validated 1-based indices for a comma list, or None (setup.sh:337-345)."""
    if not INDEX_LIST_RE.match(s):
        return None
    idx = [int(x) for x in s.split(",")]
    if any(i < 1 or i > count for i in idx):
        return None
    return idx


class Prompter:
    """`read -p` over arbitrary streams, optionally pre-seeded with answers."""

    def __init__(self, inp: TextIO | None = None, out: TextIO | None = None,
                 answers: Iterable[str] | None = None):
        self.inp = inp if inp is not None else sys.stdin
        self.out = out if out is not None else sys.stdout
        self.answers = list(answers) if answers is not None else None

    def say(self, text: str = "") -> None:
        self.out.write(text + "\n")
        self.out.flush()

    def read(self, prompt: str) -> str:
        self.out.write(prompt)
        self.out.flush()
        if self.answers is not None:
            if not self.answers:
                raise EOFError(f"no scripted answer left for prompt: {prompt.strip()}")
            ans = self.answers.pop(0)
            self.out.write(ans + "\n")
            return ans
        line = self.inp.readline()
        if line == "":
            raise EOFError(f"stdin closed at prompt: {prompt.strip()}")
        return line.rstrip("\n")

    def get_argument(self, msg: str, default: str | None = None) -> str:
        """getArgument (setup.sh:94-110): `msg (default) `; empty input -> default."""
        while True:
            if default is None:
                ans = self.read(f"{msg} ").strip()
                if ans:
                    return ans
                continue
            ans = self.read(f"{msg} ({default}) ").strip()
            return default if ans == "" else ans


def _list_options(p: Prompter, rows: list[tuple[str, str]]) -> None:
    for i, (name, ident) in enumerate(rows, 1):
        p.say(f"{i}.\t{name}  {ident}")


def _ask_networks(p: Prompter, prov: Provider, msg: str, current: str) -> str:
    nets = prov.networks()
    p.say("From the networks below:")
    _list_options(p, [(n.name, n.id) for n in nets])
    default_loc = next((i for i, n in enumerate(nets, 1) if n.name == prov.default_network), 1)
    count = len(nets)
    if current == "":
        current = ",".join(prov.network_ids([default_loc]))
    while True:
        tmp = p.get_argument(msg, current.replace('"', ""))
        current = normalize_list(current)
        tmp = normalize_list(tmp)
        if INDEX_LIST_RE.match(tmp):
            idx = parse_index_list(tmp, count)
            if idx is not None:
                return ",".join(prov.network_ids(idx))
            p.say("error: Enter a valid option or leave blank to use the default.")
            p.say(f"    Values should be comma separated between 1 and {count}.")
        elif tmp == current:
            return current
        else:
            p.say("error: Enter a valid option or leave blank to use the default.")
            p.say(f"    Values should be comma separated between 1 and {count}.")


def _ask_package(p: Prompter, prov: Provider, current: str) -> str:
    pkgs = prov.packages()
    p.say("From the packages below:")
    _list_options(p, [(k.name, k.id) for k in pkgs])
    loc = next((i for i, k in enumerate(pkgs, 1) if k.name == prov.default_package), 1)
    count = len(pkgs)
    if current == "":
        current = prov.package_id(loc)
    while True:
        tmp = p.get_argument("What KVM package should the master and nodes run on:", current.replace('"', ""))
        if PACKAGE_RE.match(tmp):
            i = int(tmp)
            if 1 <= i <= count:
                current = prov.package_id(i)
                p.say(f"entered {tmp} and got {current}")
                return current
            p.say("error: Enter a valid option or leave blank to use the default.")
            p.say(f"    Value should be between 1 and {count}.")
        elif tmp == current.replace('"', ""):
            return current
        else:
            p.say("error: Enter a valid option or leave blank to use the default.")
            p.say(f"    Value should be between 1 and {count}.")


def get_config_from_user(cfg: ClusterConfig, prov: Provider, p: Prompter) -> ClusterConfig:
    """The 8 prompts in reference order (setup.sh:264-450)."""
    p.say(SEP)
    cfg.KUBERNETES_NAME = p.get_argument("Name your Kubernetes environment:", cfg.KUBERNETES_NAME.replace('"', ""))
    p.say(SEP)
    desc_default = cfg.KUBERNETES_NAME if cfg.KUBERNETES_DESCRIPTION in ("", None) else cfg.KUBERNETES_DESCRIPTION
    cfg.KUBERNETES_DESCRIPTION = p.get_argument("Describe this Kubernetes environment:", desc_default.replace('"', ""))
    p.say(SEP)
    while True:
        v = p.get_argument("Hostname of the master:", cfg.RANCHER_MASTER_HOSTNAME.replace('"', ""))
        if valid_hostname(v):
            break
        p.say("error: Enter a valid hostname or leave blank to use the default.")
        p.say("    Must start with a letter and can only include letters and numbers")
    cfg.RANCHER_MASTER_HOSTNAME = v
    p.say(SEP)
    while True:
        v = p.get_argument("Enter a string to use for appending to hostnames of all the nodes:",
                           cfg.KUBERNETES_NODE_HOSTNAME_BEGINSWITH.replace('"', ""))
        if valid_hostname(v):
            break
        p.say("error: Enter a valid value or leave blank to use the default.")
        p.say("    Must start with a letter and can only include letters and numbers")
    cfg.KUBERNETES_NODE_HOSTNAME_BEGINSWITH = v
    p.say(SEP)
    # HARD LIMIT: 1-9 nodes allowed only since this setup has no HA (setup.sh:297)
    while True:
        v = p.get_argument("How many nodes should this Kubernetes cluster have:", str(cfg.KUBERNETES_NUMBER_OF_NODES))
        if valid_node_count(v):
            break
        p.say("error: Enter a valid value (number between 1-9) or leave blank to use the default.")
    cfg.KUBERNETES_NUMBER_OF_NODES = int(v)
    p.say(SEP)
    cfg.RANCHER_MASTER_NETWORKS = _ask_networks(
        p, prov, "What networks should the master be a part of, provide comma separated values:", cfg.RANCHER_MASTER_NETWORKS)
    p.say(SEP)
    cfg.KUBERNETES_NODE_NETWORKS = _ask_networks(
        p, prov, "What networks should the nodes be a part of, provide comma separated values:", cfg.KUBERNETES_NODE_NETWORKS)
    p.say(SEP)
    cfg.HOST_PACKAGE = _ask_package(p, prov, cfg.HOST_PACKAGE).replace('"', "")
    return cfg


def verify_config(cfg: ClusterConfig, p: Prompter, backend: str = "local") -> None:
    """verifyConfig (setup.sh:452-483): summary, then loop until yes/no; `no` exits 0."""
    p.say("#" * 80)
    p.say("Verify that the following configuration is correct:")
    p.say("")
    p.say(f"Name of kubernetes environment: {cfg.KUBERNETES_NAME}")
    p.say(f"Kubernetes environment description: {cfg.KUBERNETES_DESCRIPTION}")
    p.say(f"Master hostname: {cfg.RANCHER_MASTER_HOSTNAME}")
    p.say(f"All node hostnames will start with: {cfg.KUBERNETES_NODE_HOSTNAME_BEGINSWITH}")
    p.say(f"Kubernetes environment will have {cfg.KUBERNETES_NUMBER_OF_NODES} nodes")
    p.say(f"Master server will be part of these networks: {cfg.RANCHER_MASTER_NETWORKS}")
    p.say(f"Kubernetes nodes will be a part of these networks: {cfg.KUBERNETES_NODE_NETWORKS}")
    p.say(f"This package will be used for all the hosts: {cfg.HOST_PACKAGE}")
    p.say("")
    p.say("Make sure the above information is correct before answering:")
    cli = "triton" if backend == "triton" else "./tk8s"
    p.say(f'    to view list of networks call "{cli} networks -l"')
    p.say(f'    to view list of packages call "{cli} packages -l"')
    p.say("WARN: Make sure that the nodes and master are part of networks that can communicate with "
          "each other and this system from which the setup is running.")
    while True:
        yn = p.read("Is the above config correct (yes | no)? ").strip()
        if yn == "yes":
            return
        if yn == "no":
            raise WizardAbort(0)
        p.say("Please answer yes or no.")


# ---- non-interactive answers -----------------------------------------------------------
ANSWER_KEYS = ["name", "description", "master_hostname", "node_prefix", "nodes",
               "master_networks", "node_networks", "package", "confirm"]


def _index_of(rows: list, key) -> str:
    """Map a name/id/1-based index to the index string the prompt expects."""
    if key is None or key == "":
        return ""
    s = str(key)
    if s.isdigit():
        return s
    for i, r in enumerate(rows, 1):
        if s in (r.name, r.id):
            return str(i)
    raise ValueError(f"unknown option {s!r}; choose one of {[r.name for r in rows]}")


def answers_to_script(answers: dict, prov: Provider) -> list[str]:
    """Turn an answers mapping into the raw line sequence the prompts consume ("" = default)."""
    a = {k.lower(): v for k, v in answers.items()}
    nets = prov.networks()
    pkgs = prov.packages()

    def netlist(v) -> str:
        if v is None or v == "":
            return ""
        items = v if isinstance(v, (list, tuple)) else str(v).split(",")
        return ",".join(_index_of(nets, x) for x in items)

    return [
        str(a.get("name", "") or ""),
        str(a.get("description", "") or ""),
        str(a.get("master_hostname", "") or ""),
        str(a.get("node_prefix", "") or ""),
        str(a.get("nodes", "") or ""),
        netlist(a.get("master_networks")),
        netlist(a.get("node_networks")),
        _index_of(pkgs, a.get("package")),
        str(a.get("confirm", "yes")),
    ]


def load_answers(path: str) -> dict:
    text = Path(path).read_text()
    if path.endswith(".json"):
        return json.loads(text)
    import yaml

    data = yaml.safe_load(text)
    if isinstance(data, list):
        return dict(zip(ANSWER_KEYS, data))
    return dict(data or {})


def run_wizard(cfg: ClusterConfig, prov: Provider, answers: dict | None = None,
               inp: TextIO | None = None, out: TextIO | None = None) -> ClusterConfig:
    script = answers_to_script(answers, prov) if answers is not None else None
    p = Prompter(inp, out if out is not None else (io.StringIO() if script is not None and out is None else None), script)
    get_config_from_user(cfg, prov, p)
    verify_config(cfg, p, backend=prov.name)
    return cfg
