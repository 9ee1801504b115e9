"""HCL subset: parser, ``${...}`` interpolation and the ``rancher.tf`` renderer.

Terraform is not available offline, so the repo ships its own small engine (provision.py)
that reads the same files the reference's Terraform reads: module definitions
(terraform/{master,host}/{main,vars}.tf, reference terraform/master/main.tf:1-36,
vars.tf:1-23) and the generated root config ``terraform/rancher.tf`` (setup.sh:162-198).

Supported: blocks with string labels, ``key = value`` attributes, strings with ``${...}``
interpolation (nested quotes inside, e.g. ``"${file("x")}"``), numbers, booleans, lists,
maps, ``#``/``//``/``/* */`` comments, HCL2 bare expressions (``list(string)``,
``when = destroy``). Interpolation functions: ``file(path)``, ``join(sep, list)``; references
``var.X``, ``TYPE.NAME.ATTR``, ``self.ATTR``. Duplicate attributes keep the LAST value and are
reported (the reference declares ``tags`` twice, terraform/master/main.tf:6-8 and 33-35).
"""
from __future__ import annotations

import os
import re
from pathlib import Path

from .utils.record import field, record as dataclass


class HclError(ValueError):
    pass


@dataclass
class Block:
    type: str
    labels: list[str]
    attrs: dict[str, Any] = field(default_factory=dict)
    blocks: list["Block"] = field(default_factory=list)
    duplicates: list[str] = field(default_factory=list)

    def children(self, type_: str) -> list["Block"]:
        return [b for b in self.blocks if b.type == type_]


# ---- tokenizer ---------------------------------------------------------------------------
_PUNCT = set("{}[]=,:()")


def _tokens(text: str) -> list[tuple[str, Any, int]]:
    toks: list[tuple[str, Any, int]] = []
    i, n, line = 0, len(text), 1
    while i < n:
        c = text[i]
        if c == "\n":
            line += 1
            i += 1
        elif c in " \t\r":
            i += 1
        elif c == "#" or text.startswith("//", i):
            while i < n and text[i] != "\n":
                i += 1
        elif text.startswith("/*", i):
            j = text.find("*/", i + 2)
            if j < 0:
                raise HclError(f"line {line}: unterminated comment")
            line += text.count("\n", i, j)
            i = j + 2
        elif c == '"':
            s, i2 = _read_string(text, i + 1, line)
            line += text.count("\n", i, i2)
            toks.append(("str", s, line))
            i = i2
        elif c in _PUNCT:
            toks.append((c, c, line))
            i += 1
        else:
            m = re.compile(r"[A-Za-z0-9_\-.]+").match(text, i)
            if not m:
                raise HclError(f"line {line}: unexpected character {c!r}")
            word = m.group(0)
            if re.fullmatch(r"-?\d+(\.\d+)?", word):
                toks.append(("num", float(word) if "." in word else int(word), line))
            elif word in ("true", "false"):
                toks.append(("bool", word == "true", line))
            else:
                toks.append(("ident", word, line))
            i = m.end()
    return toks


def _read_string(text: str, i: int, line: int) -> tuple[str, int]:
    """Read a string body starting after the opening quote; `${...}` may contain quotes."""
    out = []
    n = len(text)
    while i < n:
        c = text[i]
        if c == "\\" and i + 1 < n:
            nxt = text[i + 1]
            out.append({"n": "\n", "t": "\t", '"': '"', "\\": "\\"}.get(nxt, "\\" + nxt))
            i += 2
        elif c == '"':
            return "".join(out), i + 1
        elif text.startswith("${", i):
            depth, j = 0, i
            in_str = False
            while j < n:
                ch = text[j]
                if in_str:
                    if ch == "\\":
                        j += 1
                    elif ch == '"':
                        in_str = False
                elif ch == '"':
                    in_str = True
                elif ch == "{":
                    depth += 1
                elif ch == "}":
                    depth -= 1
                    if depth == 0:
                        break
                j += 1
            if j >= n:
                raise HclError(f"line {line}: unterminated interpolation")
            out.append(text[i : j + 1])
            i = j + 1
        else:
            out.append(c)
            i += 1
    raise HclError(f"line {line}: unterminated string")


# ---- parser ------------------------------------------------------------------------------
class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else ("eof", None, -1)

    def take(self, kind=None):
        tok = self.peek()
        if kind and tok[0] != kind:
            raise HclError(f"line {tok[2]}: expected {kind}, got {tok[0]} {tok[1]!r}")
        self.i += 1
        return tok

    def body(self, until: str | None) -> Block:
        blk = Block("body", [])
        while True:
            tok = self.peek()
            if tok[0] == "eof":
                if until:
                    raise HclError("unexpected end of file")
                return blk
            if until and tok[0] == until:
                self.take()
                return blk
            if tok[0] == ",":
                self.take()
                continue
            if tok[0] not in ("ident", "str"):
                raise HclError(f"line {tok[2]}: expected attribute or block, got {tok[1]!r}")
            name = self.take()[1]
            if self.peek()[0] in ("=", ":"):
                self.take()
                if name in blk.attrs:
                    blk.duplicates.append(name)
                blk.attrs[name] = self.value()
            else:
                labels = []
                while self.peek()[0] in ("str", "ident"):
                    labels.append(self.take()[1])
                self.take("{")
                inner = self.body("}")
                blk.blocks.append(Block(name, labels, inner.attrs, inner.blocks, inner.duplicates))

    def value(self):
        tok = self.peek()
        if tok[0] in ("str", "num", "bool"):
            return self.take()[1]
        if tok[0] == "ident" and self.peek(1)[0] == "(":  # function call / type constraint, e.g.
            name = self.take()[1]                           # list(string), join(",", x): kept as an
            depth, parts = 0, [name]                        # interpolation
            while True:
                t = self.take()
                if t[0] == "eof":
                    raise HclError(f"line {tok[2]}: unterminated call of {name}")
                depth += t[0] == "("
                depth -= t[0] == ")"
                parts.append(f'"{t[1]}"' if t[0] == "str" else str(t[1]).lower() if t[0] == "bool" else str(t[1]))
                if depth == 0:
                    break
            return "${" + "".join(parts) + "}"
        if tok[0] == "ident":  # bare reference (HCL2 style), kept as an interpolation
            return "${" + self.take()[1] + "}"
        if tok[0] == "[":
            self.take()
            items = []
            while self.peek()[0] != "]":
                items.append(self.value())
                if self.peek()[0] == ",":
                    self.take()
            self.take("]")
            return items
        if tok[0] == "{":
            self.take()
            m = self.body("}")
            if m.blocks:
                raise HclError(f"line {tok[2]}: blocks are not allowed inside a map value")
            return dict(m.attrs)
        raise HclError(f"line {tok[2]}: unexpected {tok[1]!r}")


_TOKENS_VERSION = 1
_TOKEN_MEMO: dict[str, list] = {}
_TOKEN_CACHE = None


def _cached_tokens(text: str) -> list[tuple[str, Any, int]]:
    """_tokens(text), remembered in this process and across runs in the parse cache
    (utils/pcache.py, keyed by the whole text: the character scanner was ~2-4 ms of every
    provision on the MI355X host). Only for the module files (parse_dir), which are the same in
    every workspace: the generated root (rancher.tf) names the workspace's own paths, and caching
    it would grow the table by one entry per workspace. Tokens are immutable tuples, so callers
    can share them."""
    global _TOKEN_CACHE
    toks = _TOKEN_MEMO.get(text)
    if toks is None:
        if _TOKEN_CACHE is None:
            from .utils.pcache import PersistentCache

            _TOKEN_CACHE = PersistentCache(f"hcl-tokens-{_TOKENS_VERSION}", limit=64)
        toks = _TOKEN_CACHE.get(text)
        if not isinstance(toks, list):
            toks = _tokens(text)
            _TOKEN_CACHE.put(text, toks)
        _TOKEN_MEMO[text] = toks
    return toks


def parse(text: str, cache: bool = False) -> Block:
    return _Parser(_cached_tokens(text) if cache else _tokens(text)).body(None)


def parse_file(path: str | os.PathLike, cache: bool = False) -> Block:
    return parse(Path(path).read_text(), cache)


def parse_dir(path: str | os.PathLike) -> Block:
    """Merge every *.tf in a directory (Terraform module semantics)."""
    root = Block("body", [])
    for f in sorted(Path(path).glob("*.tf")):
        b = parse_file(f, cache=True)
        root.attrs.update(b.attrs)
        root.blocks.extend(b.blocks)
        root.duplicates.extend(b.duplicates)
    return root


# ---- interpolation -----------------------------------------------------------------------
_INTERP = re.compile(r"\$\{")


def _split_interps(s: str) -> list[tuple[bool, str]]:
    """[(is_expr, text)] pieces of a string."""
    out, i = [], 0
    while True:
        m = _INTERP.search(s, i)
        if not m:
            if i < len(s):
                out.append((False, s[i:]))
            return out
        if m.start() > i:
            out.append((False, s[i : m.start()]))
        depth, j, in_str = 0, m.start() + 1, False
        while j < len(s):
            ch = s[j]
            if in_str:
                if ch == '"':
                    in_str = False
            elif ch == '"':
                in_str = True
            elif ch == "{":
                depth += 1
            elif ch == "}":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        out.append((True, s[m.start() + 2 : j].strip()))
        i = j + 1


def eval_expr(expr: str, ctx: dict) -> Any:
    expr = expr.strip()
    m = re.fullmatch(r'join\(\s*"([^"]*)"\s*,\s*(.+)\)', expr, re.S)
    if m:
        v = eval_expr(m.group(2), ctx)
        return m.group(1).join(map(str, v if isinstance(v, list) else [v]))
    m = re.fullmatch(r'file\(\s*"(.*)"\s*\)', expr, re.S)
    if m:
        p = Path(interpolate(m.group(1), ctx)).expanduser()
        base = ctx.get("__dir__")
        if not p.is_absolute() and base:
            p = Path(base) / p
        try:
            return p.read_text()
        except OSError as e:
            raise HclError(f"file({m.group(1)!r}): {e}") from e
    if len(expr) >= 2 and expr[0] == expr[-1] == '"':
        return interpolate(expr[1:-1], ctx)
    parts = expr.split(".")
    cur: Any = ctx
    for p in parts:
        if isinstance(cur, dict) and p in cur:
            cur = cur[p]
        elif isinstance(cur, list) and p.isdigit() and int(p) < len(cur):
            cur = cur[int(p)]
        else:
            raise HclError(f"unknown reference ${{{expr}}}")
    return cur


def interpolate(value: Any, ctx: dict) -> Any:
    """Resolve ``${...}`` in strings (recursively in lists/maps). A string that is exactly one
    interpolation keeps the referenced value's type (lists stay lists, as in HCL 0.9)."""
    if isinstance(value, list):
        return [interpolate(v, ctx) for v in value]
    if isinstance(value, dict):
        return {k: interpolate(v, ctx) for k, v in value.items()}
    if not isinstance(value, str) or "${" not in value:
        return value
    pieces = _split_interps(value)
    if len(pieces) == 1 and pieces[0][0]:
        return eval_expr(pieces[0][1], ctx)
    out = []
    for is_expr, text in pieces:
        if is_expr:
            v = eval_expr(text, ctx)
            out.append(",".join(map(str, v)) if isinstance(v, list) else str(v))
        else:
            out.append(text)
    return "".join(out)


# ---- renderer (updateTerraformConfig, setup.sh:162-198) -----------------------------------
def _q(s: str) -> str:
    return '"' + str(s).replace("\\", "\\\\").replace('"', '\\"') + '"'


def render_provider(kind: str, account: str, key_path: str, key_id: str, url: str) -> str:
    return (
        f'provider "{kind}" {{\n'
        f"    account = {_q(account)}\n"
        f'    key_material = "${{file("{key_path}")}}"\n'
        f"    key_id = {_q(key_id)}\n"
        f"    url = {_q(url)}\n"
        "}\n"
    )


def render_module(name: str, source: str, networks: list[str], pub_key_path: str, package: str,
                  image: str | None = None) -> str:
    nets = ",".join(_q(n) for n in networks)
    lines = [
        "",
        f'module "{name}" {{',
        f"    source = {_q(source)}",
        f"    hostname = {_q(name)}",
        f"    networks = [{nets}]",
        f'    root_authorized_keys = "${{file("{pub_key_path}")}}"',
    ]
    if image:
        lines.append(f"    image = {_q(image)}")
    lines += [f"    package = {_q(package)}", "}"]
    return "\n".join(lines) + "\n"


def render_root(provider_kind: str, account: str, key_path: str, pub_key_path: str, key_id: str, url: str,
                master: str, master_networks: list[str], hosts: list[str], host_networks: list[str],
                package: str, form: str = "tk8s") -> str:
    """``form`` "tk8s": modules terraform/{master,host} (resource tk8s_machine, the engine's own
    type); "compat": terraform/compat/{master,host} (terraform_data + the tk8s CLI), which stock
    Terraform plans and applies as well."""
    prefix = "compat/" if form == "compat" else ""
    out = render_provider(provider_kind, account, key_path, key_id, url) if form != "compat" else ""
    out += render_module(master, prefix + "master", master_networks, pub_key_path, package)
    for h in hosts:
        out += render_module(h, prefix + "host", host_networks, pub_key_path, package)
    return out
