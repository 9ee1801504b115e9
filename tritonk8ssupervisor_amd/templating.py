"""Jinja2 subset used by the playbook engine (``{{ expr }}`` templates and ``when:`` tests).

Expressions are parsed with Python's ``ast`` and evaluated by a whitelist interpreter — no
``eval``. Supported: literals, names, attribute/subscript access (dicts by key), comparisons,
``in``/``not in``, ``and``/``or``/``not``, arithmetic, a few string/dict methods, and filters
``x | f(args)``: b64decode, b64encode, replace, default/d, int, float, string, lower, upper,
trim, to_json, from_json, length, bool, join, list, first, last, basename, dirname.

Reference playbooks rely on e.g. ``project_id['content'] | b64decode | replace('\\n', '')``
(ansible/roles/rancherhost/tasks/main.yml:15) and ``'rancher-agent' not in containers.stdout``
(rancherhost/tasks/main.yml:9).
"""
from __future__ import annotations

import ast
import base64
import json
import os
import re
from typing import Any


class TemplateError(ValueError):
    pass


class Undefined(TemplateError):
    pass


_ALLOWED_METHODS = {
    str: {"find", "startswith", "endswith", "replace", "strip", "split", "lower", "upper", "rstrip", "lstrip",
          "splitlines", "format", "count", "join"},
    dict: {"get", "keys", "values", "items"},
    list: {"index", "count"},
}


def _b64decode(s):
    return base64.b64decode(s).decode(errors="replace")


def _default(v, d="", boolean=False):
    if isinstance(v, _UndefinedValue) or (boolean and not v):
        return d
    return v


FILTERS = {
    "b64decode": _b64decode,
    "b64encode": lambda s: base64.b64encode(str(s).encode()).decode(),
    "replace": lambda s, a, b: str(s).replace(a, b),
    "default": _default,
    "d": _default,
    "int": lambda v, d=0: int(v) if str(v).strip().lstrip("-").isdigit() else d,
    "float": float,
    "string": str,
    "lower": lambda s: str(s).lower(),
    "upper": lambda s: str(s).upper(),
    "trim": lambda s: str(s).strip(),
    "to_json": lambda v: json.dumps(v),
    "from_json": lambda s: json.loads(s),
    "length": len,
    "count": len,
    "bool": lambda v: v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes", "on"),
    "join": lambda v, sep="": sep.join(map(str, v)),
    "list": list,
    "first": lambda v: v[0],
    "last": lambda v: v[-1],
    "basename": os.path.basename,
    "dirname": os.path.dirname,
}


class _UndefinedValue:
    def __init__(self, name):
        self.name = name

    def __bool__(self):
        return False

    def __repr__(self):
        return f"Undefined({self.name})"


def _split_filters(expr: str) -> list[str]:
    parts, depth, cur, quote = [], 0, [], None
    i = 0
    while i < len(expr):
        c = expr[i]
        if quote:
            cur.append(c)
            if c == "\\" and i + 1 < len(expr):
                cur.append(expr[i + 1])
                i += 1
            elif c == quote:
                quote = None
        elif c in "'\"":
            quote = c
            cur.append(c)
        elif c in "([{":
            depth += 1
            cur.append(c)
        elif c in ")]}":
            depth -= 1
            cur.append(c)
        elif c == "|" and depth == 0 and not (i + 1 < len(expr) and expr[i + 1] == "|"):
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(c)
        i += 1
    parts.append("".join(cur))
    return [p.strip() for p in parts]


_WORDS = re.compile(r"\b(true|false|none|True|False|None)\b")


def _sub_words(seg: str) -> str:
    return _WORDS.sub(lambda m: {"true": "True", "false": "False", "none": "None"}.get(m.group(1), m.group(1)), seg)


def _pyify(expr: str) -> str:
    """Jinja literals (true/false/none) -> Python, leaving quoted strings untouched."""
    res: list[str] = []
    seg: list[str] = []
    quote, prev = None, ""
    for c in expr:
        if quote:
            res.append("\\n" if c == "\n" else c)
            if c == quote and prev != "\\":
                quote = None
        elif c in "'\"":
            res.append(_sub_words("".join(seg)))
            seg = []
            res.append(c)
            quote = c
        else:
            seg.append(c)
        prev = c
    res.append(_sub_words("".join(seg)))
    return "".join(res)


class _Eval:
    def __init__(self, variables: dict, strict: bool):
        self.vars = variables
        self.strict = strict

    def __call__(self, node):
        m = getattr(self, "v_" + type(node).__name__, None)
        if m is None:
            raise TemplateError(f"unsupported expression element {type(node).__name__}")
        return m(node)

    def v_Expression(self, n):
        return self(n.body)

    def v_Constant(self, n):
        return n.value

    def v_Name(self, n):
        if n.id in self.vars:
            return self.vars[n.id]
        if self.strict:
            raise Undefined(f"'{n.id}' is undefined")
        return _UndefinedValue(n.id)

    def v_List(self, n):
        return [self(e) for e in n.elts]

    def v_Tuple(self, n):
        return tuple(self(e) for e in n.elts)

    def v_Dict(self, n):
        return {self(k): self(v) for k, v in zip(n.keys, n.values)}

    def _get(self, base, key, label):
        if isinstance(base, _UndefinedValue):
            if self.strict:
                raise Undefined(f"'{base.name}' is undefined")
            return _UndefinedValue(f"{base.name}.{key}")
        if isinstance(base, dict):
            if key in base:
                return base[key]
        elif isinstance(base, (list, tuple, str)) and isinstance(key, int):
            try:
                return base[key]
            except IndexError:
                pass
        if self.strict:
            raise Undefined(f"{label} has no attribute/key {key!r}")
        return _UndefinedValue(f"{label}.{key}")

    def v_Attribute(self, n):
        base = self(n.value)
        if isinstance(base, (str, dict, list)) and n.attr in _ALLOWED_METHODS.get(type(base), ()):
            if not (isinstance(base, dict) and n.attr in base):
                return getattr(base, n.attr)
        return self._get(base, n.attr, ast.unparse(n.value))

    def v_Subscript(self, n):
        base = self(n.value)
        key = self(n.slice)
        return self._get(base, key, ast.unparse(n.value))

    def v_Call(self, n):
        fn = self(n.func)
        if not callable(fn) or getattr(fn, "__self__", None) is None:
            raise TemplateError(f"call of {ast.unparse(n.func)} not allowed")
        return fn(*[self(a) for a in n.args])

    def v_UnaryOp(self, n):
        v = self(n.operand)
        if isinstance(n.op, ast.Not):
            return not v
        if isinstance(n.op, ast.USub):
            return -v
        raise TemplateError("unsupported unary op")

    def v_BoolOp(self, n):
        if isinstance(n.op, ast.And):
            v = True
            for e in n.values:
                v = self(e)
                if not v:
                    return v
            return v
        v = False
        for e in n.values:
            v = self(e)
            if v:
                return v
        return v

    def v_BinOp(self, n):
        a, b = self(n.left), self(n.right)
        ops = {ast.Add: lambda: a + b, ast.Sub: lambda: a - b, ast.Mult: lambda: a * b,
               ast.Div: lambda: a / b, ast.Mod: lambda: a % b, ast.FloorDiv: lambda: a // b}
        f = ops.get(type(n.op))
        if f is None:
            raise TemplateError("unsupported operator")
        return f()

    def v_Compare(self, n):
        left = self(n.left)
        for op, comp in zip(n.ops, n.comparators):
            right = self(comp)
            ok = {ast.Eq: lambda: left == right, ast.NotEq: lambda: left != right, ast.Lt: lambda: left < right,
                  ast.LtE: lambda: left <= right, ast.Gt: lambda: left > right, ast.GtE: lambda: left >= right,
                  ast.In: lambda: left in right, ast.NotIn: lambda: left not in right,
                  ast.Is: lambda: left is right, ast.IsNot: lambda: left is not right}[type(op)]()
            if not ok:
                return False
            left = right
        return True

    def v_IfExp(self, n):
        return self(n.body) if self(n.test) else self(n.orelse)


def evaluate(expr: str, variables: dict, strict: bool = True) -> Any:
    parts = _split_filters(expr.strip())
    try:
        tree = ast.parse(_pyify(parts[0]) or "None", mode="eval")
    except SyntaxError as e:
        raise TemplateError(f"cannot parse {parts[0]!r}: {e}") from e
    val = _Eval(variables, strict and len(parts) == 1)(tree)
    for f in parts[1:]:
        m = re.fullmatch(r"([A-Za-z_][A-Za-z0-9_]*)\s*(\((.*)\))?", f, re.S)
        if not m:
            raise TemplateError(f"bad filter {f!r}")
        name, args = m.group(1), m.group(3)
        if name not in FILTERS:
            raise TemplateError(f"unknown filter {name!r}")
        argv = []
        if args and args.strip():
            argv = list(_Eval(variables, strict)(ast.parse("(" + _pyify(args) + ",)", mode="eval")))
        if isinstance(val, _UndefinedValue) and name not in ("default", "d"):
            if strict:
                raise Undefined(f"'{val.name}' is undefined")
        val = FILTERS[name](val, *argv)
    if isinstance(val, _UndefinedValue) and strict:
        raise Undefined(f"'{val.name}' is undefined")
    return val


_TPL = re.compile(r"\{\{(.*?)\}\}", re.S)


def render(value: Any, variables: dict, strict: bool = True) -> Any:
    """Render `{{ }}` templates in strings (recursively in lists/dicts). A string that is a single
    template returns the native value (so lists/dicts survive)."""
    if isinstance(value, list):
        return [render(v, variables, strict) for v in value]
    if isinstance(value, dict):
        return {k: render(v, variables, strict) for k, v in value.items()}
    if not isinstance(value, str) or "{{" not in value:
        return value
    m = _TPL.fullmatch(value.strip())
    if m:
        return evaluate(m.group(1), variables, strict)
    return _TPL.sub(lambda mm: _to_str(evaluate(mm.group(1), variables, strict)), value)


def _to_str(v: Any) -> str:
    if isinstance(v, (dict, list)):
        return json.dumps(v)
    return "" if v is None else str(v)


def test(expr: Any, variables: dict) -> bool:
    """`when:` semantics: bare expressions, legacy `{{ }}` wrapped ones, lists (AND), bools."""
    if isinstance(expr, bool):
        return expr
    if isinstance(expr, list):
        return all(test(e, variables) for e in expr)
    s = str(expr).strip()
    m = _TPL.fullmatch(s)
    if m:
        s = m.group(1)
    v = evaluate(s, variables)
    if isinstance(v, str):
        return v.strip().lower() in ("1", "true", "yes", "on")
    return bool(v)
