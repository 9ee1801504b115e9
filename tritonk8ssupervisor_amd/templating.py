"""Templating for the playbook engine (``{{ expr }}`` templates and ``when:`` tests).

Two tiers with one semantics:

* fast path -- a Jinja subset parsed with Python's ``ast`` and evaluated by a whitelist
  interpreter (no ``eval``): literals, names, attribute/subscript access (dicts by key),
  comparisons, ``in``/``not in``, ``and``/``or``/``not``, arithmetic, a few string/dict methods,
  filters ``x | f(args)`` (b64decode, b64encode, replace, default/d, int, float, string, lower,
  upper, trim, to_json, from_json, length, bool, join, list, first, last, basename, dirname) and
  the Ansible tests. It costs microseconds per expression, which matters on a bring-up that
  renders hundreds of them in ~30 ms (jinja2 alone takes ~44 ms to import and ~1.4 ms to
  compile one expression);
* anything outside the subset (other filters such as ``map``/``sum``/``regex_replace``,
  ``lookup(...)``, statements) is rendered by real Jinja2 in a sandbox with the Ansible filters,
  tests and lookups registered -- so nothing silently diverges or fails for lack of support.
  tests/test_playbook.py renders every template the shipped roles contain through both tiers
  and requires identical results.

Reference playbooks rely on e.g. ``project_id['content'] | b64decode | replace('\\n', '')``
(ansible/roles/rancherhost/tasks/main.yml:15) and ``'rancher-agent' not in containers.stdout``
(rancherhost/tasks/main.yml:9).
"""
from __future__ import annotations

import _ast  # the node classes and the parse flag; the ``ast`` module (unparse) only for messages
import json
import os
import re


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
    import base64

    return base64.b64decode(s).decode(errors="replace")


def _b64encode(s):
    import base64

    return base64.b64encode(str(s).encode()).decode()


def _unparse(node) -> str:
    import ast

    return ast.unparse(node)


def _default(v, d="", boolean=False):
    if isinstance(v, _UndefinedValue) or (boolean and not v):
        return d
    return v


FILTERS = {
    "b64decode": _b64decode,
    "b64encode": _b64encode,
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
            raise _Unsupported(f"unsupported expression element {type(node).__name__}")
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

    def _get(self, base, key, node):
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
            raise Undefined(f"{_unparse(node)} has no attribute/key {key!r}")
        return _UndefinedValue(f"{_unparse(node)}.{key}")

    def v_Attribute(self, n):
        base = self(n.value)
        if isinstance(base, (str, dict, list)) and n.attr in _ALLOWED_METHODS.get(type(base), ()):
            if not (isinstance(base, dict) and n.attr in base):
                return getattr(base, n.attr)
        return self._get(base, n.attr, n.value)

    def v_Subscript(self, n):
        base = self(n.value)
        key = self(n.slice)
        return self._get(base, key, n.value)

    def _lenient(self, node):
        saved, self.strict = self.strict, False
        try:
            return self(node)
        finally:
            self.strict = saved

    def v_Call(self, n):
        if isinstance(n.func, _ast.Name) and n.func.id == "__filter__":
            name = n.args[0].value
            if name not in FILTERS:
                raise _Unsupported(f"unknown filter {name!r}")
            val = self._lenient(n.args[1])
            if isinstance(val, _UndefinedValue) and name not in ("default", "d"):
                if self.strict:
                    raise Undefined(f"'{val.name}' is undefined")
                return val  # propagate to the enclosing (strict) expression
            return FILTERS[name](val, *[self(a) for a in n.args[2:]])
        if isinstance(n.func, _ast.Name) and n.func.id == "__test__":
            return _jinja_test(n.args[0].value, self._lenient(n.args[1]))
        if isinstance(n.func, _ast.Name) and n.func.id not in self.vars:
            raise _Unsupported(f"function {n.func.id}()")  # lookup(), query(), range() ...
        fn = self(n.func)
        if not callable(fn) or getattr(fn, "__self__", None) is None:
            raise TemplateError(f"call of {_unparse(n.func)} not allowed")
        return fn(*[self(a) for a in n.args])

    def v_UnaryOp(self, n):
        v = self(n.operand)
        if isinstance(n.op, _ast.Not):
            return not v
        if isinstance(n.op, _ast.USub):
            return -v
        raise TemplateError("unsupported unary op")

    def v_BoolOp(self, n):
        if isinstance(n.op, _ast.And):
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
        ops = {_ast.Add: lambda: a + b, _ast.Sub: lambda: a - b, _ast.Mult: lambda: a * b,
               _ast.Div: lambda: a / b, _ast.Mod: lambda: a % b, _ast.FloorDiv: lambda: a // b}
        f = ops.get(type(n.op))
        if f is None:
            raise TemplateError("unsupported operator")
        return f()

    def v_Compare(self, n):
        left = self(n.left)
        for op, comp in zip(n.ops, n.comparators):
            right = self(comp)
            ok = {_ast.Eq: lambda: left == right, _ast.NotEq: lambda: left != right, _ast.Lt: lambda: left < right,
                  _ast.LtE: lambda: left <= right, _ast.Gt: lambda: left > right, _ast.GtE: lambda: left >= right,
                  _ast.In: lambda: left in right, _ast.NotIn: lambda: left not in right,
                  _ast.Is: lambda: left is right, _ast.IsNot: lambda: left is not right}[type(op)]()
            if not ok:
                return False
            left = right
        return True

    def v_IfExp(self, n):
        return self(n.body) if self(n.test) else self(n.orelse)


_KEYWORDS = {"and", "or", "not", "in", "is", "if", "else", "True", "False", "None"}
_OPEN = {")": "(", "]": "[", "}": "{"}


def _operand_start(out: list[str]) -> int:
    """Index in ``out`` where the postfix expression ending at ``out[-1]`` starts
    (atom followed by ``.name`` / ``[...]`` / ``(...)`` trailers)."""
    i = len(out) - 1
    while i >= 0:
        t = out[i]
        if t in _OPEN:
            depth = 0
            while i >= 0:
                if out[i] in _OPEN:
                    depth += 1
                elif out[i] in _OPEN.values():
                    depth -= 1
                    if depth == 0:
                        break
                i -= 1
            if i < 0:
                raise TemplateError("unbalanced brackets before filter")
        elif not (t[:1].isalnum() or t[:1] in "_'\"") or t in _KEYWORDS - {"True", "False", "None"}:
            raise TemplateError(f"filter/test without an operand near {t!r}")
        # out[i] is the first token of this piece; a trailer continues the chain
        if i > 1 and out[i - 1] == ".":
            i -= 2
            continue
        prev = out[i - 1] if i > 0 else ""
        if out[i] in _OPEN.values() and prev and (prev in _OPEN or ((prev[:1].isalpha() or prev[:1] == "_")
                                                                    and prev not in _KEYWORDS)):
            i -= 1
            continue
        return i
    raise TemplateError("filter/test without an operand")


def _rewrite(expr: str) -> str:
    """Jinja filters/tests -> calls the evaluator understands, with Jinja precedence:
    ``x | f(a) + 1`` -> ``__filter__('f', x, a) + 1``; ``x is not defined`` -> ``not __test__('defined', x)``."""
    import io
    import tokenize  # only on a rewrite-cache miss (_rewritten)

    try:
        toks = [t for t in tokenize.generate_tokens(io.StringIO(expr).readline)
                if t.type not in (tokenize.NEWLINE, tokenize.NL, tokenize.ENDMARKER, tokenize.INDENT, tokenize.DEDENT)]
    except (tokenize.TokenError, IndentationError, SyntaxError) as e:
        raise TemplateError(f"cannot tokenize {expr!r}: {e}") from e
    words = [t.string for t in toks]
    out: list[str] = []
    i = 0
    while i < len(words):
        w = words[i]
        nxt = words[i + 1] if i + 1 < len(words) else ""
        if w == "|" and nxt and (nxt[:1].isalpha() or nxt[:1] == "_"):
            start = _operand_start(out)
            operand = " ".join(out[start:])
            del out[start:]
            name, i = nxt, i + 2
            args = ""
            if i < len(words) and words[i] == "(":
                depth, j = 0, i
                while j < len(words):
                    depth += words[j] == "(" or words[j] in ("[", "{")
                    depth -= words[j] == ")" or words[j] in ("]", "}")
                    if depth == 0:
                        break
                    j += 1
                args = _rewrite(" ".join(words[i + 1:j])) if j > i + 1 else ""
                i = j + 1
            out += ["__filter__", "(", repr(name), ",", "(", operand, ")"] + ([",", args] if args.strip() else []) + [")"]
            continue
        if w == "is" and out:
            neg = nxt == "not"
            k = i + 2 if neg else i + 1
            if k < len(words):
                start = _operand_start(out)
                operand = " ".join(out[start:])
                del out[start:]
                name = words[k]
                out += (["not"] if neg else []) + ["__test__", "(", repr(name.lower()), ",", "(", operand, ")", ")"]
                i = k + 1
                continue
        if w == "~":
            w = "+"  # Jinja string concatenation (string operands)
        out.append(w)
        i += 1
    return " ".join(out)


def _jinja_test(name: str, v: Any) -> bool:
    undef = isinstance(v, _UndefinedValue)
    if name == "defined":
        return not undef
    if name == "undefined":
        return undef
    if undef:
        raise Undefined(f"'{v.name}' is undefined")
    r = v if isinstance(v, dict) else {}
    table = {
        "none": lambda: v is None, "string": lambda: isinstance(v, str),
        "number": lambda: isinstance(v, (int, float)) and not isinstance(v, bool),
        "mapping": lambda: isinstance(v, dict), "sequence": lambda: isinstance(v, (list, tuple, str)),
        "iterable": lambda: isinstance(v, (list, tuple, str, dict)),
        "true": lambda: v is True, "false": lambda: v is False, "boolean": lambda: isinstance(v, bool),
        "failed": lambda: bool(r.get("failed")), "failure": lambda: bool(r.get("failed")),
        "succeeded": lambda: not r.get("failed"), "success": lambda: not r.get("failed"),
        "changed": lambda: bool(r.get("changed")), "skipped": lambda: bool(r.get("skipped")),
    }
    if name not in table:
        raise _Unsupported(f"unknown test {name!r}")
    return table[name]()


class _Unsupported(TemplateError):
    """Outside the fast subset: hand the expression to real Jinja2."""


def evaluate(expr: str, variables: dict, strict: bool = True) -> Any:
    try:
        return _evaluate_subset(expr, variables, strict)
    except _Unsupported:
        return jinja_evaluate(expr, variables, strict)


_REWRITE_VERSION = 1  # bump when _rewrite / _pyify change what they produce
_PARSED: dict[str, Any] = {}  # expression text -> its parsed tree (or the _Unsupported it raised)


_REWRITES = None  # expression text -> rewritten Python source, kept across processes


def _rewritten(expr: str) -> str:
    """_rewrite(_pyify(expr)), remembered across bring-ups (utils/pcache.py): the rewrite needs
    the stdlib tokenizer, whose first use in a process compiles a large regex."""
    global _REWRITES
    if _REWRITES is None:
        from .utils.pcache import PersistentCache

        _REWRITES = PersistentCache(f"jinja-rewrite-{_REWRITE_VERSION}")
    src = _REWRITES.get(expr)
    if src is None:
        src = _rewrite(_pyify(expr.strip()))
        _REWRITES.put(expr, src)
    return src


def _parse(expr: str):
    """The rewritten, parsed form of an expression, computed once per distinct text: a play
    evaluates the same few expressions for every host (the tokenizer is most of the cost)."""
    hit = _PARSED.get(expr)
    if hit is None:
        try:
            src = _rewritten(expr)
            hit = compile(src or "None", "<template>", "eval", _ast.PyCF_ONLY_AST)  # = ast.parse(mode="eval")
        except TemplateError as e:
            hit = _Unsupported(str(e))
        except SyntaxError as e:
            hit = _Unsupported(f"cannot parse {expr!r}: {e}")
        if len(_PARSED) >= 4096:
            _PARSED.clear()
        _PARSED[expr] = hit
    if isinstance(hit, _Unsupported):
        raise _Unsupported(str(hit))
    return hit


def _evaluate_subset(expr: str, variables: dict, strict: bool = True) -> Any:
    tree = _parse(expr)
    val = _Eval(variables, strict)(tree)
    if isinstance(val, _UndefinedValue) and strict:
        raise Undefined(f"'{val.name}' is undefined")
    return val


# ---- real Jinja2 (sandboxed) for everything outside the subset ----------------------------------
_JINJA = {}


def _flatten(xs, levels=None):
    out = []
    for x in xs:
        if isinstance(x, (list, tuple)) and (levels is None or levels > 0):
            out.extend(_flatten(x, None if levels is None else levels - 1))
        else:
            out.append(x)
    return out


def _jinja_env(strict: bool):
    env = _JINJA.get(strict)
    if env is not None:
        return env
    import jinja2
    import jinja2.sandbox

    env = jinja2.sandbox.ImmutableSandboxedEnvironment(
        undefined=jinja2.StrictUndefined if strict else jinja2.Undefined, keep_trailing_newline=True)
    for name in ("b64decode", "b64encode", "to_json", "from_json", "bool", "basename", "dirname"):
        env.filters[name] = FILTERS[name]
    env.filters.update({
        "regex_replace": lambda s, pat, rep="": re.sub(pat, rep, str(s)),
        "regex_search": lambda s, pat: (m.group(0) if (m := re.search(pat, str(s))) else None),
        "dict2items": lambda d: [{"key": k, "value": v} for k, v in d.items()],
        "items2dict": lambda xs: {x["key"]: x["value"] for x in xs},
        "combine": lambda *ds: {k: v for d in ds for k, v in d.items()},
        "to_yaml": lambda v: __import__("yaml").safe_dump(v, default_flow_style=False),
        "from_yaml": lambda s: __import__("yaml").safe_load(s),
        "quote": lambda s: __import__("shlex").quote(str(s)),
        "flatten": _flatten,
    })
    for name in ("changed", "failed", "failure", "succeeded", "success", "skipped"):
        env.tests[name] = (lambda n: (lambda v: _jinja_test(n, v)))(name)

    @jinja2.pass_context
    def lookup(ctx, kind, *terms, **kw):
        out = []
        for t in terms:
            if kind == "file":
                out.append(open(os.path.expanduser(str(t))).read().rstrip("\n"))
            elif kind == "template":
                with open(os.path.expanduser(str(t))) as f:
                    out.append(render_text(f.read(), dict(ctx.get_all())))
            elif kind == "env":
                out.append(os.environ.get(str(t), ""))
            else:
                raise TemplateError(f"lookup plugin {kind!r} is not supported")
        return out[0] if len(out) == 1 else ",".join(out)

    env.globals["lookup"] = lookup
    env.globals["query"] = lambda kind, *t: [lookup(kind, x) for x in t]
    _JINJA[strict] = env
    return env


def _jinja_errors():
    import jinja2
    import jinja2.exceptions

    return jinja2.exceptions.UndefinedError, (jinja2.exceptions.TemplateError, jinja2.exceptions.SecurityError)


def jinja_evaluate(expr: str, variables: dict, strict: bool = True) -> Any:
    undefined_error, errors = _jinja_errors()
    try:
        val = _jinja_env(strict).compile_expression(expr.strip(), undefined_to_none=False)(**variables)
    except undefined_error as e:
        raise Undefined(str(e)) from e
    except errors as e:
        raise TemplateError(f"{expr!r}: {e}") from e
    import jinja2

    if isinstance(val, jinja2.Undefined):
        if strict:
            raise Undefined(f"{expr!r} is undefined")
        return _UndefinedValue(expr.strip())
    return val


def render_text(text: str, variables: dict, strict: bool = True) -> str:
    """A whole template (statements included) through real Jinja2: file templates."""
    undefined_error, errors = _jinja_errors()
    try:
        return _jinja_env(strict).from_string(text).render(**variables)
    except undefined_error as e:
        raise Undefined(str(e)) from e
    except errors as e:
        raise TemplateError(str(e)) from e


_TPL = re.compile(r"\{\{(.*?)\}\}", re.S)


def _single(text: str):
    """The match when ``text`` is exactly ONE ``{{ expr }}`` (then the value keeps its type);
    ``{{ a }}{{ b }}`` is two templates concatenated, not one expression."""
    m = _TPL.fullmatch(text.strip())
    return m if m and "{{" not in m.group(1) and "}}" not in m.group(1) else None


def render(value: Any, variables: dict, strict: bool = True) -> Any:
    """Render `{{ }}` templates in strings (recursively in lists/dicts). A string that is a single
    template returns the native value (so lists/dicts survive)."""
    if isinstance(value, list):
        return [render(v, variables, strict) for v in value]
    if isinstance(value, dict):
        return {k: render(v, variables, strict) for k, v in value.items()}
    if not isinstance(value, str) or ("{{" not in value and "{%" not in value):
        return value
    if "{%" in value:  # statements: real Jinja2
        return render_text(value, variables, strict)
    m = _single(value)
    if m:
        out = evaluate(m.group(1), variables, strict)
    else:
        out = _TPL.sub(lambda mm: _to_str(evaluate(mm.group(1), variables, strict)), value)
    # a variable whose value is itself a template (group_vars: `x: "{{ y }}/z"`) renders in turn,
    # as Ansible's lazy templating does (bounded: a self-reference cannot loop)
    for _ in range(8):
        if not (isinstance(out, str) and "{{" in out):
            break
        m = _single(out)
        out = evaluate(m.group(1), variables, strict) if m else \
            _TPL.sub(lambda mm: _to_str(evaluate(mm.group(1), variables, strict)), out)
    return out


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
    m = _single(s)
    if m:
        s = m.group(1)
    v = evaluate(s, variables)
    if isinstance(v, str):
        return v.strip().lower() in ("1", "true", "yes", "on")
    return bool(v)
