"""Minimal stand-in for ``ansible.module_utils.basic`` (Ansible is not installed offline).

Implements the contract a module sees from real Ansible: arguments arrive as
``{"ANSIBLE_MODULE_ARGS": {...}}`` (a file named by argv[1], or stdin), are checked and typed
against ``argument_spec`` (required, defaults, choices, str/int/float/bool/list/dict/path/raw),
``_ansible_check_mode`` sets ``check_mode``, and ``exit_json``/``fail_json`` print one JSON object
and exit 0/1. Used by tests/test_ansible_library.py only.
"""
import json
import os
import sys


class AnsibleModule:
    def __init__(self, argument_spec, supports_check_mode=False, **_):
        raw = open(sys.argv[1]).read() if len(sys.argv) > 1 else sys.stdin.read()
        args = json.loads(raw)["ANSIBLE_MODULE_ARGS"]
        self.check_mode = bool(args.pop("_ansible_check_mode", False))
        if self.check_mode and not supports_check_mode:
            self.exit_json(skipped=True, msg="remote module does not support check mode")
        unknown = set(args) - set(argument_spec)
        if unknown:
            self.fail_json(msg=f"Unsupported parameters: {', '.join(sorted(unknown))}")
        self.params = {}
        for k, spec in argument_spec.items():
            if k not in args or args[k] is None:
                if spec.get("required"):
                    self.fail_json(msg=f"missing required arguments: {k}")
                self.params[k] = spec.get("default")
                continue
            v = args[k]
            t = spec.get("type", "str")
            if t == "str":
                v = str(v)
            elif t == "int":
                v = int(v)
            elif t == "float":
                v = float(v)
            elif t == "bool":
                v = v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes", "on")
            elif t == "list":
                v = v if isinstance(v, list) else [x for x in str(v).split(",") if x]
                if spec.get("elements") == "str":
                    v = [str(x) for x in v]
            elif t == "dict":
                v = dict(v)
            elif t == "path":
                v = os.path.expanduser(str(v))
            if "choices" in spec and v not in spec["choices"]:
                self.fail_json(msg=f"value of {k} must be one of: {', '.join(map(str, spec['choices']))}, got: {v}")
            self.params[k] = v

    def exit_json(self, **kw):
        kw.setdefault("changed", False)
        print(json.dumps(kw, default=str))
        sys.exit(0)

    def fail_json(self, **kw):
        kw["failed"] = True
        print(json.dumps(kw, default=str))
        sys.exit(1)
