"""YAML loading through libyaml when the C extension is present (5-10x faster than the pure
Python loader; the playbook engine parses every role file on each bring-up)."""
from __future__ import annotations

import yaml

_Loader = getattr(yaml, "CSafeLoader", yaml.SafeLoader)


def load(text: str):
    return yaml.load(text, Loader=_Loader)  # noqa: S506 - CSafeLoader/SafeLoader only


def load_all(text: str):
    return yaml.load_all(text, Loader=_Loader)  # noqa: S506
