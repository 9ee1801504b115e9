"""Shared helpers of the built-in apps: where to listen, where the other Services are."""
from __future__ import annotations

import json
import os
import urllib.request

from ..utils.k8senv import env_name
from ..utils.net import host_port


def bind_host() -> str:
    return os.environ.get("POD_IP") or "0.0.0.0"


def listen_port(default: int) -> int:
    v = os.environ.get("PORT")
    return int(v) if v else host_port(default)


def service_address(names, default_port: int) -> tuple[str, int] | None:
    """Address of the first Service in ``names``: the kubelet's Service env vars first (Services
    that existed when this pod started), then the API (``TK8S_K8S_API``) for later ones."""
    for n in names:
        e = env_name(n)
        h = os.environ.get(f"{e}_SERVICE_HOST")
        if h:
            return h, int(os.environ.get(f"{e}_SERVICE_PORT") or host_port(default_port))
    api = os.environ.get("TK8S_K8S_API")
    if not api:
        return None
    ns = os.environ.get("POD_NAMESPACE", "default")
    for n in names:
        try:
            with urllib.request.urlopen(f"{api}/api/v1/namespaces/{ns}/services/{n}", timeout=5) as r:
                s = json.loads(r.read())
            return s["spec"]["clusterIP"], host_port(int(s["spec"]["ports"][0]["port"]))
        except (OSError, ValueError, KeyError, IndexError):
            continue
    return None
