"""Kubelet-style container environment: Service links and the downward API.

Service links (``enableServiceLinks``, on by default): for every Service of the pod's namespace
that exists when the pod starts, ``<NAME>_SERVICE_HOST`` / ``_SERVICE_PORT`` (+ ``_SERVICE_PORT_<PORT
NAME>``) and the Docker-link style ``<NAME>_PORT`` / ``<NAME>_PORT_<port>_<PROTO>[_PROTO|_PORT|_ADDR]``,
plus ``KUBERNETES_SERVICE_HOST``/``_PORT`` for the API server. The Guestbook frontend of the
reference's walkthrough finds its redis Services this way (docs/detailed.md:285-370). Ports are
the ones cluster processes actually use (utils.net.host_port).

``field_path`` resolves ``valueFrom.fieldRef`` (metadata.name/namespace/uid/labels['k']/
annotations['k'], spec.nodeName/serviceAccountName, status.podIP/hostIP).
"""
from __future__ import annotations

import re
from urllib.parse import urlsplit

from .net import host_port


def env_name(name: str) -> str:
    return re.sub(r"[^A-Z0-9_]", "_", name.upper())


def service_env(services: list[dict], api_base: str | None = None) -> dict[str, str]:
    env: dict[str, str] = {}
    for s in services:
        spec = s.get("spec", {})
        ip, ports = spec.get("clusterIP"), spec.get("ports") or []
        if not ip or ip == "None" or not ports:
            continue
        n = env_name(s["metadata"]["name"])
        first = ports[0]
        env[f"{n}_SERVICE_HOST"] = ip
        env[f"{n}_SERVICE_PORT"] = str(host_port(first["port"]))
        env[f"{n}_PORT"] = f"{first.get('protocol', 'TCP').lower()}://{ip}:{host_port(first['port'])}"
        for p in ports:
            hp, proto = host_port(p["port"]), p.get("protocol", "TCP")
            if p.get("name") and not str(p["name"]).isdigit():
                env[f"{n}_SERVICE_PORT_{env_name(str(p['name']))}"] = str(hp)
            pre = f"{n}_PORT_{p['port']}_{proto.upper()}"
            env[pre] = f"{proto.lower()}://{ip}:{hp}"
            env[f"{pre}_PROTO"] = proto.lower()
            env[f"{pre}_PORT"] = str(hp)
            env[f"{pre}_ADDR"] = ip
    if api_base:
        u = urlsplit(api_base if "://" in api_base else "http://" + api_base)
        env["KUBERNETES_SERVICE_HOST"] = u.hostname or ""
        env["KUBERNETES_SERVICE_PORT"] = str(u.port or 80)
    return env


_INDEXED = re.compile(r"^metadata\.(labels|annotations)\['([^']+)'\]$")


def field_path(pod: dict, path: str, pod_ip: str = "", host_ip: str = "") -> str:
    md, spec = pod.get("metadata", {}), pod.get("spec", {})
    m = _INDEXED.match(path)
    if m:
        return str(md.get(m.group(1), {}).get(m.group(2), ""))
    simple = {
        "metadata.name": md.get("name", ""), "metadata.namespace": md.get("namespace", ""),
        "metadata.uid": md.get("uid", ""), "spec.nodeName": spec.get("nodeName", ""),
        "spec.serviceAccountName": spec.get("serviceAccountName", "default"),
        "status.podIP": pod_ip, "status.hostIP": host_ip, "status.podIPs": pod_ip,
    }
    if path not in simple:
        raise ValueError(f"unsupported fieldRef fieldPath {path!r}")
    return str(simple[path])
