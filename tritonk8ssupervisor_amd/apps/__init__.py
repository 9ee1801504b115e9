"""Built-in stand-ins for the container images the reference's walkthroughs deploy.

Pods here are processes (agent/runtime.py), so there is no image to pull. A container that names
an image but no command runs the catalogue entry for that image's repository name: the apps of
the reference's acceptance demos (docs/detailed.md:261-370) -- Ghost from the dashboard, the
Guestbook (redis leader + followers + frontend) with kubectl -- plus a static page for
nginx/httpd. Each app binds the pod's own IP (``POD_IP``) and the port its image uses, shifted
by utils.net.host_port when the cluster runs without root.
"""
from __future__ import annotations

import sys

_CATALOGUE: dict[str, tuple[str, tuple[str, ...]]] = {
    "redis": ("redis", ()),
    "redis-master": ("redis", ()),
    "redis-leader": ("redis", ()),
    "gb-redisslave": ("redis", ("--follow", "redis-master,redis-leader")),
    "gb-redis-follower": ("redis", ("--follow", "redis-leader,redis-master")),
    "redis-slave": ("redis", ("--follow", "redis-master,redis-leader")),
    "redis-follower": ("redis", ("--follow", "redis-leader,redis-master")),
    "gb-frontend": ("guestbook", ()),
    "guestbook": ("guestbook", ()),
    "ghost": ("ghost", ()),
    "nginx": ("static", ()),
    "httpd": ("static", ()),
}


def image_name(image: str) -> str:
    """Repository name of an image reference: registry/path/NAME:tag@digest -> NAME."""
    return image.split("@", 1)[0].rsplit("/", 1)[-1].split(":", 1)[0].lower()


def resolve(image: str | None) -> list[str] | None:
    """argv that runs the built-in app for ``image`` (None if the image is not in the catalogue)."""
    if not image:
        return None
    hit = _CATALOGUE.get(image_name(image))
    if hit is None:
        return None
    module, extra = hit
    return [sys.executable, "-S", "-m", f"tritonk8ssupervisor_amd.apps.{module}", *extra]


def catalogue() -> dict[str, str]:
    return {name: module for name, (module, _) in _CATALOGUE.items()}
