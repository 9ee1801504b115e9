"""httpserver.Router matches plain segment patterns without a regex and compiles the others on
first use (compiling the control plane's ~120 routes up front was 3.8 ms of its start on the
MI355X host). It must answer as trying every route's regex in order would -- with dots in
literal segments taken literally."""
from __future__ import annotations

import re
from urllib.parse import unquote

import pytest

from tritonk8ssupervisor_amd.controlplane.httpserver import HttpError, Router, _literal_prefix, _segments


@pytest.mark.parametrize("pattern,prefix", [
    (r"/(ping|healthz)?", "/"), (r"/api/?", "/api"), (r"/v1/kv/(?P<key>.+)", "/v1/kv/"),
    (r"/apis/metrics.k8s.io/v1beta1/?", "/apis/metrics"), (r"/api/v1/nodes", "/api/v1/nodes"),
    (r"/a+b", "/a"), (r"/x{2}", "/"), (r"/p*q", "/"), (r"/\.well-known", "/"), (r"/a[bc]", "/a"),
])
def test_literal_prefix(pattern, prefix):
    assert _literal_prefix(pattern) == prefix
    assert all(m.startswith(prefix) for m in ("/", "/api", "/aab") if re.fullmatch(pattern, m))


def _eager(routes, method, path):
    allowed = False
    for m, _, pat, _, h, _ in routes:
        mt = re.compile("^" + re.sub(r"\.(?!\+)", r"\\.", pat) + "$").match(path)
        if mt:
            if m == method or (m == "GET" and method == "HEAD"):
                return h, {k: unquote(v) for k, v in mt.groupdict().items()}
            allowed = True
    return 405 if allowed else 404


def test_the_control_planes_routes_answer_as_eager_matching(tmp_path):
    from tritonk8ssupervisor_amd.controlplane.server import ControlPlane

    cp = ControlPlane("127.0.0.1", 0, str(tmp_path), 5.0, None, 0, 0)
    assert all(r[3] is None for r in cp.router.routes)  # nothing compiled up front
    assert sum(_segments(r[2]) is None for r in cp.router.routes) <= 4  # nearly all are plain segments
    paths = ["/", "/ping", "/healthz", "/version", "/metrics", "/api", "/api/", "/api/v1", "/api/v1/nodes",
             "/api/v1/nodes/x", "/api/v1/nodes/x/status", "/apis/apps/v1", "/apis/metrics.k8s.io/v1beta1",
             "/apis/metricsXk8s.io/v1beta1", "/v1/kv/a/b/c", "/v1/cluster/wait", "/v1/scripts/t:1:s",
             "/r/projects/1a7/kubernetes/api/v1/namespaces/default/pods", "/r/projects/1a7/kubernetes-dashboard:9090",
             "/api/v1/namespaces/kube-system/pods/p/log", "/api/v1/namespaces/ns/pods/p/status",
             "/apis/batch/v1/namespaces/ns/jobs/j", "/openapi/v3/apis/apps/v1", "/v2-beta/projects/1a7", "/nope",
             "/api/v1/watch/pods", "/apis/apps/v1/namespaces/kube-system/daemonsets", "/api/v1/nodes/",
             "/apis/apps/v1/namespaces/ns/deployments/d/scale", "/apis/apps/v1/namespaces/ns/jobs/d/scale",
             "/api/v1/namespaces//pods", "/apis//v1/x", "/v1/kv/", "/api/v1/", "/apis/apps/", "/apis/apps/v1/",
             "/r/projects/1a7/kubernetes/apis/metrics.k8s.io/v1beta1/", "/openapi/v3/api/v1", "no-slash",
             "/api/v1/nodes/a%2Fb", "/v1/kv/a%20b/c"]
    for method in ("GET", "POST", "PUT", "DELETE", "PATCH", "HEAD"):
        for path in paths:
            try:
                got = cp.router.match(method, path)
            except HttpError as e:
                got = e.status
            want = _eager(cp.router.routes, method, path)
            assert got == want, (method, path)


def test_a_route_added_later_still_matches_in_order():
    r = Router()
    r.add("GET", r"/a/(?P<x>[^/]+)", "first")
    r.add("GET", r"/a/b", "second")
    assert r.match("GET", "/a/b") == ("first", {"x": "b"})
    with pytest.raises(HttpError) as e:
        r.match("POST", "/a/b")
    assert e.value.status == 405


@pytest.mark.parametrize("pattern,spec", [
    (r"/api/v1/nodes", ((("lit", "api"), ("lit", "v1"), ("lit", "nodes")), False)),
    (r"/api/?", ((("lit", "api"),), True)),
    (r"/v1/kv/(?P<key>.+)", ((("lit", "v1"), ("lit", "kv"), ("rest", "key")), False)),
    (r"/a/(?P<k>x|y)/(?P<n>[^/]+)", ((("lit", "a"), ("choice", "k", frozenset({"x", "y"})), ("param", "n")), False)),
    (r"/(ping|healthz)?", None), (r"/o/(?P<gv>api/[^/]+|apis/[^/]+/[^/]+)", None), (r"/x/(?P<r>.+)/?", None),
])
def test_segment_specs(pattern, spec):
    assert _segments(pattern) == spec


def test_routes_added_after_a_match_are_seen():
    r = Router()
    r.add("GET", r"/a/b", "ab")
    assert r.match("GET", "/a/b")[0] == "ab"
    r.add("GET", r"/c/(?P<x>[^/]+)", "c")
    r.add("GET", r"/(ping|healthz)?", "ping")
    assert r.match("GET", "/c/1") == ("c", {"x": "1"})
    assert r.match("GET", "/healthz")[0] == "ping" and r.match("GET", "/")[0] == "ping"


def test_random_paths_route_as_eager_matching(tmp_path):
    """Property check over generated paths: the lazy/segment router and trying every route's regex
    in order (dots in literal segments taken literally) pick the same handler and groups, or fail
    with the same status."""
    from hypothesis import given, settings, strategies as st

    from tritonk8ssupervisor_amd.controlplane.server import ControlPlane

    cp = ControlPlane("127.0.0.1", 0, str(tmp_path), 5.0, None, 0, 0)
    words = st.sampled_from(["api", "apis", "v1", "v1beta1", "apps", "batch", "namespaces", "kube-system", "default",
                             "pods", "nodes", "status", "log", "exec", "scale", "deployments", "jobs", "watch", "kv",
                             "metrics.k8s.io", "metricsXk8sXio", "r", "projects", "1a7", "kubernetes", "openapi", "v3",
                             "v2-beta", "registrationtokens", "scripts", "env", "kubectl", "cluster", "wait", "events",
                             "x:y", "", "%2F", "ping", "healthz", "version"])

    @settings(max_examples=400, deadline=None)
    @given(st.lists(words, min_size=0, max_size=9), st.booleans(), st.sampled_from(["GET", "POST", "PUT", "DELETE", "HEAD"]))
    def check(parts, trailing, method):
        path = "/" + "/".join(parts) + ("/" if trailing and parts else "")
        try:
            got = cp.router.match(method, path)
        except HttpError as e:
            got = e.status
        assert got == _eager(cp.router.routes, method, path), (method, path)

    check()
