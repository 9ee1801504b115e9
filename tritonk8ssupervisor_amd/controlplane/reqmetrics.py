"""API server request metrics for ``/metrics``, named as kube-apiserver exports them:

* ``apiserver_request_total{verb,group,resource,subresource,code}`` -- a counter per request;
* ``apiserver_request_duration_seconds{verb,group,resource,subresource}`` -- a histogram of the
  time to the response's first byte (WATCH requests only start their stream, so they are left
  out of the histogram, as kube-apiserver does).

``verb`` is the Kubernetes one: LIST and WATCH for collection GETs, GET for one object, POST,
PUT, PATCH, DELETE. Requests outside the Kubernetes API (the Rancher API, the KV store, the
dashboard) count under ``resource="(other)"``. Classification is string slicing only -- it runs
on every request of the control plane.
"""
from __future__ import annotations

BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


def classify(method: str, path: str, watch: bool) -> tuple[str, str, str, str]:
    """(verb, group, resource, subresource) of a request path."""
    if path.startswith("/r/projects/"):
        parts = path.split("/", 5)  # '', r, projects, pid, kubernetes, rest
        path = "/" + parts[5] if len(parts) > 5 and parts[4] == "kubernetes" else "/"
    segs = [s for s in path.split("/") if s]
    if len(segs) >= 2 and segs[0] == "api":
        group, rest = "", segs[2:]
    elif len(segs) >= 3 and segs[0] == "apis":
        group, rest = segs[1], segs[3:]
    else:
        return method, "", "(other)", ""
    if len(rest) >= 3 and rest[0] == "namespaces":
        rest = rest[2:]
    if not rest:
        return method, group, "(discovery)" if method == "GET" else "(other)", ""
    resource = rest[0]
    sub = rest[2] if len(rest) > 2 else ""
    verb = method
    if method == "GET" and len(rest) == 1:
        verb = "WATCH" if watch else "LIST"
    return verb, group, resource, sub


class RequestMetrics:
    def __init__(self) -> None:
        self.counts: dict[tuple, int] = {}
        self.hist: dict[tuple, list] = {}  # key -> [bucket counts..., count, sum]

    def observe(self, method: str, path: str, watch: bool, code: int, seconds: float) -> None:
        verb, group, resource, sub = classify(method, path, watch)
        key = (verb, group, resource, sub)
        ck = key + (code,)
        self.counts[ck] = self.counts.get(ck, 0) + 1
        if verb == "WATCH":
            return
        h = self.hist.get(key)
        if h is None:
            h = self.hist[key] = [0] * (len(BUCKETS) + 2)
        for i, b in enumerate(BUCKETS):
            if seconds <= b:
                h[i] += 1
        h[-2] += 1
        h[-1] += seconds

    def lines(self) -> list[str]:
        out = ["# TYPE apiserver_request_total counter"]
        for (verb, group, res, sub, code), n in sorted(self.counts.items()):
            out.append(f'apiserver_request_total{{verb="{verb}",group="{group}",resource="{res}",'
                       f'subresource="{sub}",code="{code}"}} {n}')
        out.append("# TYPE apiserver_request_duration_seconds histogram")
        for (verb, group, res, sub), h in sorted(self.hist.items()):
            lab = f'verb="{verb}",group="{group}",resource="{res}",subresource="{sub}"'
            for b, n in zip(BUCKETS, h):
                out.append(f'apiserver_request_duration_seconds_bucket{{{lab},le="{b:g}"}} {n}')
            out.append(f'apiserver_request_duration_seconds_bucket{{{lab},le="+Inf"}} {h[-2]}')
            out.append(f"apiserver_request_duration_seconds_count{{{lab}}} {h[-2]}")
            out.append(f"apiserver_request_duration_seconds_sum{{{lab}}} {h[-1]:.6f}")
        return out
