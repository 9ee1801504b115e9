"""Keep-alive HTTP/JSON client for the tk8s control plane (stdlib only, import-light: the
connection is utils/http1.py, not http.client)."""
from __future__ import annotations

import json
import threading
import time
from urllib.parse import urlencode, urlsplit

from ..utils.http1 import Connection


class ApiError(RuntimeError):
    def __init__(self, status: int, message: str, body: Any = None):
        super().__init__(f"HTTP {status}: {message}")
        self.status = status
        self.body = body


class Client:
    """One persistent connection per client; safe to share between threads (serialised)."""

    def __init__(self, base: str, token: str | None = None, prefix: str = "", timeout: float = 30.0):
        u = urlsplit(base if "://" in base else "http://" + base)
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or 80
        self.base = f"http://{self.host}:{self.port}"
        self.prefix = prefix.rstrip("/")
        self.token = token
        self.timeout = timeout
        self._conn: Connection | None = None
        self._lock = threading.Lock()

    def _connection(self, timeout: float) -> Connection:
        if self._conn is None:
            self._conn = Connection(self.host, self.port, timeout=timeout)
        else:
            self._conn.set_timeout(timeout)
        return self._conn

    def close(self) -> None:
        with self._lock:
            if self._conn is not None:
                self._conn.close()
                self._conn = None

    def request(self, method: str, path: str, body: Any = None, query: dict | None = None,
                timeout: float | None = None, raw: bool = False, ok=(200, 201, 202, 204),
                content_type: str | None = None) -> Any:
        url = path if path.startswith("/") else "/" + path
        if query:
            url += ("&" if "?" in url else "?") + urlencode({k: v for k, v in query.items() if v is not None})
        headers = {"Connection": "keep-alive"}
        data = None
        if body is not None:
            if isinstance(body, (bytes, str)):
                data = body.encode() if isinstance(body, str) else body
                headers["Content-Type"] = "text/plain"
            else:
                data = json.dumps(body).encode()
                headers["Content-Type"] = content_type or "application/json"
        if self.token:
            headers["Authorization"] = f"Bearer {self.token}"
        t = self.timeout if timeout is None else timeout
        with self._lock:
            for attempt in range(2):  # one transparent reconnect for a dropped keep-alive
                conn = self._connection(t)
                reused = conn.connected
                try:
                    resp = conn.request(method, url, body=data, headers=headers)
                    payload, status, ctype = resp.body, resp.status, resp.header("content-type")
                    if not conn.connected:  # the server closed it (Connection: close)
                        self._conn = None
                    break
                except OSError as e:
                    conn.close()
                    self._conn = None
                    # only a keep-alive connection the server dropped while idle is retried: a
                    # fresh connection's failure or a timeout is the caller's to see
                    if attempt or not reused or isinstance(e, TimeoutError):
                        raise
        if raw:
            if status not in ok:
                raise ApiError(status, payload[:300].decode(errors="replace"))
            return payload.decode(errors="replace")
        parsed: Any = payload.decode(errors="replace")
        if "json" in ctype and payload:
            parsed = json.loads(payload)
        if status not in ok:
            msg = parsed.get("message") if isinstance(parsed, dict) else str(parsed)[:300]
            raise ApiError(status, msg or "error", parsed)
        return parsed

    # ---- convenience --------------------------------------------------------------------
    def get(self, path: str, **kw) -> Any:
        return self.request("GET", path, **kw)

    def post(self, path: str, body: Any = None, **kw) -> Any:
        return self.request("POST", path, body=body if body is not None else {}, **kw)

    def put(self, path: str, body: Any = None, **kw) -> Any:
        return self.request("PUT", path, body=body if body is not None else {}, **kw)

    def delete(self, path: str, **kw) -> Any:
        return self.request("DELETE", path, **kw)

    def k8s(self, path: str) -> str:
        return self.prefix + path

    def wait_up(self, timeout: float = 30.0, interval: float = 0.01) -> bool:
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            try:
                if self.request("GET", "/ping", raw=True, timeout=2.0) == "pong":
                    return True
            except (ApiError, OSError):
                pass
            time.sleep(interval)
        return False

    def watch(self, path: str, since: int, timeout: float = 30.0, query: dict | None = None) -> tuple[int, list[dict]]:
        # batch=1: the long-poll form (one JSON batch per request), not the Kubernetes stream
        q = {"watch": "1", "batch": "1", "resourceVersion": str(since), "timeoutSeconds": str(timeout)}
        q.update(query or {})
        r = self.get(path, query=q, timeout=timeout + 10)
        return int(r["resourceVersion"]), r["events"]


def client_from_kubeconfig(cfg: dict) -> Client:
    """Build a Client from a kubeconfig dict written by the control plane."""
    cur = cfg.get("current-context")
    ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == cur)
    cluster = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
    user = next(u["user"] for u in cfg["users"] if u["name"] == ctx["user"])
    u = urlsplit(cluster["server"])
    return Client(f"{u.scheme}://{u.netloc}", token=user.get("token"), prefix=u.path)
