"""A tiny threaded HTTP server base for the built-in web apps."""
from __future__ import annotations

import json
import sys
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .common import bind_host, listen_port


class Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, fmt, *args):  # access log on the pod's stdout (kubectl logs)
        sys.stdout.write("%s - %s\n" % (self.address_string(), fmt % args))
        sys.stdout.flush()

    def send(self, code: int, body, ctype: str = "text/plain; charset=utf-8") -> None:
        data = body.encode() if isinstance(body, str) else body
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        if self.command != "HEAD":
            self.wfile.write(data)

    def send_json(self, code: int, obj) -> None:
        self.send(code, json.dumps(obj), "application/json")

    def body_json(self):
        n = int(self.headers.get("Content-Length") or 0)
        return json.loads(self.rfile.read(n) or b"{}")


def serve(handler: type[Handler], default_port: int, what: str) -> int:
    host, port = bind_host(), listen_port(default_port)
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    print(f"{what} listening on {host}:{port}", flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0
