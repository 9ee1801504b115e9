"""``nginx`` / ``httpd`` stand-in: a static welcome page on port 80 (shifted when not root)."""
from __future__ import annotations

import html
import os

from .httpapp import Handler, serve


class Static(Handler):
    server_version = "tk8s-static/1.0"

    def do_GET(self):
        who = html.escape(f"{os.environ.get('POD_NAME', '?')} on {os.environ.get('NODE_NAME', '?')}")
        return self.send(200, "<!DOCTYPE html><html><head><title>Welcome to nginx!</title></head><body>"
                              f"<h1>Welcome to nginx!</h1><p>Served by tk8s pod {who}.</p></body></html>",
                         "text/html; charset=utf-8")

    do_HEAD = do_GET


def main(argv=None) -> int:
    return serve(Static, 80, "tk8s static")


if __name__ == "__main__":
    raise SystemExit(main())
