"""``ghost`` stand-in: the blog the reference deploys from the Kubernetes dashboard
(docs/detailed.md:261-283: image ``ghost``, port 2368, external Service).

  GET  /                          the blog front page (title "Ghost"), newest post first
  GET  /ghost/api/v0.1/posts      {"posts": [...]}
  POST /ghost/api/v0.1/posts      {"posts": [{"title": ..., "html": ...}]} (or the bare post) -> 201
"""
from __future__ import annotations

import html
import threading
import time
from urllib.parse import urlsplit

from .httpapp import Handler, serve

_lock = threading.Lock()
POSTS = [{"id": 1, "title": "Welcome to Ghost",
          "html": "<p>You're live! This blog is a tk8s pod on an AMD Instinct MI355X cluster.</p>",
          "published_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}]


def _is_posts(path: str) -> bool:
    return path.startswith("/ghost/api/") and path.rstrip("/").endswith("/posts")


class Ghost(Handler):
    server_version = "tk8s-ghost/1.0"

    def do_GET(self):
        path = urlsplit(self.path).path
        with _lock:
            posts = list(POSTS)
        if _is_posts(path):
            return self.send_json(200, {"posts": posts})
        if path in ("/", "/index.html"):
            items = "".join(f"<article><h2>{html.escape(p['title'])}</h2>{p['html']}</article>" for p in reversed(posts))
            return self.send(200, "<!doctype html><html><head><meta charset='utf-8'><title>Ghost</title></head>"
                                  "<body><header><h1>Ghost</h1><p>Just a blogging platform</p></header>"
                                  f"{items}</body></html>", "text/html; charset=utf-8")
        return self.send(404, "not found\n")

    do_HEAD = do_GET

    def do_POST(self):
        if not _is_posts(urlsplit(self.path).path):
            return self.send(404, "not found\n")
        try:
            body = self.body_json()
            post = (body.get("posts") or [body])[0]
            title = str(post["title"])
        except (ValueError, KeyError, TypeError, IndexError, AttributeError):
            return self.send_json(422, {"errors": [{"message": "a post needs a title"}]})
        with _lock:
            new = {"id": len(POSTS) + 1, "title": title, "html": f"<p>{html.escape(str(post.get('html', '')))}</p>",
                   "published_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
            POSTS.append(new)
        return self.send_json(201, {"posts": [new]})


def main(argv=None) -> int:
    return serve(Ghost, 2368, "tk8s ghost")


if __name__ == "__main__":
    raise SystemExit(main())
