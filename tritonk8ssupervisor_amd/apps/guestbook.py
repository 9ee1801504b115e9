"""``gb-frontend`` stand-in: the Guestbook web tier of the reference's kubectl walkthrough.

docs/detailed.md:285-370 deploys ``guestbook-all-in-one.yaml`` and opens the frontend through a
LoadBalancer Service. The frontend image serves a page plus ``guestbook.php``:

  GET /guestbook.php?cmd=set&key=K&value=V  -> SET K V on the redis leader -> {"message": "Updated"}
  GET /guestbook.php?cmd=get&key=K          -> GET K from a redis follower -> {"data": "<value>"}

Same API here, against the ``redis-master``/``redis-leader`` and ``redis-slave``/``redis-follower``
Services (Service env vars first, like GET_HOSTS_FROM=env; the API for later Services).
"""
from __future__ import annotations

from urllib.parse import parse_qs, urlsplit

from .common import service_address
from .httpapp import Handler, serve
from .resp import RespError, call

LEADERS = ("redis-master", "redis-leader")
FOLLOWERS = ("redis-slave", "redis-follower", "redis-replica")

INDEX = """<!doctype html>
<html><head><meta charset="utf-8"><title>Guestbook</title></head>
<body style="font-family: sans-serif; width: 50%; margin-left: 20px">
<h2>Guestbook</h2>
<form id="guestbook"><input id="msg" placeholder="Messages" autofocus> <button>Submit</button></form>
<div id="messages"></div>
<script>
const key = "messages";
async function load() {
  const d = await (await fetch(`guestbook.php?cmd=get&key=${key}`)).json();
  return (d.data || "").split(",").filter(Boolean);
}
async function show() {
  const box = document.getElementById("messages");
  box.innerHTML = "";
  for (const m of await load()) { const p = document.createElement("p"); p.textContent = m; box.appendChild(p); }
}
document.getElementById("guestbook").addEventListener("submit", async (e) => {
  e.preventDefault();
  const msgs = await load();
  msgs.push(document.getElementById("msg").value);
  await fetch(`guestbook.php?cmd=set&key=${key}&value=${encodeURIComponent(msgs.join(","))}`);
  document.getElementById("msg").value = "";
  show();
});
show();
</script></body></html>
"""


def _redis(names, fallback=()) -> tuple[str, int]:
    addr = service_address(names, 6379) or (service_address(fallback, 6379) if fallback else None)
    if addr is None:
        raise LookupError(f"no redis Service among {', '.join(tuple(names) + tuple(fallback))}")
    return addr


class Frontend(Handler):
    server_version = "tk8s-gb-frontend/1.0"

    def do_GET(self):
        u = urlsplit(self.path)
        if u.path in ("/", "/index.html"):
            return self.send(200, INDEX, "text/html; charset=utf-8")
        if u.path == "/healthz":
            return self.send(200, "ok\n")
        if u.path != "/guestbook.php":
            return self.send(404, "not found\n")
        q = {k: v[-1] for k, v in parse_qs(u.query, keep_blank_values=True).items()}
        key = q.get("key", "messages")
        try:
            if q.get("cmd") == "set":
                call(*_redis(LEADERS), "SET", key, q.get("value", ""))
                return self.send_json(200, {"message": "Updated"})
            v = call(*_redis(FOLLOWERS, LEADERS), "GET", key)
            return self.send_json(200, {"data": (v or b"").decode(errors="replace")})
        except (OSError, RespError, LookupError) as e:
            return self.send_json(503, {"error": str(e)})

    do_HEAD = do_GET


def main(argv=None) -> int:
    return serve(Frontend, 80, "tk8s gb-frontend")


if __name__ == "__main__":
    raise SystemExit(main())
