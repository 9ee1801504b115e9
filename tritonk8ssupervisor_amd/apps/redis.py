"""``redis`` image stand-in: a RESP2 key-value server with leader/follower replication.

The Guestbook of the reference's kubectl walkthrough (docs/detailed.md:285-370) runs a redis
leader (``redis`` image) and followers (``gb-redisslave`` / ``gb-redis-follower``) behind two
Services; pods here are processes, so this is what those images run (apps/__init__.py maps the
names). It speaks RESP2 for what the Guestbook and ``redis-cli`` use -- strings, lists, keys,
INFO/ROLE/REPLICAOF -- and replicates by snapshot: a follower pulls ``TK8S.DUMP`` from its leader
every ``--sync-interval`` seconds and refuses writes (``READONLY``), like a Redis replica.
"""
from __future__ import annotations

import argparse
import asyncio
import fnmatch
import json

from .common import bind_host, listen_port, service_address
from .resp import RespError, Status, command, encode

OK = Status("OK")
WRITES = {"SET", "DEL", "INCR", "INCRBY", "DECR", "APPEND", "RPUSH", "LPUSH", "LPOP", "RPOP", "FLUSHALL", "FLUSHDB"}


class _WrongType(Exception):
    pass


async def read_command(reader: asyncio.StreamReader) -> list[bytes] | None:
    line = await reader.readline()
    if not line:
        return None
    if line[:1] != b"*":  # inline command (telnet / nc)
        return line.split()
    args = []
    for _ in range(int(line[1:].strip())):
        hdr = await reader.readline()
        if hdr[:1] != b"$":
            raise ValueError(f"expected a bulk string, got {hdr[:20]!r}")
        args.append((await reader.readexactly(int(hdr[1:].strip()) + 2))[:-2])
    return args


async def read_bulk(reader: asyncio.StreamReader) -> bytes | None:
    line = await reader.readline()
    if not line:
        raise ConnectionError("leader closed the connection")
    t, rest = line[:1], line[1:].rstrip(b"\r\n")
    if t == b"-":
        raise RespError(rest.decode(errors="replace"))
    if t != b"$":
        raise ValueError(f"expected a bulk reply, got {line[:20]!r}")
    n = int(rest)
    return None if n < 0 else (await reader.readexactly(n + 2))[:-2]


class Redis:
    def __init__(self, sync_interval: float = 0.1):
        self.data: dict[bytes, bytes | list[bytes]] = {}
        self.leader: tuple[str, int] | None = None
        self.follow_names: list[str] = []
        self.link = "down"
        self.sync_interval = sync_interval
        self.syncs = 0
        self.clients = 0

    @property
    def follower(self) -> bool:
        return self.leader is not None or bool(self.follow_names)

    # ---- commands -------------------------------------------------------------------------
    def execute(self, args: list[bytes]):
        name = args[0].decode(errors="replace").upper()
        if self.follower and name in WRITES:
            return RespError("READONLY You can't write against a read only replica.")
        fn = getattr(self, "c_" + name.lower().replace(".", "_"), None)
        if fn is None:
            return RespError(f"ERR unknown command '{name}'")
        try:
            return fn(*args[1:])
        except TypeError:
            return RespError(f"ERR wrong number of arguments for '{name.lower()}' command")
        except _WrongType:
            return RespError("WRONGTYPE Operation against a key holding the wrong kind of value")
        except ValueError:
            return RespError("ERR value is not an integer or out of range")

    def _str(self, k: bytes) -> bytes | None:
        v = self.data.get(k)
        if isinstance(v, list):
            raise _WrongType
        return v

    def _list(self, k: bytes, create: bool = False) -> list[bytes]:
        v = self.data.get(k)
        if v is None:
            if not create:
                return []
            v = self.data[k] = []
        if not isinstance(v, list):
            raise _WrongType
        return v

    def _drop_empty(self, k: bytes) -> None:
        if self.data.get(k) == []:
            del self.data[k]

    def c_ping(self, msg=None):
        return Status("PONG") if msg is None else msg

    def c_echo(self, msg):
        return msg

    def c_get(self, k):
        return self._str(k)

    def c_set(self, k, v, *_options):
        self.data[k] = v
        return OK

    def c_del(self, *keys):
        if not keys:
            raise TypeError
        return sum(self.data.pop(k, None) is not None for k in keys)

    def c_exists(self, *keys):
        return sum(k in self.data for k in keys)

    def c_type(self, k):
        v = self.data.get(k)
        return Status("none" if v is None else "list" if isinstance(v, list) else "string")

    def c_incrby(self, k, n):
        v = int(self._str(k) or b"0") + int(n)
        self.data[k] = str(v).encode()
        return v

    def c_incr(self, k):
        return self.c_incrby(k, b"1")

    def c_decr(self, k):
        return self.c_incrby(k, b"-1")

    def c_append(self, k, v):
        self.data[k] = (self._str(k) or b"") + v
        return len(self.data[k])

    def c_strlen(self, k):
        return len(self._str(k) or b"")

    def c_rpush(self, k, *values):
        if not values:
            raise TypeError
        lst = self._list(k, True)
        lst.extend(values)
        return len(lst)

    def c_lpush(self, k, *values):
        if not values:
            raise TypeError
        lst = self._list(k, True)
        for v in values:
            lst.insert(0, v)
        return len(lst)

    def c_lpop(self, k):
        lst = self._list(k)
        v = lst.pop(0) if lst else None
        self._drop_empty(k)
        return v

    def c_rpop(self, k):
        lst = self._list(k)
        v = lst.pop() if lst else None
        self._drop_empty(k)
        return v

    def c_llen(self, k):
        return len(self._list(k))

    def c_lrange(self, k, start, stop):
        lst = self._list(k)
        n, s, e = len(lst), int(start), int(stop)
        s = max(0, n + s) if s < 0 else s
        e = n + e if e < 0 else e
        return lst[s:e + 1]

    def c_keys(self, pattern=b"*"):
        p = pattern.decode("latin-1")
        return sorted(k for k in self.data if fnmatch.fnmatchcase(k.decode("latin-1"), p))

    def c_dbsize(self):
        return len(self.data)

    def c_flushall(self, *_):
        self.data.clear()
        return OK

    c_flushdb = c_flushall

    def c_select(self, _db):
        return OK

    def c_command(self, *_):
        return []

    def c_client(self, *_):
        return OK

    def c_role(self):
        if self.follower:
            host, port = self.leader or ("", 0)
            return [b"slave", host.encode(), port, b"connected" if self.link == "up" else b"connect", self.syncs]
        return [b"master", 0, []]

    def c_info(self, *_):
        lines = ["# Server", "redis_version:7.0.0-tk8s", "# Clients", f"connected_clients:{self.clients}",
                 "# Replication", f"role:{'slave' if self.follower else 'master'}"]
        if self.follower:
            host, port = self.leader or ("", 0)
            lines += [f"master_host:{host}", f"master_port:{port}", f"master_link_status:{self.link}",
                      f"tk8s_syncs:{self.syncs}"]
        lines += ["# Keyspace", f"db0:keys={len(self.data)}"]
        return ("\r\n".join(lines) + "\r\n").encode()

    def c_replicaof(self, host, port):
        if host.upper() == b"NO" and port.upper() == b"ONE":
            self.leader, self.follow_names, self.link = None, [], "down"
        else:
            self.leader, self.follow_names = (host.decode(), int(port)), []
        return OK

    c_slaveof = c_replicaof

    def c_tk8s_dump(self):
        """Snapshot for followers (latin-1 keeps arbitrary bytes through JSON)."""
        snap = {k.decode("latin-1"): (v.decode("latin-1") if isinstance(v, bytes) else [x.decode("latin-1") for x in v])
                for k, v in self.data.items()}
        return json.dumps(snap).encode()

    def load(self, blob: bytes) -> None:
        snap = json.loads(blob)
        self.data = {k.encode("latin-1"): (v.encode("latin-1") if isinstance(v, str) else [x.encode("latin-1") for x in v])
                     for k, v in snap.items()}

    # ---- network --------------------------------------------------------------------------
    async def handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        self.clients += 1
        try:
            while True:
                args = await read_command(reader)
                if args is None:
                    break
                if not args:
                    continue
                if args[0].upper() == b"QUIT":
                    writer.write(encode(OK))
                    await writer.drain()
                    break
                writer.write(encode(self.execute(args)))
                await writer.drain()
        except (ConnectionError, asyncio.IncompleteReadError, ValueError):
            pass
        finally:
            self.clients -= 1
            writer.close()

    async def follow_loop(self) -> None:
        loop = asyncio.get_running_loop()
        while True:
            if self.leader is None and self.follow_names:
                addr = await loop.run_in_executor(None, service_address, list(self.follow_names), 6379)
                if addr is not None and self.follow_names:
                    self.leader = addr
            if self.leader is None:
                await asyncio.sleep(0.2)
                continue
            target = self.leader
            try:
                r, w = await asyncio.wait_for(asyncio.open_connection(*target), 2.0)
                try:
                    while self.leader == target:
                        w.write(command("TK8S.DUMP"))
                        await w.drain()
                        self.load(await asyncio.wait_for(read_bulk(r), 5.0) or b"{}")
                        self.link = "up"
                        self.syncs += 1
                        await asyncio.sleep(self.sync_interval)
                finally:
                    w.close()
            except (OSError, asyncio.TimeoutError, ConnectionError, ValueError, RespError):
                self.link = "down"
                if self.follow_names:
                    self.leader = None  # resolve the leader Service again
                await asyncio.sleep(0.3)


async def serve(a: argparse.Namespace) -> None:
    db = Redis(a.sync_interval)
    if a.replicaof:
        db.leader = (a.replicaof[0], int(a.replicaof[1]))
    if a.follow:
        db.follow_names = [n for n in a.follow.split(",") if n]
    host, port = bind_host(), a.port or listen_port(6379)
    server = await asyncio.start_server(db.handle, host, port, reuse_address=True)
    print(f"tk8s-redis {'follower' if db.follower else 'leader'}: Ready to accept connections tcp on {host}:{port}",
          flush=True)
    follower = asyncio.create_task(db.follow_loop())
    try:
        async with server:
            await server.serve_forever()
    finally:
        follower.cancel()


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="tk8s-redis", description=__doc__.splitlines()[0])
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--replicaof", nargs=2, metavar=("HOST", "PORT"))
    ap.add_argument("--follow", default=None, help="comma list of leader Service names (follower mode)")
    ap.add_argument("--sync-interval", type=float, default=0.1)
    a, _ = ap.parse_known_args(argv)  # image args (redis-server flags) are accepted and ignored
    try:
        asyncio.run(serve(a))
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
