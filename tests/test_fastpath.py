"""The import-light replacements on the bring-up path behave like the stdlib pieces they stand
in for: utils/record.py (dataclasses), utils/pool.py (concurrent.futures), utils/http1.py
(http.client), utils/ids.py (uuid.uuid5), utils/yamlio.py's parse cache (PyYAML) -- and
./setup.sh's interpreter does not import the heavy modules at all."""
import os
import socket
import subprocess
import sys
import threading
import uuid
from pathlib import Path

import pytest
import yaml

from tritonk8ssupervisor_amd.utils import yamlio
from tritonk8ssupervisor_amd.utils.http1 import Connection, ProtocolError
from tritonk8ssupervisor_amd.utils.ids import uuid5
from tritonk8ssupervisor_amd.utils.pool import Pool, as_completed
from tritonk8ssupervisor_amd.utils.record import asdict, field, fields, record

REPO = Path(__file__).resolve().parents[1]


# ---- record ---------------------------------------------------------------------------------
@record
class Point:
    x: int
    y: int = 0
    tags: list = field(default_factory=list)


@record(frozen=True)
class Key:
    name: str
    n: int = 1


@record
class Outer:
    p: Point
    ps: list = field(default_factory=list)


def test_record_init_repr_eq():
    a = Point(1)
    assert (a.x, a.y, a.tags) == (1, 0, [])
    assert Point(1, 2, ["t"]) == Point(x=1, y=2, tags=["t"]) and Point(1) != Point(2)
    assert repr(Point(1, 2)) == "Point(x=1, y=2, tags=[])"
    assert Point(1).tags is not Point(1).tags  # fresh default per instance
    assert [f.name for f in fields(Point)] == ["x", "y", "tags"]
    with pytest.raises(TypeError):
        Point()
    with pytest.raises(TypeError):
        Point(1, 2, [], 4)
    with pytest.raises(TypeError):
        Point(1, x=2)
    with pytest.raises(TypeError):
        Point(1, z=3)
    with pytest.raises(TypeError):
        hash(Point(1))  # eq without frozen: unhashable, as with dataclasses


def test_record_frozen_and_asdict():
    k = Key("a")
    assert {k: 1}[Key("a", 1)] == 1
    with pytest.raises(AttributeError):
        k.name = "b"
    o = Outer(Point(1, tags=["x"]), [Point(2)])
    d = asdict(o)
    assert d == {"p": {"x": 1, "y": 0, "tags": ["x"]}, "ps": [{"x": 2, "y": 0, "tags": []}]}
    d["p"]["tags"].append("y")
    assert o.p.tags == ["x"]  # deep copy


# ---- pool -----------------------------------------------------------------------------------
def test_pool_map_order_errors_and_as_completed():
    with Pool(4) as p:
        assert p.map(lambda v: v * v, range(10)) == [v * v for v in range(10)]

        def boom(v):
            if v == 3:
                raise ValueError("three")
            return v

        with pytest.raises(ValueError):
            p.map(boom, range(5))
        gates = [threading.Event() for _ in range(3)]
        futs = [p.submit(g.wait) for g in gates]
        done = as_completed(futs)
        try:
            for i in (1, 2, 0):  # finish them in this order; as_completed yields them the same way
                gates[i].set()
                assert futs.index(next(done)) == i
        finally:
            for g in gates:
                g.set()
        assert len(p._threads) <= 4
    with pytest.raises(RuntimeError):
        p.submit(lambda: 1)


def test_pool_reuses_idle_workers():
    p = Pool(8)
    for _ in range(20):
        p.submit(lambda: None).result()
    assert len(p._threads) == 1
    p.shutdown()


# ---- http1 ----------------------------------------------------------------------------------
def _serve(responses):
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    seen = []

    def run():
        c, _ = srv.accept()
        f = c.makefile("rb")
        for resp in responses:
            req = b""
            while not req.endswith(b"\r\n\r\n"):
                line = f.readline()
                if not line:
                    return
                req += line
            n = next((int(ln.split(b":")[1]) for ln in req.split(b"\r\n") if ln.lower().startswith(b"content-length")), 0)
            seen.append(req + f.read(n))
            c.sendall(resp)
        c.close()
        srv.close()

    threading.Thread(target=run, daemon=True).start()
    return srv.getsockname()[1], seen


def test_http1_content_length_chunked_and_keepalive():
    port, seen = _serve([b"HTTP/1.1 100 Continue\r\n\r\nHTTP/1.1 200 OK\r\nContent-Length: 5\r\nX-A: 1\r\n\r\nhello",
                         b"HTTP/1.1 201 Created\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n2;ext=1\r\nde\r\n0\r\n\r\n",
                         b"HTTP/1.1 204 No Content\r\n\r\n",
                         b"HTTP/1.0 200 OK\r\n\r\nuntil close"])
    c = Connection("127.0.0.1", port, timeout=5)
    r = c.request("GET", "/a")
    assert (r.status, r.body, r.header("x-a")) == (200, b"hello", "1")
    r = c.request("POST", "/b", body=b'{"k":1}', headers={"Content-Type": "application/json"})
    assert (r.status, r.body) == (201, b"abcde")
    assert c.request("DELETE", "/c").status == 204
    r = c.request("GET", "/d")
    assert r.body == b"until close" and not c.connected
    assert seen[0].startswith(b"GET /a HTTP/1.1\r\n") and b"Host: 127.0.0.1:" in seen[0]
    assert seen[1].endswith(b'\r\n\r\n{"k":1}') and b"Content-Length: 7" in seen[1]


def test_http1_truncated_response_is_an_error():
    port, _ = _serve([b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\n\r\nshort"])
    c = Connection("127.0.0.1", port, timeout=5)
    with pytest.raises(ProtocolError):
        c.request("GET", "/")
    assert not c.connected


# ---- ids ------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["tk8s/machine/kubenode1", "", "ünïcode/名"])
def test_uuid5_matches_the_stdlib(name):
    ns = "5f1c0d3e-8a4b-4c6e-9b1a-7e2f3d4c5b6a"
    assert uuid5(ns, name) == str(uuid.uuid5(uuid.UUID(ns), name))


# ---- yaml parse cache ------------------------------------------------------------------------
def test_yaml_cache_returns_exactly_the_parse(tmp_path, monkeypatch):
    monkeypatch.setenv("TK8S_YAML_CACHE", str(tmp_path / "c"))
    text = "a: 1\nb: [yes, no, on, '0x1f', 0x1f, 1e3, 1.5e3, ~]\nc: {d: e}\n0: zero\n"
    want = yaml.safe_load(text)
    assert yamlio.load(text) == want                # miss: parsed and stored
    assert len(os.listdir(tmp_path / "c")) == 1
    first = yamlio.load(text)
    assert first == want and yamlio.load(text) is not first   # hit: a fresh copy each time
    first["a"] = 2
    assert yamlio.load(text)["a"] == 1
    assert yamlio.load_all("---\nx: 1\n---\ny: 2\n") == [{"x": 1}, {"y": 2}]
    stamp = "when: 2024-01-02 03:04:05\n"       # a timestamp marshal cannot hold: not cached
    assert yamlio.load(stamp) == yaml.safe_load(stamp)
    assert len(os.listdir(tmp_path / "c")) == 2


def test_yaml_cache_entry_must_match_the_text(tmp_path, monkeypatch):
    import marshal

    monkeypatch.setenv("TK8S_YAML_CACHE", str(tmp_path))
    text = "k: v\n"
    yamlio.load(text)
    (entry,) = tmp_path.iterdir()
    entry.write_bytes(marshal.dumps(("k: other\n", {"k": "forged"})))  # same key, different text
    assert yamlio.load(text) == {"k": "v"}


def test_flat_mapping_is_what_yaml_reads(tmp_path, monkeypatch):
    monkeypatch.setenv("TK8S_YAML_CACHE", str(tmp_path))
    data = {"master": "127.0.1.2", "kubernetes_name": 'k8s "dev"\tü', "n": 3, "b": True, "z": None}
    text = yamlio.flat_mapping(data)
    assert yaml.safe_load(text) == data
    assert yamlio.load(text) == data
    with pytest.raises(ValueError):
        yamlio.flat_mapping({"a": [1]})


def test_setup_cli_does_not_import_the_heavy_modules(tmp_path):
    """What ./setup.sh's interpreter loads before the bring-up starts (cli/fast.py, cli/main.py,
    orchestrator.py): none of the modules the fast path replaced."""
    code = ("import sys; from tritonk8ssupervisor_amd.cli import main; from tritonk8ssupervisor_amd import orchestrator, "
            "playbook, playbook_modules, provision; from tritonk8ssupervisor_amd.provider import local; "
            "from tritonk8ssupervisor_amd.controlplane import client; "
            "bad = {'yaml', 'dataclasses', 'inspect', 'concurrent.futures', 'logging', 'uuid', 'http.client', "
            "'urllib.request', 'email.parser', 'ssl', 'tempfile', 'hashlib', 'typing', 'runpy', 'argparse', 'gettext', "
            "'configparser', 'copy', 'shutil', 'ast', 'tokenize', 'base64'} & set(sys.modules); "
            "print(sorted(bad))")
    r = subprocess.run([sys.executable, "-S", "-c", code], cwd=REPO, capture_output=True, text=True, timeout=60,
                       env={**os.environ, "PYTHONPATH": str(REPO)})
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "[]", r.stdout


def test_pool_never_strands_a_task_behind_a_waiting_worker():
    """Tasks that wait on tasks submitted after them (each needs a worker of its own): with
    enough workers allowed, every one of them runs, however the workers happen to be idle."""
    for _ in range(200):
        p = Pool(3)
        p.submit(lambda: None).result()  # one worker, idle
        gates = [threading.Event() for _ in range(3)]
        futs = [p.submit(gates[0].wait), p.submit(lambda: (gates[0].set(), gates[1].wait())),
                p.submit(lambda: gates[1].set())]
        try:
            for f in futs:
                f.result(timeout=10)
        finally:
            for g in gates:
                g.set()
            p.shutdown()


@pytest.mark.parametrize("argv", [
    ["setup"],
    ["setup", "--answers", "a.json", "--yes", "--json", "--port", "18080", "--timeout", "300", "--rccl-timeout", "120"],
    ["setup", "--answers=a.yml", "--no-validate", "--rccl", "off", "-v", "--backend", "baremetal", "--inventory", "i.yml"],
    ["setup", "--nodes", "4", "--package", "mi355x-2gpu", "--name", "x y", "--dry-run", "--platform", "kubeadm",
     "--hbm-bytes", "4096", "--md5-bytes", "1024", "--probe-iters", "1", "--node-grace", "2.5", "--rocprof",
     "--rocprof-counters", "SQ_WAVES", "--rccl-max-bytes", "1024", "--resume", "--master-hostname", "m",
     "--node-prefix", "n", "--verbose"],
])
def test_fast_setup_parser_builds_what_argparse_builds(argv):
    from tritonk8ssupervisor_amd.cli import main as cli

    fast = cli._fast_setup_args(argv)
    assert fast is not None
    slow = cli.build_parser().parse_args(argv)
    assert vars(fast) == vars(slow)


@pytest.mark.parametrize("argv", [
    ["setup", "--help"], ["setup", "--ans", "a.json"], ["setup", "--rccl", "maybe"], ["setup", "--nodes", "two"],
    ["setup", "--timeout", "-1"], ["setup", "--yes=1"], ["setup", "--answers"], ["setup", "-vv"], ["status"],
])
def test_fast_setup_parser_leaves_the_rest_to_argparse(argv):
    from tritonk8ssupervisor_amd.cli import main as cli

    assert cli._fast_setup_args(argv) is None


def test_ini_reader_matches_configparser():
    import configparser

    from tritonk8ssupervisor_amd.playbook import read_ini_section

    texts = ["[defaults]\nhost_key_checking = False\nforks=0\n# comment\n; other\nRetry_Files_Enabled: no\n[ssh]\nx = 1\n",
             "", "[other]\na = 1\n", "[defaults]\nlong = a\n  continued\n", "[defaults]\nx = %(y)s\ny = 2\n"]
    for t in texts:
        cp = configparser.ConfigParser()
        cp.read_string(t)
        assert read_ini_section(t, "defaults") == (dict(cp["defaults"]) if cp.has_section("defaults") else {}), t


@pytest.mark.parametrize("cidr", ["127.0.1.0/24", "10.0.0.0/30", "192.168.4.0/22", "10.9.0.0/31", "10.9.0.7/32"])
def test_ipv4_hosts_match_ipaddress(cidr):
    import ipaddress

    from tritonk8ssupervisor_amd.provider.local import _ipv4_hosts

    assert list(_ipv4_hosts(cidr)) == [str(a) for a in ipaddress.ip_network(cidr).hosts()]


def test_late_site_finder_only_adds_site_dirs_for_third_party_imports():
    code = ("import sys; import tritonk8ssupervisor_amd; n = len(sys.path); import ntpath, pathlib; "
            "assert len(sys.path) == n, 'a stdlib probe added the site dirs'; import yaml; "
            "assert len(sys.path) > n; print('ok')")
    r = subprocess.run([sys.executable, "-S", "-c", code], cwd=REPO, capture_output=True, text=True, timeout=60,
                       env={**os.environ, "PYTHONPATH": str(REPO)})
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr


@pytest.mark.parametrize("argv", [
    ["--await-url", "run/registration-url", "--name", "kubenode1", "--ip", "127.0.1.3"],
    ["http://127.0.0.1:1/v1/scripts/T", "--name", "n", "--tool-dir", "/a", "--tool-dir", "/b", "--gpus", "0,1",
     "--timeout", "5", "--smi-interval", "0", "--smi-delay", "1.5", "--labels", "a=b,c=d", "--sandbox", "/s"],
    ["--device-plugin", "grpc", "--url", "http://u"],
])
def test_agent_fast_parser_matches_argparse(argv):
    from tritonk8ssupervisor_amd.agent import agent as ag

    assert ag._parse_fast(argv) == ag._parse_argparse(argv)


@pytest.mark.parametrize("argv", [["--help"], ["--name=x"], ["--device-plugin", "other", "--url", "u"], ["a", "b"],
                                  ["--timeout", "soon", "--url", "u"], ["--name"]])
def test_agent_fast_parser_defers_the_rest(argv):
    from tritonk8ssupervisor_amd.agent import agent as ag

    assert ag._parse_fast(argv) is None


def test_controlplane_fast_parser():
    from tritonk8ssupervisor_amd.controlplane import server

    a = server._parse_fast(["--host", "127.0.1.1", "--port", "0", "--advertise", "127.0.1.1", "--state-dir", "/s",
                            "--node-grace", "2.5", "--dns-port", "0", "--ingress-port", "0", "--ready-file", "/r"])
    assert a == {"host": "127.0.1.1", "port": 0, "advertise": "127.0.1.1", "state_dir": "/s", "node_grace": 2.5,
                 "dns_port": 0, "ingress_port": 0, "ready_file": "/r"}
    assert server._parse_fast(["--help"]) is None and server._parse_fast(["--port=1"]) is None
    assert server._parse_fast(["--port", "x"]) is None


def test_daemon_entries_skip_runpy_and_ssl():
    """The control plane and agent start with -c '<pkg>.__main__' imports: no runpy, and the control
    plane (plain HTTP) keeps ssl out of asyncio."""
    code = ("import sys; sys.argv = ['-c', '--help']; "
            "import tritonk8ssupervisor_amd.controlplane.__main__")
    r = subprocess.run([sys.executable, "-S", "-c", code], cwd=REPO, capture_output=True, text=True, timeout=60,
                       env={**os.environ, "PYTHONPATH": str(REPO)})
    assert r.returncode == 0 and "tk8s-controlplane" in r.stdout, r.stderr
    code = ("import sys; sys.modules.setdefault('ssl', None); import asyncio, tritonk8ssupervisor_amd.controlplane.server; "
            "print(sorted({'runpy', 'argparse', 'uuid', 'secrets', 'html'} & set(sys.modules)), sys.modules['ssl'])")
    r = subprocess.run([sys.executable, "-S", "-c", code], cwd=REPO, capture_output=True, text=True, timeout=60,
                       env={**os.environ, "PYTHONPATH": str(REPO)})
    assert r.returncode == 0 and r.stdout.strip() == "[] None", (r.stdout, r.stderr)


def test_uuid4_and_token_hex_shapes():
    import re
    import uuid

    from tritonk8ssupervisor_amd.utils.ids import token_hex, uuid4

    u = uuid4()
    assert uuid.UUID(u).version == 4 and str(uuid.UUID(u)) == u and uuid.UUID(u).variant == uuid.RFC_4122
    assert uuid4() != u
    assert re.fullmatch(r"[0-9a-f]{40}", token_hex(20))
