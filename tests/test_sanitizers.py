"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the xGMI
allocator, the JSON/args helpers (native/tests/host_selftest.cpp) and the restart supervisor
(tk8s-supervise), built with g++ -fsanitize=address,undefined and exercised on the CPU."""
import json
import os
import shutil
import signal
import subprocess
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
NATIVE = REPO / "native"
SAN = ["-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _build(tmp_path, name, sources):
    out = tmp_path / name
    r = subprocess.run(["g++", *SAN, f"-I{NATIVE / 'include'}", *map(str, sources), "-o", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def test_host_selftest_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "selftest", [NATIVE / "tests" / "host_selftest.cpp", NATIVE / "src" / "topology.cpp"])
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=ENV, timeout=120)
    assert r.returncode == 0 and "host selftest ok" in r.stdout, r.stdout + r.stderr


def test_supervisor_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "tk8s-supervise", [NATIVE / "tools" / "tk8s_supervise.cpp"])
    cnt = tmp_path / "n"
    r = subprocess.run([str(exe), "--pidfile", str(tmp_path / "a.pid"), "--restart", "on-failure", "--max-restarts", "3",
                        "--backoff-ms", "5", "--", "sh", "-c", f"echo x >> {cnt}; exit 4"],
                       capture_output=True, text=True, env=ENV, timeout=60)
    assert r.returncode == 4 and cnt.read_text().count("x") == 4, r.stderr[-2000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    pf = tmp_path / "b.pid"
    p = subprocess.Popen([str(exe), "--pidfile", str(pf), "--log", str(tmp_path / "b.log"), "--", "sleep", "600"],
                         env=ENV, start_new_session=True, stderr=subprocess.PIPE, text=True)
    deadline = time.monotonic() + 10
    while not pf.exists() and time.monotonic() < deadline:
        time.sleep(0.01)
    child = json.loads(pf.read_text())["child"]
    os.kill(child, signal.SIGKILL)
    while json.loads(pf.read_text() or "{}").get("child") == child and time.monotonic() < deadline:
        time.sleep(0.01)
    p.send_signal(signal.SIGTERM)
    assert p.wait(20) == 0 or p.returncode in (128 + signal.SIGTERM, -signal.SIGTERM, 143)
    err = p.stderr.read() + (tmp_path / "b.log").read_text()
    assert "AddressSanitizer" not in err and "runtime error" not in err, err[-2000:]
