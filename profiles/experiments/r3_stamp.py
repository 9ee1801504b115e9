#!/usr/bin/env python3
"""Run a command, stamp every stderr line with ms since launch into LOG; stdout passes through.

    r3_stamp.py LOG [KEY=VALUE ...] -- CMD ARGS...
"""
import os
import subprocess
import sys
import threading
import time

log = sys.argv[1]
i = sys.argv.index("--")
env = dict(os.environ)
for kv in sys.argv[2:i]:
    k, _, v = kv.partition("=")
    env[k] = v
cmd = sys.argv[i + 1:]
t0 = time.monotonic()
p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)


def pump_err():
    with open(log, "w") as f:
        f.write(f"launch unix_ms={time.time() * 1e3:.3f}\n")
        for line in p.stderr:
            f.write(f"{(time.monotonic() - t0) * 1e3:9.3f} {line.decode(errors='replace')}")


th = threading.Thread(target=pump_err, daemon=True)
th.start()
out = p.stdout.read()
rc = p.wait()
th.join(5)
with open(log, "a") as f:
    f.write(f"exit {rc} after {(time.monotonic() - t0) * 1e3:.3f} ms\n")
sys.stdout.buffer.write(out)
sys.exit(rc)
