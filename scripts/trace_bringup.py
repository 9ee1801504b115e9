#!/usr/bin/env python3
"""Cross-process timeline of one ``./setup.sh`` bring-up (TK8S_TRACE=1).

Runs the bench's bring-up (1 worker by default) in a scratch workspace with tracing on, then
merges the setup's event log with every ``TRACE`` line the control plane and node agents
printed to their logs, in wall-clock order, relative to the moment ``./setup.sh`` was launched.
Repeats ``--runs`` times (1 s apart, like the bench) and prints each timeline; ``--out FILE``
keeps them as JSON.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def one(root: Path, nodes: int, package: str = "mi355x-1gpu", rccl: str = "off") -> list[tuple[float, str, str]]:
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    init_workspace(root)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, root / f)
    (root / "answers.json").write_text(json.dumps({"nodes": nodes, "package": package, "confirm": "yes"}))
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_TRACE="1",
               TK8S_HOST_REGISTRY=str(root / "hostreg"))
    t0 = time.time()
    p = subprocess.run(["./setup.sh", "--answers", "answers.json", "--yes", "--json", "--port", "0", "--rccl", rccl],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    out: list[tuple[float, str, str]] = [(0.0, "launcher", "./setup.sh launched")]
    for line in p.stdout.splitlines():
        if line.startswith("ALL NODES READY"):
            out.append((float("nan"), "setup", line))
    for line in (root / ".tk8s" / "events.jsonl").read_text().splitlines():
        e = json.loads(line)
        what = (e["event"] + "".join(f" {k}={e[k]}" for k in ("phase", "task", "name") if k in e))[:110]
        if e.get("timing_ms"):  # the module's own breakdown (facts gathering, tk8s_kube, ...)
            what += " " + json.dumps(e["timing_ms"], separators=(",", ":"))
        out.append(((e["ts"] - t0) * 1000, "setup", what))
    for log in (root / ".tk8s").rglob("*"):
        if not log.is_file() or log.suffix in (".json", ".jsonl", ".pid", ".lock"):
            continue
        try:
            text = log.read_text(errors="replace")
        except OSError:
            continue
        for line in text.splitlines():
            if line.startswith("TRACE "):
                _, ts, where, what = (line.split(" ", 3) + [""])[:4]
                out.append(((float(ts) - t0) * 1000, where, what))
    for log in (root / ".tk8s").rglob("pods/kube-system_rccl-allreduce-*/log"):  # the ranks' own reports
        for line in log.read_text(errors="replace").splitlines():
            if line.startswith("{"):
                try:
                    r = json.loads(line)
                except ValueError:
                    continue
                keep = {k: v for k, v in r.items() if not isinstance(v, (list, dict))}
                out.append((float("inf"), "rank", json.dumps(keep)))
    subprocess.run(["./setup.sh", "-c", "--yes"], cwd=root, env=env, capture_output=True, timeout=120)
    if p.returncode != 0:
        raise SystemExit(f"setup failed ({p.returncode}):\n{p.stdout[-2000:]}\n{p.stderr[-2000:]}")
    return sorted((x for x in out if x[0] == x[0]), key=lambda x: x[0])  # (reports last: ms = inf)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=1)
    ap.add_argument("--package", default="mi355x-1gpu", help="cpu-only: BASELINE configs[1]'s workers")
    ap.add_argument("--rccl", default="off", help="on: also time the post-Ready RCCL fabric Job")
    ap.add_argument("--out")
    a = ap.parse_args()
    from tritonk8ssupervisor_amd.utils.build_native import build

    build()  # as bench.py does: incremental, and it makes the host's unpacked RCCL (fabric Job ranks)
    runs = []
    for i in range(a.runs):
        root = Path(tempfile.mkdtemp(prefix="tk8s-trace-"))
        try:
            tl = one(root, a.nodes, a.package, a.rccl)
        finally:
            shutil.rmtree(root, ignore_errors=True)
        runs.append([{"ms": round(t, 2) if t != float("inf") else None, "where": w, "what": x} for t, w, x in tl])
        print(f"--- run {i}", flush=True)
        for t, w, x in tl:
            print(f"{t:8.2f} {w:10s} {x}", flush=True)
        time.sleep(1.0)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(runs, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
