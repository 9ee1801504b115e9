"""CPU and memory usage of the node and of its pods, for the metrics API (``kubectl top``) and the
HorizontalPodAutoscaler: what the kubelet's resource metrics endpoint answers.

A pod's usage is the sum over the processes of its containers (``members``: every container runs
in a session of its own, agent/runtime.py; a child that moved to another process group or session
is still followed through its parent chain): CPU from ``utime + stime`` deltas between two
samples, memory from the resident set. The node's comes from ``/proc/stat`` and ``/proc/meminfo``.
"""
from __future__ import annotations

import os
import time

_TICK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
_PAGE = os.sysconf("SC_PAGE_SIZE") if hasattr(os, "sysconf") else 4096


def _proc_table() -> dict[int, tuple[int, int, int, int, int]]:
    """pid -> (process group, cpu ticks, resident bytes, parent pid, session, start time in clock
    ticks since boot) for every readable process: with its start time a pid names one process
    even after the pid is reused."""
    out = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat", "rb") as f:
                raw = f.read().decode(errors="replace")
            rest = raw[raw.rindex(")") + 2:].split()
            # fields after "(comm)": state ppid pgrp session ... utime(14) stime(15) ... rss(24)
            out[int(d)] = (int(rest[2]), int(rest[11]) + int(rest[12]), int(rest[21]) * _PAGE, int(rest[1]),
                           int(rest[3]), int(rest[19]))
        except (OSError, ValueError, IndexError):
            continue
    return out


def members(table: dict, root: int, children: dict | None = None) -> set[int]:
    """The processes of the container whose first process is ``root`` (the leader of a session and
    process group of its own): its session and process group, and everything descending from
    them -- a job-control shell's pipelines (new process groups) and ``setsid`` children stay
    counted while their parent chain leads back. (A double fork that orphans itself to init
    leaves the chain: the limits of a watchdog without cgroups.)"""
    if children is None:
        children = child_map(table)
    mine = {p for p, v in table.items() if p == root or v[0] == root or v[4] == root}
    stack = list(mine)
    while stack:
        for c in children.get(stack.pop(), ()):
            if c not in mine:
                mine.add(c)
                stack.append(c)
    return mine


def child_map(table: dict) -> dict[int, list[int]]:
    out: dict[int, list[int]] = {}
    for p, v in table.items():
        out.setdefault(v[3], []).append(p)
    return out


def _node_cpu_ticks() -> tuple[int, int]:
    with open("/proc/stat") as f:
        vals = [int(x) for x in f.readline().split()[1:]]
    idle = vals[3] + (vals[4] if len(vals) > 4 else 0)
    return sum(vals), idle


def _node_memory() -> int:
    info = {}
    with open("/proc/meminfo") as f:
        for line in f:
            k, v = line.split(":", 1)
            info[k] = int(v.split()[0]) * 1024
    return info.get("MemTotal", 0) - info.get("MemAvailable", info.get("MemFree", 0))


class UsageSampler:
    """Call ``sample(groups)`` periodically; ``groups``: pod key -> {container name: pgid}."""

    def __init__(self):
        self.prev: dict[tuple[str, str], tuple[float, int]] = {}
        self.prev_node: tuple[int, int] | None = None

    def sample(self, groups: dict[str, dict[str, int]]) -> dict:
        now = time.time()
        table = _proc_table()
        kids = child_map(table)
        pods = {}
        for key, containers in groups.items():
            cs = []
            for name, pgid in containers.items():
                procs = [table[p] for p in members(table, pgid, kids)]
                ticks = sum(v[1] for v in procs)
                rss = sum(v[2] for v in procs)
                last = self.prev.get((key, name))
                self.prev[(key, name)] = (now, ticks)
                cores = 0.0
                if last is not None and now > last[0] and ticks >= last[1]:
                    cores = (ticks - last[1]) / _TICK / (now - last[0])
                cs.append({"name": name, "cpu_cores": cores, "memory_bytes": rss})
            pods[key] = cs
        live = {(k, n) for k, c in groups.items() for n in c}
        self.prev = {k: v for k, v in self.prev.items() if k in live}
        node = {"cpu_cores": 0.0, "memory_bytes": 0}
        try:
            total, idle = _node_cpu_ticks()
            if self.prev_node is not None and total > self.prev_node[0]:
                busy = (total - self.prev_node[0]) - (idle - self.prev_node[1])
                node["cpu_cores"] = busy / (total - self.prev_node[0]) * (os.cpu_count() or 1)
            self.prev_node = (total, idle)
            node["memory_bytes"] = _node_memory()
        except (OSError, ValueError, IndexError):
            pass
        return {"timestamp": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(now)), "node": node, "pods": pods}
