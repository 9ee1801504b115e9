"""Wall-clock trace points for the bring-up's cross-process critical path (``TK8S_TRACE=1``).

Each process (setup, control plane, node agents) prints ``TRACE <unix time> <where> <what>``
to its own log; ``scripts/trace_bringup.py`` merges them with the setup's event log, so the
hops between processes (pod exit -> status report -> node condition -> readiness long-poll)
can be timed on the GPU box without a profiler. Off by default: one env lookup at import.
"""
import os
import time

ON = bool(os.environ.get("TK8S_TRACE"))


def trace(where: str, what: str) -> None:
    if ON:
        print(f"TRACE {time.time():.6f} {where} {what}", flush=True)
