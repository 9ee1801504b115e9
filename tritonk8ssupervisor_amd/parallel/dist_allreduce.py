"""torch.distributed all-reduce validator, one process per rank: the PyTorch twin of ``tk8s-rccl`` (N3).

``--backend gloo`` (CPU tensors) is the cluster fabric check when the GPUs are faked
(``TK8S_FAKE_GPUS``, CPU-only hosts and tests); ``--backend nccl`` (= RCCL on ROCm, tensors on
the pod's one visible MI355X) is what a PyTorch user's job sees on the real cluster
(manifests/examples/torch-allreduce-job.yaml). It follows the native job's protocol step by
step so the control-plane path is exercised unchanged: rank 0 publishes its rendezvous address to the control-plane KV store
(HTTP PUT), the other ranks long-poll it (GET ``?wait=``), then every rank runs an
RCCL-tests-style sweep with an exact result check and prints ONE JSON line with the same keys
as native/tools/tk8s_rccl.cpp (``ok``, ``nranks``, ``rank``, ``peak_busbw_gbps``, ``results``).

``--group-index I --devices d0,..,dk-1`` is the fabric Job's one-pod-per-node shape (ranks
I*k .. I*k+k-1, like ``tk8s-rccl --group-index``): torch.distributed has one default group per
process, so the pod runs its k ranks as child processes and prints ONE merged line for the pod.

With ``NCCL_DEBUG`` set (INFO), RCCL's log goes to a file of the rank's own (``NCCL_DEBUG_FILE``,
unless the caller named one); the rank copies it to stderr and reports in its JSON line which
transport RCCL's channels took (``transport``: counts of ``via P2P/...``, ``via SHM/...``,
``via NET/...`` connections, and whether the communicator's init completed) -- what tells
whether ranks in separate pods still go GPU to GPU over xGMI.

Fail fast (the same contract as tk8s-rccl, native/include/tk8s/failfast.h):
``--op-timeout`` (alias ``--timeout``, default 20 s) bounds the rendezvous fetch, the process
group's init and every collective (gloo's own timeout); a failure prints ``{"ok": false,
"phase": ...}`` and exits 2; a watchdog thread ends a rank whose phase makes no progress for
op-timeout + 10 s (exit 4, as tk8s-rccl's). Fault points (``TK8S_FAULTS``, ``[:rank]`` targets one rank):
``rccl.hang@<phase>`` (the rank stops), ``rccl.exit@<phase>`` (exit 3), ``rccl.crash@<phase>``
(abort) for phases uid / init / sweep / check -- how the CPU tests kill or hang one rank of a
2- or 8-rank job and show every other rank still ends within its deadline.

Check (N6 semantics): rank r contributes ``(r + 1) * p[i]`` with ``p[i] = (i % m) + 1``;
every element must equal ``n (n + 1) / 2 * p[i]`` exactly. ``m`` keeps every partial sum an
exactly representable integer: 251 for fp32 (< 2^24), 4 for bf16 (sums <= 256 up to n = 8).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import urllib.request


SA_TOKEN = "/var/run/secrets/kubernetes.io/serviceaccount/token"
WATCHDOG_GRACE_S = 10.0
WATCHDOG_EXIT = 4  # = tk8s::kWatchdogExit (native/include/tk8s/failfast.h)


class Phases:
    """The rank's current phase, a no-progress watchdog over it, and its fault points."""

    def __init__(self, rank: int | None, nranks: int, op_timeout: float):
        import threading

        self.rank, self.nranks, self.op_timeout = rank, nranks, op_timeout
        self.phase, self.deadline, self.started = "start", 0.0, 0.0
        self.lock = threading.Lock()
        if op_timeout > 0:
            threading.Thread(target=self._watch, name="watchdog", daemon=True).start()

    def enter(self, phase: str) -> None:
        with self.lock:
            self.phase, self.started = phase, time.monotonic()
            self.deadline = self.started + self.op_timeout + WATCHDOG_GRACE_S
        self._faults(phase)

    def _watch(self) -> None:
        while True:
            time.sleep(0.05)
            with self.lock:
                if not self.deadline or time.monotonic() < self.deadline:
                    continue
                phase, waited = self.phase, time.monotonic() - self.started
            print(json.dumps({"ok": False, "rank": self.rank, "nranks": self.nranks, "phase": phase, "timed_out": True,
                              "watchdog": True, "error": f"watchdog: no progress in phase {phase} for {waited:.0f} s"}),
                  flush=True)
            os._exit(WATCHDOG_EXIT)

    def _faults(self, phase: str) -> None:
        from ..utils.faults import _parse

        for point, target, arg in _parse(os.environ.get("TK8S_FAULTS", "")):
            if target != phase or not point.startswith("rccl."):
                continue
            if arg is not None and (self.rank is None or arg != str(self.rank)):
                continue
            kind = point[len("rccl."):]
            sys.stderr.write(f"dist_allreduce rank {self.rank}: TK8S_FAULTS {point}@{phase}\n")
            sys.stderr.flush()
            if kind == "exit":
                os._exit(3)
            if kind == "crash":
                os.abort()
            if kind == "hang":
                while True:
                    time.sleep(1)


def _kv_headers() -> dict:
    """The pod's ServiceAccount token (the control plane's KV answers no anonymous caller):
    TK8S_KV_TOKEN, else the token file the agent mounted (process pods name it in
    TK8S_SERVICEACCOUNT_TOKEN_FILE, image pods have it at the Kubernetes path)."""
    tok = os.environ.get("TK8S_KV_TOKEN", "")
    for path in (os.environ.get("TK8S_SERVICEACCOUNT_TOKEN_FILE", ""), SA_TOKEN):
        if tok or not path:
            continue
        try:
            with open(path) as f:
                tok = f.read().strip()
        except OSError:
            pass
    return {"Authorization": f"Bearer {tok}"} if tok else {}


def _publish(url: str, value: str) -> None:
    urllib.request.urlopen(urllib.request.Request(url, data=value.encode(), method="PUT", headers=_kv_headers()),
                           timeout=10).read()


def _fetch(url: str, timeout: float) -> str:
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        wait = max(1, min(10, int(deadline - time.monotonic())))  # a long-poll never outlives the deadline
        try:
            v = urllib.request.urlopen(urllib.request.Request(url + f"?wait={wait}", headers=_kv_headers()),
                                       timeout=wait + 5).read().decode().strip()
            if v:
                return v
        except OSError:
            time.sleep(0.02)
    raise TimeoutError(f"no rendezvous address at {url} after {timeout:.0f}s")


def rccl_transport(text: str) -> dict:
    """What RCCL's ``NCCL_DEBUG=INFO`` log says about the channels it connected: per transport
    (P2P, SHM, NET, ...) the number of ``via <transport>/...`` connections and their forms, and
    whether ``Init COMPLETE`` was logged."""
    import re

    counts: dict[str, int] = {}
    forms: dict[str, int] = {}
    for m in re.finditer(r"\bvia ([A-Z0-9]+)(/[\w/.:-]*)?", text):
        counts[m.group(1)] = counts.get(m.group(1), 0) + 1
        form = m.group(1) + (m.group(2) or "")
        forms[form] = forms.get(form, 0) + 1
    return {"counts": counts, "forms": forms, "init_complete": "Init COMPLETE" in text,
            "lines": text.count("\n")}


def _debug_file() -> str | None:
    """Route RCCL's INFO log to a file of this rank's (before RCCL is loaded), if NCCL_DEBUG is on."""
    if not os.environ.get("NCCL_DEBUG"):
        return None
    if not os.environ.get("NCCL_DEBUG_FILE"):
        import tempfile

        os.environ["NCCL_DEBUG_FILE"] = os.path.join(tempfile.gettempdir(), f"tk8s-rccl-{os.getpid()}.log")
    return os.environ["NCCL_DEBUG_FILE"]


def sweep(rank: int, n: int, min_bytes: int, max_bytes: int, factor: int, iters: int, warmup: int,
          dtype: str = "float32", device: str = "cpu", phases: Phases | None = None) -> dict:
    import torch
    import torch.distributed as dist

    sync = torch.cuda.synchronize if device != "cpu" else (lambda: None)
    dt = {"float32": torch.float32, "bfloat16": torch.bfloat16}[dtype]
    esize = torch.tensor([], dtype=dt).element_size()
    results, ok, peak = [], True, 0.0
    size = max(min_bytes, esize)
    while size <= max_bytes:
        count = max(1, size // esize)
        pat = (torch.arange(count, dtype=torch.int64, device=device) % (251 if dt == torch.float32 else 4) + 1)
        want = (pat * (n * (n + 1) // 2)).to(dt)
        buf = torch.empty(count, dtype=dt, device=device)
        if phases is not None:
            phases.enter("sweep")
        for _ in range(warmup):
            buf.copy_(pat * (rank + 1))
            dist.all_reduce(buf)
        times = []
        bad = 0
        for _ in range(max(1, iters)):
            buf.copy_(pat * (rank + 1))
            sync()
            dist.barrier()
            t = time.perf_counter()
            dist.all_reduce(buf)
            sync()
            times.append(time.perf_counter() - t)
            if phases is not None and phases.phase != "check":
                phases.enter("check")
            bad = max(bad, int((buf != want).sum()))
        sec = sorted(times)[len(times) // 2]
        algbw = count * esize / sec / 1e9
        busbw = algbw * 2 * (n - 1) / n if n > 1 else 0.0  # 0 at n = 1 (no fabric)
        peak = max(peak, busbw)
        ok &= bad == 0
        results.append({"bytes": count * esize, "count": count, "time_us": sec * 1e6, "algbw_gbps": algbw,
                        "busbw_gbps": busbw, "bad": bad})
        size *= factor
    return {"ok": ok, "results": results, "peak_busbw_gbps": peak if n > 1 else None,
            "peak_algbw_gbps": max((r["algbw_gbps"] for r in results), default=0.0)}


def _rank_group(a, argv: list[str], k: int) -> int:
    """Run ranks group_index*k .. +k-1 as child processes; one merged JSON line for the pod."""
    import subprocess

    rest, skip = [], False
    for i, tok in enumerate(argv):  # drop --group-index/--devices (and their values), keep the rest
        if skip:
            skip = False
            continue
        if tok in ("--group-index", "--devices"):
            skip = True
            continue
        if tok.startswith(("--group-index=", "--devices=")):
            continue
        rest.append(tok)
    first = a.group_index * k
    procs = [subprocess.Popen([sys.executable, "-m", __spec__.name if __spec__ else "tritonk8ssupervisor_amd.parallel.dist_allreduce",
                               "--rank", str(first + j), *rest], stdout=subprocess.PIPE, text=True)
             for j in range(k)]
    outs = []
    # every child is bounded by its own deadlines and watchdog; this is the backstop over them
    bound = 6 * a.timeout + 4 * WATCHDOG_GRACE_S if a.timeout > 0 else None
    for pr in procs:
        try:
            out, _ = pr.communicate(timeout=bound)
        except subprocess.TimeoutExpired:
            pr.kill()
            out, _ = pr.communicate()
            out = json.dumps({"ok": False, "error": f"rank process did not end within {bound:.0f}s", "timed_out": True})
        line = (out or "").strip().splitlines()
        try:
            outs.append(json.loads(line[-1]) if line else {"ok": False, "error": f"rank exited {pr.returncode}"})
        except ValueError:
            outs.append({"ok": False, "error": line[-1][:200]})
    merged = dict(outs[0])
    merged.update(ok=all(o.get("ok") for o in outs), mode="rank_group", rank=first, first_rank=first, local_ranks=k,
                  peak_busbw_gbps=(min((o.get("peak_busbw_gbps") or 0.0 for o in outs), default=0.0)
                                   if a.nranks > 1 else None),
                  init_seconds=max((o.get("init_seconds", 0.0) for o in outs), default=0.0))
    errs = [o["error"] for o in outs if o.get("error")]
    if errs:
        merged["error"] = "; ".join(errs)
    print(json.dumps(merged))
    return 0 if merged["ok"] else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--rank", type=int)
    ap.add_argument("--group-index", type=int, help="the pod's index: ranks group-index*k .. +k-1")
    ap.add_argument("--devices", default="", help="the pod's GPUs, comma separated (k = their count)")
    ap.add_argument("--nranks", type=int, required=True)
    ap.add_argument("--kv-url", required=True)
    ap.add_argument("--min-bytes", type=int, default=1024)
    ap.add_argument("--max-bytes", type=int, default=4 << 20)
    ap.add_argument("--factor", type=int, default=4)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--dtype", choices=["float32", "bfloat16"], default="float32")
    ap.add_argument("--op-timeout", "--timeout", dest="timeout", type=float, default=20.0,
                    help="bound on each wait: rendezvous, init, every collective (s)")
    ap.add_argument("--backend", choices=["gloo", "nccl"], default="gloo", help="nccl = RCCL on ROCm (GPU tensors)")
    a = ap.parse_args(argv)
    if a.rank is None:
        if a.group_index is None:
            ap.error("one of --rank / --group-index is required")
        devs = [d for d in a.devices.split(",") if d.strip()] or ["0"]
        if len(devs) > 1:
            return _rank_group(a, argv if argv is not None else sys.argv[1:], len(devs))
        a.rank = a.group_index
    t0 = time.monotonic()
    debug_file = _debug_file() if a.backend == "nccl" else None
    host = os.environ.get("NODE_IP", "127.0.0.1")
    ph = Phases(a.rank, a.nranks, a.timeout)
    try:
        ph.enter("uid")
        import torch.distributed as dist
        from datetime import timedelta

        # Rank 0 binds the rendezvous store on an ephemeral port itself and publishes the port it
        # got: picking a free port and binding it later left a window in which another process on
        # the host took it (EADDRINUSE on the shared GPU box).
        if a.rank == 0:
            store = dist.TCPStore(host, 0, world_size=a.nranks, is_master=True,
                                  timeout=timedelta(seconds=a.timeout), wait_for_workers=False)
            _publish(a.kv_url, f"{host}:{store.port}")
        else:
            sh, sp = _fetch(a.kv_url, a.timeout).rsplit(":", 1)
            store = dist.TCPStore(sh, int(sp), world_size=a.nranks, is_master=False,
                                  timeout=timedelta(seconds=a.timeout))
        ph.enter("init")
        device = "cpu"
        if a.backend == "nccl":
            import torch

            torch.cuda.set_device(0)  # the device plugin exposes exactly this pod's GPU(s)
            device = "cuda:0"
        dist.init_process_group(a.backend, store=store, rank=a.rank, world_size=a.nranks,
                                timeout=timedelta(seconds=a.timeout))
        init_s = time.monotonic() - t0
        res = sweep(a.rank, a.nranks, a.min_bytes, a.max_bytes, a.factor, a.iters, a.warmup, a.dtype, device, ph)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - reported as the pod result
        print(json.dumps({"ok": False, "rank": a.rank, "nranks": a.nranks, "phase": ph.phase,
                          "timed_out": "timeout" in str(e).lower() or isinstance(e, TimeoutError),
                          "error": f"{type(e).__name__}: {e}"}), flush=True)
        os._exit(2)  # a failed process group's teardown can block on the dead peer
    with ph.lock:
        ph.deadline = 0.0
    out = {"ok": res["ok"], "backend": a.backend, "mode": "multi_process", "nranks": a.nranks, "rank": a.rank,
           "dtype": a.dtype, "init_seconds": round(init_s, 4), "peak_busbw_gbps": res["peak_busbw_gbps"],
           "peak_algbw_gbps": res["peak_algbw_gbps"], "op_timeout_s": a.timeout,
           "sweep": {"min_bytes": a.min_bytes, "max_bytes": a.max_bytes, "factor": a.factor, "iters": a.iters,
                     "warmup": a.warmup, "dtypes": [a.dtype]}, "results": res["results"]}
    if a.nranks == 1:
        out["fabric"] = "1 GPU: no fabric"
    if a.backend == "nccl":  # same tuning report as tk8s-rccl
        for k in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS"):
            out[k.lower()] = os.environ.get(k) or "auto"
        out["peak_links_equivalent"] = res["peak_busbw_gbps"] / 153.0 if a.nranks > 1 else None
    if debug_file and "%" not in debug_file:
        try:
            with open(debug_file, errors="replace") as f:
                text = f.read()
            sys.stderr.write(text)
            sys.stderr.flush()
            out["transport"] = rccl_transport(text)
        except OSError as e:
            out["transport"] = {"error": f"{debug_file}: {e}"}
    print(json.dumps(out))
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
