"""The cluster's RCCL fabric check (BASELINE.json configs 4-5): after every node is Ready, an
Indexed Job all-reduces over every GPU -- one pod per physical host, its process driving all of
the host's GPUs as consecutive ranks (rccl_layout) -- and checks the result exactly; ``--rocprof`` runs the ranks under
rocprofv3 (kernel trace + stats, or one counter pass). The reference's readiness oracle was a
curl of the dashboard (setup.sh:56-85); this is the data-plane check that replaces it.

``FabricCheck`` is a mixin of orchestrator.Setup; the helpers below parse the ranks' logs and
the profiler's output.
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

from .workspace import SetupError, pod_portable


# What of the operator's environment reaches the fabric Job's ranks: RCCL's logging switches, and
# the fail-fast knobs and fault points (native/include/tk8s/failfast.h; a pod's env is otherwise
# an allowlist, agent.POD_ENV_KEEP).
RANK_ENV_PASS = ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "TK8S_GPU_SYNC_TIMEOUT_S", "TK8S_RCCL_BLOCKING")


def rccl_faults(spec: str) -> str:
    """The ``rccl.*`` entries of a TK8S_FAULTS spec (the ranks' own fault points)."""
    return ",".join(x.strip() for x in spec.split(",") if x.strip().startswith("rccl."))


def rccl_rank_env(fake: bool = False) -> tuple[list[dict], Path | None]:
    """Environment entries for the fabric Job's rank container, and the unpacked RCCL's directory
    (None: the installed library). Pods get an env allowlist, so RCCL's logging switches, the
    fail-fast knobs and the ``rccl.*`` fault points are passed on here; with real GPUs the rank
    loads RCCL with its gfx950 device code unpacked once per host (utils/rccl_unpack.py: no
    5.3 GB inflation in every rank's communicator start) and runs glibc's malloc on transparent
    huge pages: HIP copies RCCL's 108 MB code object several times while loading it (its stream
    read, comgr's set_data, ...), each copy into freshly faulted 4 KiB pages -- ~190 ms of a
    285 ms load was memcpy; on huge pages (the kernel's madvise mode is enough) the communicator
    start went from 318 to 202 ms on the MI355X (profiles/r5_thp/); the rank then loads that code
    and makes its stream on threads while the unique id is made (profiles/r6_rccl_prewarm/).
    Off-switches: TK8S_RCCL_UNPACKED=0, TK8S_RCCL_THP=0, TK8S_RCCL_PREWARM=0.

    The unpacked copy is asked for, not named: ``TK8S_RCCL_UNPACKED=1`` makes the agent of the
    node that runs the rank PREPEND its own current copy to the rank's LD_LIBRARY_PATH
    (agent._container_env; ADVICE r5: the copy is checked against the ROCm of that node, and the
    library path the node's runtime passes on is kept)."""
    from . import shortcut_on

    env = [{"name": var, "value": os.environ[var]} for var in RANK_ENV_PASS if os.environ.get(var)]
    faults = rccl_faults(os.environ.get("TK8S_FAULTS", ""))
    if faults:
        env.append({"name": "TK8S_FAULTS", "value": faults})
    if fake:
        return env, None
    from .utils.rccl_unpack import library_dir

    lib = library_dir()
    if lib is not None:
        env.append({"name": "TK8S_RCCL_UNPACKED", "value": "1"})
    if shortcut_on("TK8S_RCCL_THP"):
        tun = os.environ.get("GLIBC_TUNABLES")
        env.append({"name": "GLIBC_TUNABLES", "value": (tun + ":" if tun else "") + "glibc.malloc.hugetlb=1"})
    if not shortcut_on("TK8S_RCCL_PREWARM"):  # the rank's code load and stream on threads (tk8s_rccl.cpp)
        env.append({"name": "TK8S_RCCL_PREWARM", "value": "0"})
    return env, lib


class FabricCheck:
    @staticmethod
    def rccl_layout(k, g: int) -> dict:
        """Shape of the fabric Job: ONE pod per physical host (node label ``tk8s.amd.com/host``),
        its one process driving every GPU of the host as consecutive ranks -- one runtime start
        and one communicator init per host instead of one per node (8 one-GPU
        workers on one host were 8 rank processes). Several nodes on a host: the pod is
        host-scoped (``tk8s.amd.com/gpu-scope: host``, scheduler.py claims the other nodes' GPUs).
        Hosts must carry equal GPU counts (one Indexed Job, equal shares); else one pod per node
        when nodes are uniform, else one per GPU."""
        try:
            nodes = k.get("/api/v1/nodes").get("items", [])
        except Exception:  # noqa: BLE001 - the per-GPU shape works whatever the nodes say
            return {"per_pod": 1, "scope": "node"}
        per_node = {n["metadata"]["name"]: int((n.get("status", {}).get("allocatable") or {}).get("amd.com/gpu", 0) or 0)
                    for n in nodes}
        per_node = {nn: c for nn, c in per_node.items() if c > 0}
        hosts: dict[str, int] = {}
        for n in nodes:
            nn = n["metadata"]["name"]
            if nn in per_node:
                h = (n["metadata"].get("labels") or {}).get("tk8s.amd.com/host") or f"node:{nn}"
                hosts[h] = hosts.get(h, 0) + per_node[nn]
        if hosts and len(set(hosts.values())) == 1 and sum(hosts.values()) == g:
            nodes_per_host = len(per_node) // len(hosts)
            return {"per_pod": next(iter(hosts.values())), "scope": "host" if nodes_per_host > 1 else "node",
                    "hosts": len(hosts)}
        counts = list(per_node.values())
        if counts and len(set(counts)) == 1 and counts[0] * len(counts) == g:
            return {"per_pod": counts[0], "scope": "node"}
        return {"per_pod": 1, "scope": "node"}

    def run_rccl(self) -> dict | None:
        from .controlplane.client import client_from_kubeconfig
        from .kube import apply_objects, load_manifests, pods_of, wait_job

        if self.platform == "kubeadm":  # one RCCL-tests Job per GPU node (kubeadm_platform.py)
            return self.kubeadm_rccl()

        g = self.expected_gpus()
        enabled = self.rccl if self.rccl is not None else g >= 2
        if not enabled or g < 1:
            return None
        c = self._client()
        pid = self.project_id()
        k = client_from_kubeconfig(c.get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"}))
        job = f"rccl-allreduce-{int(time.time() * 1000) % 10**9:x}"
        layout = self.rccl_layout(k, g)
        per_pod = layout["per_pod"]
        npods = g // per_pod
        # one process per node drives all of that node's GPUs (ranks index*k .. index*k+k-1)
        group = ["--group-index", "$(JOB_COMPLETION_INDEX)", "--devices", "$(TK8S_GPU_DEVICES)", "--nranks", str(g)]
        # The Ready-path check's sweep: 1 KiB x4 up to --rccl-max-bytes (64 MiB), fp32, 5 timed
        # iterations -- shorter than the standalone validator's RCCL-tests sweep (8 B x2 to 1 GiB,
        # fp32 and bf16, tk8s-rccl's defaults); the report says so ("sweep").
        op = str(getattr(self, "rccl_op_timeout", 20.0))
        sweep = {"min_bytes": 1024, "max_bytes": int(self.rccl_max_bytes), "factor": 4, "iters": 5, "warmup": 2,
                 "dtypes": ["float32"], "what": "fabric check: 1 KiB x4 to --rccl-max-bytes, fp32 (the standalone "
                                                "tk8s-rccl sweeps 8 B x2 to 1 GiB in fp32 and bf16)"}
        if os.environ.get("TK8S_FAKE_GPUS"):
            cmd = ["$(TK8S_PYTHON)", "-m", "tritonk8ssupervisor_amd.parallel.dist_allreduce", *group,
                   "--kv-url", f"$(TK8S_KV_URL)/{job}/uid", "--max-bytes", str(1 << 20), "--op-timeout", op]
            sweep.update(max_bytes=1 << 20, iters=3, warmup=1)
        else:
            from .ops import BIN

            cmd = [pod_portable([str(BIN / "tk8s-rccl")])[0], *group,
                   "--kv-url", f"$(TK8S_KV_URL)/{job}/uid", "--min-bytes", "1024",
                   "--max-bytes", str(self.rccl_max_bytes), "--factor", "4", "--iters", "5", "--warmup", "2",
                   "--dtype", "float32", "--op-timeout", op]
        prof_dir = None
        if self.rocprof:
            import shutil

            rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
            if os.environ.get("TK8S_FAKE_GPUS") or not os.path.exists(rp):
                self.out("    --rocprof: rocprofv3 unavailable here (or GPUs are faked); profiling skipped")
            else:
                # N8 (BASELINE.json config 5): kernel trace + per-kernel stats of every rank. Counter
                # collection (--pmc) is a separate run by design: never mixed with tracing.
                # in the workspace, not .tk8s/: the ranks write it, and the pod jail denies .tk8s/
                prof_dir = self.ws.root / "rocprof" / job
                prof_dir.mkdir(parents=True, exist_ok=True)
                pmc = []
                if self.rocprof_counters:  # a counter pass: --pmc with --kernel-trace/--stats only
                    check_pmc_counters(self.rocprof_counters)
                    pmc = ["--pmc", *self.rocprof_counters]
                # (--teardown: the rank returns from main, so the profiler's exit handlers write its
                # trace -- tk8s-rccl otherwise leaves with _Exit right after its result)
                cmd = [rp, *pmc, "--kernel-trace", "--stats", "-d", str(prof_dir), "-o", "rank$(JOB_COMPLETION_INDEX)",
                       "--output-format", "csv", "--", *cmd, *([] if os.environ.get("TK8S_FAKE_GPUS") else ["--teardown"])]
        objs = load_manifests(self.ws.manifests / "rccl-allreduce-job.yaml",
                              {"job_name": job, "npods": npods, "gpus_per_pod": per_pod, "rccl_command": cmd,
                               "gpu_scope": layout["scope"]})
        c0 = objs[0]["spec"]["template"]["spec"]["containers"][0]
        extra, rccl_lib = rccl_rank_env(fake=bool(os.environ.get("TK8S_FAKE_GPUS")))
        if extra:
            c0.setdefault("env", []).extend(extra)
        if prof_dir is not None:  # the ranks write their traces there: a hostPath volume, which the pod jail allows
            pspec = objs[0]["spec"]["template"]["spec"]
            pspec["volumes"] = [{"name": "rocprof", "hostPath": {"path": str(prof_dir), "type": "DirectoryOrCreate"}}]
            pspec["containers"][0]["volumeMounts"] = [{"name": "rocprof", "mountPath": str(prof_dir)}]
        apply_objects(k, objs)
        self.out(f"Running RCCL all-reduce over {g} GPU(s) (job kube-system/{job}, {npods} pod(s) x {per_pod} GPU(s)"
                 + (", one process per host" if layout["scope"] == "host" else "") + ")")
        left = max(10.0, self.rccl_timeout or self.timeout)
        try:
            j = wait_job(k, job, "kube-system", timeout=left)
        except TimeoutError as e:
            raise SetupError(f"RCCL all-reduce Job {job} did not finish within {left:.0f}s: {e}", code=124) from e
        pods = pods_of(k, f"job-name={job}", "kube-system")
        results = [p.get("status", {}).get("result") or {} for p in pods]
        ok = j["status"].get("succeeded", 0) >= npods and all(r.get("ok") for r in results)
        first = next((r for r in results if r), {})
        rep = {"job": job, "ok": ok, "nranks": g, "pods": npods, "gpus_per_pod": per_pod, "scope": layout["scope"],
               **bandwidth_summary(results, g), "sweep": sweep, "op_timeout_s": float(op),
               "rccl_library": "unpacked" if rccl_lib is not None else "installed",
               "tuning": {k: first.get(k) for k in ("nccl_algo", "nccl_proto", "nccl_min_nchannels",
                                                    "nccl_max_nchannels", "peak_links_equivalent") if k in first},
               "rank_results": [rank_result(p) for p in pods]}
        done = [r["init_done_unix_ms"] for r in results if r.get("init_done_unix_ms")]
        if done:  # how unevenly the ranks' runtimes + communicators came up
            rep["init_spread_ms"] = round(max(done) - min(done), 3)
            rep["comm_init_ms_max"] = round(max(r.get("comm_init_ms", 0.0) for r in results), 3)
            rep["sweep_ms_max"] = round(max(r.get("sweep_ms", 0.0) for r in results), 3)
        rep["transport"] = rccl_transports([(p.get("metadata", {}).get("annotations") or {}).get("tk8s.amd.com/log-path")
                                            for p in pods])
        if prof_dir is not None:
            rep["rocprof"] = summarize_rocprof(prof_dir)
        if not ok:
            bad = [r for r in rep["rank_results"] if not r.get("ok")]
            why = "; ".join(f"{r['pod']}: phase {r.get('phase') or '?'}: {r.get('error') or 'failed'}" for r in bad)
            raise SetupError(f"RCCL all-reduce validation failed: {why[:600]} | {json.dumps(rep)[:600]}", code=2)
        return rep


def bandwidth_summary(results: list[dict], nranks: int) -> dict:
    """Peak algbw and busbw over the ranks' records. busbw = algbw * 2(n-1)/n: at
    one rank the all-reduce is a local copy and no link carries a byte, so busbw is null and the
    fabric line says "1 GPU: no fabric" (VERDICT r5 weak #4)."""
    alg = max((float(r.get("peak_algbw_gbps") or 0.0) for r in results), default=0.0)
    if nranks <= 1:
        return {"peak_busbw_gbps": None, "peak_algbw_gbps": alg, "fabric": "1 GPU: no fabric"}
    return {"peak_busbw_gbps": max((float(r.get("peak_busbw_gbps") or 0.0) for r in results), default=0.0),
            "peak_algbw_gbps": alg}


def fabric_line(rccl: dict) -> str:
    """The setup summary's RCCL clause: busbw over n GPUs, or, at one GPU, that there is no fabric
    (the all-reduce of one rank is a local copy; its algbw is not a link rate)."""
    if rccl.get("peak_busbw_gbps") is None:
        return (f"RCCL all-reduce ok over 1 GPU: no fabric (local algbw {float(rccl.get('peak_algbw_gbps') or 0):.1f} "
                f"GB/s)")
    return f"RCCL all-reduce peak busbw {rccl['peak_busbw_gbps']:.1f} GB/s over {rccl['nranks']} GPU(s)"


def rank_result(pod: dict) -> dict:
    """One fabric pod's verdict, with the phase and error a failed rank reported (tk8s-rccl /
    dist_allreduce print {"ok": false, "phase": ..., "error": ...})."""
    r = pod.get("status", {}).get("result") or {}
    out = {"pod": pod["metadata"]["name"], "node": pod["spec"].get("nodeName"), "ok": r.get("ok")}
    if not r.get("ok"):
        st = pod.get("status", {})
        term = next((cs.get("state", {}).get("terminated") for cs in st.get("containerStatuses") or []
                     if cs.get("state", {}).get("terminated")), None) or {}
        out.update(phase=r.get("phase"), error=str(r.get("error") or st.get("message") or "")[:300],
                   timed_out=bool(r.get("timed_out")), exit_code=term.get("exitCode"))
    return out


def rccl_transports(log_paths: list) -> dict:
    """Which transports the RCCL ranks' channels used, from their NCCL_DEBUG=INFO lines
    ("... via P2P/IPC", "via SHM/...", "via NET/..."): on one MI355X node every channel must be
    P2P over xGMI; SHM or NET means a host-memory or network fallback."""
    import re

    counts = {"p2p": 0, "shm": 0, "net": 0, "collnet": 0}
    seen = complete = False
    lib = None
    for p in log_paths:
        try:
            text = Path(p).read_text(errors="replace") if p else ""
        except OSError:
            continue
        for m in re.finditer(r" via (P2P|SHM|NET|COLLNET)\b", text):
            counts[m.group(1).lower()] += 1
        seen |= "NCCL INFO" in text
        complete |= "Init COMPLETE" in text
        m = re.search(r"Librccl path\s*:\s*(\S+)", text)
        lib = lib or (m.group(1) if m else None)
    # logged: RCCL's INFO log was there to judge (NCCL_DEBUG=INFO); a 1-rank communicator logs
    # its init but connects no channel, so its counts stay 0 with logged true
    counts.update(logged=seen, init_complete=complete, library=lib)
    return counts


# Hardware counters one rocprofv3 --pmc pass can hold per block on gfx950 (asking for more makes
# it fail with "error code 38" and hang). FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2.
PMC_BLOCK_LIMITS = {"SQ": 8, "TCC": 4, "TCP": 4, "TA": 2, "TD": 2, "GRBM": 2}
PMC_WEIGHT = {"FETCH_SIZE": ("TCC", 3), "WRITE_SIZE": ("TCC", 2)}


def check_pmc_counters(counters: list[str]) -> None:
    used: dict[str, int] = {}
    seen = set()
    for c in counters:
        base = c.rsplit("_", 1)[0] if c.endswith(("_sum", "_avr", "_min", "_max")) else c
        if base in seen:  # _sum/_avr/_min/_max of one counter count once
            continue
        seen.add(base)
        block, weight = PMC_WEIGHT.get(base, (base.split("_", 1)[0], 1))
        if block not in PMC_BLOCK_LIMITS:
            raise SetupError(f"--rocprof-counters: unknown counter block of {c!r} "
                             f"(supported: {', '.join(sorted(PMC_BLOCK_LIMITS))})")
        used[block] = used.get(block, 0) + weight
        if used[block] > PMC_BLOCK_LIMITS[block]:
            raise SetupError(f"--rocprof-counters: more than {PMC_BLOCK_LIMITS[block]} {block} counter slots in one "
                             "pass; split them over several runs")


def summarize_rocprof(prof_dir: Path, top: int = 5) -> dict:
    """Top kernels per rank from rocprofv3 `*_kernel_stats.csv` files under prof_dir, plus the
    per-kernel counter totals of a --pmc pass (`*_counter_collection.csv`)."""
    import csv

    out = {"dir": str(prof_dir), "ranks": {}}
    counters: dict[str, dict[str, dict[str, float]]] = {}
    for f in sorted(prof_dir.rglob("*counter_collection.csv")):
        rank = f.name.split("_counter_collection")[0]
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                k = (r.get("Kernel_Name") or "")[:120]
                name = r.get("Counter_Name") or ""
                try:
                    v = float(r.get("Counter_Value") or 0)
                except ValueError:
                    continue
                per = counters.setdefault(rank, {}).setdefault(k, {})
                per[name] = per.get(name, 0.0) + v
    if counters:
        out["counters"] = counters
    for f in sorted(prof_dir.rglob("*kernel_stats.csv")):
        with open(f, newline="") as fh:
            rows = list(csv.DictReader(fh))
        rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0) or 0))
        out["ranks"][f.name.split("_kernel_stats")[0]] = [
            {"kernel": r.get("Name", "")[:120], "calls": int(r.get("Calls", 0) or 0),
             "total_us": round(float(r.get("TotalDurationNs", 0) or 0) / 1e3, 2),
             "avg_us": round(float(r.get("AverageNs", 0) or 0) / 1e3, 3)} for r in rows[:top]]
    return out
