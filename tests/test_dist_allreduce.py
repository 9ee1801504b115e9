"""Multi-process all-reduce validator on CPU (gloo): the CPU twin of tk8s-rccl (N3/N6), with the
rank-0 address exchanged through the control-plane KV store exactly like the RCCL unique id."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

from test_controlplane import _start, _stop

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("nranks,dtype", [(2, "float32"), (3, "bfloat16")])
def test_gloo_allreduce_ranks_agree_exactly(tmp_path, nranks, dtype):
    p, c = _start(tmp_path)
    try:
        url = f"{c.base}/v1/kv/job-{nranks}/uid"
        procs = [subprocess.Popen([sys.executable, "-m", "tritonk8ssupervisor_amd.parallel.dist_allreduce", "--rank", str(r),
                                   "--nranks", str(nranks), "--kv-url", url, "--max-bytes", str(256 << 10), "--dtype", dtype],
                                  cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                  env={**os.environ, "TK8S_KV_TOKEN": c.token})  # the KV answers no anonymous caller
                 for r in range(nranks)]
        outs = [json.loads(pr.communicate(timeout=120)[0].strip().splitlines()[-1]) for pr in procs]
    finally:
        _stop(p)
    assert [o["rank"] for o in outs] == list(range(nranks))
    for o in outs:
        assert o["ok"] and o["nranks"] == nranks and o["dtype"] == dtype
        assert all(r["bad"] == 0 for r in o["results"])
        assert o["peak_busbw_gbps"] > 0
        sizes = [r["bytes"] for r in o["results"]]
        assert sizes[0] == 1024 and sizes[-1] == 256 << 10


def test_missing_peer_times_out_with_a_json_error(tmp_path):
    p, c = _start(tmp_path)
    try:
        r = subprocess.run([sys.executable, "-m", "tritonk8ssupervisor_amd.parallel.dist_allreduce", "--rank", "1",
                            "--nranks", "2", "--kv-url", f"{c.base}/v1/kv/none/uid", "--timeout", "1"],
                           cwd=REPO, capture_output=True, text=True, timeout=60, env={**os.environ, "TK8S_KV_TOKEN": c.token})
    finally:
        _stop(p)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 2 and not out["ok"] and "TimeoutError" in out["error"]
