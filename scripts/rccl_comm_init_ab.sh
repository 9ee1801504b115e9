#!/usr/bin/env bash
# RCCL knobs that could shorten the 1-rank communicator start (comm_init_ms, ~205 ms), interleaved,
# 3 rounds, unpacked RCCL with huge-page malloc, as the fabric Job runs the rank.
set -o pipefail
out=gpurun_out/r5_rccl_commknobs
mkdir -p $out /tmp/cik
timeout -k 10 600 python3 -c "from tritonk8ssupervisor_amd.utils.build_native import build; build()" > $out/build.log 2>&1
lib=$(python3 -c "from tritonk8ssupervisor_amd.utils.rccl_unpack import library_dir; print(library_dir() or '')")
[[ -n "$lib" ]] || exit 3
for r in 1 2 3; do
  for v in base NCCL_CUMEM_ENABLE=0 NCCL_RUNTIME_CONNECT=1 NCCL_TUNER_PLUGIN=none NCCL_MAX_NCHANNELS=2; do
    sleep 1.5
    rm -f /tmp/cik/u
    if [[ $v == base ]]; then e=""; else e="$v"; fi
    env $e LD_LIBRARY_PATH=$lib GLIBC_TUNABLES=glibc.malloc.hugetlb=1 TK8S_TRACE=1 timeout -k 10 120 \
      ./tritonk8ssupervisor_amd/bin/tk8s-rccl --group-index 0 --devices 0 --nranks 1 --uid-file /tmp/cik/u \
      --max-bytes 4194304 --iters 3 --warmup 1 > /tmp/cik/out.json 2> /tmp/cik/err.txt || exit 1
    python3 - "$v" >> $out/results.txt <<'PY'
import json, sys
t = {}
for line in open("/tmp/cik/err.txt"):
    if line.startswith("TRACE "):
        _, ts, _, what = line.rstrip("\n").split(" ", 3)
        t.setdefault(what, float(ts))
d = json.loads(open("/tmp/cik/out.json").read().strip().splitlines()[-1])
ms = lambda a, b: round((t[b] - t[a]) * 1e3, 1) if a in t and b in t else None
print(sys.argv[1], {"comm_init_ms": round(d.get("comm_init_ms", 0), 1), "sweep_ms": round(d.get("sweep_ms", 0), 3),
                    "busbw": d.get("peak_busbw_gbps"), "total": ms("main", "exit")})
PY
  done
done
cat $out/results.txt
