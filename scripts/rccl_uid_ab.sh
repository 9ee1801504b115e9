#!/usr/bin/env bash
# ncclGetUniqueId's share of the fabric rank's start (trace: "ncclGetUniqueId" -> "unique id
# published"), with RCCL's bootstrap interface knobs, interleaved, 3 rounds, unpacked RCCL.
set -o pipefail
out=gpurun_out/r5_rccl_uid
mkdir -p $out /tmp/uid
timeout -k 10 600 python3 -c "from tritonk8ssupervisor_amd.utils.build_native import build; build()" > $out/build.log 2>&1
lib=$(python3 -c "from tritonk8ssupervisor_amd.utils.rccl_unpack import library_dir; print(library_dir() or '')")
[[ -n "$lib" ]] || exit 3
for r in 1 2 3; do
  for v in base NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 NCCL_NET_PLUGIN=none; do
    sleep 1.5
    rm -f /tmp/uid/u
    if [[ $v == base ]]; then e=""; else e="$v"; fi
    env $e LD_LIBRARY_PATH=$lib GLIBC_TUNABLES=glibc.malloc.hugetlb=1 TK8S_TRACE=1 timeout -k 10 120 \
      ./tritonk8ssupervisor_amd/bin/tk8s-rccl --group-index 0 --devices 0 --nranks 1 --uid-file /tmp/uid/u \
      --max-bytes 4194304 --iters 3 --warmup 1 > /tmp/uid/out.json 2> /tmp/uid/err.txt || exit 1
    python3 - "$v" >> $out/results.txt <<'PY'
import json, sys
t = {}
for line in open("/tmp/uid/err.txt"):
    if line.startswith("TRACE "):
        _, ts, _, what = line.rstrip("\n").split(" ", 3)
        t.setdefault(what, float(ts))
d = json.loads(open("/tmp/uid/out.json").read().strip().splitlines()[-1])
ms = lambda a, b: round((t[b] - t[a]) * 1e3, 1) if a in t and b in t else None
print(sys.argv[1], {"to_hip": ms("main", "hip runtime up"), "uid": ms("ncclGetUniqueId", "unique id published"),
                    "comm_init_ms": round(d.get("comm_init_ms", 0), 1), "total": ms("main", "exit")})
PY
  done
done
cat $out/results.txt
