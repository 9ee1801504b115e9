#!/usr/bin/env bash
# Is the k-concurrent-process start-up cost host-wide or per GPU? k copies of hsa_init_costs
# (ROCr only: hsa_init, agents, queues) start together, (a) with the GPU visible and (b) with
# no GPU visible (ROCR_VISIBLE_DEVICES=99: KFD open + CPU agent only). If (b) also slows down
# with k, the serialised part is host-wide (KFD process creation / topology), not per device.
# Binary built on the CPU host: g++ ... native/bench/hsa_init_costs.cpp -o build/bench/hsa_init_costs
set -euo pipefail
OUT=gpurun_out/conc
mkdir -p "$OUT"
BIN=build/bench/hsa_init_costs
run() {  # run <label> <k> [env...]
  local label=$1 k=$2; shift 2
  for i in $(seq "$k"); do env "$@" timeout -k 5 60 "$BIN" > "$OUT/$label.k$k.$i.json" & done
  wait
  sleep 1.5
}
sleep 1.5
for rep in 1 2; do
  for k in 1 2 4 8; do run "gpu.r$rep" "$k"; run "nogpu.r$rep" "$k" ROCR_VISIBLE_DEVICES=99; done
done
python3 - "$OUT" <<'PY'
import json, sys, glob, statistics, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{out}/*.json")):
    name = f.split("/")[-1]
    label, rep, k = name.split(".")[0], name.split(".")[1], int(name.split(".")[2][1:])
    try:
        d = json.load(open(f))
    except ValueError:
        continue
    agg[(label, k)].append(d.get("hsa_init_ms"))
summary = {f"{label} k={k}": {"median_hsa_init_ms": round(statistics.median([x for x in v if x is not None]), 1),
                               "max": round(max(x for x in v if x is not None), 1), "n": len(v)}
           for (label, k), v in sorted(agg.items())}
json.dump(summary, open(f"{out}/hsa_concurrency_summary.json", "w"), indent=1)
print(json.dumps(summary, indent=1))
PY
