# Does the validation pod's `tk8s-probe --reuse` (which never calls HIP) still start the HIP
# runtime / open the KFD, e.g. through the fat-binary registration of libtk8s.so at load time?
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/reuse_cost; mkdir -p $o
echo '{"ok":true}' > /tmp/r.json
python3 - > $o/times.json <<'PY'
import json, subprocess, time
ts = []
for _ in range(4):
    time.sleep(0.5)
    t = time.perf_counter()
    subprocess.run(["tritonk8ssupervisor_amd/bin/tk8s-probe", "--reuse", "/tmp/r.json"], check=True, stdout=subprocess.DEVNULL)
    ts.append(round((time.perf_counter() - t) * 1000, 2))
print(json.dumps({"reuse_ms": ts}))
PY
sleep 1
AMD_LOG_LEVEL=4 timeout -k 5 30 tritonk8ssupervisor_amd/bin/tk8s-probe --reuse /tmp/r.json > $o/log4.txt 2>&1
cat $o/times.json; wc -l $o/log4.txt
