#!/usr/bin/env python3
"""Feasibility check for GPU isolation of pods: inside an unprivileged user + mount namespace,
replace the KFD topology node list and /dev/dri with views that hold only the allowed GPUs, then
ask tk8s-gpuinfo what it sees. Prints one block per case."""
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "tritonk8ssupervisor_amd" / "bin"
TOPO = Path(os.path.realpath("/sys/class/kfd/kfd")) / "topology" / "nodes"


def nodes():
    out = []
    for d in sorted(TOPO.iterdir(), key=lambda p: int(p.name)):
        props = dict(ln.split() for ln in (d / "properties").read_text().splitlines() if len(ln.split()) == 2)
        out.append((int(d.name), int(props.get("simd_count", 0)), int(props.get("drm_render_minor", 0) or 0)))
    return out


SCRIPT = r"""
set -u
T="$1"; shift; KEEP="$1"; shift; MINORS="$1"; shift
S=$(mktemp -d /tmp/tk8s-iso.XXXXXX)
i=0
for n in $KEEP; do cp -r "$T/$n" "$S/$i" 2>/dev/null; i=$((i+1)); done
mkdir -p "$S/dri"
mount --bind /dev/dri "$S/dri" || { echo bind-dri-failed; exit 3; }
mount -t tmpfs tk8s-topo "$T" || { echo mount-topo-failed; exit 4; }
cp -r "$S"/[0-9]* "$T"/ && echo "topo-view: $(ls $T | tr '\n' ' ')"
mount -t tmpfs tk8s-dri /dev/dri || { echo mount-dri-failed; exit 5; }
for m in $MINORS; do touch /dev/dri/renderD$m && mount --bind "$S/dri/renderD$m" /dev/dri/renderD$m; done
echo "dri-view: $(ls /dev/dri | tr '\n' ' ')"
"$@"
echo "rc=$?"
"""


def case(title, keep, minors):
    print(f"=== {title}: keep nodes {keep}, render minors {minors}", flush=True)
    r = subprocess.run(["unshare", "-Urm", "--propagation", "private", "bash", "-c", SCRIPT, "iso", str(TOPO),
                        " ".join(map(str, keep)), " ".join(map(str, minors)), str(BIN / "tk8s-gpuinfo")],
                       capture_output=True, text=True, timeout=25)
    print(r.stdout[-3000:], r.stderr[-2000:], f"unshare rc={r.returncode}", flush=True)


ns = nodes()
print("nodes:", ns)
cpu = [n for n, simd, _ in ns if simd == 0]
gpu = [(n, m) for n, simd, m in ns if simd > 0]
print("=== plain userns, no masking", flush=True)
r = subprocess.run(["unshare", "-Urm", str(BIN / "tk8s-gpuinfo")], capture_output=True, text=True, timeout=25)
print(r.stdout[-2000:], r.stderr[-1000:], f"rc={r.returncode}", flush=True)
case("no GPU", cpu, [])
if gpu:
    case("first GPU only", cpu + [gpu[0][0]], [gpu[0][1]])
