set -e
echo "tmp entries: $(ls -a /tmp | wc -l)  home=$HOME entries: $(ls -a $HOME | wc -l)"
J=$GRAFT_REPO_ROOT/tritonk8ssupervisor_amd/bin/tk8s-gpujail
W=$(mktemp -d /tmp/jt-XXXX); mkdir -p $W/.tk8s/machines/n1/pods/p $W/ansible/tmp $HOME/.local/state/tk8s $HOME/.cache
ARGS="--deny $W/.tk8s --deny $W/ansible/tmp --deny $HOME/.ssh --deny $HOME/.local/state/tk8s --read-only $GRAFT_REPO_ROOT --read-only $W --read-only $HOME --allow $HOME/.cache --allow $W/.tk8s/machines/n1/pods/p --scope-signals"
echo "rules: $($J $ARGS --plan | wc -l)"
python3 - "$J" $ARGS <<'PY'
import subprocess, sys, time
J, args = sys.argv[1], sys.argv[2:]
def t(cmd, n=30):
    v = []
    for _ in range(n):
        s = time.perf_counter(); subprocess.run(cmd); v.append(time.perf_counter() - s)
    v.sort(); return v[len(v) // 2] * 1e3
print("true %.2f ms, jail(no rules) %.2f ms, jail(policy) %.2f ms" % (t(["/bin/true"]), t([J, "--", "/bin/true"]), t([J, *args, "--", "/bin/true"])))
PY
