#!/bin/bash
# MI355X cluster bring-up wizard (same surface as the reference's setup.sh):
#   ./setup.sh            create: prompts, provisioning, configuration, readiness wait
#   ./setup.sh -c         teardown: destroy machines and reset configuration
# Non-interactive: ./setup.sh --answers answers.yaml --yes   (see docs/usage.md)
set -o errexit
set -o pipefail
# (no subshells or extra execs before the burn-in preload below: the shebang is bash itself and
# the script's directory comes from a parameter expansion, not $(dirname))
case "$0" in */*) cd "${0%/*}" ;; esac
PY="${TK8S_PYTHON:-python3}"
# TK8S_SHORTCUTS=0: the plain path, every start-up shortcut off (tritonk8ssupervisor_amd/__init__.py
# SHORTCUT_SWITCHES has the full list; these are the ones acted on before Python starts)
if [[ "${TK8S_SHORTCUTS:-1}" == 0 ]]; then
    export TK8S_PRELOAD_BURNIN=0 TK8S_HOST_BURNIN=0 TK8S_NO_PYCACHE_PREFIX=1
    PYFLAGS=""  # site processing as usual (-S and the late site finder are a shortcut too)
else
    PYFLAGS="-S"
fi
if [[ "${1:-}" == "-c" ]]; then
    shift
    exec "$PY" $PYFLAGS -c 'from tritonk8ssupervisor_amd.cli.fast import run; run()' clean "$@"
fi
# A non-interactive bring-up (--answers) preloads the GPU burn-in: tk8s-hsaprobe starts now, maps
# the ROCr runtime (~11 ms before its main()) while the CLI's interpreter starts, and waits on
# fd 7 for the plan (which GPUs, where the result goes) that earlyburn.py writes -- or for EOF
# when this run has no early burn-in (see tk8s_hsaprobe.cpp, --plan-stdin).
if [[ -z "${TK8S_FAKE_GPUS:-}" && "${TK8S_PRELOAD_BURNIN:-1}" != 0 && " $* " == *" --answers"* ]]; then
    for d in "${TK8S_HOME:-}" "${PYTHONPATH%%:*}" "$PWD"; do
        probe="$d/tritonk8ssupervisor_amd/bin/tk8s-hsaprobe"
        if [[ -n "$d" && -x "$probe" ]]; then
            exec 7> >(exec "$probe" --plan-stdin > /dev/null 2>&1)
            export TK8S_EARLY_PROBE_FD=7 TK8S_EARLY_PROBE_PID=$! TK8S_EARLY_PROBE_BIN="$probe"
            break
        fi
    done
fi
# -S: skip site-packages .pth processing at start-up (tritonk8ssupervisor_amd/__init__.py adds
# the site directories back); -c instead of -m: no runpy. The CLI's start-up is part of the
# bring-up time.
exec "$PY" $PYFLAGS -c 'from tritonk8ssupervisor_amd.cli.fast import run; run()' setup "$@"
