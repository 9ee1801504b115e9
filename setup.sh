#!/bin/bash
# MI355X cluster bring-up wizard (same surface as the reference's setup.sh):
#   ./setup.sh            create: prompts, provisioning, configuration, readiness wait
#   ./setup.sh -c         teardown: destroy machines and reset configuration
# Non-interactive: ./setup.sh --answers answers.yaml --yes   (see docs/usage.md)
set -o errexit
set -o pipefail
# (no subshells or extra execs before the CLI's interpreter: the shebang is bash itself and the
# script's directory comes from a parameter expansion, not $(dirname))
case "$0" in */*) cd "${0%/*}" ;; esac
PY="${TK8S_PYTHON:-python3}"
# TK8S_SHORTCUTS=0: the plain path, every start-up shortcut off (tritonk8ssupervisor_amd/__init__.py
# SHORTCUT_SWITCHES has the full list; these are the ones acted on before Python starts)
if [[ "${TK8S_SHORTCUTS:-1}" == 0 ]]; then
    export TK8S_HOST_BURNIN=0 TK8S_NO_PYCACHE_PREFIX=1 TK8S_SKIP_SITE=0
fi
PYFLAGS="-S"
if [[ "${TK8S_SKIP_SITE:-1}" == 0 ]]; then
    PYFLAGS=""  # site processing as usual (-S and the late site finder are a shortcut too)
fi
if [[ "${1:-}" == "-c" ]]; then
    shift
    exec "$PY" $PYFLAGS -c 'from tritonk8ssupervisor_amd.cli.fast import run; run()' clean "$@"
fi
# -S: skip site-packages .pth processing at start-up (tritonk8ssupervisor_amd/__init__.py adds
# the site directories back); -c instead of -m: no runpy. The CLI's start-up is part of the
# bring-up time.
exec "$PY" $PYFLAGS -c 'from tritonk8ssupervisor_amd.cli.fast import run; run()' setup "$@"
