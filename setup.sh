#!/usr/bin/env bash
# MI355X cluster bring-up wizard (same surface as the reference's setup.sh):
#   ./setup.sh            create: prompts, provisioning, configuration, readiness wait
#   ./setup.sh -c         teardown: destroy machines and reset configuration
# Non-interactive: ./setup.sh --answers answers.yaml --yes   (see docs/usage.md)
set -o errexit
set -o pipefail
cd "$(dirname "$0")"
PY="${TK8S_PYTHON:-python3}"
if [[ "${1:-}" == "-c" ]]; then
    shift
    exec "$PY" -S -c 'from tritonk8ssupervisor_amd.cli.fast import run; run()' clean "$@"
fi
# -S: skip site-packages .pth processing at start-up (tritonk8ssupervisor_amd/__init__.py adds
# the site directories back); -c instead of -m: no runpy. The CLI's start-up is part of the
# bring-up time.
exec "$PY" -S -c 'from tritonk8ssupervisor_amd.cli.fast import run; run()' setup "$@"
