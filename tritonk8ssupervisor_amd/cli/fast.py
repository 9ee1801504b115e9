"""Entry point of ./setup.sh: ``python -S -c 'from tritonk8ssupervisor_amd.cli.fast import run; run()' ARGS``.

``python -m`` goes through runpy and importlib.util (~2-3 ms on the MI355X host); a ``-c`` import
of this module does not, and the CLI's start-up is part of the bring-up time. sys.argv is
``['-c', <command>, ...]``, the same positions as under ``-m``.
"""
import sys


def run() -> None:
    if len(sys.argv) > 1 and sys.argv[1] == "setup":
        # before anything else is imported: the GPU burn-in is the bring-up's critical path
        from ..earlyburn import launch

        launch(sys.argv[2:])
    from .main import main

    raise SystemExit(main())
