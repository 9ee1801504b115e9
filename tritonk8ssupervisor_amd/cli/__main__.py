import sys

if len(sys.argv) > 1 and sys.argv[1] == "setup":
    # before anything else is imported: the GPU burn-in is the bring-up's critical path
    from ..earlyburn import launch

    launch(sys.argv[2:])

from .main import main  # noqa: E402

raise SystemExit(main())
