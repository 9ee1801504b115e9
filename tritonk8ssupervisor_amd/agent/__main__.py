from .agent import main

raise SystemExit(main())
