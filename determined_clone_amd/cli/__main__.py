import sys

from determined_clone_amd.cli.cli import main

sys.exit(main())
