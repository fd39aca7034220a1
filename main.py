#!/usr/bin/env python
"""gfedntm_amd command line (reference-compatible flags; see gfedntm_amd/cli.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gfedntm_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    main()
