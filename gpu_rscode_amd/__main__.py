"""``python -m gpu_rscode_amd`` — the Python CLI (see gpu_rscode_amd/utils/cli.py)."""
import sys

from .utils.cli import main

sys.exit(main())
