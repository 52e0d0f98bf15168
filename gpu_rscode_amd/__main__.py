"""``python -m gpu_rscode_amd`` — the Python CLI (see gpu_rscode_amd/utils/cli.py)."""
import os
import sys

# before anything initialises HIP: RCCL peers of the --dist mode need dmabuf IPC on this driver
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from .utils.cli import main  # noqa: E402

sys.exit(main())
