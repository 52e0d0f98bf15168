"""File formats, timing/metrics and the Python CLI."""
from . import fileformat, timing

__all__ = ["fileformat", "timing"]
