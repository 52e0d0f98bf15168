"""Codec models: systematic Reed-Solomon over GF(2^8) / GF(2^4)-nibbles."""
from .rs import ReedSolomon, UnrecoverableError, alloc_rows, flat_rows

__all__ = ["ReedSolomon", "UnrecoverableError", "alloc_rows", "flat_rows"]
