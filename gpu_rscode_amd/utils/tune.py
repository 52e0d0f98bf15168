"""``GFRS_TUNE``: the one switchboard for measured thresholds and A/B aids (Python side).

The native code reads the same variable (``csrc/include/gfrs/tune.h``): comma-separated
``key=value`` pairs, e.g. ``GFRS_TUNE=fp4=tm,gf16_mfma=1``. Python keys: ``gf16_mfma`` (0 | 1: never /
always the GF(2^16) matrix-core engine where supported), ``fp4_batch_min_cols`` (batched GF(2^8)
launches take the FP4 kernels from this many columns per stripe) and ``row_align`` (``alloc_rows``
pitch alignment of rows >= 8 MiB). Read on every call, so a test may switch them in-process.
"""
from __future__ import annotations

import os


def tune_str(key: str) -> str | None:
    env = os.environ.get("GFRS_TUNE", "")
    for item in env.split(","):
        k, sep, v = item.partition("=")
        if sep and k.strip() == key:
            return v.strip()
    return None


def tune_int(key: str, default: int) -> int:
    v = tune_str(key)
    try:
        return int(v) if v is not None else default
    except ValueError:
        return default


def with_tune(env: dict | None = None, **keys) -> dict:
    """A copy of ``env`` (default: os.environ) whose GFRS_TUNE also holds ``keys`` (for subprocesses)."""
    e = dict(os.environ if env is None else env)
    items = [x for x in e.get("GFRS_TUNE", "").split(",") if x and x.partition("=")[0] not in keys]
    items += [f"{k}={v}" for k, v in keys.items()]
    e["GFRS_TUNE"] = ",".join(items)
    return e
