"""Parallelism: torch.distributed stripe sharding (RCCL/xGMI), per-step parity placement, and the
host streaming pipeline."""
from .dist import (DistContext, DistributedRS, broadcast_matrix, gather_columns, init_distributed, scatter_columns,
                   shard_range)
from .placement import MODES as PLACEMENT_MODES
from .placement import ParityExchange, even_splits

__all__ = ["DistContext", "DistributedRS", "PLACEMENT_MODES", "ParityExchange", "broadcast_matrix", "even_splits",
           "gather_columns", "init_distributed", "scatter_columns", "shard_range"]
