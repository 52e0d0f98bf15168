"""Parallelism: torch.distributed stripe sharding (RCCL/xGMI) and the host streaming pipeline."""
from .dist import (DistContext, DistributedRS, broadcast_matrix, gather_columns, init_distributed, scatter_columns,
                   shard_range)

__all__ = ["DistContext", "DistributedRS", "broadcast_matrix", "gather_columns", "init_distributed",
           "scatter_columns", "shard_range"]
