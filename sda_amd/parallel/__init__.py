"""Multi-GPU aggregation: one process per GPU, torch.distributed over RCCL/xGMI."""
from .comm import Comm  # noqa: F401
from .engine import DistributedAggregator  # noqa: F401
