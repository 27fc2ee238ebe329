"""Process-group layer: one process per GPU, torch.distributed over RCCL (xGMI)."""
from .comm import Comm, init, world  # noqa: F401
