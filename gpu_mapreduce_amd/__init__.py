"""gpu_mapreduce_amd — an MI355X-native MapReduce engine.

Same API surface as MR-MPI / baoxuezhao GPU-mapreduce (MapReduce object,
KeyValue/KeyMultiValue, OINK scripting, C and Python bindings), re-built for
AMD Instinct MI355X (gfx950): device-resident KV/KMV in HBM, hand-written
HIP/CDNA4 kernels for hashing, partitioning, radix sort, group-by, segmented
reduce and text/graph maps, and an RCCL all-to-all shuffle over xGMI with one
process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).
"""
from ._ext import C, so_path  # noqa: F401
from .parallel.comm import Comm, init, world  # noqa: F401
from .runtime.keyvalue import KeyValue, to_bytes  # noqa: F401
from .runtime.mapreduce import MapReduce, MultiValue  # noqa: F401

__version__ = "0.1.0"
