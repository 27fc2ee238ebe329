"""map_device alone (2^27 tasks -> (t % 2^20, 1)), 4 times: run under
rocprofv3 --kernel-trace to see the count / scan / write split."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_mapreduce_amd.parallel.comm import Comm  # noqa: E402
from gpu_mapreduce_amd.runtime.mapreduce import MapReduce  # noqa: E402

MAP = """
__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long t, mrd::Emit& out) {
  out.emit((long long)(t & 1048575), (int)1);
}
"""
comm = Comm(device="cuda")
for _ in range(4):
    mr = MapReduce(comm)
    mr.map_device(1 << 27, MAP)
    torch.cuda.synchronize()
