"""Device functors from Python: a histogram of hashed integers, with the map
and the reduce written as HIP device code that the engine compiles at run
time for the GPU (gfx950) and runs over HBM-resident pairs — no host
callback touches a pair.

    python examples/python/device_functors.py [ntask=50000000] [nbucket=4096]

(needs a GPU MapReduce; multi-GPU: torchrun --nproc-per-node 8 ...)"""
import struct
import sys

import gpu_mapreduce_amd as g

ntask = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
nbucket = int(sys.argv[2]) if len(sys.argv) > 2 else 4096

MAP = f"""
// task t -> (bucket of a splitmix64 hash of t, 1)
__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long t, mrd::Emit& out) {{
  unsigned long long x = (unsigned long long)t + 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  out.emit((long long)(x % {nbucket}ull), (int)1);
}}
"""

# the reduce as a fold: every 256-value chunk of a key gets its own thread,
# the chunks' accumulators merge in a tree — a hot bucket costs no more
FOLD = """
struct mr_acc { long long n; };
__device__ void mr_init(mrd::Bytes key, mr_acc& a) { a.n = 0; }
__device__ void mr_add(mr_acc& a, mrd::Bytes v) { a.n += v.as<int>(); }
__device__ void mr_merge(mr_acc& a, const mr_acc& b) { a.n += b.n; }
__device__ void mr_finish(mrd::Bytes key, const mr_acc& a, mrd::Emit& out) { out.emit(key.as<long long>(), a.n); }
"""


def main():
    comm = g.init()
    if not comm.is_cuda:
        print("device functors need a GPU MapReduce; nothing to do on the CPU engine")
        return 0
    mr = g.MapReduce(comm)
    npairs = mr.map_device(ntask, MAP)
    nkeys = mr.collate()
    mr.reduce_device(FOLD)
    counts = {}
    mr.scan_kv(lambda k, v: counts.__setitem__(struct.unpack("<q", k)[0], struct.unpack("<q", v)[0]))
    total = comm.allreduce(sum(counts.values()), "sum")
    if comm.rank == 0:
        print(f"{npairs} pairs, {nkeys} buckets, total count {total}")
    assert total == ntask
    return 0


if __name__ == "__main__":
    sys.exit(main())
