"""tri_find_mr (the 4-collate MapReduce pipeline) on one R-MAT graph, twice
(the second run is warm); prints the per-stage times of each run.

    python tools/trimr_time.py SCALE [ooc [HBM_MIB [HOST_MIB]]]
    env: REPS (runs, default 2), CHECK=1 (TriangleGraph count as the check),
         FPATH (spool directory), BIG (an in-HBM run at that scale first), COPYBW=1

ooc: under an HBM budget (default 256 MiB) and a host budget (default 2 GiB),
spool files in a temporary directory; each stage also shows this rank's
host <-> device bytes and its time against the 50 GB/s PCIe floor."""
import os
import shutil
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_mapreduce_amd as g  # noqa: E402
from gpu_mapreduce_amd import C  # noqa: E402
from gpu_mapreduce_amd.models.pagerank import GRAPH500  # noqa: E402
from gpu_mapreduce_amd.models.triangles import tri_find_mr  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ooc = len(sys.argv) > 2 and sys.argv[2] == "ooc"
hbm = (int(sys.argv[3]) if len(sys.argv) > 3 else 256) << 20
host = (int(sys.argv[4]) if len(sys.argv) > 4 else 2048) << 20
if os.environ.get("NUMA") == "1":  # bind like bench.py's ranks (parallel/comm.py bind_numa_local)
    from gpu_mapreduce_amd.parallel.comm import bind_numa_local
    print("numa cpus", bind_numa_local(0), "of", len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else "?")
comm = g.Comm(device=os.environ.get("DEV", "cuda:0"))
if os.environ.get("PREPIN"):  # PREPIN=MiB: the pinned host arena before the job (gpu_mapreduce_amd/hostpin.py)
    from gpu_mapreduce_amd import hostpin
    print(f"prepin {os.environ['PREPIN']} MiB: {hostpin.prepin(int(os.environ['PREPIN'])):.1f} ms", flush=True)
if os.environ.get("HEARTBEAT"):  # a line every N s: long out-of-core runs are not taken for hung
    import threading
    import time as _t

    def _beat(every=float(os.environ["HEARTBEAT"]), t0=_t.perf_counter()):
        while True:
            _t.sleep(every)
            print(f"alive {(_t.perf_counter() - t0):.0f} s", flush=True)
    threading.Thread(target=_beat, daemon=True).start()
if os.environ.get("BIG"):  # first the bench's in-HBM run at scale BIG (the pool holds its peak after it)
    big = int(os.environ["BIG"])
    kb = C.map_rmat((1 << big) * 16, big, *GRAPH500, 0.0, 1, 0, comm.device)
    eb = kb.kdata.view(torch.int64).view(-1, 2)
    for _ in range(2):
        tri_find_mr(comm, eb)
    del kb, eb
    torch.cuda.synchronize()
    from gpu_mapreduce_amd.runtime import hbm_pool
    print("after BIG pool:", hbm_pool.stats(0), flush=True)
    if os.environ.get("TRIM") in ("1", "2"):
        hbm_pool.trim(0)
        print("trimmed pool:", hbm_pool.stats(0), flush=True)
    if os.environ.get("TRIM") == "2":  # the pinned host blocks cached by the caching host allocator too
        torch._C._host_emptyCache()
        print("host cache emptied", flush=True)
if os.environ.get("COPYBW") == "1":  # pinned <-> HBM copy rates in this process state
    import time
    h = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
    dv = torch.empty(1 << 30, dtype=torch.uint8, device=comm.device)
    for name, f in (("H2D", lambda: dv.copy_(h, non_blocking=True)), ("D2H", lambda: h.copy_(dv, non_blocking=True))):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        print(f"copy {name} 1 GiB pinned: {3 * (1 << 30) / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)
    t0 = time.perf_counter()
    for _ in range(20):
        x = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
        del x
    print(f"pinned 64 MiB alloc+free (caching host allocator): {(time.perf_counter() - t0) / 20 * 1e3:.2f} ms", flush=True)
    del h, dv
kv = C.map_rmat((1 << scale) * 16, scale, *GRAPH500, 0.0, 1, 0, comm.device)
if os.environ.get("BIG"):
    import resource
    print("host maxrss GB", resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, flush=True)
e = kv.kdata.view(torch.int64).view(-1, 2)
if os.environ.get("CHECK") == "1":  # the specialised TriangleGraph count as the check
    from gpu_mapreduce_amd.models.triangles import TriangleGraph
    want = TriangleGraph(comm, e, 1 << scale).count()
    print(f"check: TriangleGraph count {want}", flush=True)
    torch.cuda.empty_cache() if torch.cuda.is_available() else None
fdir = os.environ.get("FPATH") or None  # spool directory (default: a temporary one)
if fdir:
    import subprocess
    print(subprocess.run(["df", "-h", fdir], capture_output=True, text=True).stdout, flush=True)
for rep in range(int(os.environ.get("REPS", "2"))):
    root = tempfile.mkdtemp(prefix="mrh_trimr_", dir=fdir) if ooc else ""
    try:
        r = (tri_find_mr(comm, e, hbm_budget=hbm, host_budget=host, fpath=root, memsize=64) if ooc
             else tri_find_mr(comm, e))
    finally:
        if root:
            shutil.rmtree(root, ignore_errors=True)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    tot = sum(s["ms"] for s in r["stages"])
    if os.environ.get("PREPIN"):
        print("   arena", hostpin.stats(), flush=True)
    print(f"rep {rep}: {tot:.1f} ms, {r['triangles']} triangles"
          + (f" (check {want}: {'equal' if int(r['triangles']) == int(want) else 'DIFFERENT'})"
             if os.environ.get("CHECK") == "1" else ""), flush=True)
    if ooc:
        print(f"   spool files {r['spool_files']}, host {r['spool_host_bytes'] / 1e9:.2f} GB, "
              f"disk {r['spool_disk_bytes'] / 1e9:.2f} GB", flush=True)
    if torch.cuda.is_available():
        from gpu_mapreduce_amd.runtime import hbm_pool
        print("   pool:", hbm_pool.stats(0), flush=True)
    for s in r["stages"]:
        line = f"   {s['op']:<24} {s['ms']:9.2f} ms  in {s['pairs_in']:>12}  out {s['pairs_out']:>12}"
        b = s.get("h2d_bytes", 0) + s.get("d2h_bytes", 0)
        if ooc:
            floor = b / 50e6
            line += (f"  pcie {b / 1e6:9.1f} MB  floor {floor:7.2f} ms  x{s['ms'] / max(floor, 1e-3):6.1f}"
                     f"  disk {s.get('disk_bytes', 0) / 1e6:7.1f} MB")
        print(line, flush=True)
