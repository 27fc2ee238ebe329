"""Repeat tests/test_graph_mr.py::test_graph_mr_commands_out_of_core's sssp_mr
script (128 KiB HBM budget) K times in one process against scipy's Dijkstra;
prints which runs lose or change a vertex.   python tools/sssp_ooc_repeat.py [K]"""
import io
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from scipy.sparse import csr_matrix  # noqa: E402
from scipy.sparse.csgraph import dijkstra  # noqa: E402

from gpu_mapreduce_amd.oink.interp import OINK  # noqa: E402
from gpu_mapreduce_amd.parallel.comm import Comm  # noqa: E402
from test_graph_mr import parse_sources, weighted_graph  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = 3000
d = tempfile.mkdtemp()
os.chdir(d)
from pathlib import Path  # noqa: E402
e, w = weighted_graph(Path(d), n, 4 * n, 5)
G = csr_matrix((w, (e[:, 0], e[:, 1])), shape=(n, n))
comm = Comm(device="cuda")
bad = 0
for rep in range(K):
    out = io.StringIO()
    o = OINK(comm, screen=out, logfile="log.oink")
    o.file(text="set memsize -16384 maxpage 8\nsssp_mr 2 777 -i graph.w -o tmp.ssspmr NULL\n")
    rows = np.loadtxt("tmp.ssspmr.0", ndmin=2)
    start = 0
    msg = []
    for s0, it, cnt in parse_sources(out.getvalue()):
        r = rows[start:start + cnt]
        start += cnt
        dd = dijkstra(G, indices=s0)
        got = {int(v): dv for v, dv, _ in r}
        want = {i for i in range(n) if np.isfinite(dd[i])}
        miss, extra = sorted(want - set(got)), sorted(set(got) - want)
        wrong = [v for v in got if v in want and abs(got[v] - dd[v]) > 1e-4 * max(1.0, dd[v])]
        msg.append(f"src {s0} it {it} n {cnt} missing {miss[:8]} extra {extra[:8]} wrong {len(wrong)}")
        bad += bool(miss or extra or wrong)
    print(f"rep {rep}: " + " | ".join(msg), flush=True)
print("bad sources", bad, "of", 2 * K)
