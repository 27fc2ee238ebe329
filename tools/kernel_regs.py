#!/usr/bin/env python3
"""Per-kernel duration and register / scratch / LDS usage from a rocprofv3
--kernel-trace database (register spills show up as scratch_size > 0).

    python tools/kernel_regs.py DB [name-substring]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    q = ("select name, count(*), avg(duration), max(vgpr_count), max(accum_vgpr_count), max(scratch_size), "
         "max(lds_size) from kernels where name like ? group by name order by sum(duration) desc")
    for r in c.execute(q, (f"%{pat}%",)):
        print(f"{r[0][:70]:<70} x{r[1]:<5} {r[2] / 1e3:9.1f} us  vgpr {r[3]} agpr {r[4]} scratch {r[5]} lds {r[6]}")


if __name__ == "__main__":
    main()
