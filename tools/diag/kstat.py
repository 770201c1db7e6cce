"""Per-kernel count / average / min duration (us) from a rocprofv3 rocpd database (--kernel-trace
without --stats writes only the .db): python tools/diag/kstat.py <db> [name-substring ...]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pats = sys.argv[2:] or [""]
for p in pats:
    for name, n, avg, mn in c.execute("select name, count(*), avg(end-start)/1000.0, min(end-start)/1000.0 from kernels "
                                      "where name like ? group by name order by sum(end-start) desc limit 8",
                                      (f"%{p}%",)):
        print(f"{avg:9.1f} us avg {mn:9.1f} min x{n:4d}  {name[:110]}")
