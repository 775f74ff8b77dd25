"""Per-kernel summary of a rocprofv3 results database: python tools/prof_db.py DB [N]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = c.execute('select name, count(*), avg(end-start)/1000.0, sum(end-start)/1000.0 from kernels '
                 'group by name order by sum(end-start) desc limit ?', (n,)).fetchall()
for r in rows:
    print(f'{r[3]:10.1f} us total {r[1]:5d} x {r[2]:8.2f} us  {r[0][:120]}')
