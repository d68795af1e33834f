"""Per-kernel average durations from a rocprofv3 rocpd database (development)."""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
disp = [t for (t,) in c.execute("select name from sqlite_master where name like 'rocpd_kernel_dispatch_%'")][0]
sym = [t for (t,) in c.execute("select name from sqlite_master where name like 'rocpd_info_kernel_symbol_%'")][0]
names = dict(c.execute(f"select id, kernel_name from {sym}"))
acc = defaultdict(list)
for kid, st, en in c.execute(f"select kernel_id, start, end from {disp}"):
    acc[names.get(kid, kid)].append(en - st)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{len(v):5d} {sum(v)/len(v)/1e3:10.2f} us  {k[:110]}")
