#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 rocpd SQLite database (the default output of
`rocprofv3 --kernel-trace -o NAME`): `python tools/rocpd_stats.py DB [--top N] [--start-frac F]`.
``--start-frac`` drops the first fraction of the trace's time span (warm-up)."""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--start-frac", type=float, default=0.0)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute("""select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
                    join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
t0 = min(r[1] for r in rows)
t1 = max(r[2] for r in rows)
cut = t0 + (t1 - t0) * a.start_frac
agg = {}
for name, s, e in rows:
    if s < cut:
        continue
    n, tot = agg.get(name, (0, 0))
    agg[name] = (n + 1, tot + (e - s))
total = sum(v[1] for v in agg.values())
print(f"window {(t1 - cut) / 1e6:.3f} ms, kernel-busy {total / 1e6:.3f} ms, {sum(v[0] for v in agg.values())} dispatches")
for name, (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
    print(f"{tot / 1e6:9.3f} ms {100 * tot / total:5.1f}% {n:7d}x  {name[:150]}")
