"""Kernel stats (calls, total / average ns per kernel) from a rocprofv3 rocpd database
(`rocprofv3 --kernel-trace` without --output-format csv writes <name>_results.db).
python scripts/rocpd_stats.py <db> [steps]"""
import collections
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    names = {i: n for i, n in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    agg = collections.defaultdict(lambda: [0, 0])
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        a = agg[names.get(kid, str(kid))]
        a[0] += 1
        a[1] += e - s
    return agg


if __name__ == "__main__":
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    agg = stats(sys.argv[1])
    tot = sum(v[1] for v in agg.values())
    print("total %.2f ms per step" % (tot / 1e6 / steps))
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print("%9.3f ms/step %5d calls  %s" % (v[1] / 1e6 / steps, v[0], k[:110]))
