"""Per-kernel duration summary from a rocprofv3 SQLite results database (rocpd schema).
usage: python tools/prof_db.py <results.db> [name-substring ...]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    subs = sys.argv[2:]
    c = sqlite3.connect(db)
    rows = c.execute("select k.display_name, d.end - d.start from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol k on d.kernel_id = k.id"
                     ).fetchall()
    agg = defaultdict(list)
    for name, dur in rows:
        if not subs or any(x in name for x in subs):
            agg[name].append(dur / 1000.0)
    total = sum(sum(v) for v in agg.values())
    print(f"{'%':>5} {'calls':>6} {'avg us':>9} {'min us':>9}  kernel")
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{100 * sum(v) / total:5.1f} {len(v):6d} {sum(v) / len(v):9.1f} {min(v):9.1f}  {name[:90]}")


if __name__ == "__main__":
    main()
