"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_stats.csv) per kernel."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    q = """select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
           join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""
    rows = {}
    for name, st, en in con.execute(q):
        rows.setdefault(name, []).append((en - st) * 1e-3)  # ns -> us
    return rows


def main(path, top=30):
    if os.path.isdir(path):
        c = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = c[0]
    rows = from_db(path)
    tot = sum(sum(v) for v in rows.values())
    out = sorted(((sum(v), len(v), k) for k, v in rows.items()), reverse=True)
    print(f"{'total_us':>12} {'calls':>7} {'avg_us':>9} {'pct':>6}  kernel")
    for t, n, k in out[:top]:
        print(f"{t:12.1f} {n:7d} {t / n:9.2f} {100 * t / tot:6.2f}  {k[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])
