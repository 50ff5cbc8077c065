"""Summarise a rocprofv3 rocpd database (or kernel_stats.csv) into a per-kernel table.
usage: python tools/prof_summary.py gpurun_out/prof/run_results.db [--steps N]"""
import sqlite3
import sys


def main(path, steps=None):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = 'kernel_name' if 'kernel_name' in cols else 'name'
    rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name_col} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':90s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for n, cnt, s, a, mn, mx in rows:
        print(f"{n[:90]:90s} {cnt:6d} {s/1e6:10.3f} {a/1e3:9.1f} {mn/1e3:9.1f} {mx/1e3:9.1f} {100*s/tot:6.2f}")
    print(f"total kernel time {tot/1e6:.3f} ms")


if __name__ == '__main__':
    main(sys.argv[1])
