"""Summarise a rocprofv3 rocpd database into per-kernel tables.
usage: python tools/prof_summary.py DB [--by-grid] [--window MARKER] [--steps K]
--by-grid splits a kernel name by launch grid (tells GEMM shapes apart).
--window keeps only the dispatches between the first two launches of the MARKER kernel
(bench.py brackets its timed region with torch.cuda._sleep, i.e. a spin_kernel), so
autotuning and warm-up launches drop out; --steps K adds a per-step column."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--by-grid', action='store_true')
    ap.add_argument('--match', default=None, help='substring filter on the kernel name')
    ap.add_argument('--window', default=None, help='marker kernel name substring')
    ap.add_argument('--steps', type=int, default=0)
    ap.add_argument('--sequence', action='store_true',
                    help='with --window and --steps: list one step\'s dispatches in launch order, '
                         'each averaged over the steps')
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    q = "select name, grid_x, workgroup_x, end-start, start from kernels order by start"
    rows = c.execute(q).fetchall()
    if a.window:
        marks = [i for i, r in enumerate(rows) if a.window in r[0]]
        if len(marks) < 2:
            raise SystemExit(f'fewer than two {a.window} dispatches in {a.db}')
        t0, t1 = rows[marks[0]][4], rows[marks[1]][4]
        rows = [r for r in rows if t0 < r[4] < t1 and a.window not in r[0]]
    if a.sequence:
        if not (a.window and a.steps) or len(rows) % a.steps:
            raise SystemExit('--sequence needs --window, --steps and a whole number of dispatches per step')
        n = len(rows) // a.steps
        tot = 0.0
        print(f"{'#':>4s} {'kernel':80s} {'blocks':>7s} {'avg_us':>9s} {'min_us':>9s} {'cum_ms':>8s}")
        for i in range(n):
            ds = [rows[k * n + i][3] for k in range(a.steps)]
            name, gx, wx = rows[i][0], rows[i][1], rows[i][2]
            tot += sum(ds) / len(ds)
            print(f"{i:4d} {name[:80]:80s} {gx // max(wx, 1):7d} {sum(ds) / len(ds) / 1e3:9.1f} {min(ds) / 1e3:9.1f} "
                  f"{tot / 1e6:8.3f}")
        return
    agg = {}
    for name, gx, wx, d, _ in rows:
        if a.match and a.match not in name:
            continue
        key = (name, gx // max(wx, 1)) if a.by_grid else (name, None)
        s = agg.setdefault(key, [0, 0, 1e18, 0])
        s[0] += 1
        s[1] += d
        s[2] = min(s[2], d)
        s[3] = max(s[3], d)
    tot = sum(v[1] for v in agg.values())
    ps = f" {'ms/step':>8s}" if a.steps else ''
    print(f"{'kernel':88s} {'blocks':>7s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}"
          + ps)
    for (n, g), (cnt, s, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        gs = '' if g is None else str(g)
        st = f" {s / 1e6 / a.steps:8.3f}" if a.steps else ''
        print(f"{n[:88]:88s} {gs:>7s} {cnt:6d} {s/1e6:10.3f} {s/cnt/1e3:9.1f} {mn/1e3:9.1f} {mx/1e3:9.1f} {100*s/tot:6.2f}"
              + st)
    per = f", {tot / 1e6 / a.steps:.3f} ms/step" if a.steps else ''
    print(f"total kernel time {tot/1e6:.3f} ms over {sum(v[0] for v in agg.values())} dispatches{per}")


if __name__ == '__main__':
    main()
