"""Per-stream busy time of bench.py's timed window from a rocprofv3 database: how much of the
fused step each stream (BERT / speech+image / fusion) has a kernel running, their overlap,
and each stream's busy time split by kernel class.
    python tools/stream_timeline.py gpurun_out/prof_bench_f16/run_results.db [--steps 10]"""
import argparse
import sqlite3
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for s, e in iv:
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--marker', default='spin')
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute('select name, stream_id, queue_id, start, end from kernels order by start').fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    t0, t1 = rows[marks[0]][4], rows[marks[1]][3]
    rows = [r for r in rows if r[3] >= t0 and r[4] <= t1 and a.marker not in r[0]]
    wall = (t1 - t0) / a.steps / 1e6
    by = defaultdict(list)
    for name, sid, qid, s, e in rows:
        by[(sid, qid)].append((s, e, name))
    print(f'window {wall:.3f} ms/step, {len(rows)} dispatches')
    allv = []
    for k, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
        iv = [(s, e) for s, e, _ in v]
        allv += iv
        names = defaultdict(float)
        for s, e, n in v:
            names[n.split('(')[0][:60]] += (e - s)
        top = sorted(names.items(), key=lambda x: -x[1])[:4]
        print(f'stream {k}: {len(v) / a.steps:.0f} kernels/step, busy {union(iv) / a.steps / 1e6:.3f} ms/step, '
              f'sum {sum(e - s for s, e in iv) / a.steps / 1e6:.3f}; top: ' +
              ', '.join(f'{n} {t / a.steps / 1e6:.2f}' for n, t in top))
    print(f'any stream busy {union(allv) / a.steps / 1e6:.3f} ms/step')
    ks = sorted(by.keys(), key=lambda k: -len(by[k]))[:2]
    if len(ks) == 2:
        A = sorted((s, e) for s, e, _ in by[ks[0]])
        B = sorted((s, e) for s, e, _ in by[ks[1]])
        both = union(A) + union(B) - union(A + B)
        print(f'both of the two busiest streams busy: {both / a.steps / 1e6:.3f} ms/step')


if __name__ == '__main__':
    main()
