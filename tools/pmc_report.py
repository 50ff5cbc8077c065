"""Per-kernel roofline table from one rocprofv3 kernel-trace database plus PMC passes of the
same command (tools/pmc_encoders.sh):

  dur_us    average dispatch duration (kernel trace)
  rd_MB     HBM-side read bytes  = 2 x FETCH_SIZE (KB) (gfx950: FETCH_SIZE reports half of
            16-B/lane streaming reads, MI355X_MICROARCH.md §HBM/rocprofv3)
  wr_MB     HBM-side write bytes = WRITE_SIZE (KB)
  GB/s      (rd + wr) / dur, and its fraction of the 8 TB/s HBM3E peak
  mfma%     SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the share of
            SIMD-cycles the matrix cores were busy while the kernel ran (= its fraction of the
            dense MFMA peak for the instruction it issues)

usage: python tools/pmc_report.py TRACE_DB PMC_DIR [--min-us 5]"""
import argparse
import csv
import glob
import os
import sqlite3
from collections import defaultdict

HBM_PEAK_GBS = 8000.0
SIMDS = 256 * 4
XCDS = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('pmc')
    ap.add_argument('--min-us', type=float, default=5.0)
    a = ap.parse_args()
    dur = defaultdict(list)
    for name, gx, d in sqlite3.connect(a.db).execute('select name, grid_x, end-start from kernels'):
        dur[(name, int(gx))].append(d / 1e3)
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(a.pmc, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row['Kernel_Name'], int(float(row['Grid_Size'])))
                # one row per (dispatch, counter); GRBM appears in every pass: keep it per pass
                cnt[key][row['Counter_Name'] + ('@' + os.path.basename(os.path.dirname(f)))].append(
                    float(row['Counter_Value']))
    print(f"{'kernel':70s} {'grid':>9s} {'dur_us':>8s} {'rd_MB':>8s} {'wr_MB':>8s} {'GB/s':>7s} {'hbm%':>5s} {'mfma%':>6s}")
    rows = []
    for key, ds in dur.items():
        d = sum(ds) / len(ds)
        if d < a.min_us or key not in cnt:
            continue
        c = {k: sum(v) / len(v) for k, v in cnt[key].items()}
        get = lambda n: next((v for k, v in c.items() if k.split('@')[0] == n), None)  # noqa: E731
        fetch, write = get('FETCH_SIZE'), get('WRITE_SIZE')
        rd = 2 * fetch * 1024 / 1e6 if fetch is not None else None
        wr = write * 1024 / 1e6 if write is not None else None
        gbs = (rd + wr) / 1e3 / (d / 1e6) if rd is not None and wr is not None else None
        mf = None
        busy = get('SQ_VALU_MFMA_BUSY_CYCLES')
        if busy is not None:
            grbm = next(v for k, v in c.items() if k.startswith('GRBM_GUI_ACTIVE@') and
                        any(k2.split('@')[0] == 'SQ_VALU_MFMA_BUSY_CYCLES' and k2.split('@')[1] == k.split('@')[1]
                            for k2 in c))
            mf = 100 * busy / (grbm / XCDS * SIMDS)
        rows.append((d * len(ds), key, d, rd, wr, gbs, mf))
    f = lambda v, fmt: (fmt % v) if v is not None else '-'  # noqa: E731
    for _, (name, g), d, rd, wr, gbs, mf in sorted(rows, key=lambda r: -r[0]):
        print(f"{name[:70]:70s} {g:9d} {d:8.1f} {f(rd, '%8.1f'):>8s} {f(wr, '%8.1f'):>8s} {f(gbs, '%7.0f'):>7s} "
              f"{f(gbs and 100 * gbs / HBM_PEAK_GBS, '%5.1f'):>5s} {f(mf, '%6.1f'):>6s}")


if __name__ == '__main__':
    main()
