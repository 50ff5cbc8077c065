"""Per-kernel average of every counter in one rocprofv3 --pmc pass (CSV), with the stall split
of the SQ wave-cycle counters (MI355X_MICROARCH.md "rocprofv3 PMC slots"):

    python tools/pmc_sq.py PMC_DIR [--min-waves 0]

Columns: dispatches, then each counter's per-dispatch mean; if the SQ wave-cycle counters are
present, wait% / inst-stall% / active% of SQ_WAVE_CYCLES and the LDS bank-conflict share of the
LDS-array cycles."""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('pmc')
    a = ap.parse_args()
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(a.pmc, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                cnt[(row['Kernel_Name'], int(float(row['Grid_Size'])))][row['Counter_Name']].append(float(row['Counter_Value']))
    names = sorted({n for v in cnt.values() for n in v})
    print('kernel'.ljust(72), 'n', ' '.join(n[:14].rjust(14) for n in names), 'wait% stall% active% ldsconf%')
    rows = []
    for key, c in cnt.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        wc = m.get('SQ_WAVE_CYCLES') or 0
        ext = ''
        if wc:
            ext = ' %5.1f %6.1f %7.1f' % (100 * m.get('SQ_WAIT_ANY', 0) / wc, 100 * m.get('SQ_WAIT_INST_ANY', 0) / wc,
                                          100 * m.get('SQ_ACTIVE_INST_ANY', 0) / wc)
        if m.get('SQ_LDS_IDX_ACTIVE'):
            ext += ' %8.1f' % (100 * m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE'])
        rows.append((wc * len(next(iter(c.values()))), key, len(next(iter(c.values()))), m, ext))
    for _, (name, g), n, m, ext in sorted(rows, key=lambda r: -r[0]):
        print(name[:72].ljust(72), n, ' '.join(('%14.4g' % m[k]) if k in m else '-'.rjust(14) for k in names), ext)


if __name__ == '__main__':
    main()
