"""Average PMC counter values per dispatch from tools/pmc.sh output dirs (rocprofv3 CSV)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get('Counter_Name') or row.get('counter_name')
                v = float(row.get('Counter_Value') or row.get('counter_value') or 0)
                kname = row.get('Kernel_Name', '')[:60]
                grid = row.get('Grid_Size', '')
                vals[(kname, grid, name)].append(v)
    for (k, g, n), v in sorted(vals.items()):
        print(f'{k:60s} grid={g:>9s} {n:28s} n={len(v):3d} avg={sum(v) / len(v):.4g}')


if __name__ == '__main__':
    main(sys.argv[1])
