"""Per-dispatch SQ counter table from a rocprofv3 --pmc CSV (k_encode / k_modofdm rows in order).

usage: python tools/pmc_table.py <counter_collection.csv | rocprofv3 output directory>
A directory is searched (recursively) for its *counter_collection.csv files, which are read together."""
import csv
import glob
import os
import sys
from collections import defaultdict


def csv_files(path):
    if os.path.isdir(path):
        found = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))
        if not found:
            sys.exit(f"{path}: no *counter_collection.csv below this directory")
        return found
    return [path]


def main():
    if len(sys.argv) != 2:
        sys.exit(__doc__)
    rows = defaultdict(dict)
    names = {}
    for f in csv_files(sys.argv[1]):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
            names[d] = r["Kernel_Name"][:28]
    ctrs = sorted({c for v in rows.values() for c in v})
    print("disp kernel                      " + " ".join(f"{c[3:]:>14s}" for c in ctrs))
    for d in sorted(rows):
        print(f"{d:4d} {names[d]:28s} " + " ".join(f"{rows[d].get(c, 0):14.4g}" for c in ctrs))


if __name__ == "__main__":
    main()
