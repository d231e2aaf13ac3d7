"""Per-dispatch SQ counter table from a rocprofv3 --pmc CSV (k_encode / k_modofdm rows in order)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
rows = defaultdict(dict)
names = {}
for r in csv.DictReader(open(path)):
    d = int(r["Dispatch_Id"])
    rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
    names[d] = r["Kernel_Name"][:28]
ctrs = sorted({c for v in rows.values() for c in v})
print("disp kernel                      " + " ".join(f"{c[3:]:>14s}" for c in ctrs))
for d in sorted(rows):
    print(f"{d:4d} {names[d]:28s} " + " ".join(f"{rows[d].get(c, 0):14.4g}" for c in ctrs))
