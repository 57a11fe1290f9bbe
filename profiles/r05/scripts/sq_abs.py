"""Per-kernel averages of a rocprofv3 --pmc counter CSV: absolute per dispatch, and per wave (/ SQ_WAVES when
collected in the same pass)."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"].split("(")[0][-60:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    c = {n: sum(x) / len(x) for n, x in v.items()}
    print(f"{sys.argv[2] if len(sys.argv) > 2 else ''} {k} dispatches {len(next(iter(v.values())))}: " +
          ", ".join(f"{n} {val:.4g}" for n, val in sorted(c.items())))
