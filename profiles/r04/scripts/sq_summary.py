"""Per-kernel averages of a rocprofv3 --pmc counter CSV, as ratios to SQ_WAVE_CYCLES (one line per kernel)."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"].split("(")[0][-60:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    c = {n: sum(x) / len(x) for n, x in v.items()}
    w = c.get("SQ_WAVE_CYCLES", 1.0)
    print(f"{sys.argv[2] if len(sys.argv) > 2 else ''} {k} dispatches {len(next(iter(v.values())))}: " +
          ", ".join(f"{n} {val / w:.3f}" for n, val in sorted(c.items()) if n != "SQ_WAVE_CYCLES") +
          f" (SQ_WAVE_CYCLES {w:.4g})")
