"""Summarise profiles/pmc.sh passes: per kernel, the median per launch of every counter, and HBM bytes
= 2 x FETCH_SIZE (KiB) x 1024 + WRITE_SIZE (KiB) x 1024 (gfx950: FETCH_SIZE counts half of a wide
streaming read, MI355X_MICROARCH.md §HBM).  Usage: python profiles/pmc.py gpurun_out/pmc_<tag> [out.json]
The summary carries "_meta": per translation unit of the kernels measured, the library's source digest
(annety_amd.build.source_digest) of the tree the passes ran from, and the bench arguments; bench.py reports the file
as `traffic` only while those digests are the current ones."""
import collections
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from annety_amd.build import kernel_unit, source_digest  # noqa: E402

src = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)  # (dispatch, kernel, counter) -> summed over dimensions
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, k, c), v in per.items():
        name = k.replace("void ", "").replace("annety_crc::(anonymous namespace)::", "").split("(")[0]
        vals[name][c].append(v)
res = {}
for k, cs in vals.items():
    m = {c: statistics.median(v) for c, v in cs.items()}
    m["launches"] = max(len(v) for v in cs.values())
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        m["hbm_bytes_per_launch"] = int(2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024)
    if "TCC_HIT_sum" in m and m.get("TCC_MISS_sum") is not None:
        t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
        m["l2_hit_rate"] = m["TCC_HIT_sum"] / t if t else None
    res[k] = m
args = ""
if os.path.exists(os.path.join(src, "args.txt")):
    args = open(os.path.join(src, "args.txt")).read().strip()
units = sorted({kernel_unit(k) for k in res if k.startswith(("crc32_", "lhc_"))})
res["_meta"] = {"source_digest": {u: source_digest(u) for u in units}, "bench_args": args,
                "counters": "FETCH_SIZE, WRITE_SIZE, TCC_HIT_sum + TCC_MISS_sum: one rocprofv3 --pmc pass each"}
print(json.dumps(res, indent=1))
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump(res, f, indent=1)
