"""Summarise a profiles/collect.sh run into committed files under profiles/.

<tag>_kernel_stats.csv   rocprofv3 --stats kernel summary of the bench command
<tag>_pmc_traffic.json   per-launch HBM bytes of the hot kernel from separate FETCH_SIZE / WRITE_SIZE
                         passes, with the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE
                         (KiB) counts half of a wide coalesced streaming read -> bytes = 2*FETCH*1024;
                         WRITE_SIZE (KiB) exact -> bytes = WRITE*1024.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

src, tag = sys.argv[1], sys.argv[2]
dst = os.path.dirname(os.path.abspath(__file__))


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(src, pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))

def counter(name):
    vals = [float(r["Counter_Value"]) for r in rows(f"{'fetch' if name == 'FETCH_SIZE' else 'write'}/**/*counter_collection.csv")
            if r["Counter_Name"] == name and "crc32_" in r["Kernel_Name"]]
    return vals

fetch = counter("FETCH_SIZE")
write = counter("WRITE_SIZE")
trace = [r for r in rows("kt/**/*kernel_trace.csv") if "crc32_" in r["Kernel_Name"]]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace]
res = {
    "payloads": 1 << 20,
    "len": 1024,
    "kernel": trace[0]["Kernel_Name"] if trace else None,
    "launches_traced": len(durs),
    "kernel_ms_avg_rocprof": statistics.mean(durs) if durs else None,
    "fetch_size_kib_median": statistics.median(fetch) if fetch else None,
    "write_size_kib_median": statistics.median(write) if write else None,
}
if fetch and write:
    res["hbm_bytes_per_launch"] = int(2 * res["fetch_size_kib_median"] * 1024 + res["write_size_kib_median"] * 1024)
    res["algorithmic_bytes_per_launch"] = (1 << 30) + 4 * (1 << 20)
    res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / res["algorithmic_bytes_per_launch"]
with open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
