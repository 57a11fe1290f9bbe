"""Per-kernel averages of a rocprofv3 --kernel-trace --stats run: from its kernel_stats CSV, or from its SQLite
database through /opt/rocm/bin/rocpd2summary (rocprofv3's default output format). Prints one line per product kernel
(calls, average and min/max in us) and writes the compact table as CSV.
Usage: python profiles/r06/kt_summary.py <run dir or .db or kernel_stats.csv> <out.csv>"""
import csv
import glob
import os
import subprocess
import sys
import tempfile

src, out = sys.argv[1], sys.argv[2]
if os.path.isdir(src):
    dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
    src = (csvs or dbs)[0]
if src.endswith(".db"):
    tmp = tempfile.mkdtemp()
    subprocess.run(["/opt/rocm/bin/rocpd2summary", "-i", src, "-f", "csv", "-d", tmp, "-o", "kt"], check=True,
                   capture_output=True)
    src = glob.glob(os.path.join(tmp, "*kernels_summary.csv"))[0]
rows = []
for r in csv.DictReader(open(src)):
    name = r.get("Name") or r.get("KERNEL_NAME") or ""
    if "annety_crc" not in name:
        continue
    short = name.replace("void ", "").replace("annety_crc::(anonymous namespace)::", "").split("(")[0]
    avg = float(r.get("Average (Nsec)") or r.get("AverageNs") or 0) / 1e3
    mn = float(r.get("Min (Nsec)") or r.get("MinNs") or 0) / 1e3
    mx = float(r.get("Max (Nsec)") or r.get("MaxNs") or 0) / 1e3
    rows.append((short, int(r.get("Calls") or 0), round(avg, 3), round(mn, 3), round(mx, 3)))
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "calls", "avg_us", "min_us", "max_us"])
    w.writerows(rows)
for r in rows:
    print(f"{r[0]:60s} {r[1]:6d} avg {r[2]:9.3f} us  min {r[3]:9.3f}  max {r[4]:9.3f}")
