"""Print the top kernels of a rocprofv3 --stats run (kernel_stats.csv under DIR)."""
import csv
import glob
import re
import sys

d = sys.argv[1]
files = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
if not files:
    sys.exit(f"no kernel_stats.csv under {d}")
rows = list(csv.DictReader(open(files[0])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{files[0]}: total kernel time {tot / 1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    m = re.search(r"k_\w+(<[^>]*>)?", r["Name"])
    name = m.group(0) if m else r["Name"][:60]
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {100 * float(r['TotalDurationNs']) / tot:5.1f}% "
          f"n={r['Calls']:>7} avg={float(r['AverageNs']) / 1e3:8.2f} us  {name}")
