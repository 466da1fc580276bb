"""Top kernels of a rocprofv3 --stats kernel_stats.csv: python tools/kstats.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:80]:80s} calls={r['Calls']:>6} avg_us={float(r['AverageNs']) / 1e3:10.2f} "
          f"tot_ms={float(r['TotalDurationNs']) / 1e6:9.2f}")
