"""Kernel timeline of a rocprofv3 --kernel-trace CSV: per dispatch its start
offset, duration and queue, from the first dispatch whose name matches
--from (its last occurrence, or the n-th with --nth) for --window ms, plus the
busy time per queue in that window.
python tools/timeline.py TRACE_DIR [--from whatif_seed] [--nth -4] [--window 40]"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    pat = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--from=")), "whatif_seed")
    nth = int(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--nth=")), "-4"))
    window = float(next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--window=")), "40")) * 1e6
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"),
                             r["Kernel_Name"]))
    rows.sort()
    starts = [r for r in rows if pat in r[3]]
    if not starts:
        raise SystemExit(f"no dispatch matches {pat}")
    t0 = starts[nth][0]
    busy = {}
    for s, e, q, name in rows:
        if s < t0 or s > t0 + window:
            continue
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  q{q:>3}  {name[:90]}")
        busy[q] = busy.get(q, 0) + (e - s)
    for q, b in sorted(busy.items()):
        print(f"queue {q}: busy {b / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
