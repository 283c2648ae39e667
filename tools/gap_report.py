"""GPU idle gaps between consecutive dispatches of one bench step, from a
rocprofv3 --kernel-trace (+ --memory-copy-trace) CSV directory.
usage: python tools/gap_report.py <dir> [first-kernel-of-step]"""
import csv
import glob
import sys

d = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_extract_hist"
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48]))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
ev.sort()
starts = [i for i, e in enumerate(ev) if first in e[2]]
if len(starts) < 3:
    sys.exit(f"fewer than 3 steps found starting with {first}")
i0, i1 = starts[-2], starts[-1]  # the last complete step
step = ev[i0:i1]
t0 = step[0][0]
tot_gap = 0
prev_end = t0
for s, e, n in step:
    gap = max(0, s - prev_end)
    tot_gap += gap
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {n}")
    prev_end = max(prev_end, e)
print(f"step span {(step[-1][1] - t0) / 1e3:.1f} us, idle {tot_gap / 1e3:.1f} us")
