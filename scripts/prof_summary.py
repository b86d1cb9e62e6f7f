"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'total/step(us)':>14} {'calls/step':>10} {'avg(us)':>9} {'%':>6}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e3/steps:14.2f} {int(r['Calls'])/steps:10.1f} {float(r['AverageNs'])/1e3:9.2f} "
          f"{100*float(r['TotalDurationNs'])/tot:6.1f}  {r['Name'][:100]}")
print(f"sum of kernel time per step: {tot/1e3/steps:.1f} us over {sum(int(r['Calls']) for r in rows)/steps:.0f} launches")
