#!/usr/bin/env python3
"""Per-step kernel table of the graph-replayed training steps from a rocprofv3 kernel trace.

    python scripts/graph_steady_state.py <run_kernel_trace.csv> [marker_substring]

Steady state = the longest run of kernels without a ``copyBuffer`` (copies happen in setup, in the
eager warm-up steps and in the host reads after the timed region; the replayed multi-step graphs
issue none). A step is delimited by the
marker kernel (default: the optimizer launch, ``adam``). Prints mean us per step for each kernel,
the kernel time per step and the first-start to last-end span per step."""
import collections
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[-1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "adam"
    rows = list(csv.DictReader(open(path)))
    name_key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the longest run of kernels without a copy (the timed graph replays; copies happen in setup,
    # eager warm-up steps and the host reads after the timed region)
    cuts = [-1] + [i for i, r in enumerate(rows) if "copyBuffer" in r[name_key]] + [len(rows)]
    a, b = max(zip(cuts[:-1], cuts[1:]), key=lambda ab: ab[1] - ab[0])
    ss = rows[a + 1:b]
    # steps: from the kernel after one marker to the next marker (inclusive)
    idx = [i for i, r in enumerate(ss) if marker in r[name_key]]
    if len(idx) < 3:
        print("too few steps in the steady state", len(idx))
        return
    steps = []
    for a, b in zip(idx[:-1], idx[1:]):
        steps.append(ss[a + 1:b + 1])
    steps = steps[1:]                      # (the first one may start inside a graph)
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    span = 0.0
    ktime = 0.0
    for st in steps:
        t0 = min(int(r["Start_Timestamp"]) for r in st)
        t1 = max(int(r["End_Timestamp"]) for r in st)
        span += (t1 - t0) / 1e3
        for r in st:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            tot[r[name_key]] += d
            cnt[r[name_key]] += 1
            ktime += d
    n = len(steps)
    print(f"steady state: {n} steps without a copyBuffer (marker '{marker}')")
    print(f"{'us/step':>9} {'calls/step':>10}  kernel")
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"{tot[k] / n:9.2f} {cnt[k] / n:10.2f}  {k[:110]}")
    print(f"kernel time per step {ktime / n:.1f} us; first-start to last-end per step {span / n:.1f} us")


if __name__ == "__main__":
    main()
