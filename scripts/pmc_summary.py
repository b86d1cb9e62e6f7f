#!/usr/bin/env python3
"""Per-kernel table of a rocprofv3 ``--pmc`` run (``scripts/gpu_steps.sh pmc_*``).

    python scripts/pmc_summary.py gpurun_out/prof_pmc_cml [--trace gpurun_out/prof_stats] [--top 20]

Reads ``*counter_collection.csv`` under the directory (one row per dispatch x counter) and prints,
per kernel, the mean value of every counter per dispatch. Durations come from the same CSV's
start / end timestamps when present, else from a kernel-trace run's ``*kernel_trace.csv``
(``--trace``; mean over that run's dispatches of the kernel). With FETCH_SIZE / WRITE_SIZE (KB)
it adds the HBM-side bytes and GB/s; with SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_WAIT_ANY /
SQ_VALU_MFMA_BUSY_CYCLES it adds the wait share and MFMA-busy share.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os


def _find(d, pat):
    out = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    return out


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    return None


def load_counters(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in _find(d, "*counter_collection.csv"):
        seen = set()
        for r in csv.DictReader(open(p)):
            k = _col(r, "Kernel_Name", "Kernel-Name", "KernelName")
            c = _col(r, "Counter_Name", "Counter-Name")
            v = _col(r, "Counter_Value", "Counter-Value")
            if k is None or c is None or v is None:
                continue
            did = _col(r, "Dispatch_Id", "Dispatch-Id", "Correlation_Id")
            per[k][c].append(float(v))
            s, e = _col(r, "Start_Timestamp"), _col(r, "End_Timestamp")
            if s is not None and e is not None and (k, did) not in seen:
                seen.add((k, did))
                dur[k].append((float(e) - float(s)) / 1e3)
    return per, dur


def load_trace(d):
    dur = collections.defaultdict(list)
    for p in _find(d, "*kernel_trace.csv"):
        for r in csv.DictReader(open(p)):
            k = _col(r, "Kernel_Name")
            s, e = _col(r, "Start_Timestamp"), _col(r, "End_Timestamp")
            if k is not None and s is not None and e is not None:
                dur[k].append((float(e) - float(s)) / 1e3)
    return dur


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="+", help="one or more runs (e.g. a FETCH_SIZE pass and a WRITE_SIZE pass)")
    ap.add_argument("--trace", default=None, help="kernel-trace run for durations")
    ap.add_argument("--top", type=int, default=20)
    args = ap.parse_args(argv)
    per, dur = collections.defaultdict(lambda: collections.defaultdict(list)), collections.defaultdict(list)
    for d in args.dir:
        p1, d1 = load_counters(d)
        for k, v in p1.items():
            for c, vals in v.items():
                per[k][c].extend(vals)
        for k, v in d1.items():
            dur[k].extend(v)
    if args.trace:
        tdur = load_trace(args.trace)
        for k, v in tdur.items():
            if not dur.get(k):
                dur[k] = v
    mean = lambda v: sum(v) / len(v) if v else float("nan")      # noqa: E731
    counters = sorted({c for k in per for c in per[k]})
    rank = sorted(per, key=lambda k: -(mean(dur.get(k, [])) * len(dur.get(k, [])) if dur.get(k) else 0.0))
    hdr = f"{'us/call':>9} {'calls':>6} " + " ".join(f"{c.replace('SQ_', '')[:12]:>12}" for c in counters)
    extra = []
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        extra.append("GB/s")
    if "SQ_WAVE_CYCLES" in counters and "SQ_WAIT_ANY" in counters:
        extra.append("wait%")
    if "SQ_BUSY_CYCLES" in counters and "SQ_VALU_MFMA_BUSY_CYCLES" in counters:
        extra.append("mfma%")
    print(hdr + "".join(f" {e:>7}" for e in extra) + "  kernel")
    for k in rank[:args.top]:
        d = mean(dur.get(k, []))
        vals = {c: mean(per[k].get(c, [])) for c in counters}
        line = f"{d:9.2f} {len(per[k][counters[0]]) if counters else 0:6d} " + " ".join(
            f"{vals[c]:12.4g}" for c in counters)
        if "GB/s" in extra:
            line += f" {(vals['FETCH_SIZE'] + vals['WRITE_SIZE']) * 1024 / (d * 1e3) if d == d and d > 0 else 0:7.0f}"
        if "wait%" in extra:
            line += f" {100 * vals['SQ_WAIT_ANY'] / max(vals['SQ_WAVE_CYCLES'], 1):7.1f}"
        if "mfma%" in extra:
            # SQ_BUSY_CYCLES counts quad-cycles per SE; MFMA busy counts cycles per SIMD, summed:
            # reported as the raw ratio (compare kernels, not absolute utilisation)
            line += f" {100 * vals['SQ_VALU_MFMA_BUSY_CYCLES'] / max(vals['SQ_BUSY_CYCLES'], 1):7.1f}"
        print(line + "  " + k[:90])


if __name__ == "__main__":
    main()
