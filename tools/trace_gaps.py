#!/usr/bin/env python3
"""Inter-kernel gaps from a rocprofv3 --kernel-trace CSV.

usage: trace_gaps.py <kernel_trace.csv> [last_n_steps]

Prints, over the last N routing steps (a step ends at k_finalize), the time
per step inside kernels, the time between consecutive dispatches (start of
kernel i+1 minus end of kernel i) summed per (kernel i -> kernel i+1) pair,
and the step wall time (k_finalize end to k_finalize end)."""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(swmx?::Params.*", "", name)
    name = name.replace("void swx::", "")
    return name


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    ev.sort()
    fin = [i for i, e in enumerate(ev) if e[2].startswith("k_finalize")]
    if len(fin) < last + 1:
        last = len(fin) - 1
    lo, hi = fin[-last - 1], fin[-1]
    seg = ev[lo:hi + 1]
    busy = defaultdict(float)
    cnt = defaultdict(int)
    gaps = defaultdict(float)
    gcnt = defaultdict(int)
    for a, b in zip(seg, seg[1:]):
        busy[b[2]] += (b[1] - b[0]) / 1e3
        cnt[b[2]] += 1
        g = (b[0] - a[1]) / 1e3
        key = "%s -> %s" % (a[2], b[2])
        gaps[key] += g
        gcnt[key] += 1
    wall = (seg[-1][1] - seg[0][1]) / 1e3
    print("steps %d  wall %.1f us/step" % (last, wall / last))
    print("kernel time per step:")
    for k in sorted(busy, key=lambda k: -busy[k]):
        print("  %-40s %8.2f us/step  %6.2f calls/step  %7.2f us avg" % (
            k, busy[k] / last, cnt[k] / last, busy[k] / cnt[k]))
    print("  %-40s %8.2f" % ("total", sum(busy.values()) / last))
    print("gaps per step (next start - prev end):")
    for k in sorted(gaps, key=lambda k: -gaps[k]):
        print("  %-60s %8.2f us/step  %7.2f us avg  (%d)" % (k, gaps[k] / last, gaps[k] / gcnt[k], gcnt[k]))
    print("  %-60s %8.2f" % ("total", sum(gaps.values()) / last))


if __name__ == "__main__":
    main()


def per_position(path, last=50):
    """Average duration of the i-th kernel of a step (step = finalize to finalize)."""
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    ev = [e for e in ev if not e[2].startswith("__amd")]
    fin = [i for i, e in enumerate(ev) if e[2].startswith("k_finalize")]
    acc = defaultdict(list)
    for a, b in zip(fin[-last - 1:], fin[-last:]):
        for pos, e in enumerate(ev[a + 1:b + 1]):
            acc[(pos, e[2])].append((e[1] - e[0]) / 1e3)
    for (pos, name), v in sorted(acc.items()):
        print("  %2d %-40s n=%4d avg %8.2f min %8.2f max %8.2f" % (pos, name, len(v), sum(v) / len(v), min(v), max(v)))
