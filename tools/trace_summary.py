#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel count/avg/total, and GPU busy vs wall time over
the last K windows (a window starts at each k_gen_storm launch).

    python tools/trace_summary.py gpurun_out/prof/run_kernel_trace.csv [--last K]
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=30)
    ap.add_argument("--marker", default="k_window_start")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(starts) > a.last:
        rows = rows[starts[-a.last - 1]:starts[-1]]
    win = len([r for r in rows if a.marker in r[2]])
    per = collections.defaultdict(list)
    for s, e, n in rows:
        per[n].append(e - s)
    wall = rows[-1][1] - rows[0][0]
    busy = 0
    last_end = 0
    for s, e, _ in rows:
        s = max(s, last_end)
        if e > s:
            busy += e - s
        last_end = max(last_end, e)
    print(f"windows={win} wall/window={wall / win / 1e3:.1f} us  busy/window={busy / win / 1e3:.1f} us  "
          f"launches/window={len(rows) / win:.1f}")
    print(f"{'kernel':60s} {'n/win':>6s} {'avg_us':>8s} {'us/win':>8s}")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n[:60]:60s} {len(d) / win:6.1f} {sum(d) / len(d) / 1e3:8.2f} {sum(d) / win / 1e3:8.2f}")


if __name__ == "__main__":
    main()
