"""HBM traffic per launch from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE collected in
separate runs, as MI355X_MICROARCH.md's HBM section prescribes). Writes a JSON summary that
bench.py reports as roofline.traffic for the dominant kernel.
Usage: pmc_traffic.py <fetch_csv> <write_csv> <out_json> [workload=storm] [n_gpus=1] [--last K]
Per kernel: the median bytes per launch, and over the last K windows (a window starts at each
k_window_start* launch, as tools/trace_summary.py counts them) the launches and bytes per window;
`step` sums every kernel over those windows. Kernel names keep their template arguments and lose
only the namespaces and the argument list, so anonymous-namespace kernels keep their own names
(round 4's summaries collapsed them into one "" entry).
The summary is stamped with the kernel-source hash, the workload and the GPU count; bench.py uses it
only for a run of the same code and configuration."""
import csv
import json
import os
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_hash  # noqa: E402

MARKER = "k_window_start"


def kernel_name(raw: str) -> str:
    """'void tgsim::(anonymous namespace)::k_rest<(tgsim::Kind)1>(tgsim::X, int)' -> 'k_rest<(Kind)1>'."""
    s = raw.replace("(anonymous namespace)::", "").replace("tgsim::", "")
    if s.startswith("void "):
        s = s[5:]
    depth = 0
    for i, ch in enumerate(s):  # the argument list is the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return s[:i].strip()
    return s.strip()


def per_kernel(path, counter, last):
    rows = []
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        rows.append((int(row["Dispatch_Id"]), kernel_name(row["Kernel_Name"]),
                     float(row["Counter_Value"]) * 1024.0))  # rocprofv3 reports KiB
    rows.sort()
    per = defaultdict(list)
    for _, k, v in rows:
        per[k].append(v)
    starts = [i for i, r in enumerate(rows) if r[1].startswith(MARKER)]
    win = defaultdict(float)
    nwin = defaultdict(int)
    n = 0
    if starts:
        first = starts[-last] if len(starts) >= last else starts[0]
        n = len([i for i in starts if i >= first])
        for _, k, v in rows[first:]:
            win[k] += v
            nwin[k] += 1
    return ({k: float(np.median(x)) for k, x in per.items()}, {k: len(x) for k, x in per.items()},
            {k: win[k] / n for k in win} if n else {}, {k: nwin[k] / n for k in nwin} if n else {}, n)


def main():
    argv = list(sys.argv[1:])
    last = 5
    if "--last" in argv:
        i = argv.index("--last")
        last = int(argv[i + 1])
        del argv[i:i + 2]
    fmed, fcnt, fwin, fnw, nwin = per_kernel(argv[0], "FETCH_SIZE", last)
    wmed, _, wwin, _, _ = per_kernel(argv[1], "WRITE_SIZE", last)
    kernels = {}
    for k in sorted(set(fmed) | set(wmed)):
        f, w = fmed.get(k, 0.0), wmed.get(k, 0.0)
        kernels[k] = {"fetch_size_raw": f, "fetch_bytes": 2 * f, "write_bytes": w, "traffic_bytes": 2 * f + w,
                      "launches": fcnt.get(k, 0), "launches_per_window": fnw.get(k, 0.0),
                      "traffic_bytes_per_window": 2 * fwin.get(k, 0.0) + wwin.get(k, 0.0)}
    assert "" not in kernels, "a kernel name parsed to ''"
    out = {
        "source_hash": source_hash(),
        "workload": argv[3] if len(argv) > 3 else "storm",
        "n_gpus": int(argv[4]) if len(argv) > 4 else 1,
        "note": "per-launch medians; fetch_bytes = 2 x FETCH_SIZE (gfx950 tallies 128-B read requests at "
                "64 B: MI355X_MICROARCH.md, HBM section); write_bytes = WRITE_SIZE; Infinity-Cache hits are "
                "included in both. *_per_window: sums over the last `windows` windows (each starts at a "
                "k_window_start* launch) / windows",
        "windows": nwin,
        "step": {"traffic_bytes_per_window": sum(v["traffic_bytes_per_window"] for v in kernels.values()),
                 "fetch_bytes_per_window": 2 * sum(fwin.values()) / 1.0,
                 "write_bytes_per_window": sum(wwin.values()),
                 "launches_per_window": sum(fnw.values())},
        "kernels": kernels,
    }
    json.dump(out, open(argv[2], "w"), indent=1)
    for k, v in kernels.items():
        print(f"{k[:40]:40s} fetch {v['fetch_bytes'] / 1e6:8.2f} MB  write {v['write_bytes'] / 1e6:8.2f} MB  "
              f"per window {v['traffic_bytes_per_window'] / 1e6:8.2f} MB ({v['launches_per_window']:.1f} launches)")
    print(f"step: {out['step']['traffic_bytes_per_window'] / 1e6:.1f} MB per window over {nwin} windows")


if __name__ == "__main__":
    main()
