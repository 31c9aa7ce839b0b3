#!/usr/bin/env python3
"""Bytes the topic fill moved per launch (rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE passes of
tools/bench_topics.py, tools/gpu_topics_pmc.sh) against the 4 B per delivery it must write, and the
store rate those bytes give at the fill's timed duration (the jsonl line of the same tree).
Usage: topics_pmc_summary.py <outdir> <n>"""
import csv
import json
import os
import re
import sys

import numpy as np


DUR = []


def per_kernel(path, counter):
    v = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = re.sub(r"\(.*", "", name).split("::")[-1].replace("void ", "")
        v.setdefault(name, []).append(float(row["Counter_Value"]) * 1024.0)  # rocprofv3 reports KiB
        if counter == "WRITE_SIZE" and name == "k_sub_fill":  # the launch's own duration (ns)
            DUR.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return {k: float(np.median(x)) for k, x in v.items()}


def main():
    out, n = sys.argv[1], int(sys.argv[2])
    w = per_kernel(os.path.join(out, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    f = per_kernel(os.path.join(out, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    line = json.loads(open(os.path.join(out, "topics_fanout.jsonl")).read().strip().splitlines()[-1])
    need = 4.0 * line["deliveries"]
    wb = w.get("k_sub_fill", 0.0)
    res = {"n_instances": n, "deliveries": line["deliveries"], "alg_write_bytes": need,
           "k_sub_fill_write_bytes": wb, "k_sub_fill_fetch_bytes": 2 * f.get("k_sub_fill", 0.0),
           "write_over_alg": wb / need if need else None, "ms_fill": line["ms_fill"],
           "pmc_write_GBps": wb / (line["ms_fill"] * 1e-3) / 1e9,
           "k_sub_fill_ms_under_pmc": float(np.median(DUR)) / 1e6 if DUR else None,
           "frac_hbm": wb / (line["ms_fill"] * 1e-3) / 8e12,
           "note": "fetch doubled for gfx950 (MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
           "kernels_write": w, "kernels_fetch_raw": f}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
