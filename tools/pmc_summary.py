"""Per-kernel medians of rocprofv3 --pmc counter collections (one or more run_counter_collection.csv),
with the per-dispatch duration. Usage: pmc_summary.py <csv> [<csv> ...]"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np

vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("tgsim::", "")
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        dur[name].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0)
for k in sorted(vals):
    print(f"{k}: dur_us {np.median(dur[k]):.2f}")
    for c in sorted(vals[k]):
        print(f"    {c:28s} {np.median(vals[k][c]):14.4g}")
