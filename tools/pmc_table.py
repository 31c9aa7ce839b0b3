"""Per-kernel medians of every counter in rocprofv3 --pmc CSVs (one or more passes).
Usage: pmc_table.py <counter_collection.csv> [...]"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np

v = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = re.sub(r"\(.*", "", name).replace("tgsim::", "").replace("void ", "")
        v[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        v[name]["_vgpr"] = [float(row["VGPR_Count"])]
        v[name]["_lds"] = [float(row["LDS_Block_Size"])]
counters = sorted({c for k in v.values() for c in k})
print("kernel".ljust(26) + "".join(c[:18].rjust(19) for c in counters))
for k in sorted(v):
    print(k[:25].ljust(26) + "".join((f"{np.median(v[k][c]):19.4g}" if c in v[k] else " " * 19) for c in counters))
