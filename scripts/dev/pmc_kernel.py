"""Per-launch averages of every PMC counter in rocprofv3 counter_collection.csv files, for the
kernels whose name starts with a prefix. Usage: pmc_kernel.py <prefix> <csv> [<csv> ...]"""
import csv
import json
import sys
from collections import defaultdict

prefix = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if name.startswith(prefix):
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
print(json.dumps(out, indent=1))
