"""Per-kernel summary of a rocprofv3 --stats kernel_stats.csv: short kernel names, calls, average and total time."""
import csv
import re
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    for x in rows[:int(sys.argv[0] and 30)]:
        m = re.search(r"(k_\w+(<[^>]*>)?|rocprim|__amd_\w+)", x["Name"])
        print("%-44s %5s %10.1f us %9.2f ms" % (m.group(1) if m else x["Name"][:44], x["Calls"],
                                                float(x["AverageNs"]) / 1000, float(x["TotalDurationNs"]) / 1e6))
