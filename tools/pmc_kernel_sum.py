"""Per-launch counter values of one kernel from rocprofv3 --pmc CSV output:
    python tools/pmc_kernel_sum.py DIR KERNEL_SUBSTRING
sums each counter over its dimensions (SE / XCC instances) per dispatch and
averages over the kernel's dispatches; prints JSON."""
import csv
import glob
import json
import os
import sys


def per_launch(d, kernel):
    per = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if kernel in r.get("Kernel_Name", ""):
                    c = per.setdefault(r["Counter_Name"], {})
                    k = r.get("Dispatch_Id", "0")
                    c[k] = c.get(k, 0.0) + float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in sorted(per.items())}


if __name__ == "__main__":
    print(json.dumps(per_launch(sys.argv[1], sys.argv[2]), indent=1))
