"""Per-dispatch averages of the PMC counters a rocprofv3 --pmc pass recorded for one kernel."""
import collections
import csv
import sys


def summary(paths, kernel):
    out = {}
    for path in paths:
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for k, v in agg.items():
            out[k] = v / max(1, len(disp[k]))
    return out


if __name__ == "__main__":
    kern = sys.argv[1]
    for k, v in sorted(summary(sys.argv[2:], kern).items()):
        print(f"{k:28s} {v:16.0f}")
