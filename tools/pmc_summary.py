"""Per-kernel averages of rocprofv3 --pmc counter CSVs (sum over a dispatch's instances, averaged
over dispatches). Usage: pmc_summary.py CSV [CSV ...] (kernels whose name contains 'sparse' or
'pass_terms', or $PMC_MATCH when set)."""
import collections
import csv
import os
import sys


def main() -> None:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")
            k = r["Kernel_Name"].split("::")[-1].split("(")[0] if "::" in r["Kernel_Name"] else k
            match = os.environ.get("PMC_MATCH")
            if (match not in k) if match else ("sparse" not in k and "pass_terms" not in k):
                continue
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            seen[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    for k, cs in per.items():
        print(k)
        for c, v in sorted(cs.items()):
            n = max(len(seen[(k, c)]), 1)
            print(f"  {c:28s} {v / n:16.1f}")


if __name__ == "__main__":
    main()
