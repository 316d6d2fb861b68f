"""Step timeline from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): the last N
dispatches with start / end relative to the first of them (us), their duration and the idle gap
before each, so the fixed costs of a step (launch gaps, small kernels) can be read off."""
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"_GLOBAL__N_1\w*?\d+(\w+?)(I|E|v)", name)
    return (m.group(1) if m else name)[:44]


def main(path: str, last: int = 40) -> None:
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ev = ev[-last:]
    t0 = ev[0][0]
    prev_end = None
    print("start_us,end_us,dur_us,gap_us,kernel")
    for st, en, name in ev:
        gap = (st - prev_end) / 1e3 if prev_end is not None else 0.0
        print(f"{(st - t0) / 1e3:.1f},{(en - t0) / 1e3:.1f},{(en - st) / 1e3:.1f},{gap:.1f},{short(name)}")
        prev_end = en if prev_end is None else max(prev_end, en)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
