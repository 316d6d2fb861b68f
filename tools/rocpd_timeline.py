"""Kernel timeline of the last N dispatches in a rocprofv3 rocpd database (run_results.db): one
row per dispatch with start / end relative to the first of them (us), duration, queue (stream)
and a short kernel name - to see which kernels of a step overlap."""
import re
import sqlite3
import sys


def short(name: str) -> str:
    m = re.search(r"_GLOBAL__N_1\d+(\w+?)(I|E)", name)
    if m:
        return m.group(1)
    return name[:40]


def main(path: str, last: int = 60) -> None:
    con = sqlite3.connect(path)
    tables = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tables if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tables if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in con.execute(f"pragma table_info({disp})")]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else "0")
    rows = list(con.execute(
        f"select d.start, d.end, d.{qcol}, s.kernel_name from {disp} d join {sym} s"
        f" on d.kernel_id = s.id order by d.start"))
    rows = rows[-last:]
    t0 = rows[0][0]
    print("start_us,end_us,dur_us,queue,kernel")
    for st, en, q, name in rows:
        print(f"{(st - t0) / 1e3:.1f},{(en - t0) / 1e3:.1f},{(en - st) / 1e3:.1f},{q},{short(name)}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
