"""Per-kernel duration summary (calls, total, average, min, max in ns) from a rocprofv3 rocpd
SQLite database (run_results.db), as CSV rows sorted by total time - the --stats view for runs
whose output format is the database."""
import sqlite3
import sys


def main(path: str) -> None:
    con = sqlite3.connect(path)
    tables = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tables if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tables if t.startswith("rocpd_info_kernel_symbol"))
    rows = con.execute(
        f"select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start),"
        f" min(d.end - d.start), max(d.end - d.start) from {disp} d join {sym} s"
        f" on d.kernel_id = s.id group by s.kernel_name order by sum(d.end - d.start) desc")
    total = None
    print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage")
    out = list(rows)
    total = sum(r[2] for r in out) or 1
    for name, calls, tot, avg, mn, mx in out:
        print(f'"{name}",{calls},{tot},{avg:.1f},{mn},{mx},{100.0 * tot / total:.2f}')


if __name__ == "__main__":
    main(sys.argv[1])
