"""HBM bytes per launch of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE,
KB per dispatch summed over instances), gfx950-corrected as MI355X_MICROARCH.md prescribes
(FETCH_SIZE counts 1/2 of a wide coalesced stream's bytes: read bytes = 2 * 1024 * FETCH_SIZE).

Usage: pmc_traffic.py FETCH_CSV WRITE_CSV BENCH_JSON_LOG ROOFLINE_FIELD > json
The kernel name, the shape key (bench.traffic_key) and the algorithmic bytes per launch are read
from the bench line the profiled run printed (its ROOFLINE_FIELD object: roofline,
roofline_scan or roofline_sparse), so the file can only describe the run it was measured on."""
import collections
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def per_dispatch(path: str, kernel: str, counter: str) -> list[float]:
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel + "(" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(acc.values())


def bench_line(log: str) -> dict:
    for line in reversed(Path(log).read_text().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {log}")


def main() -> None:
    fcsv, wcsv, log, field = sys.argv[1:5]
    from bench import traffic_key

    b = bench_line(log)
    roof = b[field]
    cfg = b["config"]
    kernel = roof["kernel"]
    if field == "roofline_sparse":
        key = f"sparse_scan_{cfg['corpus']}_n{cfg['n_chunks']}_q{cfg['batch_per_gpu']}"
    else:
        form = {"dense_scan_i8": 1, "dense_gemm_scan_w4": 2}.get(kernel.split("_kernel")[0], 0)
        key = traffic_key(form, cfg["n_chunks"], cfg["dim"], cfg["batch_per_gpu"], cfg["corpus"])
    f = per_dispatch(fcsv, kernel, "FETCH_SIZE")
    w = per_dispatch(wcsv, kernel, "WRITE_SIZE")
    if not f or not w:
        raise SystemExit(f"kernel {kernel} not found in the counter files")
    fk, wk = sum(f) / len(f), sum(w) / len(w)
    rd, wr = fk * 1024 * 2, wk * 1024
    alg = float(roof["algorithmic_bytes_per_launch"])
    print(json.dumps({
        "key": key, "kernel": kernel, "workload": cfg["workload"],
        "method": ("rocprofv3 --pmc, one pass per counter (FETCH_SIZE; WRITE_SIZE), no tracing "
                   "domains; KB; read bytes = FETCH_SIZE*1024*2 (gfx950 correction)"),
        "launches_sampled": len(f),
        "fetch_size_kb_per_launch": fk, "write_size_kb_per_launch": wk,
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (rd + wr) / alg,
    }, indent=1))


if __name__ == "__main__":
    main()
