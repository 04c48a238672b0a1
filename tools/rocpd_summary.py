"""Summarise rocprofv3 rocpd databases (tools/profile_round.sh output) into the
files committed under profiles/<tag>/:

  kernel_stats.csv         per-kernel calls / total / average / min / max (ns) of the
                           block line's --kernel-trace --stats pass (<src>/kt)
  kernel_stats_<w>.csv     the same for the other workloads' passes (<src>/kt_<w>)
  pmc_traffic.json         per-kernel average HBM bytes per dispatch from the separate
                           FETCH_SIZE and WRITE_SIZE passes (<src>/fetch*, <src>/write*),
                           corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
                           read bytes = 2 x FETCH_SIZE (FETCH_SIZE tallies 128-B
                           requests at 64 B), write bytes = WRITE_SIZE; both in KiB.
                           Dispatches are grouped by (kernel, grid size) and each kernel
                           keeps its largest-grid group: the config-2 / config-3
                           full-resolution launch, not the 120x240 inner blocks that
                           share its symbol.

usage: python tools/rocpd_summary.py gpurun_out/<tag> profiles/<tag>
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sqlite3
import sys


def _db(d):
    f = glob.glob(os.path.join(d, "*.db"))
    if not f:
        raise SystemExit(f"no rocpd database under {d}")
    return sqlite3.connect(f[0])


def kernel_stats(d):
    c = _db(d)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [{"Name": r[0], "Calls": r[1], "TotalDurationNs": r[2], "AverageNs": round(r[3], 1),
             "Percentage": round(100.0 * r[2] / tot, 2), "MinNs": r[4], "MaxNs": r[5]} for r in rows]


def pmc(dirs, counter):
    """kernel -> (dispatches, average value, grid size) of its largest-grid dispatches."""
    best = {}
    for d in dirs:
        c = _db(d)
        rows = c.execute(
            "select kernel_name, grid_size, count(*), avg(value) from counters_collection "
            "where counter_name = ? group by kernel_name, grid_size", (counter,)).fetchall()
        for name, grid, n, v in rows:
            if name not in best or grid > best[name][2]:
                best[name] = (n, v, grid)
    return best


def write_stats(path, ks):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(ks[0].keys()))
        w.writeheader()
        w.writerows(ks)


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    ks = kernel_stats(os.path.join(src, "kt"))
    write_stats(os.path.join(dst, "kernel_stats.csv"), ks)
    for d in sorted(glob.glob(os.path.join(src, "kt_*"))):
        if os.path.isdir(d) and glob.glob(os.path.join(d, "*.db")):
            write_stats(os.path.join(dst, "kernel_stats_" + os.path.basename(d)[3:] + ".csv"),
                        kernel_stats(d))
    fetch = pmc(sorted(p for p in glob.glob(os.path.join(src, "fetch*")) if os.path.isdir(p)),
                "FETCH_SIZE")
    write = pmc(sorted(p for p in glob.glob(os.path.join(src, "write*")) if os.path.isdir(p)),
                "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) | set(write)):
        f, w = fetch.get(name), write.get(name)
        fk = f[1] if f else None
        wk = w[1] if w else None
        rd = None if fk is None else 2.0 * fk * 1024.0
        wr = None if wk is None else wk * 1024.0
        out[name] = {"dispatches": max(f[0] if f else 0, w[0] if w else 0),
                     "grid_size": (f or w)[2],
                     "fetch_size_kib": fk, "write_size_kib": wk,
                     "read_bytes": rd, "write_bytes": wr,
                     "hbm_bytes": None if rd is None or wr is None else rd + wr}
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump({"correction": "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; per "
                                 "dispatch of each kernel's largest grid",
                   "kernels": out}, f, indent=1)
    for r in ks[:14]:
        t = out.get(r["Name"], {})
        hb = t.get("hbm_bytes")
        print(f"{r['AverageNs'] / 1e3:9.1f} us x{r['Calls']:4d}  "
              f"{'' if hb is None else f'{hb / 1e9:7.3f} GB'}  {r['Name'][:110]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
