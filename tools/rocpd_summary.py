"""Summarise rocprofv3 rocpd databases (tools/profile_round.sh output) into the
files committed under profiles/<tag>/:

  kernel_stats.csv   per-kernel calls / total / average / min / max (ns) from the
                     --kernel-trace --stats pass
  pmc_traffic.json   per-kernel average HBM bytes per dispatch from the separate
                     FETCH_SIZE and WRITE_SIZE passes, corrected as
                     MI355X_MICROARCH.md §HBM prescribes for gfx950:
                     read bytes = 2 x FETCH_SIZE (FETCH_SIZE tallies 128-B
                     requests at 64 B), write bytes = WRITE_SIZE; both in KiB.

usage: python tools/rocpd_summary.py gpurun_out/p2 profiles/r01_v2
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


def pmc(d, counter):
    c = _db(d)
    rows = c.execute(
        "select kernel_name, count(*), avg(value) from counters_collection where counter_name = ? "
        "group by kernel_name", (counter,)).fetchall()
    return {r[0]: (r[1], r[2]) for r in rows}


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    ks = kernel_stats(os.path.join(src, "kt"))
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(ks[0].keys()))
        w.writeheader()
        w.writerows(ks)
    fetch = pmc(os.path.join(src, "fetch"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "write"), "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) | set(write)):
        fk = fetch.get(name, (0, None))[1]
        wk = write.get(name, (0, None))[1]
        rd = None if fk is None else 2.0 * fk * 1024.0
        wr = None if wk is None else wk * 1024.0
        out[name] = {"dispatches": max(fetch.get(name, (0,))[0], write.get(name, (0,))[0]),
                     "fetch_size_kib": fk, "write_size_kib": wk,
                     "read_bytes": rd, "write_bytes": wr,
                     "hbm_bytes": None if rd is None or wr is None else rd + wr}
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump({"correction": "read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE; per dispatch",
                   "kernels": out}, f, indent=1)
    for r in ks[:12]:
        t = out.get(r["Name"], {})
        hb = t.get("hbm_bytes")
        print(f"{r['AverageNs'] / 1e3:9.1f} us x{r['Calls']:4d}  "
              f"{'' if hb is None else f'{hb / 1e9:7.3f} GB'}  {r['Name'][:110]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
