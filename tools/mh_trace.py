"""Summarise MSFNO_MH_TRACE files (csrc/mlp_fused_h.hip, diagnostic build path): per
workgroup the CU it ran on (HW_ID / XCC_ID) and the 100-MHz real-time clock at entry, after
the prologue's x1 loads, after the last MFMA step and once its stores are issued.

Prints the phase durations, how the first dispatch wave pairs blocks on CUs, and how the
two workgroups a CU holds overlap: the fraction of CU-time in which both are in a
load / store phase, one is, or both compute.
usage: python tools/mh_trace.py <trace file> [launch index, default last]"""
import struct
import sys
from collections import defaultdict

import numpy as np


def launches(path):
    data = open(path, "rb").read()
    off, out = 0, []
    while off < len(data):
        (n,) = struct.unpack_from("<Q", data, off)
        off += 8
        a = np.frombuffer(data, dtype=np.uint64, count=5 * n, offset=off).reshape(n, 5)
        off += 40 * n
        out.append(a.copy())
    return out


def main(path, which=-1):
    L = launches(path)
    a = L[which]
    n = len(a)
    hw = (a[:, 0] & 0xFFFFFFFF).astype(np.int64)
    xcc = (a[:, 0] >> 32).astype(np.int64)
    cu = xcc * 256 + ((hw >> 8) & 0xFF)           # XCC, SE / SH / CU bits of HW_ID
    t = a[:, 1:].astype(np.int64)
    t0 = t[:, 0].min()
    t = (t - t0) * 10  # ns
    pro, comp, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    print(f"{len(L)} launches in file; launch {which}: {n} workgroups on {len(set(cu))} CUs, "
          f"span {t[:, 3].max() / 1e3:.1f} us")
    for name, v in (("prologue (x1 loads)", pro), ("MFMA steps", comp), ("epilogue (stores)", epi)):
        print(f"  {name:22s} mean {v.mean() / 1e3:7.2f} us  p10 {np.percentile(v, 10) / 1e3:7.2f}"
              f"  p90 {np.percentile(v, 90) / 1e3:7.2f}")
    first = defaultdict(list)
    for b in range(min(n, 512)):
        first[cu[b]].append(b)
    pairs = [v for v in first.values() if len(v) == 2]
    d = [abs(v[1] - v[0]) for v in pairs]
    print(f"  first 512 blocks: {len(first)} CUs, {len(pairs)} with two; block-index gap of a "
          f"pair: min {min(d) if d else 0}, median {int(np.median(d)) if d else 0}, max {max(d) if d else 0}")
    # per CU: sweep the phase changes; CU-time by the resident workgroups' phase mix
    acc = defaultdict(int)
    for c in set(cu):
        ev = []
        for i in np.where(cu == c)[0]:
            ev += [(t[i, 0], i, "m"), (t[i, 1], i, "c"), (t[i, 2], i, "m"), (t[i, 3], i, None)]
        ev.sort(key=lambda e: e[0])
        state, last = {}, ev[0][0]
        for time, i, ph in ev:
            ph_list = sorted(state.values())
            acc["".join(ph_list) or "idle"] += time - last
            last = time
            if ph is None:
                state.pop(i, None)
            else:
                state[i] = ph
    tot = sum(acc.values())
    names = {"mm": "both load/store", "cm": "one loads/stores, one computes", "cc": "both compute",
             "m": "alone, load/store", "c": "alone, compute", "idle": "idle"}
    print("  CU-time by resident workgroups' phases: " + ", ".join(
        f"{names.get(k, k)} {v / tot:.2f}" for k, v in sorted(acc.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -1)
