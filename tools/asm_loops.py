"""Per-loop instruction census of a kernel in a hipcc -S listing: for every loop
header, the MFMA / ds_read / scratch (spill) / s_nop counts between the header and
its back edge.  usage: python tools/asm_loops.py <file.s> <kernel symbol substring>"""
import re
import sys
from collections import Counter


def main(path, sub):
    s = open(path).read()
    starts = [m.start() for m in re.finditer(r"^(_Z\S*):", s, re.M)]
    for st in starts:
        name = s[st:s.index(":", st)]
        if sub not in name:
            continue
        body = s[st:s.index(".Lfunc_end", st)].splitlines()
        print(name)
        for k, line in enumerate(body):
            if not line.startswith(".LBB"):
                continue
            lab = line.split(":")[0]
            # a loop: some later branch jumps back to this label
            back = [j for j, l in enumerate(body) if j > k and "branch" in l and l.strip().endswith(lab)]
            if not back:
                continue
            c = Counter()
            for l in body[k:back[-1] + 1]:
                t = l.strip().split()
                if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
                    c[t[0].split("_e32")[0]] += 1
            scratch = sum(v for kk, v in c.items() if kk.startswith("scratch_"))
            print(f"  loop {lab} lines {k}-{back[-1]}: mfma {c['v_mfma_f32_32x32x16_bf16']} "
                  f"ds_read_b128 {c['ds_read_b128']} scratch {scratch} s_nop {c['s_nop']} "
                  f"accvgpr {c['v_accvgpr_read_b32'] + c['v_accvgpr_write_b32'] + c['v_accvgpr_mov_b32']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
