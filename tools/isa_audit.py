"""ISA audit of libmsfno.so's gfx950 code objects ("Co-residency hazard").

On gfx950 a packed-FP32 VALU op (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32) whose
src1 feeds the LOW lane from its HIGH half -- op_sel:[0,1,...] -- returns wrong low
results in lanes 48..63 while MFMAs of another wave execute on the same CU
(tools/gen_pk_opsel_sweep.py, profiles/r05_pk/pk_sweep.log).  Every other op_sel
combination measured correct.  The library must therefore contain no such instruction;
this module extracts the gfx950 code objects of a fat binary (clang offload bundles,
plain or compressed -- "CCOB", as ROCm's own libraries and torch ship them, unpacked with
clang-offload-bundler), disassembles them with llvm-objdump and lists the offenders.  The
same audit covers what co-runs with the block's MFMA kernels: RCCL's kernels (torch's
bundled librccl.so, /opt/rocm's) and torch's own (libtorch_hip.so).

    python tools/isa_audit.py [lib.so ...]    (default: the in-tree libmsfno.so;
                                               exit 1 if any is found)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
CMAGIC = b"CCOB"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
ANY = re.compile(r"v_pk_(add|mul|fma)_f32\b")
# src1 op_sel bit set with src0's clear: op_sel:[0,1] (add / mul) or op_sel:[0,1,x] (fma)
BAD = re.compile(r"v_pk_(add|mul|fma)_f32\b.*\bop_sel:\[0,1[\],]")


def code_objects(path):
    """(target triple, ELF bytes) of every gfx code object in the bundles of `path`."""
    data = open(path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24: off + 24 + ts].decode()
            off += 24 + ts
            if "amdgcn" in triple and es:
                out.append((triple, data[pos + eo: pos + eo + es]))
        pos = data.find(MAGIC, pos + 1)
    return out


def compressed_gfx950(path, td):
    """Files holding the gfx950 code object of every compressed bundle ("CCOB" header:
    magic, u16 version, u16 method, u32 total size, ...) in `path`."""
    data = open(path, "rb").read()
    out = []
    pos = data.find(CMAGIC)
    while pos >= 0:
        ver, _meth, total = struct.unpack_from("<HHI", data, pos + 4)
        if ver in (2, 3) and 32 < total <= len(data) - pos:
            blob = os.path.join(td, f"b{pos}.ccob")
            with open(blob, "wb") as fh:
                fh.write(data[pos: pos + total])
            targets = subprocess.run([BUNDLER, "--list", "--type=o", f"--input={blob}"],
                                     capture_output=True, text=True).stdout.split()
            if TARGET in targets:
                co = blob[:-5] + ".co"
                subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={blob}",
                                f"--targets={TARGET}", f"--output={co}"], check=True)
                out.append(co)
            os.remove(blob)
            pos = data.find(CMAGIC, pos + total)
        else:
            pos = data.find(CMAGIC, pos + 4)
    return out


def scan(co, bad, counts):
    """Disassemble one code object; offenders into `bad`, packed-op forms into `counts`."""
    p = subprocess.Popen([OBJDUMP, "-d", "--mcpu=gfx950", co], stdout=subprocess.PIPE,
                         text=True)
    sym = "?"
    for line in p.stdout:
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            sym = m.group(1)
        elif ANY.search(line):
            f = re.search(r"op_sel:\[[0-9,]+\]", line)
            counts[f.group(0) if f else "op_sel default"] = counts.get(
                f.group(0) if f else "op_sel default", 0) + 1
            if BAD.search(line):
                bad.append(f"{sym}: {line.split('//')[0].strip()}")
    if p.wait() != 0:
        raise RuntimeError(f"llvm-objdump failed on {co}")


def audit(path, counts=None):
    """Returns (number of gfx950 code objects disassembled, list of offending
    'kernel: instruction' lines); `counts` (a dict) receives the packed-FP32 ops by
    op_sel form."""
    counts = {} if counts is None else counts
    bad = []
    n = 0
    with tempfile.TemporaryDirectory() as td:
        cos = []
        for i, (triple, elf) in enumerate(code_objects(path)):
            if "gfx950" not in triple:
                continue
            f = os.path.join(td, f"co{i}.elf")
            with open(f, "wb") as fh:
                fh.write(elf)
            cos.append(f)
        cos += compressed_gfx950(path, td)
        for co in cos:
            scan(co, bad, counts)
            os.remove(co)
            n += 1
    return n, bad


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    libs = sys.argv[1:] or [os.path.join(
        here, "..", "modulated-spherical-fourier-neural-operator_amd", "msfno_amd", "libmsfno.so")]
    rc = 0
    for lib in libs:
        counts = {}
        n, bad = audit(lib, counts)
        print(f"{lib}: {n} gfx950 code objects, packed-FP32 ops by form {counts}, "
              f"{len(bad)} op_sel:[0,1] instructions")
        for b in bad[:20]:
            print("  ", b)
        rc |= 1 if bad or n == 0 else 0
    return rc


if __name__ == "__main__":
    sys.exit(main())
