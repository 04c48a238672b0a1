import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{d}/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void msfno::(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, c in acc.items():
    ds = list(dur[k].values())
    ms = sum(ds) / len(ds)
    print(f"== {k}: {len(ds)} dispatch-passes, avg {ms:.3f} ms (profiled)")
    for n in sorted(c):
        v = sum(c[n]) / len(c[n])
        print(f"   {n:28s} {v:11.4g}")
    if "GRBM_GUI_ACTIVE" in c:
        g = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"])
        clk = g / 8 / (ms * 1e-3) / 1e9
        print(f"   clock_GHz {clk:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            mb = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(c["SQ_VALU_MFMA_BUSY_CYCLES"])
            print(f"   mfma_busy_frac {mb / (1024 * g / 8):.3f}")
        if "SQ_WAVE_CYCLES" in c:
            wc = sum(c["SQ_WAVE_CYCLES"]) / len(c["SQ_WAVE_CYCLES"])
            wi = sum(c["SQ_WAIT_INST_ANY"]) / len(c["SQ_WAIT_INST_ANY"])
            wa = sum(c["SQ_WAIT_ANY"]) / len(c["SQ_WAIT_ANY"])
            print(f"   wait_any/wave {wa / wc:.3f}  wait_inst/wave {wi / wc:.3f}")
