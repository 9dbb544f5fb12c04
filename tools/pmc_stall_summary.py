"""Stall breakdown per kernel of tools/r05_pmc_stall.sh: shares of wave time parked on
s_waitcnt / barriers (SQ_WAIT_ANY), stalled at issue (SQ_WAIT_INST_ANY: MFMA dependency or a busy
pipe; of it the LDS issue stalls SQ_WAIT_INST_LDS) and issuing (SQ_ACTIVE_INST_ANY) -- the
three are disjoint and sum to SQ_WAVE_CYCLES (MI355X_MICROARCH.md PMC table) -- with MFMA busy
and LDS instructions per MFMA.  Usage: python tools/pmc_stall_summary.py DIR [min_dispatch]"""
import collections
import csv
import glob
import sys


def main(root, skip=0):
    rows = collections.defaultdict(dict)
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void nrt::", ""))
            rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[key]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for (did, name), c in rows.items():
        if did < skip:
            continue
        a = agg[name[:64]]
        a["n"] += 1
        a["ms"] += c["ns"] / 1e6
        a["clk"] += c["GRBM_GUI_ACTIVE"] / 8
        for k, v in c.items():
            if k.startswith("SQ_"):
                a[k] += v
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["ms"]):
        wc = max(a["SQ_WAVE_CYCLES"], 1)
        print(f"{name:64s} n {int(a['n']):3d} ms {a['ms'] / a['n']:7.3f} busy "
              f"{a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['clk'] * 1024):.3f} waves/simd "
              f"{4 * wc / (a['clk'] * 1024):.2f} parked {a['SQ_WAIT_ANY'] / wc:.3f} issue-stall "
              f"{a['SQ_WAIT_INST_ANY'] / wc:.3f} (lds {a['SQ_WAIT_INST_LDS'] / wc:.3f}) active "
              f"{a['SQ_ACTIVE_INST_ANY'] / wc:.3f} lds/mfma {a['SQ_INSTS_LDS'] / max(a['SQ_INSTS_MFMA'], 1):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
