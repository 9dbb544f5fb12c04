"""Per-dispatch summary of a rocprofv3 --pmc run (SQ counters of tools/r05_train_prof.sh):
MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1,024 SIMDs), clock = GRBM_GUI_ACTIVE /
8 XCDs), resident waves per SIMD (4 x SQ_WAVE_CYCLES / clock cycles / 1,024), VALU per MFMA and
the share of wave time waiting on an instruction dependency.  Usage: python
tools/pmc_dispatch_summary.py DIR [skip_dispatches_below]"""
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
    for (did, name), c in sorted(rows.items()):
        if did < skip:
            continue
        clk = c["GRBM_GUI_ACTIVE"] / 8
        a = agg[name[:60]]
        a["n"] += 1
        a["ms"] += c["ns"] / 1e6
        a["busy_cyc"] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["clk"] += clk
        a["wave_cyc"] += c["SQ_WAVE_CYCLES"]
        a["valu"] += c["SQ_INSTS_VALU"]
        a["mfma"] += c["SQ_INSTS_MFMA"]
        a["wait"] += c["SQ_WAIT_INST_ANY"]
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["ms"]):
        print(f"{name:60s} n {int(a['n']):3d} ms/disp {a['ms'] / a['n']:7.3f} busy "
              f"{a['busy_cyc'] / (a['clk'] * 1024):.3f} waves/simd {4 * a['wave_cyc'] / (a['clk'] * 1024):.2f} "
              f"valu/mfma {a['valu'] / max(a['mfma'], 1):6.2f} wait {a['wait'] / max(a['wave_cyc'], 1):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
