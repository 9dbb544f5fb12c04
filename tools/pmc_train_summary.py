"""Summarise tools/pmc_train.sh: per backward kernel dispatch, MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES
over clock cycles x 1,024 SIMDs, clock = GRBM_GUI_ACTIVE / 8 XCDs), the executed MFMA rate
(SQ_INSTS_MFMA x 4,096 FLOP of a v_mfma_f32_32x32x2_f32 / kernel time, and its fraction of the
157.3 TF/s FP32 matrix peak), resident waves per SIMD (SQ_WAVE_CYCLES counts quad-cycles:
4 x SQ_WAVE_CYCLES / clock cycles / 1,024), VALU per MFMA and the share of wave time waiting on
an instruction dependency (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)."""
import collections
import csv
import glob
import json
import sys


def main(root="gpurun_out/pmc_train"):
    out = {}
    for opt in ("1", "0"):
        rows = collections.defaultdict(dict)
        for f in glob.glob(f"{root}/o{opt}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                key = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0])
                rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
                rows[key]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (did, name), c in sorted(rows.items()):
            clk = c["GRBM_GUI_ACTIVE"] / 8
            out.setdefault(f"bwd_colsplit={opt}", []).append({
                "kernel": name.replace("void nrt::", ""), "dispatch": did,
                "ms": round(c["ns"] / 1e6, 3),
                "mfma_busy": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * 1024), 3),
                "mfma_tflops": round(c["SQ_INSTS_MFMA"] * 4096 / c["ns"] / 1e3, 1),
                "frac_fp32_peak": round(c["SQ_INSTS_MFMA"] * 4096 / c["ns"] / 1e3 / 157.3, 3),
                "waves_per_simd": round(4 * c["SQ_WAVE_CYCLES"] / (clk * 1024), 2),
                "valu_per_mfma": round(c["SQ_INSTS_VALU"] / max(c["SQ_INSTS_MFMA"], 1), 2),
                "wait_inst_frac": round(c["SQ_WAIT_INST_ANY"] / max(c["SQ_WAVE_CYCLES"], 1), 3),
                "clock_ghz": round(clk / c["ns"], 2)})
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:])
