"""HBM traffic of one march launch from the FETCH_SIZE / WRITE_SIZE passes of tools/pmc.sh
-> profiles/pmc_<kernel>.json (read by bench.py for roofline.traffic).

Corrections (MI355X_MICROARCH.md, HBM): on gfx950 FETCH_SIZE reports half of the bytes of a
16-B/lane streaming read (x2 here; the ring's buffer_load...lds weight pieces and the ray loads are
that access form); WRITE_SIZE counts bytes for 16-B stores and per-lane atomics; both are in KiB.
Usage: python tools/pmc_traffic.py gpurun_out/pmc/p1 gpurun_out/pmc/p2 [size] [precision] [kernel]
       [scene] [profile-name]
  scene: write profiles/pmc_<scene>_<precision>_<profile-name>.json (bench.py --scene lines; profile-name is
  the kernel's nrt_profile name, default the kernel) instead of profiles/pmc_<kernel>.json.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(run_dir, name, kernel="k_march16"):
    import glob
    path = os.path.join(run_dir, "run_counter_collection.csv")
    if not os.path.exists(path):
        found = glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True)
        path = found[0] if found else path
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name and kernel in r["Kernel_Name"] and "scan_best" not in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"{name} for {kernel} not found in {path}")
    # the first dispatch is the timed frame (--steps 1 --warmup 0); bench.py's later untimed
    # evaluation-counting frame adds one device atomic per wave-evaluation and is not counted
    first = min(vals, key=int)
    return vals[first], len(vals)


def main():
    fetch_dir, write_dir = sys.argv[1], sys.argv[2]
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 800
    precision = sys.argv[4] if len(sys.argv) > 4 else "fp16"
    kernel = sys.argv[5] if len(sys.argv) > 5 else "k_march16"
    scene = sys.argv[6] if len(sys.argv) > 6 else None
    pname = sys.argv[7] if len(sys.argv) > 7 else kernel
    fetch_kib, n1 = counter(fetch_dir, "FETCH_SIZE", kernel)
    write_kib, n2 = counter(write_dir, "WRITE_SIZE", kernel)
    read_b = 2 * fetch_kib * 1024
    write_b = write_kib * 1024
    out = {
        "kernel": kernel, "size": size, "precision": precision,
        "fetch_size_kib": fetch_kib, "write_size_kib": write_kib, "dispatches": [n1, n2],
        "hbm_read_bytes": read_b, "hbm_write_bytes": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "note": "FETCH_SIZE x2 (gfx950 16-B/lane read correction), WRITE_SIZE as reported; "
                "separate rocprofv3 --pmc passes of bench.py --size %d --steps 1 --warmup 0 "
                "--no-extra-legs; the timed frame's launch (first dispatch)" % size,
    }
    if scene:
        out["scene"] = scene
        out["note"] = out["note"].replace("bench.py --size %d" % size, "bench.py --scene %s --size %d" % (scene, size))
        path = os.path.join(ROOT, "profiles", f"pmc_{scene}_{precision}_{pname}.json")
    else:
        path = os.path.join(ROOT, "profiles", f"pmc_{kernel}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
