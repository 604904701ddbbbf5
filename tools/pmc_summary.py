"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (avg per dispatch).

    python tools/pmc_summary.py [pmc_dir] [--json profiles/pmc_<workload>.json --kernels a,b]

With --json, writes the HBM traffic of one plan execute (the sum over the
listed kernels of one dispatch each) in bytes, with the gfx950 corrections of
MI355X_MICROARCH.md's HBM section applied:
  * FETCH_SIZE (KB) counts half the bytes of wide coalesced reads -> x2;
  * WRITE_SIZE (KB) is exact for 16-B/lane stores; narrower stores are
    reported as counted (uncalibrated, stated in the JSON).
bench.py reads `hbm_bytes_per_launch` from that file into roofline.traffic.
"""
import argparse
import collections
import csv
import glob
import json

ap = argparse.ArgumentParser()
ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
ap.add_argument("--json")
ap.add_argument("--kernels", default="")
ap.add_argument("--source", default="", help="provenance tag stored in the JSON")
args = ap.parse_args()

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{args.root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
for k, cs in avg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} avg/dispatch = {v:.4g}  (n={len(acc[k][c])})")

if args.json:
    want = [w for w in args.kernels.split(",") if w]
    per = {}
    total = 0.0
    for k, cs in avg.items():
        if want and not any(k.startswith(w) for w in want):
            continue
        fetch = 2.0 * cs.get("FETCH_SIZE", 0.0) * 1024
        write = cs.get("WRITE_SIZE", 0.0) * 1024
        hit, miss = cs.get("TCC_HIT_sum", 0.0), cs.get("TCC_MISS_sum", 0.0)
        per[k] = {"fetch_bytes_x2": fetch, "write_bytes": write,
                  "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
                  "counters_per_dispatch": cs}
        busy = cs.get("SQ_BUSY_CYCLES")
        if busy:  # issue-side shares (per SQ, summed over SEs): what bounds the kernel
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
                      "SQ_WAIT_ANY"):
                if c in cs and cs.get("SQ_WAVE_CYCLES"):
                    per[k][c.lower() + "_per_wave_cycle"] = cs[c] / cs["SQ_WAVE_CYCLES"]
        total += fetch + write
    out = {"hbm_bytes_per_launch": total, "per_kernel": per, "source": args.source,
           "note": "FETCH_SIZE doubled (gfx950 wide-read correction); WRITE_SIZE as counted; "
                   "SQ_* per dispatch, *_per_wave_cycle = counter / SQ_WAVE_CYCLES"}
    with open(args.json, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))
