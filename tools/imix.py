"""Dynamic instruction mix per wave of the engine kernels from one rocprofv3 PMC pass (8 SQ counters,
tools/gpu_imix.sh): per kernel, the counters' mean over the full-grid launches divided by the waves
of a launch (the physics kernel: one wave per env and env-step; the imitation kernel: two envs per
wave). Writes JSON to stdout.

  python tools/imix.py DIR --config standstill
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

COUNTERS = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
            "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="standstill")
    a = ap.parse_args()
    rows = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [(grid, value)]
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") in COUNTERS:
                    rows[r["Kernel_Name"]][r["Counter_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    out = {"method": "rocprofv3 --pmc " + " ".join(COUNTERS) + " --kernel-trace over bench.py --steps 10, full-grid "
                     "launches; per wave", "config": a.config, "kernels": {}}
    for k, cs in rows.items():
        short = "physics_kernel_tgs" if "physics_kernel_tgs" in k else ("imitation_kernel" if "imitation_kernel" in k else None)
        if short is None:
            continue
        if short in out["kernels"] and out["kernels"][short]["launches"] >= len(cs["SQ_WAVES"]):
            continue  # two instantiations (imitation_kernel<true> is only warmed up): keep the launched one
        g = max(x[0] for x in cs["SQ_WAVES"])
        mean = {c: sum(v for gs, v in cs[c] if gs == g) / max(1, sum(1 for gs, _ in cs[c] if gs == g)) for c in cs}
        waves = mean["SQ_WAVES"]
        out["kernels"][short] = {"launches": sum(1 for gs, _ in cs["SQ_WAVES"] if gs == g), "waves": round(waves),
                                 "per_wave": {c: round(mean[c] / waves) for c in COUNTERS if c != "SQ_WAVES"}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
