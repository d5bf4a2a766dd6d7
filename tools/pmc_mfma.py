"""Summarise a rocprofv3 SQ/GRBM PMC pass of ``bench.py`` (tools/gpu_mfma.sh) into
``profiles/pmc_mfma.json``, keyed by workload, per kernel (means over launches):

* mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs): the matrix cores' busy share
  (the counter sums MFMA busy cycles over SIMDs, MI355X_MICROARCH.md §Per-instruction constants);
  kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs);
* valu_issue_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the share of a wave's lifetime issuing VALU
  (MFMA included), both in quad-cycles;
* wave-time split: SQ_ACTIVE_INST_ANY (issuing), SQ_WAIT_ANY (parked on s_waitcnt), SQ_WAIT_INST_ANY
  (issue-stalled), each / SQ_WAVE_CYCLES (disjoint, the guide's §PMC slots).
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_SIMD = 256 * 4
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import full_grid_mean  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="standstill")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_mfma.json"))
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                for k in ("physics_kernel", "imitation_kernel"):
                    if k in row["Kernel_Name"]:
                        acc[k][row["Counter_Name"]].append((int(row["Grid_Size"]), float(row["Counter_Value"])))
    res = {}
    for k, d in acc.items():
        m = {c: full_grid_mean(v) for c, v in d.items()}
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        res[k] = {"counters": {c: round(v, 1) for c, v in sorted(m.items())},
                  "kernel_cycles": round(cyc, 1),
                  "mfma_util": round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * N_SIMD), 5) if cyc else None,
                  "valu_issue_frac": round(m.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, 4) if wc else None,
                  "issuing_frac": round(m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4) if wc else None,
                  "waitcnt_frac": round(m.get("SQ_WAIT_ANY", 0.0) / wc, 4) if wc else None,
                  "issue_stall_frac": round(m.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4) if wc else None}
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    key = f"{a.config}:{a.num_envs}"
    phys = res.get("physics_kernel", {})
    out[key] = {"kernels": res, "mfma_util": phys.get("mfma_util"), "valu_issue_frac": phys.get("valu_issue_frac"),
                "method": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY "
                          "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F32 "
                          "GRBM_GUI_ACTIVE --kernel-trace over bench.py (one pass); mfma_util = MFMA busy cycles / "
                          "(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out[key], indent=1))


if __name__ == "__main__":
    main()
