"""Trim rocprofv3 per-dispatch CSVs in place to the engine's own kernels (physics, imitation,
motion_state, copy_rows), so the raw counters travel back from a gpurun session (<= 64 MiB) and
tools/pmc_traffic.py / pmc_mfma.py can be re-run on them here.

  python tools/trim_csv.py gpurun_out
"""
import csv
import glob
import os
import sys

KEEP = ("physics_kernel", "imitation_kernel", "motion_state_kernel", "copy_rows_kernel")


def main(root):
    for pat in ("*counter_collection.csv", "*kernel_trace.csv"):
        for f in glob.glob(os.path.join(root, "**", pat), recursive=True):
            with open(f, newline="") as fh:
                rd = csv.reader(fh)
                head = next(rd, None)
                if head is None or "Kernel_Name" not in head:
                    continue
                i = head.index("Kernel_Name")
                rows = [r for r in rd if any(k in r[i] for k in KEEP)]
            with open(f, "w", newline="") as fh:
                w = csv.writer(fh, quoting=csv.QUOTE_MINIMAL)
                w.writerow(head)
                w.writerows(rows)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
