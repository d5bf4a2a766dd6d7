"""Summarise two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, as the MI355X guide
prescribes) of ``bench.py`` into ``profiles/pmc_traffic.json``.

Per kernel: mean HBM bytes per launch = 2 x FETCH_SIZE (gfx950 tallies 128-B read requests at
64 B) + WRITE_SIZE, both reported by rocprofv3 in KB. The bench's ``roofline.traffic`` is the
physics kernel's entry for the same workload.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --config standstill --num-envs 4096
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise FileNotFoundError(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                acc[row["Kernel_Name"]].append((int(row["Grid_Size"]), float(row["Counter_Value"])))
    return {k: (full_grid_mean(v), len(v)) for k, v in acc.items()}


def full_grid_mean(rows):
    """Mean over the launches at the kernel's largest grid: the one-block warm-up dispatches of
    he_create_envs (he_engine.cpp warm_kernels) are not workload launches."""
    g = max(r[0] for r in rows)
    v = [x for gs, x in rows if gs == g]
    return sum(v) / len(v)


def short(name):
    for k in ("physics_kernel", "imitation_kernel", "motion_state_kernel", "copy_rows_kernel"):
        if k in name:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", default="standstill")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_dir, "FETCH_SIZE")
    write = per_kernel(a.write_dir, "WRITE_SIZE")
    kernels, launches = {}, {}
    for name in set(fetch) | set(write):
        k = short(name)
        n = max(fetch.get(name, (0.0, 0))[1], write.get(name, (0.0, 0))[1])
        # instantiations sharing a short name (imitation_kernel<false> / <true>): the one the workload
        # launches most
        if k is None or n <= launches.get(k, 0):
            continue
        launches[k] = n
        fb = 2.0 * fetch.get(name, (0.0, 0))[0] * 1024.0  # KB -> B, x2 gfx950 read correction
        wb = write.get(name, (0.0, 0))[0] * 1024.0
        kernels[k] = {"fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                      "hbm_bytes_per_launch": round(fb + wb),
                      "hbm_bytes_per_env": round((fb + wb) / a.num_envs, 1), "launches": n}
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    key = f"{a.config}:{a.num_envs}"
    out[key] = {"kernels": kernels,
                "physics_bytes_per_launch": kernels.get("physics_kernel", {}).get("hbm_bytes_per_launch"),
                "imitation_bytes_per_launch": kernels.get("imitation_kernel", {}).get("hbm_bytes_per_launch"),
                "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate --kernel-trace runs of "
                          "bench.py; FETCH_SIZE doubled (gfx950 128-B requests tallied at 64 B)"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out[key], indent=1))


if __name__ == "__main__":
    main()
