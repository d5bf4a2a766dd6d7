"""Host-side checks of the measurement tools whose output the bench line reads
(profiles/pmc_traffic.json, profiles/pmc_mfma.json): rocprofv3 counter rows are averaged over the
kernel's full-grid launches only (the one-block warm-up dispatches of he_create_envs excluded), and
two instantiations of one kernel (imitation_kernel<false> / <true>) do not overwrite each other."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size",
          "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
          "Accum_VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
PHYS = "(anonymous namespace)::physics_kernel(PhysArgs)"
IMIT_F = "void (anonymous namespace)::imitation_kernel<false>(ImitArgs)"
IMIT_T = "void (anonymous namespace)::imitation_kernel<true>(ImitArgs)"


def _write(d, counter, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for i, (name, grid, value) in enumerate(rows):
            w.writerow({k: 0 for k in FIELDS} | {"Dispatch_Id": i, "Kernel_Name": name, "Grid_Size": grid,
                                                "Counter_Name": counter, "Counter_Value": value})


def test_pmc_traffic_full_grid_and_instantiations(tmp_path):
    # warm-up dispatches (grid 64 / 256) with near-zero counts, then the workload's launches; the
    # <true> instantiation appears only as a warm-up dispatch
    fetch = [(PHYS, 64, 3.0), (IMIT_F, 256, 2.0), (IMIT_T, 256, 2.5)] + \
            [(PHYS, 262144, 4400.0)] * 3 + [(IMIT_F, 131072, 5400.0)] * 3
    write = [(PHYS, 64, 0.0), (IMIT_F, 256, 0.0), (IMIT_T, 256, 0.0)] + \
            [(PHYS, 262144, 13120.0)] * 3 + [(IMIT_F, 131072, 15000.0)] * 3
    _write(tmp_path / "f", "FETCH_SIZE", fetch)
    _write(tmp_path / "w", "WRITE_SIZE", write)
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), "--config", "standstill", "--num-envs", "4096", "--out", str(out)],
                   check=True, capture_output=True)
    r = json.load(open(out))["standstill:4096"]
    assert r["physics_bytes_per_launch"] == round((2 * 4400.0 + 13120.0) * 1024)
    assert r["imitation_bytes_per_launch"] == round((2 * 5400.0 + 15000.0) * 1024)
    assert r["kernels"]["imitation_kernel"]["launches"] == 4  # <false>: 3 workload + 1 warm-up rows


def test_pmc_mfma_full_grid(tmp_path):
    rows = []
    for counter, warm, full in (("GRBM_GUI_ACTIVE", 8.0, 8.0e6), ("SQ_VALU_MFMA_BUSY_CYCLES", 0.0, 4.1e7),
                                ("SQ_WAVE_CYCLES", 10.0, 1.0e8), ("SQ_ACTIVE_INST_VALU", 1.0, 3.4e7)):
        rows += [(PHYS, 64, warm, counter)] + [(PHYS, 262144, full, counter)] * 2
    d = tmp_path / "m"
    os.makedirs(d)
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for i, (name, grid, value, counter) in enumerate(rows):
            w.writerow({k: 0 for k in FIELDS} | {"Dispatch_Id": i, "Kernel_Name": name, "Grid_Size": grid,
                                                "Counter_Name": counter, "Counter_Value": value})
    out = tmp_path / "m.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_mfma.py"), str(d), "--out", str(out)],
                   check=True, capture_output=True)
    r = json.load(open(out))["standstill:4096"]
    assert abs(r["mfma_util"] - 4.1e7 / (1.0e6 * 1024)) < 1e-5
    assert abs(r["valu_issue_frac"] - 0.34) < 1e-4


def test_order_class_thresholds_equal_the_class_rule():
    """The dispatch order's class (he_physics.hip order_class): the kernel finds it by a binary search
    over 31 integer thresholds T[m] = ceil((m + 16) tot / (32 n)); the GPU test restates the rule as
    floor(32 c n / tot) - 16 clamped to [0, 31] (tests/test_full_size.py order_classes). Both must
    agree on every cost, the class edges included."""
    import numpy as np
    rng = np.random.default_rng(5)
    for trial in range(60):
        n = int(rng.integers(1, 3000))
        if trial % 3 == 0:
            c = rng.integers(1, 2**31, n)
        else:
            c = rng.integers(300_000, 900_000, n)
        tot = int(c.sum())
        d = 32 * n
        thr = [0] + [min(((m + 16) * tot + d - 1) // d, 2**32 - 1) for m in range(1, 32)]
        edges = [t for t in thr[1:] if t < 2**32 - 1]
        for x in list(c[:200]) + edges + [t - 1 for t in edges]:  # the class edges and just below them
            x = int(x)
            lo = 0
            for step in (16, 8, 4, 2, 1):
                if lo + step < 32 and x >= thr[lo + step]:
                    lo += step
            rule = min(max(32 * x * n // tot - 16, 0), 31)
            assert lo == rule, (n, x, lo, rule)


def test_committed_parity_records_belong_to_the_built_library():
    """bench.py reports the newest committed parity records (profiles/r*/<name>.json) with a
    device-code status; a kernel change without re-measured records would ship them as "stale".
    The library built from this tree must carry the device code the records were measured with."""
    import glob
    sys.path.insert(0, ROOT)
    from humanoid_amd import build as B
    if not os.path.exists(B.LIB):
        B.build()
    here = B.device_code_id(B.LIB)
    for name in ("parity_configs1", "parity_configs2", "dr_events"):
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name + ".json")))
        assert files, name
        rec = json.load(open(files[-1]))
        assert rec.get("device_code") == here, (files[-1], rec.get("device_code"), here)
