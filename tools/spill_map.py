"""Per-phase register spills of the physics kernel under a waves-per-SIMD bound (diagnostic for the
occupancy plan): the stamp build of he_physics.hip compiled with -DHE_MIN_WAVES=W (the
launch bound: 256 / W VGPRs), disassembled and split at its s_memtime stamps as in
tools/isa_phase_counts.py; per phase the scratch stores and loads the allocator inserted, and the
kernel's resource report.

  python tools/spill_map.py [W] [KERNEL]      (default 4, physics_kernel; physics_kernel_tgs: the TGS one)
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from humanoid_amd import build as B  # noqa: E402
from phase_profile import PHASES  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    kname = sys.argv[2] if len(sys.argv) > 2 else "physics_kernel"
    src = os.path.join(B.CSRC, "he_physics.hip")
    flags = dict(B.SOURCES)["he_physics.hip"]
    with tempfile.TemporaryDirectory() as td:
        co = os.path.join(td, "k.co")
        r = subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, "-O3", "-fPIC", "-std=c++17", "--cuda-device-only",
                            "--no-gpu-bundle-output", "-c", src, "-o", co, f"-DHE_MIN_WAVES={w}",
                            "-Rpass-analysis=kernel-resource-usage"] + flags + B.PHASES_DEFS["he_physics.hip"],
                           check=True, capture_output=True, text=True)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                             capture_output=True, text=True).stdout
    report = {}
    lines = r.stderr.splitlines()
    for i, ln in enumerate(lines):
        if "Function Name:" in ln and re.search(r"\d" + kname + r"E", ln):
            for ln2 in lines[i + 1:i + 14]:
                if "Function Name:" in ln2:
                    break
                m = re.search(r"remark:\s+([^:]+):\s+(\S+)", ln2)
                if m:
                    report[m.group(1).strip()] = m.group(2)
    L = dis.split("\n")
    # the kernel's own disassembly: from its label to the next function label
    start = next(i for i, ln in enumerate(L) if re.search(r"\d" + kname + r"E\w*>:", ln))
    end = next((i for i in range(start + 1, len(L)) if re.match(r"^[0-9a-f]+ <", L[i])), len(L))
    L = L[start:end]
    cuts = [i for i, ln in enumerate(L) if "s_memtime" in ln]
    phases = {}
    for a, b in zip(cuts, cuts[1:]):
        slot = None
        for ln in L[b:b + 80]:
            if "global_atomic_add" in ln:
                m = re.search(r"offset:(\d+)", ln)
                slot = int(m.group(1)) // 8 if m else 0
                break
        name = PHASES[slot] if slot is not None and slot < len(PHASES) else f"slot {slot}"
        seg = L[a:b]
        c = phases.setdefault(name, {"scratch_stores": 0, "scratch_loads": 0, "instructions": 0})
        c["scratch_stores"] += sum("scratch_store" in ln for ln in seg)
        c["scratch_loads"] += sum("scratch_load" in ln for ln in seg)
        c["instructions"] += sum(1 for ln in seg if re.match(r"\s+[a-z_0-9]+\s", ln))
    print(json.dumps({"waves_per_simd_bound": w, "resources": report, "phases": phases}, indent=1))


if __name__ == "__main__":
    main()
