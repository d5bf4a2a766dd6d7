"""Static instruction counts of the physics kernel per phase (diagnostic, DESIGN §4.1 "Where the wave's
time goes"): the stamp build of he_physics.hip (-DHE_PHASE_STAMPS=1, the product flags of
humanoid_amd/build.py) is disassembled, split at its s_memtime stamps, and each segment is named by
the stamp slot its global_atomic_add_x2 writes (offset / 8 = the phase id of tools/phase_profile.py).
Segments the compiler placed out of line (duplicated blocks) keep their slot's name; the counts are
static (the PGS sweep and the substep loop run several times), so set them against the phase cycles
of the same build (tools/phase_profile.py) only where a phase is straight-line code.

  python tools/isa_phase_counts.py > profiles/r04/isa_phase_counts.json
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from humanoid_amd import build as B  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from phase_profile import PHASES  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"
KEYS = ["valu", "pk", "lane", "mfma", "lds", "vmem", "smem", "salu", "wait", "nop", "branch"]


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "lane"
    if op.startswith("v_pk_"):
        return "pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op == "s_waitcnt":
        return "wait"
    if op == "s_nop":
        return "nop"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    return "salu" if op.startswith("s_") else "other"


def main():
    src = os.path.join(B.CSRC, "he_physics.hip")
    flags = dict(B.SOURCES)["he_physics.hip"]
    with tempfile.TemporaryDirectory() as td:
        co = os.path.join(td, "k.co")
        subprocess.run([B._hipcc(), "--offload-arch=" + B.ARCH, "-O3", "-fPIC", "-std=c++17", "--cuda-device-only",
                        "--no-gpu-bundle-output", "-c", src, "-o", co] + flags + B.PHASES_DEFS["he_physics.hip"],
                       check=True, capture_output=True)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                             capture_output=True, text=True).stdout
    ins = []
    for line in dis.split("\n"):
        m = re.match(r"\s+([a-z_0-9]+)\s*(.*?)\s*//", line)
        if m:
            ins.append((m.group(1), m.group(2)))
    cuts = [k for k, (op, _) in enumerate(ins) if op == "s_memtime"]
    segs = {}
    for j in range(1, len(cuts)):
        a, b = cuts[j - 1], cuts[j]
        slot = None
        for op, arg in ins[b:b + 60]:  # the stamp's atomic add names its slot
            if op.startswith("global_atomic_add"):
                m = re.search(r"offset:(\d+)", arg)
                slot = int(m.group(1)) // 8 if m else 0
                break
        name = PHASES[slot] if slot is not None and slot < len(PHASES) else f"slot {slot}"
        c = segs.setdefault(name, {k: 0 for k in KEYS + ["other", "total", "segments"]})
        for op, _ in ins[a:b]:
            c[cls(op)] += 1
            c["total"] += 1
        c["segments"] += 1
    print(json.dumps({"kernel": "physics_kernel (stamp build)", "instructions": len(ins), "phases": segs,
                      "definition": __doc__.split("\n\n")[0]}, indent=1))


if __name__ == "__main__":
    main()
