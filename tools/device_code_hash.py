"""Hash of the physics TU's device code (the .text and .rodata sections of the gfx950 code object)
for the product and the phase-stamp builds, with the product flags of humanoid_amd/build.py. Two
sources with equal hashes compile to the same machine code (used to check that removing dead
compile-time variants leaves the shipped kernel bit-identical).

  python tools/device_code_hash.py [csrc_dir]
"""
import hashlib
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from humanoid_amd import build as B  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def code_hash(src, defs):
    flags = dict(B.SOURCES)["he_physics.hip"]
    with tempfile.TemporaryDirectory() as td:
        co = os.path.join(td, "k.co")
        cmd = [B._hipcc(), "--offload-arch=" + B.ARCH, "-O3", "-fPIC", "-std=c++17", "--cuda-device-only", "--no-gpu-bundle-output",
               "-c", src, "-o", co] + flags + defs
        subprocess.run(cmd, check=True, capture_output=True)
        h = hashlib.sha256()
        for sec in (".text", ".rodata"):
            out = os.path.join(td, sec[1:])
            subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary", "--only-section=" + sec, co, out],
                           check=True)
            h.update(open(out, "rb").read())
        return h.hexdigest()[:16]


if __name__ == "__main__":
    csrc = sys.argv[1] if len(sys.argv) > 1 else B.CSRC
    src = os.path.join(csrc, "he_physics.hip")
    print("product", code_hash(src, []))
    print("phases ", code_hash(src, B.PHASES_DEFS["he_physics.hip"]))
