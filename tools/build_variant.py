"""Diagnostics: build the engine library with extra -D flags on the physics TU into
humanoid_amd/_variants/<name>.so, for A/B timing on one GPU box (HE_ENGINE_LIB=<path>).
Usage: python tools/build_variant.py NAME [--tu he_imitation.hip] [-DFOO=1 ...] [-mllvm -opt ...]
(an -amdgpu-sched-strategy= given here replaces the product's max-ilp)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from humanoid_amd import build as B  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    tu = "he_physics.hip"
    if defs[:1] == ["--tu"]:
        tu, defs = defs[1], defs[2:]
    B.build()
    out_dir = os.path.join(ROOT, "humanoid_amd", "_variants")
    os.makedirs(out_dir, exist_ok=True)
    hipcc = B._hipcc()
    flags = list(dict(B.SOURCES)[tu])
    if any(d.startswith("-amdgpu-sched-strategy=") for d in defs) and "-amdgpu-sched-strategy=max-ilp" in flags:
        i = flags.index("-amdgpu-sched-strategy=max-ilp")  # a variant's strategy replaces the product's
        del flags[i - 1:i + 1]
    obj = os.path.join(out_dir, name + "." + tu + ".o")
    cmd = [hipcc, "--offload-arch=" + B.ARCH, "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function"] + flags + defs + \
          ["-c", os.path.join(B.CSRC, tu), "-o", obj]
    subprocess.run(cmd, check=True)
    objs = [obj if src == tu else os.path.join(B.BUILD, src + ".o") for src, _ in B.SOURCES]
    lib = os.path.join(out_dir, name + ".so")
    subprocess.run([hipcc, "--offload-arch=" + B.ARCH, "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main()
