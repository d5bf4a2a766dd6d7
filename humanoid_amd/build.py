"""Build ``humanoid_amd/libhumanoid_engine.so`` for gfx950 with hipcc (in-tree, travels with the
repo to the GPU box). Usage: ``python -m humanoid_amd.build [--force]``."""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhumanoid_engine.so")
# diagnostic twin with the physics kernel's per-phase cycle stamps compiled in (tools/phase_profile.py);
# the product library leaves them out (their per-phase branches cost ~1% of the step)
PHASES_LIB = os.path.join(HERE, "libhumanoid_engine_phases.so")
PHASES_DEFS = {"he_physics.hip": ["-DHE_PHASE_STAMPS=1"]}
BUILD = os.path.join(HERE, "_build")
ARCH = os.environ.get("HE_OFFLOAD_ARCH", "gfx950")

# (source, extra flags): the imitation kernel must evaluate float32 expressions exactly as the
# reference's torch ops do (no FMA contraction); the physics kernel may contract.
SOURCES = [
    ("he_imitation.hip", ["-ffp-contract=off"]),
    # no SLP vectorisation: the compiler's own packed-FP32 pairing costs more moves than it saves;
    # the elimination issues its v_pk_fma_f32 explicitly (he_regla.h)
    # max-ilp scheduling: +1.0% against iterative-ilp (r02 A/B, 3 of 3 passes, bit-identical results),
    # which was +1% against the default (r01); iterative-minreg -4%
    ("he_physics.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize",
                        "-mllvm", "-amdgpu-sched-strategy=max-ilp"]),
    ("he_ingest.hip", []),
    ("he_rollout.hip", ["-ffp-contract=off"]),  # GAE: the Cython module's float32 rounding
    ("he_engine.cpp", ["-x", "hip"]),
]
HEADERS = ["he_kernels.h", "he_math.h", "he_imitation_env.h", "he_topo.h", "he_regla.h", "he_smpl_topo.h", os.path.join("..", "..", "include", "humanoid_engine.h"),
           os.path.join("..", "..", "include", "humanoid_rollout.h")]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


# kernels whose occupancy (waves per SIMD, the compiler's resource report) the build enforces: the
# physics kernel is one wave per env and latency-bound, and at one wave per SIMD it runs ~40 % slower
MIN_OCCUPANCY = {"he_physics.hip": ("physics_kernel", 2)}
# how many kernels of the TU match the watched name (physics_kernel and physics_kernel_tgs): a report
# that lists fewer fails the build, so neither can drop out of the check unnoticed
MIN_KERNELS = {"he_physics.hip": 2}


def _check_occupancy(src, stderr):
    """Every kernel of the TU whose name contains the watched name (the physics TU: physics_kernel and
    physics_kernel_tgs) must reach the occupancy."""
    want = MIN_OCCUPANCY.get(os.path.basename(src))
    if not want:
        return
    name, waves = want
    lines = stderr.splitlines()
    seen = 0
    for i, ln in enumerate(lines):
        if "Function Name:" in ln and name in ln:
            fn = ln.split("Function Name:")[1].split()[0]
            # every watched kernel must report its occupancy before the next function's report starts
            occ = None
            for ln2 in lines[i + 1:]:
                if "Function Name:" in ln2:
                    break
                m = re.search(r"Occupancy \[waves/SIMD\]: (\d+)", ln2)
                if m:
                    occ = int(m.group(1))
                    break
            if occ is None:
                raise RuntimeError(f"{fn}: no occupancy line in the compiler's resource report")
            if occ < waves:
                raise RuntimeError(f"{fn}: occupancy {occ} waves/SIMD < {waves} "
                                   "(register pressure; see the resource report)")
            seen += 1
    if seen < MIN_KERNELS.get(os.path.basename(src), 1):
        raise RuntimeError(f"{name}: {seen} kernel(s) in the compiler's resource report, "
                           f"{MIN_KERNELS.get(os.path.basename(src), 1)} expected")


def _compile(hipcc, cmd, src, o, force, hdr_time, verbose):
    stamp = o + ".cmd"  # a flag change rebuilds too
    same_cmd = os.path.exists(stamp) and open(stamp).read() == " ".join(cmd)
    if force or not same_cmd or _mtime(o) < max(_mtime(src), hdr_time):
        if verbose:
            print(" ".join(cmd))
        if os.path.basename(src) in MIN_OCCUPANCY:
            cmd = cmd + ["-Rpass-analysis=kernel-resource-usage"]
        # a failed compile or occupancy check leaves neither the object nor the stamp behind, so the
        # next build cannot mistake a rejected object for an up-to-date one
        _discard(o, stamp)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            _discard(o, stamp)
            raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stderr}")
        try:
            _check_occupancy(src, r.stderr)
        except RuntimeError:
            _discard(o, stamp)
            raise
        cmd = cmd[:-1] if cmd[-1] == "-Rpass-analysis=kernel-resource-usage" else cmd
        with open(stamp, "w") as f:
            f.write(" ".join(cmd))
        return True
    return False


def _discard(*paths):
    for p in paths:
        if os.path.exists(p):
            os.remove(p)


def _link(hipcc, lib, objs, force):
    if force or _mtime(lib) < max(_mtime(o) for o in objs):
        cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")


def build(force=False, verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    common = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function"]
    hdr_time = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    for lib, defs, suffix in ((LIB, {}, ".o"), (PHASES_LIB, PHASES_DEFS, ".phases.o")):
        objs = []
        for src, flags in SOURCES:
            s = os.path.join(CSRC, src)
            o = os.path.join(BUILD, src + (suffix if src in defs else ".o"))
            objs.append(o)
            cmd = [hipcc] + common + flags + defs.get(src, []) + ["-c", s, "-o", o]
            _compile(hipcc, cmd, s, o, force and lib == LIB or force and src in defs, hdr_time, verbose)
        _link(hipcc, lib, objs, force)
    return LIB


def device_code_id(lib=LIB):
    """sha256[:16] of the library's embedded device code (the ELF `.hip_fatbin` section: every gfx950
    code object linked in). Host-only changes leave it equal; any kernel change moves it. Measurement
    records (tests/test_full_size.py) store it, and bench.py reports a record as stale when it does not
    match the library it loaded."""
    import hashlib
    import struct
    with open(lib, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise RuntimeError(f"{lib}: not an ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sec(i):
        name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
        return name, off, size
    _, stroff, _ = sec(shstrndx)
    for i in range(shnum):
        name, off, size = sec(i)
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    raise RuntimeError(f"{lib}: no .hip_fatbin section")


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
