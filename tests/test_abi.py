"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every symbol the
header declares; ctypes struct layouts match the header's sizes; host-side model/topology logic."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "humanoid_engine.h")


def declared_symbols():
    import glob
    text = "".join(open(h).read() for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(he_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from humanoid_amd import engine
    lib_path = engine.LIB_PATH
    if not os.path.exists(lib_path):
        from humanoid_amd import build
        build.build()
    lib = C.CDLL(lib_path)  # loads without a GPU
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(engine.HE_SYMBOLS)
    lib.he_version.restype = C.c_int
    assert lib.he_version() == 1
    lib.he_hash_uniform.restype = C.c_float
    lib.he_hash_uniform.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
    from oracle import oracle as O
    for s, st, e in [(0, 0, 0), (1, 7, 4095), (123456789, 1 << 40, 17)]:
        assert lib.he_hash_uniform(s, st, e) == O.hash_uniform(s, st, e)


def test_build_tracks_every_kernel_header():
    """build.build() rebuilds when a header changes only if the header is in build.HEADERS: every
    header a kernel source includes must be listed (an unlisted one once left a stale library)."""
    import glob
    from humanoid_amd import build
    csrc = os.path.join(ROOT, "humanoid_amd", "csrc")
    tracked = {os.path.normpath(os.path.join(csrc, h)) for h in build.HEADERS}
    for src in glob.glob(os.path.join(csrc, "*")):
        for inc in re.findall(r'#include\s+"([^"]+)"', open(src).read()):
            path = os.path.normpath(os.path.join(csrc, inc))
            assert path in tracked, f"{os.path.basename(src)} includes {inc}, not in build.HEADERS"


def test_errors_are_reported_without_gpu():
    from humanoid_amd import _abi, engine
    lib = engine.load_library()
    h = C.c_void_p()
    p = _abi.default_sim_params()
    rc = lib.he_create(C.byref(p), 0, C.byref(h))
    assert rc != 0
    assert lib.he_last_error().decode()


def test_struct_sizes_match_header(tmp_path):
    from humanoid_amd import _abi
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "humanoid_engine.h"\n#include "humanoid_rollout.h"\n'
                   'int main(){printf("%zu %zu %zu %zu %zu %zu\\n",'
                   "sizeof(he_model),sizeof(he_sim_params),sizeof(he_imitation_params),sizeof(he_env_motion),"
                   "sizeof(he_rollout_field),sizeof(he_rollout_index));}\n")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert [int(x) for x in out] == [C.sizeof(_abi.HeModel), C.sizeof(_abi.HeSimParams),
                                     C.sizeof(_abi.HeImitationParams), C.sizeof(_abi.HeEnvMotion),
                                     C.sizeof(_abi.HeRolloutField), C.sizeof(_abi.HeRolloutIndex)]


def test_model_blob(model):
    from humanoid_amd import _abi
    hm = _abi.make_model(model)
    assert hm.num_pairs == 245
    assert abs(sum(hm.mass) - 73.995) < 1e-2
    assert list(hm.parents)[:5] == [-1, 0, 1, 2, 3]


def test_mjcf_roundtrip_matches_baked_json(model):
    xml = "/root/reference/packages/puffer-phc/puffer_phc/assets/smpl_humanoid.xml"
    if not os.path.exists(xml):
        pytest.skip("reference asset not present (GPU box)")
    from humanoid_amd.model import parse_mjcf
    m = parse_mjcf(xml)
    np.testing.assert_allclose(m.local_pos, model.local_pos)
    np.testing.assert_allclose(m.mass, model.mass)
    np.testing.assert_allclose(m.inertia, model.inertia)


def test_occupancy_guard_removes_the_rejected_object(tmp_path, monkeypatch):
    """build._compile must not leave an object (or its command stamp) behind when the occupancy check
    rejects it: the next build would otherwise see an up-to-date object and skip the check."""
    import subprocess
    import types
    from humanoid_amd import build
    src = tmp_path / "he_physics.hip"
    src.write_text("// fake")
    o = str(tmp_path / "he_physics.hip.o")
    stamp = o + ".cmd"
    remark = ("remark: Function Name: physics_kernel\nremark:     VGPRs: 256\n"
              "remark:     Occupancy [waves/SIMD]: 2\n"
              "remark: Function Name: physics_kernel_tgs\nremark:     VGPRs: 300\n"
              "remark:     Occupancy [waves/SIMD]: 1\n")

    def fake_run(cmd, capture_output=True, text=True):
        out = cmd[cmd.index("-o") + 1]
        with open(out, "w") as f:
            f.write("object")
        return types.SimpleNamespace(returncode=0, stderr=remark, stdout="")

    monkeypatch.setattr(subprocess, "run", fake_run)
    cmd = ["hipcc", "-c", str(src), "-o", o]
    with open(stamp, "w") as f:  # a stamp from an earlier build with the same command
        f.write(" ".join(cmd))
    with pytest.raises(RuntimeError, match="occupancy 1"):
        build._compile("hipcc", cmd, str(src), o, True, 0.0, False)
    assert not os.path.exists(o) and not os.path.exists(stamp)
    # a passing report keeps the object and writes the stamp
    remark = remark.replace("SIMD]: 1", "SIMD]: 2")
    assert build._compile("hipcc", cmd, str(src), o, True, 0.0, False)
    assert os.path.exists(o) and open(stamp).read() == " ".join(cmd)
    # a watched kernel whose report has no occupancy line, or a missing kernel, fails too
    full = remark
    remark = full.replace("remark:     Occupancy [waves/SIMD]: 2\n", "", 1)
    with pytest.raises(RuntimeError, match="no occupancy line"):
        build._compile("hipcc", cmd, str(src), o, True, 0.0, False)
    remark = full.split("remark: Function Name: physics_kernel_tgs")[0]
    with pytest.raises(RuntimeError, match="2 expected"):
        build._compile("hipcc", cmd, str(src), o, True, 0.0, False)
