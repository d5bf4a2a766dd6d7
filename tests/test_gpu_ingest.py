"""Device-side motion ingestion (he_ingest_clips) against the host restatement
(``motion_lib.build_tables``, itself pinned to the reference's motion_lib golden vectors in
test_oracle_golden.py): both engines sample the same motion states at the same times.

Tolerances: positions / rotations 2e-5 (fp32 FK in a different operation order); linear velocity
1e-3 abs + 1e-4 rel (the Gaussian filter accumulates in fp32 here, fp64 in scipy); angular and dof
velocities 3e-3 abs + 1e-3 rel (arccos of a near-identity rotation difference in fp32, as for the
reference loader's own fp32 path, test_oracle_golden.py)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _clips(model):
    from humanoid_amd import synthetic
    rng = np.random.default_rng(7)
    out = [synthetic.make_clip(model, rng, num_frames=t) for t in (150, 37, 5, 2, 90)]
    out.append(synthetic.make_standstill_clip(model, num_frames=20))
    return out


def test_ingest_matches_host_tables(model, he_model):
    from humanoid_amd.engine import Engine
    from humanoid_amd.motion_lib import build_tables
    clips = _clips(model)
    n = 8
    host = Engine(he_model, n, device=0)
    host.load_motions(build_tables(model, clips))
    dev = Engine(he_model, n, device=0)
    dev.ingest_clips(clips)
    rng = np.random.default_rng(1)
    k = 4096
    ids = torch.as_tensor(rng.integers(0, len(clips), k), device="cuda:0")
    lens = torch.as_tensor([(len(c["pose_quat_global"]) - 1) / 30.0 for c in clips], device="cuda:0")
    times = torch.rand(k, device="cuda:0") * lens[ids] * 1.02  # includes the clamp past the end
    a = host.motion_state(ids, times)
    b = dev.motion_state(ids, times)
    torch.cuda.synchronize()
    tol = {"rg_pos": (2e-5, 0), "rb_rot": (2e-5, 0), "dof_pos": (2e-4, 0), "body_vel": (1e-3, 1e-4),
           "body_ang_vel": (3e-3, 1e-3), "dof_vel": (3e-3, 1e-3)}
    for key, (atol, rtol) in tol.items():
        x, y = b[key].cpu().numpy(), a[key].cpu().numpy()
        if key == "rb_rot":  # sign-free
            x = np.where((x * y).sum(-1, keepdims=True) < 0, -x, x)
        np.testing.assert_allclose(x, y, atol=atol, rtol=rtol, err_msg=key)


def test_ingest_motion_clip_mapping(model, he_model):
    """Per-env motion entries sharing clips (motion i -> clip map) equal per-env copies."""
    from humanoid_amd.engine import Engine
    clips = _clips(model)
    n = 8
    mapping = np.array([3, 0, 0, 5, 1, 1, 1, 4], np.int32)
    shared = Engine(he_model, n, device=0)
    shared.ingest_clips(clips, mapping)
    copies = Engine(he_model, n, device=0)
    copies.ingest_clips([clips[i] for i in mapping])
    ids = torch.arange(n, device="cuda:0").repeat(64)
    times = torch.rand(ids.numel(), device="cuda:0") * 0.5
    a = shared.motion_state(ids, times)
    b = copies.motion_state(ids, times)
    torch.cuda.synchronize()
    for key in a:
        assert torch.equal(a[key], b[key]), key


def test_ingest_rejects_bad_input(he_model):
    from humanoid_amd.engine import Engine, EngineError
    eng = Engine(he_model, 4, device=0)
    with pytest.raises(EngineError):
        eng.ingest_clips([{"pose_quat_global": np.zeros((3, 24, 4), np.float32),
                           "root_trans_offset": np.zeros((3, 3), np.float32), "fps": 30}], np.array([0, 2], np.int32))
