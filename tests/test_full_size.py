"""Full-size (BASELINE configs[1]/[2]: 4096 envs) checks of the bench workload on the GPU, through
size-independent properties: determinism (the launch is bit-reproducible), finiteness, the
stand-still invariant of configs[1], and oracle parity on a random sample of envs taken from the
full-size run (one policy step from the GPU's own state, fp64 C oracle, the physics tolerances of
test_gpu_parity)."""
import argparse
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


def _rollout(config, model):
    import bench
    if not torch.cuda.is_available():
        pytest.skip("needs the GPU")
    args = argparse.Namespace(config=config, num_envs=4096, clips=128, seed=0, max_contacts=40)
    return bench.Rollout(args, model, 0, 0)


def _props(ro, idx):
    """configs[4]'s per-env mass scale, friction and terrain kind of the sampled envs (oracle kwargs)."""
    if ro.args.config != "dr":
        return {}
    return dict(mass_scale=ro.ms.cpu().numpy()[idx].copy(), friction=ro.fr.cpu().numpy()[idx].copy(),
                terrain_kind=ro.tk.cpu().numpy()[idx].copy())


def _state(ro):
    return (ro.eng.root_states.clone(), ro.eng.dof_state.clone(), ro.obs.clone(), ro.rew.clone())


@pytest.mark.parametrize("config", ["standstill", "imitation"])
def test_full_size_deterministic_and_finite(model, config):
    a, b = _rollout(config, model), _rollout(config, model)
    for _ in range(10):
        a.step()
        b.step()
    torch.cuda.synchronize()
    for x, y in zip(_state(a), _state(b)):
        assert torch.isfinite(x).all()
        assert torch.equal(x, y), "the step must be bit-reproducible"


def test_full_size_standstill_invariant(model):
    ro = _rollout("standstill", model)
    z0 = ro.eng.root_states[:, 2].clone()
    for _ in range(30):
        ro.step()
        # PD stand-still on the zero pose: nobody falls (resets happen only when the clip's time
        # runs out, which restarts the env at the same stand-still reference)
        assert (ro.term == 0).all()
    torch.cuda.synchronize()
    z = ro.eng.root_states[:, 2]
    assert (z - z0).abs().max().item() < 0.05
    assert (ro.eng.num_contacts == 16).all()  # 4 foot/toe boxes x 4 corners


@pytest.mark.parametrize("config", ["standstill", "imitation", "dr"])
def test_full_size_sample_matches_oracle(model, he_model, config):
    import cases  # tests/ on the path
    from humanoid_amd import _abi
    ro = _rollout(config, model)
    for _ in range(5):
        ro.step()
    torch.cuda.synchronize()
    rng = np.random.default_rng(11)
    idx = np.sort(rng.choice(4096, 48, replace=False))
    root = ro.eng.root_states.cpu().numpy()[idx].copy()
    dof = ro.eng.dof_state.view(4096, 69, 2).cpu().numpy()[idx].copy()
    cache = ro.eng.contact_cache.cpu().numpy()[idx].copy()  # the engine's warm start, for the oracle too
    ro.eng.step_actions(ro.actions, 2)
    torch.cuda.synchronize()
    tgt = ro.eng.dof_targets.cpu().numpy()[idx].copy()
    from test_gpu_parity import CondStats, _cond_close, contact_keys
    sp = _abi.default_sim_params(max_contacts=40, terrain=1 if config == "dr" else 0)
    props = _props(ro, idx)
    probes = []
    for seed in (123, 124, 125):  # the oracle's own sensitivity (see _cond_close)
        r_s, d_s = root.copy(), dof.copy()
        cases.probe_physics_step(he_model, sp, r_s, d_s, tgt, 2, cache.copy(), seed, **props)
        probes.append((r_s, d_s))
    c_o = cache.copy()
    out = O.physics_step(he_model, sp, root, dof, tgt, 2, cache=c_o, **props)
    kg = contact_keys(ro.eng.contact_cache.cpu().numpy()[idx])
    same = np.array([a == b for a, b in zip(kg, contact_keys(c_o))])
    assert same.mean() >= 0.95
    rg = ro.eng.root_states.cpu().numpy()[idx]
    dg = ro.eng.dof_state.view(4096, 69, 2).cpu().numpy()[idx]
    st = CondStats()
    _cond_close("root pos", rg[same, :3], root[same, :3], [r[same, :3] for r, _ in probes], 1e-4, stats=st)
    _cond_close("dof pos", dg[same, :, 0], dof[same, :, 0], [d[same, :, 0] for _, d in probes], 1e-4, stats=st)
    _cond_close("dof vel", dg[same, :, 1], dof[same, :, 1], [d[same, :, 1] for _, d in probes], 1e-2, 1e-3, stats=st)
    print(f"widened elements {st.widened}/{st.total}: {st.by_name}")
    assert st.frac <= 0.05


def test_full_size_dr_sample_30_steps(model, he_model):
    """configs[4] (4096 envs: mass / friction randomisation, plane / 10 deg slope / box steps) at full
    size: after 5 bench steps, 30 more policy steps of physics (actions 0) on all 4096 envs, and the
    oracle on a 48-env sample from the same state and warm-start cache (its own mass scale, friction
    and terrain). Joint angles and CoM at 1e-4 every step; envs whose contact sets or stick / slip
    states ever differ are excluded (below); at most 1% of the compared elements need the sensitivity
    widening (8 probes)."""
    import cases
    from humanoid_amd import _abi
    from test_gpu_parity import CondStats, _cond_close, contact_keys, friction_states, torsion_weights
    ro = _rollout("dr", model)
    for _ in range(5):
        ro.step()
    torch.cuda.synchronize()
    rng = np.random.default_rng(12)
    idx = np.sort(rng.choice(4096, 48, replace=False))
    root = ro.eng.root_states.cpu().numpy()[idx].copy()
    dof = ro.eng.dof_state.view(4096, 69, 2).cpu().numpy()[idx].copy()
    c_o = ro.eng.contact_cache.cpu().numpy()[idx].copy()
    props = _props(ro, idx)
    sp = _abi.default_sim_params(max_contacts=40, terrain=1)
    probes = [[root.copy(), dof.copy(), c_o.copy(), None] for _ in range(8)]  # 30 steps: 8 probes
    zero = torch.zeros_like(ro.actions)
    mism = np.zeros(len(idx), bool)
    slip = np.zeros(len(idx), bool)
    st = CondStats()
    hist = []
    for step in range(30):
        ro.eng.step_actions(zero, 2)
        tgt = ro.eng.dof_targets.cpu().numpy()[idx].copy()
        rw = np.zeros((len(idx), _abi.MAX_ROWS), np.float32)  # the oracle's row bound weights (torsion)
        O.set_row_weight_out(rw)
        try:
            out = O.physics_step(he_model, sp, root, dof, tgt, 2, cache=c_o, **props)
        finally:
            O.set_row_weight_out(None)
        for k, pr in enumerate(probes):  # fp32-level noise in every step
            pr[3] = cases.probe_physics_step(he_model, sp, pr[0], pr[1], tgt, 2, pr[2], 123 + 1000 * k + step, **props)
        torch.cuda.synchronize()
        cg = ro.eng.contact_cache.cpu().numpy()[idx]
        mism |= np.array([a != b for a, b in zip(contact_keys(cg), contact_keys(c_o))])
        tw = torsion_weights(rw, c_o)
        slip |= np.array([a != b for a, b in zip(friction_states(cg, props["friction"], tw),
                                                 friction_states(c_o, props["friction"], tw))])
        hist.append((ro.eng.dof_state.view(4096, 69, 2).cpu().numpy()[idx].copy(),
                     ro.eng.rb_state.view(4096, 24, 13).cpu().numpy()[idx].copy(), dof.copy(),
                     out["rb_state"].copy(), [p[1].copy() for p in probes], [p[3]["rb_state"].copy() for p in probes]))
    # configs[4] is the divergent-contact stress case: feet tip over step edges and slide on slopes,
    # and an env whose contact set or stick / slip state (a friction row within rounding of its
    # bound) ever differs between the fp32 engine and the fp64 oracle parts from it by the event;
    # such envs are excluded, at most 20% (r03 box: 2 contact-set + 5 stick/slip of 48)
    ok = ~(mism | slip)
    print(f"contact-set mismatch: {mism.sum()}/{len(idx)} envs, stick/slip mismatch {(slip & ~mism).sum()}")
    assert mism.mean() <= 0.1 and (mism | slip).mean() <= 0.2
    for dg, rbg, do, rbo, dps, rbps in hist:
        _cond_close("dof pos", dg[ok, :, 0], do[ok, :, 0], [d[ok, :, 0] for d in dps], 1e-4, stats=st)
        com = [cases.center_of_mass(model, r[ok]) for r in rbps]
        _cond_close("CoM", cases.center_of_mass(model, rbg[ok]), cases.center_of_mass(model, rbo[ok]), com, 1e-4,
                    stats=st)
    print(f"widened elements {st.widened}/{st.total} ({100 * st.frac:.2f}%): {st.by_name}")
    assert st.frac <= 0.01
