"""Env-step throughput of the MI355X humanoid engine (BASELINE.json metric).

One "step" = one policy step of every env on every rank: actions -> PD targets -> 2 gym.simulate()
calls of 1/60 s, each 2 physics substeps of 1/120 s (Isaac Gym's SimParams.substeps default; DESIGN
§5) solved by PhysX TGS's 4 position iterations (isaacgym_env.py:16-18) -> reward / reset /
934-float obs -> device-side reset of flagged envs
(puffer_phc/clean_pufferl/env.py:109-183 semantics; env-steps/s definition env.py:217-230).

Default workload = BASELINE configs[1]: 4096 SMPL-neutral humanoids per GPU, PD stand-still
(zero reference motion, actions = 0). `--config imitation` = configs[2] (128 synthetic clips,
one fixed U(-1,1) action sample), `--config dr` = configs[4] (mass/friction randomisation +
3 terrains). Data: synthetic clips (AMASS / SMPL are not available offline).

Multi-GPU: `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`; every rank owns
its own 4096 envs (envs are independent: no data-path collective), barrier + synchronize around the
timed region, max time over ranks, value = total env-steps of all ranks / that time.
"""
import argparse
import datetime
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

EV_STEPS = 60                  # kernel-duration pass after the timed region: events on every step
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector = FP32 matrix peak (spec)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
# SURVEY.md §8(d) canonical algorithmic counts per env-step
PHYS_FLOP_PER_SUBSTEP = 654_639            # dense-equivalent physics per physics step, n_c = 8
# SURVEY's 1,309,278 FLOP/env-step counts 2 physics steps; the engine runs gym.simulate() x 2 with
# SimParams.substeps = 2 (Isaac Gym's default), i.e. 4 physics steps of 1/120 s per env-step
IMIT_FLOP_PER_ENV_STEP = 30_000             # the imitation step (≈0.03 MFLOP)


def canonical_flop_per_physics_step(m):
    """SURVEY §8(d)'s dense-equivalent count per physics step with m contact rows (n = 75): mass
    matrix 135,756 + factorisation n^3/3 + bias 6,000 + 2 triangular solves 2 n^2 + contacts
    2 n^2 m + 2 n m^2 + 4 x 2 m^2 (654,639 at m = 3 x 8)."""
    n = 75
    return 135_756 + n ** 3 / 3 + 6_000 + 2 * n * n + 2 * n * n * m + 2 * n * m * m + 8 * m * m


def canonical_at_rows(m, physics_steps, envs, launch_ms):
    flop = canonical_flop_per_physics_step(m) * physics_steps
    tf = flop * envs / (launch_ms * 1e-3) / 1e12
    return {"rows_mean": round(m, 2), "flop_per_env_step": round(flop), "achieved": round(tf, 4),
            "frac": round(tf / FP32_PEAK_TFLOPS, 6)}
IMIT_BYTES_PER_ENV_STEP = 13_200            # fused imitation kernel share of the 16.0 KB/env-step


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--config", choices=["standstill", "imitation", "tracking", "dr"], default="standstill",
                    help="standstill = configs[1]; imitation = configs[2] with one fixed action sample; tracking = "
                         "configs[2] with the tracking action stream (computed on the device each step); dr = configs[4]")
    ap.add_argument("--clips", type=int, default=128)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-envs", type=int, default=2048)
    ap.add_argument("--cpu-steps", type=int, default=300)
    ap.add_argument("--max-contacts", type=int, default=40)
    ap.add_argument("--scheme", choices=["default", "pgs", "r02", "tgs_small"], default="default",
                    help="physics scheme: default = the reference's PhysX TGS (solver_type 1, isaacgym_env.py:16-18): "
                         "2 simulate() x 2 substeps of 1/120 s, each 4 position iterations on its factor and contact "
                         "set (DESIGN §5 'TGS'); pgs = the engine's velocity-level PGS step (rounds 1-4's default: 8 "
                         "warm-started sweeps per 1/120 s step, midpoint bias); r02 = round 2's energy-unstable step "
                         "(2 x 1/60 s, explicit bias, 8 PGS sweeps) with round 3's clamps, for the cost comparison "
                         "only (DESIGN §5); tgs_small = TGS's small-step form, 8 PGS substeps of 1/480 s per simulate() "
                         "with one sweep each")
    ap.add_argument("--solver-tolerance", type=float, default=None,
                    help="he_sim_params.solver_tolerance override (m/s; 0 = every sweep runs)")
    ap.add_argument("--no-puffer-level", action="store_true",
                    help="skip the PHCPufferEnv.step-level rate (numpy actions in, host bookkeeping)")
    ap.add_argument("--puffer-steps", type=int, default=50)
    ap.add_argument("--fused", action="store_true",
                    help="he_env_step as one launch (the imitation step in the physics kernel's epilogue); "
                         "at 4096 envs the two launches are faster (DESIGN §4.1)")
    ap.add_argument("--no-learner", action="store_true",
                    help="skip the configs[3] per-rank learner leg (rollout into the device Experience, GAE, PPO "
                         "update of the reference-size policy, RCCL gradient all-reduce)")
    ap.add_argument("--no-tracking", action="store_true",
                    help="skip the configs[2] tracking-action leg (throughput + joint-pose L2 vs ref)")
    return ap.parse_args(argv)


DATA = {
    "standstill": "synthetic: one random-free stand-still clip (identity rotations, constant root), actions = 0",
    "imitation": "synthetic: 128 AMASS-schema random-walk clips (SURVEY §8d recipe), env i -> clip i mod 128, "
                 "one U(-1,1) action sample reused",
    "dr": "synthetic: 128 random-walk clips, actions = 0, per-env mass scale U(0.8,1.2), friction U(0.5,1.25), "
          "terrain by env % 3 (plane / 10 deg slope / steps)",
    "tracking": "synthetic: 128 AMASS-schema random-walk clips, env i -> clip i mod 128, actions = "
                "clip(ref_dof_pos / scale) computed on the device every step",
}


def make_clips(args, model):
    from humanoid_amd import synthetic
    if args.config == "standstill":
        return [synthetic.make_standstill_clip(model, num_frames=150)]
    rng = np.random.default_rng(args.seed)
    return [synthetic.make_clip(model, rng, num_frames=150) for _ in range(args.clips)]


def puffer_level(args, model):
    """PHCPufferEnv.step rate (clean_pufferl/env.py:109-183 semantics): numpy actions copied to the
    device every step, fused physics + imitation + device resets, episode bookkeeping on device,
    info every 32 ticks. PCIe-inclusive; reported beside `value`, never as it."""
    import torch
    from humanoid_amd.env import EnvConfig, PHCPufferEnv
    clips = make_clips(args, model)
    cfg = EnvConfig(num_envs=args.num_envs, motion_file={f"clip{i}": c for i, c in enumerate(clips)},
                    seed=args.seed, max_contacts=args.max_contacts)
    pe = PHCPufferEnv(cfg)
    pe.reset()
    _, actions, _ = build_workload(args, model, 0)
    for _ in range(5):
        pe.step(actions)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.puffer_steps):
        pe.step(actions)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pe.close()
    return {"value": round(args.num_envs * args.puffer_steps / dt, 1), "unit": "env-steps/s",
            "steps": args.puffer_steps, "actions": "numpy [N,69] float32 (H2D each step)"}


def build_workload(args, model, rank):
    from humanoid_amd.motion_lib import build_tables, MotionTables
    n = args.num_envs
    clips = make_clips(args, model)
    assign = np.zeros(n, np.int64) if args.config == "standstill" else np.arange(n) % args.clips
    base = build_tables(model, clips)
    tables = MotionTables(gts=base.gts, grs=base.grs, lrs=base.lrs, gvs=base.gvs, gavs=base.gavs, dvs=base.dvs,
                          num_frames=base.num_frames[assign], length_starts=base.length_starts[assign],
                          lengths=base.lengths[assign], dt=base.dt[assign], fps=base.fps[assign])
    rng = np.random.default_rng(args.seed + 1 + rank)
    if args.config == "imitation":
        actions = rng.uniform(-1, 1, (1, 69)).astype(np.float32).repeat(n, 0)  # env.py:221 one sample reused
    else:
        actions = np.zeros((n, 69), np.float32)
    return tables, actions, rng


class Rollout:
    """Device-resident rollout state for one rank."""

    def __init__(self, args, model, device_index, rank):
        import torch
        from humanoid_amd import _abi
        from humanoid_amd.engine import Engine
        from humanoid_amd.model import pd_action_offset_scale
        from humanoid_amd.body_sets import frozen_dof_mask
        self.args = args
        self.model = model
        self.fused = bool(getattr(args, "fused", False))
        n = args.num_envs
        tables, actions, rng = build_workload(args, model, rank)
        sim = _abi.default_sim_params(max_contacts=args.max_contacts, terrain=1 if args.config == "dr" else 0,
                                      **scheme_params(args))
        self.eng = Engine(model, n, device=device_index, sim_params=sim, start_xy=rng.uniform(-1, 1, (n, 2)))
        dev = self.eng.device
        self.eng.load_motions(tables)
        off, sc = pd_action_offset_scale(model)
        self.eng.set_pd_params(off, sc, np.array(frozen_dof_mask(), np.int32), clip_actions=True)
        if args.config == "dr":
            self.ms = torch.as_tensor(rng.uniform(0.8, 1.2, (n, 24)).astype(np.float32), device=dev)
            self.fr = torch.as_tensor(rng.uniform(0.5, 1.25, n).astype(np.float32), device=dev)
            self.tk = torch.as_tensor((np.arange(n) % 3).astype(np.int32), device=dev)
            self.eng.set_env_properties(self.ms, self.fr, self.tk)
        self.p = _abi.imitation_params()
        self.mids = torch.arange(n, device=dev, dtype=torch.int64)
        self.st = torch.zeros(n, device=dev)
        self.so = torch.zeros(n, device=dev)
        self.go = torch.zeros(n, 3, device=dev)
        self.prog = torch.zeros(n, dtype=torch.int16, device=dev)
        self.em = self.eng.env_motion(self.mids, self.st, self.so, self.go, self.prog)
        self.obs = torch.zeros(n, 934, device=dev)
        self.rew = torch.zeros(n, device=dev)
        self.raw = torch.zeros(n, 5, device=dev)
        self.reset = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.term = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.actions = torch.as_tensor(actions, device=dev)
        self.seed = args.seed * 7919 + rank
        self.step_index = 0
        # HumanoidPHC.reset() of all envs (reference state init, humanoid_phc.py:90-103)
        ids = torch.arange(n, dtype=torch.int32, device=dev)
        phases = torch.as_tensor(rng.uniform(0, 1, n).astype(np.float32), device=dev)
        self.eng.reset_envs(self.p, self.em, ids, phases, self.obs, self.reset, self.term)
        self.eng.set_fused_step(self.fused)
        torch.cuda.synchronize()  # the setup's launches end here, before any step is enqueued

    def tracking_actions(self):
        """a = clip(ref_dof_pos / scale, -1, 1) with the reference pose at
        the env's next motion time (humanoid_phc.py motion_times = progress * dt + start + offset),
        on the device: one motion-state launch + elementwise ops."""
        import torch
        if not hasattr(self, "inv_scale"):
            from humanoid_amd.model import pd_action_offset_scale
            _, sc = pd_action_offset_scale(self.model)
            self.inv_scale = torch.as_tensor(1.0 / np.asarray(sc, np.float32), device=self.eng.device)
        t = (self.prog.float() + 1.0) * self.p.control_dt + self.st + self.so
        ref = self.eng.motion_state(self.mids, t, None)["dof_pos"]
        torch.clamp(ref * self.inv_scale, -1.0, 1.0, out=self.actions)

    def joint_pose_l2(self):
        """BASELINE metric's "joint-pose L2 vs ref": mean over envs of ||q - q_ref(t)||_2 (rad, 69
        dofs) at the env's current motion time."""
        t = self.prog.float() * self.p.control_dt + self.st + self.so
        ref = self.eng.motion_state(self.mids, t, None)["dof_pos"]
        q = self.eng.dof_state.view(self.args.num_envs, 69, 2)[..., 0]
        return (q - ref).norm(dim=1)

    def step(self, ev=None):
        """One he_env_step (fused: one launch; `--unfused`: the physics and imitation launches).
        ev: optional (start, mid, end) torch.cuda.Events; unfused, mid splits the two kernels.
        configs[2]'s tracking stream (--config tracking): the actions first, outside the events."""
        if self.args.config == "tracking":
            self.tracking_actions()
        if ev is not None:
            ev[0].record()
        if self.fused:
            self.eng.env_step(self.p, self.em, self.actions, self.obs, self.rew, self.raw, self.reset, self.term,
                              seed=self.seed, step_index=self.step_index)
            if ev is not None:
                ev[1].record()
        else:
            self.eng.step_actions(self.actions, 2)
            if ev is not None:
                ev[1].record()
            self.eng.imitation_reset_step(self.p, self.em, self.obs, self.rew, self.raw, self.reset, self.term,
                                          seed=self.seed, step_index=self.step_index)
        if ev is not None:
            ev[2].record()
        self.step_index += 1

    def set_fused(self, fused):
        self.fused = bool(fused)
        self.eng.set_fused_step(self.fused)


def _pmc_entry(name, key):
    """The committed rocprofv3 counter record `profiles/<name>` for workload key `config:num_envs`."""
    f = os.path.join(ROOT, "profiles", name)
    try:
        return json.load(open(f)).get(key) if os.path.exists(f) else None
    except Exception:
        return None


def kernel_figures(args, config, n, phys_ms, imit_ms, rows_mean):
    """The physics kernel's roofline entry and the imitation kernel's HBM entry for one workload:
    launch medians (HIP events) against SURVEY §8(d)'s canonical counts, with the committed PMC
    counter records of the same workload key (pmc_traffic.json, pmc_mfma.json) beside them."""
    key = f"{config}:{n}"
    tr, mf = _pmc_entry("pmc_traffic.json", key), _pmc_entry("pmc_mfma.json", key)
    traffic = tr.get("physics_bytes_per_launch") if tr else None
    imit_traffic = tr.get("imitation_bytes_per_launch") if tr else None
    mfma = None
    if mf:
        mfma = {"util": mf["mfma_util"], "valu_issue_frac": mf["valu_issue_frac"],
                "source": "profiles/pmc_mfma.json (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / "
                          "(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs))"}
    phys_flop = PHYS_FLOP_PER_SUBSTEP * 2 * sim_substeps(args)  # per env-step: 2 simulate() x substeps
    phys_tflops = phys_flop * n / (phys_ms * 1e-3) / 1e12
    imit_gbs = IMIT_BYTES_PER_ENV_STEP * n / (imit_ms * 1e-3) / 1e9
    # the physics kernel alone (the unfused launch): latency-bound, priced against the FP32 vector /
    # matrix peak with the canonical dense-equivalent flop count; mfma_util is the measured
    # matrix-core busy share (rocprofv3 SQ counters)
    phys = {"bound": "latency", "achieved": round(phys_tflops, 4), "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(phys_tflops / FP32_PEAK_TFLOPS, 6), "traffic": traffic,
            "kernel": f"{'physics_kernel_tgs' if scheme_params(args).get('solver_type', 1) == 1 else 'physics_kernel'} "
                      f"(fp32 VALU + MFMA; SURVEY §8d canonical 0.6546 MFLOP per physics step "
                      f"x {2 * sim_substeps(args)} physics steps per env-step)",
            "avg_launch_ms": round(phys_ms, 4), "mfma_util": mfma,
            # "report n_c as measured" -- the same count with the measured mean solver
            # rows as m (patch friction: a standing body 28 rows, not 3 x 16 slots)
            "at_measured_rows": canonical_at_rows(rows_mean, 2 * sim_substeps(args), n, phys_ms)}
    imit = {"bound": "hbm", "achieved": round(imit_gbs, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(imit_gbs / HBM_PEAK_GBS, 5),
            "avg_launch_ms": round(imit_ms, 4), "traffic": imit_traffic,
            # the bytes that reached HBM (PMC FETCH_SIZE + WRITE_SIZE per launch, profiles/pmc_traffic.json)
            # over the same launch time: with one clip (configs[1]) most motion reads hit the caches, so
            # this is well under the algorithmic figure above
            "hbm_frac_counter": (round(imit_traffic / (imit_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                                 if imit_traffic else None)}
    return phys, imit


def kernel_pass(ro, steps, before=None):
    """`steps` further steps (untimed, the same workload continuing) with HIP events around the
    launches of EVERY step, on the engine's stream (torch's current stream): per step the first
    launch (physics), the second (imitation) and the whole step, in ms. `before`: called ahead of
    each step, outside the events (the tracking leg's action launch)."""
    import torch
    ev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(steps)]
    for e in ev:
        if before is not None:
            before()
        ro.step(e)
    torch.cuda.synchronize()
    return (np.array([e[0].elapsed_time(e[1]) for e in ev]), np.array([e[1].elapsed_time(e[2]) for e in ev]),
            np.array([e[0].elapsed_time(e[2]) for e in ev]))


def solver_rows(ro):
    """Solver rows of each env's last solve: word 7 of the warm-start cache (include/humanoid_engine.h)."""
    import torch
    return ro.eng.contact_cache[:, 7].contiguous().view(torch.int32).cpu().numpy()


def config_leg(args, model, device_index, config, steps=50, warmup=10):
    """Another BASELINE config on this rank's GPU, the bench's own form (two launches per step): the
    rate over `steps` timed steps, then the kernel figures from a pass of EV_STEPS steps with events.
    configs[4] ("dr"): mass / friction randomisation + 3 terrains, the divergent-contact stress config."""
    import torch
    a = argparse.Namespace(**vars(args))
    a.config = config
    a.fused = False
    ro = Rollout(a, model, device_index, 0)
    for _ in range(warmup):
        ro.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ro.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    first, second, _ = kernel_pass(ro, EV_STEPS)
    rows = solver_rows(ro)
    phys, imit = kernel_figures(a, config, a.num_envs, float(np.median(first)), float(np.median(second)),
                                float(rows.mean()))
    nc = ro.eng.num_contacts.cpu().numpy()
    return {"value": round(a.num_envs * steps / dt, 1), "unit": "env-steps/s", "steps": steps, "warmup": warmup,
            "workload": {"standstill": "configs[1]", "imitation": "configs[2]",
                         "dr": "configs[4]: 4096 envs, per-env mass scale U(0.8,1.2), friction U(0.5,1.25), terrain "
                               "by env % 3 (plane / 10 deg slope / steps), actions = 0"}[config],
            "physics_kernel": phys, "imitation_kernel": imit,
            "contacts": {"slots_mean": round(float(nc.mean()), 3), "rows_mean": round(float(rows.mean()), 2),
                         "rows_max": int(rows.max())}}


def tracking_leg(args, model, device_index, steps=50, warmup=10, l2_steps=60):
    """configs[2] with the tracking action stream: 4096 envs over 128 clips,
    actions = clip(ref_dof_pos / scale) computed on the device every step inside the timed region;
    then the joint-pose L2 vs the reference over `l2_steps` further steps (untimed)."""
    import torch
    a = argparse.Namespace(**vars(args))
    a.config = "imitation"
    a.fused = False
    ro = Rollout(a, model, device_index, 0)
    for _ in range(warmup):
        ro.tracking_actions()
        ro.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ro.tracking_actions()
        ro.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    first, second, _ = kernel_pass(ro, EV_STEPS, before=ro.tracking_actions)
    phys, imit = kernel_figures(a, "imitation", a.num_envs, float(np.median(first)), float(np.median(second)),
                                float(solver_rows(ro).mean()))
    l2 = []
    for _ in range(l2_steps):
        ro.tracking_actions()
        ro.step()
        l2.append(ro.joint_pose_l2())
    l2 = torch.stack(l2).cpu().numpy()
    return {"value": round(a.num_envs * steps / dt, 1), "unit": "env-steps/s", "steps": steps,
            "workload": "configs[2]: 4096 envs over 128 synthetic clips, actions = clip(ref_dof_pos / scale) "
                        "computed on the device each step (inside the timed region)",
            "physics_kernel": phys, "imitation_kernel": imit,
            "joint_pose_l2_rad": {"mean": round(float(l2.mean()), 5), "p90": round(float(np.percentile(l2, 90)), 5),
                                  "steps": l2_steps,
                                  "definition": "||q - q_ref(t)||_2 over the 69 exp-map dofs per env, mean over envs x "
                                                "steps: PD tracking error against the clips' motion, not parity"},
            "parity_vs_oracle": parity_record()}


def parity_record(name="parity_configs2"):
    """BASELINE's "joint-pose L2 vs ref" as parity: the fp32 engine against the fp64 oracle on 48-env
    samples of a workload over 30 policy steps, measured by the GPU tests
    tests/test_full_size.py::test_full_size_{tracking,standstill}_parity_30_steps (the bench never runs
    the oracle outside its cpu_baseline leg); the newest committed record, profiles/r*/<name>.json
    (parity_configs2: configs[2] tracking; parity_configs1: configs[1], the headline workload)."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*",
                                          name + ".json")))
    if not files:
        return None
    with open(files[-1]) as f:
        rec = json.load(f)
    keep = ("joint_pose_l2_vs_oracle_rad", "com_err_vs_oracle_m", "envs", "steps", "envs_with_event",
            "env_steps_before_event", "post_event")
    out = {k: rec[k] for k in keep if k in rec}
    out["source"] = os.path.relpath(files[-1], os.path.dirname(os.path.abspath(__file__)))
    # the record belongs to this build only if it was measured with the same device code
    from humanoid_amd import build as B
    from humanoid_amd.engine import LIB_PATH
    try:
        here = B.device_code_id(os.environ.get("HE_ENGINE_LIB") or LIB_PATH)
    except Exception:
        here = None
    out["device_code"] = {"record": rec.get("device_code"), "loaded": here,
                          "status": "current" if rec.get("device_code") and rec.get("device_code") == here else "stale"}
    return out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def learner_leg(args, model, device_index):
    """configs[3] per rank: this rank's 4096 envs x 32 steps into the
    device Experience with the reference-size policy in the loop (16.98 M params), GAE, then the PPO
    update (4 epochs x 4 minibatches of 32768, core.py:264-380) with the gradient all-reduce on device
    tensors between backward and the clip (core.py:366-373). Runs on every rank; at N = 1 the
    collective runs on a one-rank RCCL group, so the backend the 8-GPU node uses has executed."""
    import torch
    import torch.distributed as dist
    from humanoid_amd import dist as hd, learner as L
    from humanoid_amd.env import EnvConfig, PHCPufferEnv
    own_group = False
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(_free_port())
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", device_index))
        own_group = True
    backend = dist.get_backend()
    rank = dist.get_rank()
    cfg = L.TrainConfig()
    n = args.num_envs
    a = argparse.Namespace(**vars(args))
    a.config = "imitation"
    a.fused = False
    clips = make_clips(a, model)
    pe = PHCPufferEnv(EnvConfig(num_envs=n, motion_file={f"clip{i}": c for i, c in enumerate(clips)},
                                seed=hd.rank_seed(1, rank)))
    dev = torch.device("cuda", device_index)
    torch.manual_seed(0)  # identical initial policy on every rank
    policy = L.make_policy(dev)
    opt = torch.optim.Adam(policy.parameters(), lr=cfg.learning_rate, eps=1e-5)  # core.py:89
    ex = L.make_experience(n, cfg, dev)
    env_id = np.arange(n)
    calls = [0]
    # gradients live in flat 16 MB buckets whose all-reduces start during backward (dist.GradBuckets)
    buckets = hd.GradBuckets(policy.parameters(), min_world=1)

    def sync_grads(params):
        calls[0] += buckets.finish()

    obs, _ = pe.reset()
    for it in range(2):  # iteration 0 is the warm-up (allocations, RCCL communicator setup)
        ex.reset_collection()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        obs = L.collect(pe, policy, ex, obs, env_id)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        hd.synced_running_norm_update(policy.obs_norm, ex.obs)  # phc_train.py:329-332 on global moments
        timers = {}
        calls[0] = 0
        stats = L.train(policy, opt, ex, cfg, sync_grads=sync_grads, timers=timers)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    pe.close()
    # the all-reduce alone, on the 67.9 MB flat gradient (device tensors; 10 repetitions)
    flat = torch.ones(L.num_trainable(policy), device=dev)
    dist.all_reduce(flat)
    torch.cuda.synchronize()
    tr = time.perf_counter()
    for _ in range(10):
        dist.all_reduce(flat)
    torch.cuda.synchronize()
    ar_ms = (time.perf_counter() - tr) / 10 * 1e3
    ok = bool(torch.isfinite(flat).all()) and float(flat[0]) == float(dist.get_world_size()) ** 11
    out = {"workload": f"configs[3] per rank: {n} envs x {cfg.batch_size // n} steps into the device Experience "
                       f"(policy in the loop), GAE, PPO update {cfg.update_epochs} epochs x {cfg.num_minibatches} "
                       f"minibatches of {cfg.minibatch_size}, gradient all-reduce between backward and clip",
           "backend": backend, "world_size": dist.get_world_size(), "params": L.num_trainable(policy),
           "rollout_ms": round((t1 - t0) * 1e3, 2), "gae_ms": round(timers["gae_ms"], 3),
           "update_ms": round(timers["update_ms"], 2), "allreduce_wait_ms_in_update": round(timers["allreduce_ms"], 3),
           "allreduce_calls": calls[0], "grad_buckets": len(buckets.buckets),
           "allreduce_overlapped_with_backward": buckets.overlap, "allreduce_67.9MB_ms": round(ar_ms, 3), "allreduce_ok": ok,
           "iteration_ms": round((t2 - t0) * 1e3, 2),
           "train_env_steps_per_s_per_rank": round(cfg.batch_size / (t2 - t0), 1),
           "losses": {k: round(v, 6) for k, v in stats.items() if k != "minibatches"},
           "minibatches": stats["minibatches"]}
    if own_group:
        dist.destroy_process_group()
    return out


def sim_substeps(args):
    """Physics steps per gym.simulate() of the run's scheme (he_sim_params.substeps)."""
    from humanoid_amd import _abi
    return int(scheme_params(args).get("substeps", _abi.default_sim_params().substeps))


def scheme_params(args):
    """he_sim_params overrides of the --scheme and --solver-tolerance."""
    out = {}
    if getattr(args, "scheme", "default") == "r02":
        out = dict(substeps=1, bias_midpoint=0, solver_type=0, solver_iterations=8)
    elif getattr(args, "scheme", "default") == "pgs":
        out = dict(solver_type=0, solver_iterations=8)
    elif getattr(args, "scheme", "default") == "tgs_small":
        out = dict(substeps=8, solver_type=0, solver_iterations=1)
    if getattr(args, "solver_tolerance", None) is not None:
        out["solver_tolerance"] = args.solver_tolerance
    return out


def scheme_leg(args, model, device_index, scheme="r02", steps=50, warmup=10):
    """The bench workload under another physics scheme (--scheme), timed the same way: the default
    TGS step against the engine's PGS step, round 2's scheme (2 x 1/60 s, explicit bias, 8 sweeps) and
    TGS's small-step form."""
    import torch
    a = argparse.Namespace(**vars(args))
    a.scheme = scheme
    ro = Rollout(a, model, device_index, 0)
    for _ in range(warmup):
        ro.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ro.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": round(a.num_envs * steps / dt, 1), "unit": "env-steps/s", "steps": steps,
            "workload": f"the bench workload under --scheme {scheme}: " + str(scheme_params(a))}


def cpu_model_name():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_cores():
    """The CPU cores this process may use: its affinity mask (os.sched_getaffinity) capped by the
    cgroup CPU quota (cpu.max, cgroup v2), which is how a shared GPU host grants its share; the
    CPU baseline runs one OpenMP thread per granted core."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
        except (OSError, ValueError):
            pass
    return {"affinity": aff, "cgroup_quota": quota, "granted": min(aff, quota) if quota else aff}


def cpu_baseline(args, model):
    """Oracle (C, OpenMP) full env step on a bounded sample: `cpu_envs` envs x `cpu_steps` steps."""
    from humanoid_amd import _abi
    from humanoid_amd.model import pd_action_offset_scale
    from humanoid_amd.body_sets import frozen_dof_mask
    from oracle import oracle as O
    a = argparse.Namespace(**vars(args))
    a.num_envs = args.cpu_envs
    tables, actions, rng = build_workload(a, model, 0)
    n = a.num_envs
    hm = _abi.make_model(model)
    sim = _abi.default_sim_params(max_contacts=args.max_contacts, terrain=1 if args.config == "dr" else 0,
                                  **scheme_params(args))
    mt = O.MotionTables.from_tables(tables)
    p = _abi.imitation_params()
    off, sc = pd_action_offset_scale(model)
    frozen = np.array(frozen_dof_mask(), bool)
    tgt = (off + sc * np.clip(actions, -1, 1)).astype(np.float32)
    tgt[:, frozen] = 0
    st = dict(start_times=np.zeros(n, np.float32), start_offsets=np.zeros(n, np.float32),
              global_offset=np.zeros((n, 3), np.float32), progress=np.zeros(n, np.int16),
              root_states=np.zeros((n, 13), np.float32), dof_state=np.zeros((n, 69, 2), np.float32),
              dof_targets=np.zeros((n, 69), np.float32), rb_state=np.zeros((n, 24, 13), np.float32),
              contact_forces=np.zeros((n, 24, 3), np.float32), obs=np.zeros((n, 934), np.float32),
              reset=np.zeros(n, np.uint8), terminate=np.zeros(n, np.uint8))
    O.reset_envs(p, mt, np.arange(n), rng.uniform(0, 1, n).astype(np.float32), np.arange(n), st)
    ms = fr = tk = None
    if args.config == "dr":
        ms = rng.uniform(0.8, 1.2, (n, 24)).astype(np.float32)
        fr = rng.uniform(0.5, 1.25, n).astype(np.float32)
        tk = (np.arange(n) % 3).astype(np.int32)
    cache = O.new_cache(n)  # the engine's warm start
    cores = host_cores()
    threads = O.set_threads(cores["granted"])
    t0 = time.perf_counter()
    for step in range(a.cpu_steps):
        out = O.physics_step(hm, sim, st["root_states"], st["dof_state"], tgt, 2, mass_scale=ms, friction=fr,
                             terrain_kind=tk, cache=cache)
        im = O.imitation_step(p, mt, out["rb_state"], st["dof_state"][..., 1], out["dof_force"], st["progress"],
                              np.arange(n), st["start_times"], st["start_offsets"], st["global_offset"])
        st["progress"][:] = im["progress"]
        st["rb_state"][:] = out["rb_state"]
        st["obs"] = im["obs"]
        ids = np.nonzero(im["reset"])[0]
        if len(ids):
            ph = np.array([O.hash_uniform(0, step, int(e)) for e in ids], np.float32)
            O.reset_envs(p, mt, ids, ph, np.arange(n), st)
    dt = time.perf_counter() - t0
    return {"value": n * a.cpu_steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model_name(), "nproc": os.cpu_count(), "host_cores": cores,
            "sample": f"{n} envs x {a.cpu_steps} policy steps of the C oracle (fp64 physics + imitation + resets), "
                      f"OpenMP over envs ({threads} threads), {dt:.1f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from humanoid_amd.model import load_default_model
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HE_BENCH_SHARED_DEVICE=1 (rehearsal only): every rank on cuda:0 with gloo collectives, to
    # exercise the multi-rank path on a one-GPU box; the real run is one rank per GPU over RCCL
    shared = os.environ.get("HE_BENCH_SHARED_DEVICE") == "1"
    if shared:
        local = 0
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            # a rank that fails mid-collective ends the job in minutes, not at the driver's limit
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=datetime.timedelta(seconds=300))
    torch.cuda.set_device(local)
    model = load_default_model()
    ro = Rollout(args, model, local, rank)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        ro.step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ro.step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    nc = ro.eng.num_contacts.cpu().numpy()
    dropped = ro.eng.dropped_contacts.cpu().numpy()
    rows = solver_rows(ro)
    # kernel durations: a pass of EV_STEPS further steps with HIP events around every launch; the
    # medians are the per-launch figures (compare the rocprofv3 averages of the same command)
    first, second, whole = kernel_pass(ro, EV_STEPS)
    step_ms = float(np.median(whole))
    phys_ms, imit_ms = float(np.median(first)), float(np.median(second))
    kernel_samples = {"steps": EV_STEPS, "statistic": "median", "first_launch_ms": {
        "median": round(phys_ms, 5), "mean": round(float(first.mean()), 5), "max": round(float(first.max()), 5)}}
    # the two kernels apart (unfused form), for the physics kernel's own roofline and the imitation
    # kernel's HBM share
    split = None
    if ro.fused:
        ro.set_fused(False)
        a1, a2, _ = kernel_pass(ro, EV_STEPS // 2)
        split = (float(np.median(a1)), float(np.median(a2)))
        ro.set_fused(True)
    # the headline's max-over-ranks time is settled before any optional leg runs a collective: a leg
    # that fails on one rank cannot then pair its collectives with this reduction
    if world > 1:
        t = torch.tensor([elapsed], device="cpu" if shared else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # configs[3]'s learner slice on every rank (RCCL; a one-rank RCCL group at N = 1)
    learner = None
    if not args.no_learner and args.num_envs == 4096:
        try:
            learner = learner_leg(args, model, local)
        except Exception as exc:  # report, never fake
            learner = {"value": None, "error": repr(exc)}
        if world > 1:  # every rank learns whether any rank's leg failed; the report says so
            try:
                ok = torch.tensor([0 if "error" in learner else 1], device="cpu" if shared else "cuda")
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if int(ok.item()) == 0 and "error" not in learner:
                    learner = {"value": None, "error": "the learner leg failed on another rank"}
            except Exception as exc:
                learner = {"value": None, "error": "rank agreement after the learner leg: " + repr(exc)}
    n = args.num_envs
    total_steps = n * args.steps * world
    value = total_steps / elapsed
    if rank == 0:
        if split is not None:  # fused: the one launch is the dominant kernel
            fused_ms = step_ms
            phys_ms, imit_ms = split
        phys_roof, imit_roof = kernel_figures(args, args.config, n, phys_ms, imit_ms, float(rows.mean()))
        traffic, mfma = phys_roof["traffic"], phys_roof["mfma_util"]
        if split is not None:  # the fused launch (physics + the imitation epilogue) is the dominant kernel
            phys_flop = PHYS_FLOP_PER_SUBSTEP * 2 * sim_substeps(args)
            f_tflops = (phys_flop + IMIT_FLOP_PER_ENV_STEP) * n / (fused_ms * 1e-3) / 1e12
            roof = {"bound": "latency", "achieved": round(f_tflops, 4), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(f_tflops / FP32_PEAK_TFLOPS, 6), "traffic": traffic,
                    "kernel": "physics_kernel, fused he_env_step (physics + imitation epilogue; canonical "
                              "physics + 0.03 MFLOP/env-step, SURVEY §8d)",
                    "avg_launch_ms": round(fused_ms, 4), "mfma_util": mfma}
        else:
            roof = phys_roof
        line = {
            "metric": "env-steps/sec (4096 SMPL humanoids per GPU)",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": DATA[args.config],
            "config": {"workload": {"standstill": "configs[1]: 4096 SMPL-neutral humanoids, PD stand-still, zero ref motion",
                                    "imitation": "configs[2]: 4096 humanoids over 128 synthetic clips, full PHC reward",
                                    "tracking": "configs[2] with the tracking action stream (SURVEY §8d 3(ii))",
                                    "dr": "configs[4]: 4096 envs, mass/friction randomisation + 3 terrains"}[args.config],
                       "num_envs_per_gpu": n, "simulate_calls": 2, "substeps_per_simulate": int(sim_substeps(args)),
                       "sim_dt": 1 / 60, "max_contacts": args.max_contacts,
                       "scheme": args.scheme, "parallelism": f"replicas{world}"},
            # the physics kernel is bound by the latency of its per-env serial chains (elimination,
            # Gauss-Seidel sweeps, triangular solves) at 2 waves / SIMD, not by HBM or the matrix
            # cores: priced against the FP32 vector / matrix peak with the canonical dense-equivalent
            # flop count; mfma_util is the measured matrix-core busy share (rocprofv3 SQ counters)
            "roofline": roof,
            "kernel_timing": kernel_samples,
            "contacts": {"slots_mean": round(float(nc.mean()), 3), "slots_max": int(nc.max()),
                         "capacity": args.max_contacts, "envs_dropping": int((dropped > 0).sum()),
                         "dropped_mean": round(float(dropped.mean()), 4)},
            "unfused_kernels": {"physics_kernel": phys_roof, "imitation_kernel": imit_roof},
        }
        if args.config == "standstill" and args.num_envs == 4096:
            line["parity_vs_oracle"] = parity_record("parity_configs1")
        if not args.no_tracking and world == 1 and args.scheme == "default":
            try:
                line["r02_scheme"] = scheme_leg(args, model, local)
            except Exception as exc:  # report, never fake
                line["r02_scheme"] = {"value": None, "error": repr(exc)}
            for sch in ("pgs", "tgs_small"):
                try:
                    line[f"{sch}_scheme"] = scheme_leg(args, model, local, scheme=sch)
                except Exception as exc:  # report, never fake
                    line[f"{sch}_scheme"] = {"value": None, "error": repr(exc)}
        if not args.no_tracking and world == 1 and args.num_envs == 4096:
            try:
                line["tracking_configs2"] = tracking_leg(args, model, local)
            except Exception as exc:  # report, never fake
                line["tracking_configs2"] = {"value": None, "error": repr(exc)}
        if not args.no_tracking and world == 1 and args.num_envs == 4096 and args.config == "standstill":
            try:
                line["dr_configs4"] = config_leg(args, model, local, "dr")
            except Exception as exc:  # report, never fake
                line["dr_configs4"] = {"value": None, "error": repr(exc)}
        if learner is not None:
            line["learner_configs3"] = learner
        if not args.no_puffer_level and world == 1:
            try:
                line["puffer_env_step"] = puffer_level(args, model)
            except Exception as exc:  # report, never fake
                line["puffer_env_step"] = {"value": None, "error": repr(exc)}
        if not args.no_cpu_baseline and world == 1:
            try:
                line["cpu_baseline"] = cpu_baseline(args, model)
            except Exception as exc:  # report, never fake
                line["cpu_baseline"] = {"value": None, "error": repr(exc)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
