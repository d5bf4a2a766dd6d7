"""``isaacgym.gymapi`` facade over the HIP engine: the subset of the Isaac Gym Python
API that puffer-phc calls (``envs/isaacgym_env.py:6-99``, ``envs/humanoid_phc.py:74, 127-134,
185-383, 497-554, 747-789``), with the same names, argument meaning and tensor semantics, so that
the env changes only its imports::

    from humanoid_amd.isaacgym import gymapi, gymtorch

Semantics kept: one sim per process, envs created one by one with one actor each, dof/shape
properties set per actor, ``prepare_sim`` before tensors are acquired, engine-owned state
tensors aliased by torch views (``gymtorch.wrap_tensor``), indexed writes by int32 actor ids,
``simulate`` advancing one substep, ``fetch_results`` completing them.

Engine-specific behaviour (documented, not silent):
* consecutive ``simulate`` calls are fused into one kernel launch of N substeps, issued at the
  next ``fetch_results`` / tensor write / refresh -- the results are identical to N launches;
* all envs share one articulation, PD gains and filter table (what puffer-phc does): a
  ``set_actor_dof_properties`` / ``set_actor_rigid_shape_properties`` that differs between envs
  raises ``NotImplementedError``;
* no viewer (headless only), CPU pipeline refused (the engine is GPU-only).
"""
from __future__ import annotations

import copy
import os
from typing import List

import numpy as np

from .. import _abi
from ..model import DEFAULT_MODEL_JSON, HumanoidModel, parse_mjcf

# ----------------------------------------------------------------------------------- constants
SIM_PHYSX = 1
SIM_FLEX = 2
UP_AXIS_Y = 0
UP_AXIS_Z = 1
DOF_MODE_NONE = 0
DOF_MODE_POS = 1
DOF_MODE_VEL = 2
DOF_MODE_EFFORT = 3
STATE_NONE, STATE_POS, STATE_VEL, STATE_ALL = 0, 1, 2, 3

DofPropertiesDtype = np.dtype([("hasLimits", "?"), ("lower", "<f4"), ("upper", "<f4"), ("driveMode", "<i4"),
                               ("velocity", "<f4"), ("effort", "<f4"), ("stiffness", "<f4"), ("damping", "<f4"),
                               ("friction", "<f4"), ("armature", "<f4")])


# ----------------------------------------------------------------------------------- value types
class Vec3:
    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)

    def __iter__(self):
        return iter((self.x, self.y, self.z))


class Quat:
    def __init__(self, x=0.0, y=0.0, z=0.0, w=1.0):
        self.x, self.y, self.z, self.w = float(x), float(y), float(z), float(w)


class Transform:
    def __init__(self, p=None, r=None):
        self.p = p if p is not None else Vec3()
        self.r = r if r is not None else Quat()


class PhysXParams:
    def __init__(self):
        self.num_threads = 4
        self.solver_type = 1
        self.num_position_iterations = 4
        self.num_velocity_iterations = 0
        self.contact_offset = 0.02
        self.rest_offset = 0.0
        self.bounce_threshold_velocity = 0.2
        self.max_depenetration_velocity = 10.0
        self.default_buffer_size_multiplier = 10.0
        self.use_gpu = True
        self.max_gpu_contact_pairs = 8 * 1024 * 1024
        self.num_subscenes = 0


class SimParams:
    def __init__(self):
        self.dt = 1.0 / 60.0
        self.substeps = 2  # Isaac Gym's default; the reference leaves it (isaacgym_env.py:6-35)
        self.up_axis = UP_AXIS_Z
        self.gravity = Vec3(0.0, 0.0, -9.81)
        self.use_gpu_pipeline = True
        self.num_client_threads = 0
        self.physx = PhysXParams()


class AssetOptions:
    def __init__(self):
        self.angular_damping = 0.0
        self.linear_damping = 0.0
        self.max_angular_velocity = 64.0
        self.default_dof_drive_mode = DOF_MODE_NONE
        self.fix_base_link = False


class PlaneParams:
    def __init__(self):
        self.normal = Vec3(0.0, 0.0, 1.0)
        self.distance = 0.0
        self.static_friction = 1.0
        self.dynamic_friction = 1.0
        self.restitution = 0.0


class CameraProperties:
    pass


class RigidBodyProperties:
    def __init__(self, mass, com, inertia):
        self.mass = float(mass)
        self.com = Vec3(*com)
        self.inertia = inertia


class RigidShapeProperties:
    def __init__(self, filter_=0, friction=1.0):
        self.filter = int(filter_)
        self.friction = float(friction)
        self.restitution = 0.0
        self.contact_offset = 0.02
        self.rest_offset = 0.0


class GymTensor:
    """Handle returned by ``acquire_*_tensor`` and ``gymtorch.unwrap_tensor``: a device pointer
    with shape/dtype (``GymTensor.h:20-28``: dtype 1 = f32, 2 = int32, ...)."""

    def __init__(self, data_ptr, shape, dtype, device, owner=None):
        self.data_ptr = int(data_ptr)
        self.shape = tuple(shape)
        self.dtype = dtype
        self.device = int(device)
        self.own_data = False
        self._owner = owner


# ----------------------------------------------------------------------------------- handles
class Asset:
    def __init__(self, model: HumanoidModel, options: AssetOptions):
        self.model = model
        self.options = options
        self.force_sensors = []


class _Env:
    def __init__(self, index):
        self.index = index
        self.actor = None


class Sim:
    def __init__(self, device, params: SimParams):
        self.device = device
        self.params = params
        self.envs: List[_Env] = []
        self.asset: Asset | None = None
        self.plane: PlaneParams | None = None
        self.dof_props = None
        self.shape_filters = None
        self.self_collision = None
        self.start_poses = []
        self.engine = None
        self.pending_substeps = 0


# ----------------------------------------------------------------------------------- the Gym object
class Gym:
    # -- sim ----------------------------------------------------------------------------------
    def create_sim(self, compute_device, graphics_device, physics_engine, params: SimParams):
        if compute_device < 0 or not params.use_gpu_pipeline:
            raise NotImplementedError("the HIP engine has no CPU pipeline (use device_type='cuda')")
        if physics_engine != SIM_PHYSX:
            raise NotImplementedError("only the rigid-body (SIM_PHYSX-equivalent) pipeline exists")
        if graphics_device >= 0:
            raise NotImplementedError("headless only: the engine has no viewer")
        return Sim(int(compute_device), copy.deepcopy(params))

    def destroy_sim(self, sim: Sim):
        sim.engine = None

    def add_ground(self, sim: Sim, plane: PlaneParams):
        sim.plane = copy.deepcopy(plane)

    # -- assets ---------------------------------------------------------------------------------
    def load_asset(self, sim: Sim, root: str, filename: str, options: AssetOptions = None) -> Asset:
        path = filename if os.path.isabs(filename) else os.path.join(root, filename)
        if path.endswith(".json"):
            with open(path) as f:
                model = HumanoidModel.from_json(f.read())
        elif os.path.basename(path) == "smpl_humanoid.xml" and not os.path.exists(path):
            raise FileNotFoundError(f"{path} (the baked model is at {DEFAULT_MODEL_JSON})")
        else:
            model = parse_mjcf(path)
        a = Asset(model, copy.deepcopy(options) if options is not None else AssetOptions())
        sim.asset = a
        return a

    def get_asset_rigid_body_count(self, asset: Asset) -> int:
        return asset.model.num_bodies

    def get_asset_dof_count(self, asset: Asset) -> int:
        return 3 * (asset.model.num_bodies - 1)  # one 3-dof ball joint per non-root body

    def find_asset_rigid_body_index(self, asset: Asset, name: str) -> int:
        try:
            return asset.model.body_names.index(name)
        except ValueError:
            return -1

    def create_asset_force_sensor(self, asset: Asset, body_idx: int, pose: Transform):
        asset.force_sensors.append((body_idx, pose))  # puffer-phc creates none
        return len(asset.force_sensors) - 1

    def get_asset_dof_properties(self, asset: Asset):
        m = asset.model
        p = np.zeros(3 * (m.num_bodies - 1), DofPropertiesDtype)
        p["hasLimits"] = True
        p["lower"], p["upper"] = m.dof_lower, m.dof_upper
        p["driveMode"] = asset.options.default_dof_drive_mode
        p["velocity"] = asset.options.max_angular_velocity
        p["effort"], p["stiffness"], p["damping"], p["armature"] = m.effort, m.stiffness, m.damping, m.armature
        return p

    # -- envs / actors ----------------------------------------------------------------------------
    def create_env(self, sim: Sim, lower: Vec3, upper: Vec3, num_per_row: int):
        e = _Env(len(sim.envs))
        e.sim = sim
        sim.envs.append(e)
        return e

    def begin_aggregate(self, env, max_bodies, max_shapes, self_collisions):
        return True

    def end_aggregate(self, env):
        return True

    def create_actor(self, env: _Env, asset: Asset, pose: Transform, name: str, group: int, filter_: int,
                     segmentation_id: int = 0):
        if env.actor is not None:
            raise NotImplementedError("one actor per env (the humanoid)")
        sim = env.sim
        if group != env.index:
            raise NotImplementedError("envs are independent collision groups (col_group = env_id)")
        sc = 0 if filter_ else 1  # filter 1 = self-collision off (humanoid_phc.py:337)
        if sim.self_collision is None:
            sim.self_collision = sc
        elif sim.self_collision != sc:
            raise NotImplementedError("self-collision must be the same for every env")
        env.actor = name
        sim.start_poses.append(((pose.p.x, pose.p.y, pose.p.z), (pose.r.x, pose.r.y, pose.r.z, pose.r.w)))
        return 0

    def enable_actor_dof_force_sensors(self, env, actor):
        return True  # dof forces are always produced

    def get_actor_rigid_body_properties(self, env: _Env, actor):
        m = env.sim.asset.model
        return [RigidBodyProperties(m.mass[b], m.com[b], m.inertia[b]) for b in range(m.num_bodies)]

    def set_actor_dof_properties(self, env: _Env, actor, props):
        sim = env.sim
        if sim.dof_props is None:
            sim.dof_props = np.array(props, copy=True)
        elif not all(np.array_equal(sim.dof_props[k], props[k]) for k in ("stiffness", "damping", "effort", "armature")):
            raise NotImplementedError("per-env PD gains differ: the engine shares one articulation")
        if not np.all(np.asarray(props["driveMode"]) == DOF_MODE_POS):
            raise NotImplementedError("only DOF_MODE_POS drives (control_mode isaac_pd)")
        return True

    def get_actor_rigid_shape_properties(self, env: _Env, actor):
        m = env.sim.asset.model
        fr = env.sim.plane.static_friction if env.sim.plane else 1.0
        return [RigidShapeProperties(int(m.filter_ints[b]), fr) for b in range(m.num_bodies)]

    def set_actor_rigid_shape_properties(self, env: _Env, actor, props):
        sim = env.sim
        f = np.array([p.filter for p in props], np.int32)
        if sim.shape_filters is None:
            sim.shape_filters = f
        elif not np.array_equal(sim.shape_filters, f):
            raise NotImplementedError("per-env filter tables differ")
        return True

    # -- prepare: build the engine ------------------------------------------------------------------
    def prepare_sim(self, sim: Sim):
        from ..engine import Engine
        if sim.asset is None or not sim.envs:
            raise RuntimeError("prepare_sim before load_asset/create_actor")
        m = copy.deepcopy(sim.asset.model)
        if sim.dof_props is not None:
            m.stiffness = np.asarray(sim.dof_props["stiffness"], np.float64)
            m.damping = np.asarray(sim.dof_props["damping"], np.float64)
            m.armature = np.asarray(sim.dof_props["armature"], np.float64)
            m.effort = np.asarray(sim.dof_props["effort"], np.float64)
        if sim.shape_filters is not None:
            m.filter_ints = sim.shape_filters
        sp, px, o = sim.params, sim.params.physx, sim.asset.options
        plane = sim.plane or PlaneParams()
        # physx.solver_type 1 (TGS, isaacgym_env.py:16) with num_position_iterations per physics step;
        # solver_type 0 maps onto the engine's velocity-level PGS step, num_position_iterations sweeps
        # (8 is the engine's tested count)
        if px.solver_type not in (0, 1):
            raise NotImplementedError(f"physx.solver_type {px.solver_type}: 0 (PGS) or 1 (TGS)")
        if px.solver_type == 1 and px.num_velocity_iterations != 0:
            raise NotImplementedError("TGS velocity iterations: the reference runs 0 (isaacgym_env.py:18)")
        if not 1 <= px.num_position_iterations <= 16:
            raise NotImplementedError("num_position_iterations must be in [1, 16]")
        solver = dict(solver_type=int(px.solver_type), solver_iterations=int(px.num_position_iterations))
        params = _abi.default_sim_params(
            dt=sp.dt, contact_offset=px.contact_offset, max_depenetration_velocity=px.max_depenetration_velocity,
            angular_damping=o.angular_damping, max_angular_velocity=o.max_angular_velocity,
            friction=plane.static_friction, self_collision=int(bool(sim.self_collision)), substeps=int(sp.substeps),
            **solver)
        params.gravity[:] = (sp.gravity.x, sp.gravity.y, sp.gravity.z)
        n = len(sim.envs)
        xy = np.array([p[0][:2] for p in sim.start_poses], np.float32)
        sim.engine = Engine(m, n, device=sim.device, sim_params=params, start_xy=xy)
        self._model = m
        poses = np.array([list(p[0]) + list(p[1]) for p in sim.start_poses], np.float32)
        if not (np.allclose(poses[:, 2], 0.89) and np.allclose(poses[:, 3:7], [0, 0, 0, 1])):
            import torch
            rs = torch.zeros(n, 13, device=sim.engine.device)
            rs[:, :7] = torch.from_numpy(poses).to(rs.device)
            sim.engine.set_root_state_indexed(rs, torch.arange(n, dtype=torch.int32, device=rs.device))
            # _initial_humanoid_root_states (humanoid_phc.py:522-523) is the root state tensor read
            # right after prepare_sim with the velocities zeroed: the creation poses, which the
            # Default / Hybrid state init resets to (he_create_envs set it for the z=0.89 pose only)
            sim.engine.initial_root_states.copy_(rs)
        return True

    # -- tensors ----------------------------------------------------------------------------------
    def _acquire(self, sim: Sim, kind: int):
        if sim.engine is None:
            raise RuntimeError("acquire_*_tensor before prepare_sim")
        t = sim.engine.buffer(kind)
        return GymTensor(t.data_ptr(), t.shape, 1, sim.device, owner=t)

    def acquire_actor_root_state_tensor(self, sim):
        return self._acquire(sim, _abi.BUF_ROOT_STATE)

    def acquire_dof_state_tensor(self, sim):
        return self._acquire(sim, _abi.BUF_DOF_STATE)

    def acquire_rigid_body_state_tensor(self, sim):
        return self._acquire(sim, _abi.BUF_RB_STATE)

    def acquire_net_contact_force_tensor(self, sim):
        return self._acquire(sim, _abi.BUF_CONTACT_FORCE)

    def acquire_dof_force_tensor(self, sim):
        return self._acquire(sim, _abi.BUF_DOF_FORCE)

    def acquire_force_sensor_tensor(self, sim):
        raise NotImplementedError("force sensors are not used by puffer-phc")

    def _flush(self, sim: Sim):
        if sim.pending_substeps:
            k, sim.pending_substeps = sim.pending_substeps, 0
            sim.engine.simulate(k)

    def refresh_dof_state_tensor(self, sim):
        self._flush(sim)

    refresh_actor_root_state_tensor = refresh_dof_state_tensor
    refresh_rigid_body_state_tensor = refresh_dof_state_tensor
    refresh_force_sensor_tensor = refresh_dof_state_tensor
    refresh_dof_force_tensor = refresh_dof_state_tensor
    refresh_net_contact_force_tensor = refresh_dof_state_tensor

    @staticmethod
    def _tensor(desc):
        from . import gymtorch
        return gymtorch.wrap_tensor(desc)

    def set_dof_position_target_tensor(self, sim: Sim, desc):
        self._flush(sim)
        sim.engine.set_dof_targets(self._tensor(desc))
        return True

    def set_actor_root_state_tensor_indexed(self, sim: Sim, desc, ids_desc, n: int):
        self._flush(sim)
        sim.engine.set_root_state_indexed(self._tensor(desc), self._tensor(ids_desc)[:n])
        return True

    def set_dof_state_tensor_indexed(self, sim: Sim, desc, ids_desc, n: int):
        self._flush(sim)
        sim.engine.set_dof_state_indexed(self._tensor(desc), self._tensor(ids_desc)[:n])
        return True

    def set_dof_position_target_tensor_indexed(self, sim: Sim, desc, ids_desc, n: int):
        self._flush(sim)
        sim.engine.set_dof_targets_indexed(self._tensor(desc), self._tensor(ids_desc)[:n])
        return True

    # -- stepping -----------------------------------------------------------------------------------
    def simulate(self, sim: Sim):
        sim.pending_substeps += 1

    def fetch_results(self, sim: Sim, wait: bool = True):
        self._flush(sim)
        return True

    # -- viewer (absent) -----------------------------------------------------------------------------
    def create_viewer(self, sim, props):
        raise NotImplementedError("headless only: the engine has no viewer")


_GYM = None


def acquire_gym() -> Gym:
    global _GYM
    if _GYM is None:
        _GYM = Gym()
    return _GYM
