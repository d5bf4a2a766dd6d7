"""Articulated-humanoid model constants.

Parses an MJCF humanoid (the SMPL-neutral ``smpl_humanoid.xml`` that the reference loads
through ``gym.load_asset`` at ``puffer_phc/envs/humanoid_phc.py:205-216`` and through
``SkeletonTree.from_mjcf`` at ``puffer_phc/poselib_skeleton.py:275-320``) into flat numpy
tables that the engine bakes into its device model blob.

What the reference gets from Isaac Gym's MJCF importer and what this module restates:

* kinematic tree: body order = depth-first MJCF order, ``parents`` and ``local_pos`` exactly as
  ``SkeletonTree.from_mjcf`` (``poselib_skeleton.py:298-312``);
* three hinge joints per non-root body become one 3-dof ball joint whose coordinates are an
  exponential map (``motion_lib.py:670-673``, ``humanoid_phc.py:919``); the hinge ``stiffness`` /
  ``damping`` become position-drive gains (``humanoid_phc.py:276-280``), ``armature`` is added to
  the joint-space inertia, ``range`` (deg) becomes dof limits (``humanoid_phc.py:305-323``);
* motor ``gear`` x ``ctrlrange`` becomes the drive effort limit (``dof_prop["effort"]``,
  ``humanoid_phc.py:324``) -- an engine decision, Isaac's importer is not available here;
* geom mass/inertia from ``density`` (MuJoCo conventions for sphere / capsule / box);
* the self-collision filter bitmask table of ``humanoid_phc.py:370-381`` (non-mesh row) plus the
  articulation's implicit parent/child exclusion gives the self-collision pair table.
"""
from __future__ import annotations

import json
import math
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import List

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")
DEFAULT_MODEL_JSON = os.path.join(ASSET_DIR, "smpl_humanoid_model.json")

GEOM_SPHERE, GEOM_CAPSULE, GEOM_BOX = 0, 1, 2

# humanoid_phc.py:374 -- shape filter bitmasks, non-mesh SMPL humanoid (one shape per body).
SMPL_FILTER_INTS = (0, 0, 7, 16, 12, 0, 56, 2, 33, 128, 0, 192, 0, 64, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)


@dataclass
class HumanoidModel:
    body_names: List[str]
    parents: np.ndarray          # int32 [B]
    local_pos: np.ndarray        # f64 [B,3]  joint offset in parent frame
    geom_type: np.ndarray        # int32 [B]
    geom_params: np.ndarray      # f64 [B,10]: sphere (cx,cy,cz,r) | capsule (ax,ay,az,bx,by,bz,r) | box (cx,cy,cz,ex,ey,ez,qx,qy,qz,qw)
    geom_radius: np.ndarray      # f64 [B] bounding/cast radius (sphere r, capsule r, box proxy r)
    mass: np.ndarray             # f64 [B]
    com: np.ndarray              # f64 [B,3] body frame
    inertia: np.ndarray          # f64 [B,3,3] about COM, body frame
    dof_names: List[str]
    stiffness: np.ndarray        # f64 [D]
    damping: np.ndarray          # f64 [D]
    armature: np.ndarray         # f64 [D]
    dof_lower: np.ndarray        # f64 [D] rad
    dof_upper: np.ndarray        # f64 [D] rad
    effort: np.ndarray           # f64 [D]
    filter_ints: np.ndarray      # int32 [B]
    extra: dict = field(default_factory=dict)

    # ------------------------------------------------------------------ derived tables
    @property
    def num_bodies(self) -> int:
        return len(self.body_names)

    @property
    def num_dof(self) -> int:
        return len(self.dof_names)

    @property
    def depth(self) -> np.ndarray:
        d = np.zeros(self.num_bodies, np.int32)
        for b in range(1, self.num_bodies):
            d[b] = d[self.parents[b]] + 1
        return d

    def ancestors(self, b: int) -> List[int]:
        """Bodies from the root down to ``b`` inclusive."""
        chain = []
        while b >= 0:
            chain.append(b)
            b = int(self.parents[b])
        return chain[::-1]

    def self_collision_pairs(self) -> np.ndarray:
        """[P,2] int32 body pairs that may collide: not parent/child, no shared filter bit
        (PhysX shape-filter semantics used by Isaac Gym, ``humanoid_phc.py:370-381``)."""
        pairs = []
        nb = self.num_bodies
        for i in range(nb):
            for j in range(i + 1, nb):
                if self.parents[j] == i or self.parents[i] == j:
                    continue
                if int(self.filter_ints[i]) & int(self.filter_ints[j]):
                    continue
                pairs.append((i, j))
        return np.asarray(pairs, np.int32).reshape(-1, 2)

    def total_mass(self) -> float:
        return float(self.mass.sum())

    # ------------------------------------------------------------------ serialisation
    def to_json(self) -> str:
        d = {}
        for k, v in self.__dict__.items():
            d[k] = v.tolist() if isinstance(v, np.ndarray) else v
        return json.dumps(d, indent=1)

    @classmethod
    def from_json(cls, text: str) -> "HumanoidModel":
        d = json.loads(text)
        ints = {"parents", "geom_type", "filter_ints"}
        kw = {}
        for k, v in d.items():
            if k in ("body_names", "dof_names", "extra"):
                kw[k] = v
            elif k in ints:
                kw[k] = np.asarray(v, np.int32)
            else:
                kw[k] = np.asarray(v, np.float64)
        return cls(**kw)


def load_default_model() -> HumanoidModel:
    with open(DEFAULT_MODEL_JSON) as f:
        return HumanoidModel.from_json(f.read())


# ---------------------------------------------------------------------------------------
# MJCF parsing
# ---------------------------------------------------------------------------------------

def _vec(s, n=None):
    v = np.array([float(x) for x in s.split()], np.float64)
    if n is not None and v.size != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


def _quat_wxyz_to_mat(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def _frame_from_axis(axis):
    """Rotation whose z column is ``axis`` (unit)."""
    z = axis / np.linalg.norm(axis)
    tmp = np.array([1.0, 0, 0]) if abs(z[0]) < 0.9 else np.array([0, 1.0, 0])
    x = np.cross(tmp, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=1)


def geom_mass_properties(gtype, params, density):
    """Mass, COM (body frame) and inertia about COM (body frame) of one geom (MuJoCo formulas)."""
    if gtype == GEOM_SPHERE:
        c, r = params[:3], params[3]
        m = density * 4.0 / 3.0 * math.pi * r ** 3
        return m, c.copy(), np.eye(3) * (0.4 * m * r * r)
    if gtype == GEOM_CAPSULE:
        a, b, r = params[:3], params[3:6], params[6]
        L = float(np.linalg.norm(b - a))
        mc = density * math.pi * r * r * L
        mh = density * 2.0 / 3.0 * math.pi * r ** 3  # one hemisphere
        m = mc + 2 * mh
        i_ax = mc * r * r / 2 + 2 * mh * 0.4 * r * r
        i_perp = mc * (L * L / 12 + r * r / 4) + 2 * mh * (0.4 * r * r + L * L / 4 + 3 * L * r / 8)
        R = _frame_from_axis(b - a) if L > 0 else np.eye(3)
        I = R @ np.diag([i_perp, i_perp, i_ax]) @ R.T
        return m, 0.5 * (a + b), I
    if gtype == GEOM_BOX:
        c, e, q = params[:3], params[3:6], params[6:10]
        m = density * 8.0 * e[0] * e[1] * e[2]
        Ib = m / 3.0 * np.diag([e[1] ** 2 + e[2] ** 2, e[0] ** 2 + e[2] ** 2, e[0] ** 2 + e[1] ** 2])
        R = _quat_wxyz_to_mat(np.array([q[3], q[0], q[1], q[2]]))
        return m, c.copy(), R @ Ib @ R.T
    raise ValueError(gtype)


def parse_mjcf(path: str, filter_ints=SMPL_FILTER_INTS) -> HumanoidModel:
    """Parse an MJCF humanoid with one geom per body and 0 or 3 hinge joints per body."""
    root = ET.parse(path).getroot()
    defaults_joint = {}
    dflt = root.find("default")
    if dflt is not None and dflt.find("joint") is not None:
        defaults_joint = dict(dflt.find("joint").attrib)
    wb = root.find("worldbody")
    body_root = wb.find("body")
    if body_root is None:
        raise ValueError("MJCF has no root body")

    body_names, parents, local_pos = [], [], []
    geom_type, geom_params, geom_radius, mass, com, inertia = [], [], [], [], [], []
    dof_names, stiff, damp, arm, lo, hi = [], [], [], [], [], []

    def add(node, parent):
        idx = len(body_names)
        body_names.append(node.attrib["name"])
        parents.append(parent)
        local_pos.append(_vec(node.attrib.get("pos", "0 0 0"), 3))
        geoms = node.findall("geom")
        if len(geoms) != 1:
            raise ValueError(f"body {body_names[-1]}: expected exactly one geom, found {len(geoms)}")
        g = geoms[0].attrib
        t = g.get("type", "capsule")
        density = float(g.get("density", "1000"))
        p = np.zeros(10)
        if t == "sphere":
            gt = GEOM_SPHERE
            p[:3] = _vec(g.get("pos", "0 0 0"), 3)
            p[3] = _vec(g["size"])[0]
            rad = p[3]
        elif t == "capsule":
            gt = GEOM_CAPSULE
            if "fromto" not in g:
                raise ValueError("capsule geoms must use fromto")
            ft = _vec(g["fromto"], 6)
            p[:6] = ft
            p[6] = _vec(g["size"])[0]
            rad = p[6]
        elif t == "box":
            gt = GEOM_BOX
            p[:3] = _vec(g.get("pos", "0 0 0"), 3)
            p[3:6] = _vec(g["size"], 3)
            qw = _vec(g.get("quat", "1 0 0 0"), 4)  # MJCF wxyz
            p[6:10] = [qw[1], qw[2], qw[3], qw[0]]
            rad = float(np.sort(p[3:6])[:2].mean())
        else:
            raise ValueError(f"unsupported geom type {t}")
        m, c, I = geom_mass_properties(gt, p, density)
        geom_type.append(gt)
        geom_params.append(p)
        geom_radius.append(rad)
        mass.append(m)
        com.append(c)
        inertia.append(I)
        joints = [j for j in node.findall("joint") if j.attrib.get("type", "hinge") == "hinge"]
        if parent >= 0:
            if len(joints) != 3:
                raise ValueError(f"body {body_names[-1]}: expected 3 hinge joints, found {len(joints)}")
            for j in joints:
                a = dict(defaults_joint)
                a.update(j.attrib)
                dof_names.append(a["name"])
                stiff.append(float(a.get("stiffness", 0)))
                damp.append(float(a.get("damping", 0)))
                arm.append(float(a.get("armature", 0)))
                r = _vec(a.get("range", "-180 180"), 2)
                lo.append(math.radians(r[0]))
                hi.append(math.radians(r[1]))
        for child in node.findall("body"):
            add(child, idx)

    add(body_root, -1)

    # motors: effort = gear * max|ctrlrange| (default ctrlrange from <default><motor>)
    gear = {n: 1.0 for n in dof_names}
    ctrl = 1.0
    if dflt is not None and dflt.find("motor") is not None:
        cr = dflt.find("motor").attrib.get("ctrlrange")
        if cr:
            ctrl = float(np.abs(_vec(cr)).max())
    act = root.find("actuator")
    if act is not None:
        for mtr in act.findall("motor"):
            gear[mtr.attrib["joint"]] = float(mtr.attrib.get("gear", "1")) * ctrl
    effort = [gear[n] for n in dof_names]

    nb = len(body_names)
    fi = np.asarray(filter_ints if filter_ints is not None else [0] * nb, np.int32)
    if fi.size != nb:
        raise ValueError("filter table length must equal the body count (humanoid_phc.py:377)")
    return HumanoidModel(
        body_names=body_names,
        parents=np.asarray(parents, np.int32),
        local_pos=np.asarray(local_pos),
        geom_type=np.asarray(geom_type, np.int32),
        geom_params=np.asarray(geom_params),
        geom_radius=np.asarray(geom_radius),
        mass=np.asarray(mass),
        com=np.asarray(com),
        inertia=np.asarray(inertia),
        dof_names=dof_names,
        stiffness=np.asarray(stiff),
        damping=np.asarray(damp),
        armature=np.asarray(arm),
        dof_lower=np.asarray(lo),
        dof_upper=np.asarray(hi),
        effort=np.asarray(effort),
        filter_ints=fi,
    )


def pd_action_offset_scale(model: HumanoidModel, bias_offset=False, has_smpl_pd_offset=False,
                           has_upright_start=True):
    """Restates ``humanoid_phc.py:385-456`` ``_build_pd_action_offset_scale`` (3-dof joints)."""
    lim_low = model.dof_lower.astype(np.float32).copy()
    lim_high = model.dof_upper.astype(np.float32).copy()
    # humanoid_phc.py:308-320 -- swap reversed limits; equal limits at 0 -> [-pi, pi]
    for j in range(model.num_dof):
        if lim_low[j] > lim_high[j]:
            lim_low[j], lim_high[j] = lim_high[j], lim_low[j]
        elif lim_low[j] == lim_high[j] and lim_low[j] == 0:
            lim_low[j], lim_high[j] = -np.pi, np.pi
    nj = model.num_dof // 3
    for j in range(nj):
        s = slice(3 * j, 3 * j + 3)
        if not bias_offset:
            curr_scale = max(np.max(np.abs(lim_low[s])), np.max(np.abs(lim_high[s])))
            curr_scale = min(1.2 * curr_scale, np.pi)
            lim_low[s] = -curr_scale
            lim_high[s] = curr_scale
        else:
            mid = 0.5 * (lim_high[s] + lim_low[s])
            sc = 0.7 * (lim_high[s] - lim_low[s])
            lim_low[s] = mid - sc
            lim_high[s] = mid + sc
    offset = (0.5 * (lim_high + lim_low)).astype(np.float32)
    scale = (0.5 * (lim_high - lim_low)).astype(np.float32)
    names = [n[:-2] for n in model.dof_names[::3]]
    # humanoid_phc.py:441-446 -- stronger knee
    for side in ("L_Knee", "R_Knee"):
        scale[names.index(side) * 3 + 1] = 5
    if has_smpl_pd_offset:
        if has_upright_start:
            offset[names.index("L_Shoulder") * 3] = -np.pi / 2
            offset[names.index("R_Shoulder") * 3] = np.pi / 2
        else:
            offset[names.index("L_Shoulder") * 3] = -np.pi / 6
            offset[names.index("L_Shoulder") * 3 + 2] = -np.pi / 2
            offset[names.index("R_Shoulder") * 3] = -np.pi / 3
            offset[names.index("R_Shoulder") * 3 + 2] = np.pi / 2
    return offset, scale


def limb_weights(model: HumanoidModel, groups) -> np.ndarray:
    """``humanoid_limb_and_weights`` row (``humanoid_phc.py:360-366``): limb lengths then masses."""
    lengths = np.linalg.norm(model.local_pos.astype(np.float32), axis=-1)
    ll = [lengths[g].sum() for g in groups]
    ms = [model.mass.astype(np.float32)[g].sum() for g in groups]
    return np.asarray(ll + ms, np.float32)
