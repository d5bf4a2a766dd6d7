"""Body-index sets of the SMPL humanoid used by the engine's kernels.

Same names and order as ``puffer_phc/body_sets.py:11-79`` (BODY_NAMES, DOF_NAMES, REMOVE_NAMES,
KEY_BODIES, CONTACT_BODIES, TRACK_BODIES, RESET_BODIES, EVAL_BODIES, LIMB_WEIGHT_GROUP); the
kernels take the index lists built here.
"""
from typing import List, Sequence, Tuple

BODY_NAMES: Tuple[str, ...] = (
    "Pelvis",
    "L_Hip", "L_Knee", "L_Ankle", "L_Toe",
    "R_Hip", "R_Knee", "R_Ankle", "R_Toe",
    "Torso", "Spine", "Chest", "Neck", "Head",
    "L_Thorax", "L_Shoulder", "L_Elbow", "L_Wrist", "L_Hand",
    "R_Thorax", "R_Shoulder", "R_Elbow", "R_Wrist", "R_Hand",
)
DOF_NAMES = BODY_NAMES[1:]
REMOVE_NAMES = ("L_Hand", "R_Hand", "L_Toe", "R_Toe")
KEY_BODIES = ("R_Ankle", "L_Ankle", "R_Wrist", "L_Wrist")
CONTACT_BODIES = ("R_Ankle", "L_Ankle", "R_Toe", "L_Toe")
TRACK_BODIES = BODY_NAMES
RESET_BODIES = TRACK_BODIES
EVAL_BODIES = tuple(n for n in BODY_NAMES if n not in REMOVE_NAMES)
JOINT_GROUPS = [
    ["L_Hip", "L_Knee", "L_Ankle", "L_Toe"],
    ["R_Hip", "R_Knee", "R_Ankle", "R_Toe"],
    ["Pelvis", "Torso", "Spine", "Chest", "Neck", "Head"],
    ["L_Thorax", "L_Shoulder", "L_Elbow", "L_Wrist", "L_Hand"],
    ["R_Thorax", "R_Shoulder", "R_Elbow", "R_Wrist", "R_Hand"],
]
LIMB_WEIGHT_GROUP = [[BODY_NAMES.index(n) for n in g] for g in JOINT_GROUPS]


def body_ids(names: Sequence[str], targets: Sequence[str] = None) -> List[int]:
    if targets is None:
        names, targets = BODY_NAMES, names
    return [list(names).index(t) for t in targets]


def frozen_dof_mask(num_dof: int = 69, freeze_hand=True, freeze_toe=True) -> List[int]:
    """1 for the dofs whose PD target is forced to 0 (``humanoid_phc.py:116-125``)."""
    mask = [0] * num_dof
    if freeze_hand:
        for n in ("L_Hand", "R_Hand"):
            i = DOF_NAMES.index(n) * 3
            mask[i:i + 3] = [1, 1, 1]
    if freeze_toe:
        for n in ("L_Toe", "R_Toe"):
            i = DOF_NAMES.index(n) * 3
            mask[i:i + 3] = [1, 1, 1]
    return mask
