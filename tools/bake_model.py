"""Bake the SMPL-neutral humanoid MJCF into ``humanoid_amd/assets/smpl_humanoid_model.json``.

Run in the build container (where the reference asset exists):
    python tools/bake_model.py /root/reference/packages/puffer-phc/puffer_phc/assets/smpl_humanoid.xml
The JSON holds only derived numeric constants (tree, offsets, geoms, mass properties, drive gains);
the GPU box never reads the reference tree.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from humanoid_amd.model import DEFAULT_MODEL_JSON, parse_mjcf  # noqa: E402

DEFAULT_XML = "/root/reference/packages/puffer-phc/puffer_phc/assets/smpl_humanoid.xml"


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_XML
    m = parse_mjcf(path)
    m.extra["source"] = "puffer_phc/assets/smpl_humanoid.xml (parsed by humanoid_amd.model.parse_mjcf)"
    with open(DEFAULT_MODEL_JSON, "w") as f:
        f.write(m.to_json())
    print(f"bodies={m.num_bodies} dofs={m.num_dof} mass={m.total_mass():.3f}kg "
          f"self-collision pairs={len(m.self_collision_pairs())} -> {DEFAULT_MODEL_JSON}")


if __name__ == "__main__":
    main()
