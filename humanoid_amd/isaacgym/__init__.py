"""Drop-in for the ``isaacgym`` modules puffer-phc imports (``gymapi``, ``gymtorch``), backed by
the MI355X engine. See ``gymapi.py`` for the covered API and the documented differences."""
from . import gymapi, gymtorch  # noqa: F401
