"""Import-compatible `gaussian_hierarchy`.

scene/gaussian_model.py:24 imports `gaussian_hierarchy._C.load_hierarchy, write_hierarchy`; the
model module does not import without it.  The hierarchy path is not built.
"""
from . import _C  # noqa: F401
