"""Stub of the reference hierarchy extension (submodules/gaussianhierarchy/ext.cpp:15-20).

Every entry point raises NotImplementedError: the LOD cut and .hier I/O are SURVEY §8(f) rows
F1/F4, not built.
"""


def _not_built(name):
    def fn(*_args, **_kwargs):
        raise NotImplementedError(f"gaussian_hierarchy._C.{name}: the hierarchy path (SURVEY §8(f) F1/F4) is not built")
    fn.__name__ = name
    return fn


load_hierarchy = _not_built("load_hierarchy")
write_hierarchy = _not_built("write_hierarchy")
expand_to_target = _not_built("expand_to_target")
expand_to_size = _not_built("expand_to_size")
get_interpolation_weights = _not_built("get_interpolation_weights")
