"""Drop-in `simple_knn` package (reference: submodules/simple-knn, ext.cpp:15-17)."""
from . import _C  # noqa: F401
