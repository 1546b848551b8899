"""hidegs_amd -- MI355X-native backend of the HiDeGS rasterizer boundary.

Contents: the C-ABI library (csrc/, built to libhidegs.so by hidegs_amd.build), its
ctypes binding (_lib) and the view-data-parallel gradient exchange (view_dp).
The drop-in packages diff_gaussian_rasterization / simple_knn / gaussian_hierarchy
at the repository root sit on top of it.
"""
