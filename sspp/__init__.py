"""Drop-in import surface of the reference package `sspp` (pyproject.toml:18-20).

    from sspp import _sspp               # SamplingPathPlanner{3,6,7,9}, Spline{3,6,7,9}
    from sspp import BSplines, CubicPath  # operator API

`_sspp` is the pybind11 extension built in-tree from sspp_amd/csrc/sspp_pybind.cpp; it links
sspp_amd/lib/libsspp_hip.so (the HIP kernels).  Importing it fails if it was not built.
"""
