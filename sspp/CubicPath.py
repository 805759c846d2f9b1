"""`from sspp import CubicPath` — see sspp_amd/CubicPath.py."""
from sspp_amd.CubicPath import CubicPath  # noqa: F401
