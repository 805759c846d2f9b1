"""`from sspp import BSplines` — see sspp_amd/BSplines.py."""
from sspp_amd.BSplines import *  # noqa: F401,F403
from sspp_amd.BSplines import __all__  # noqa: F401
