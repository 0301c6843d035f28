"""Source-compatibility alias: ``import pccl`` works exactly like ``import pccl_amd``."""
from pccl_amd import *  # noqa: F401,F403
from pccl_amd import __all__, __version__, cuda, hip  # noqa: F401
