"""tagan_amd — MI355X-native (gfx950) hot path of TAGAN.

Drop-in for the reference package ``src.tagan`` on the geometric + temporal
attention path: same classes, constructor arguments, ``state_dict`` keys and
forward signatures; compute runs in hand-written HIP kernels behind the C-ABI
of ``libtagan_hip.so`` (include/tagan_hip.h).  Import as ``tagan_amd`` (the
repository-root shim ``tagan_amd.py`` maps the hyphenated directory name).
"""
from .model import TAGAN  # noqa: F401
from .utils.config import TAGANConfig  # noqa: F401
from .utils.memory_bank import NodeMemoryBank  # noqa: F401
from . import layers, kernels  # noqa: F401

__version__ = "0.1.0"
