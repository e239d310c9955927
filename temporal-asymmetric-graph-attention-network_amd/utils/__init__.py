"""Utilities of the TAGAN hot path (mirror of src/tagan/utils/__init__.py)."""
from .memory_bank import NodeMemoryBank  # noqa: F401
from .config import TAGANConfig  # noqa: F401
