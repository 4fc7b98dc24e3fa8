"""Kernel bindings (ctypes foreign calls for the hot paths) and their
torch.ops.foremast.* operator registrations (``library``)."""
from . import library  # noqa: F401  (registers torch.ops.foremast.*)
