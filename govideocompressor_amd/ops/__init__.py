"""Native operators: loaders (``native``) and torch-facing kernel wrappers (``kernels``)."""
from .native import gpu_available, hip, host  # noqa: F401
