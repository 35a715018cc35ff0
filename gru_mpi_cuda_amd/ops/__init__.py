"""Native extension loader and kernel wrappers."""
from ._ext import load_ext, ext_available  # noqa: F401
