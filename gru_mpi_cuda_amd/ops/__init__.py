"""Native extension loader and kernel wrappers."""
from ._ext import load_ext, ft_layout, ext_available, check_fresh, StaleExtensionError  # noqa: F401
