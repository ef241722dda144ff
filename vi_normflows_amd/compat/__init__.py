"""Reference-compatible facade (``normflows.*`` names); see :mod:`.reference_api`."""
from .reference_api import *  # noqa: F401,F403
