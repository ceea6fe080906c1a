"""``atorch.auto.engine`` compat path (implementation: ``atorch/engine/``)."""

from ...engine import *  # noqa: F401,F403
