"""Compatibility package: the reference's ``utils`` (distributed helpers + epoch loops)."""
from .distributed_utils import *  # noqa: F401,F403
from .train_eval_utils import *  # noqa: F401,F403
