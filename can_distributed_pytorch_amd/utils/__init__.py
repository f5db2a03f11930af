from .checkpoint import save_checkpoint, load_checkpoint, save_train_state, load_train_state  # noqa: F401
from .flat import FlatArena  # noqa: F401
from .metrics import JsonlLogger, StepTimer  # noqa: F401
