from .trainer import build_trainer, TorchStepper  # noqa: F401
from .train_eval import train_one_epoch, train_one_epoch_native, evaluate, evaluate_per_image  # noqa: F401
