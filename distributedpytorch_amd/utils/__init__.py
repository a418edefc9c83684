from .seed import set_seed
from .checkpoint import save_model, load_model_state, save_training_state, load_training_state, strip_prefix
from .metrics import MetricsLogger, LossCurves, Throughput

__all__ = [
    "set_seed", "save_model", "load_model_state", "save_training_state", "load_training_state",
    "strip_prefix", "MetricsLogger", "LossCurves", "Throughput",
]
