"""Training: loss, device engine (HIP graphs), ``train_model`` + callbacks."""
from .engine import MetricAccumulator, Trainer, flatten_predictions, predict
from .fit import (Callback, EarlyStopping, History, JSONLLogger, LearningRateScheduler, MCCCustom, ModelCheckpoint,
                  train_model)
from .loss import calculate_weights, weighted_bce_with_logits

__all__ = ["Trainer", "MetricAccumulator", "predict", "flatten_predictions", "train_model", "calculate_weights",
           "weighted_bce_with_logits", "History", "Callback", "EarlyStopping", "ModelCheckpoint",
           "LearningRateScheduler", "JSONLLogger", "MCCCustom"]
