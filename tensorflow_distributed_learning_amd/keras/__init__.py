"""Keras-style API (tf.keras equivalent) on the MI355X engine."""
from . import activations, backend, callbacks, datasets, initializers, layers, losses, metrics  # noqa: F401
from . import mixed_precision, optimizers, regularizers, schedules, utils  # noqa: F401
from . import applications  # noqa: F401
from .layers import Input, Layer  # noqa: F401
from .models import Model, Sequential, load_model, model_from_config, clone_model  # noqa: F401


class models:  # noqa: N801 - tf.keras.models namespace
    Model = Model
    Sequential = Sequential
    load_model = staticmethod(load_model)
    model_from_config = staticmethod(model_from_config)
    clone_model = staticmethod(clone_model)
