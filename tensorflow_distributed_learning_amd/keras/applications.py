"""``tf.keras.applications`` (offline): the ResNet50 architecture (``weights=None``: nothing is
downloaded) and its ``preprocess_input`` / ``decode_predictions`` helpers.

Keras semantics reproduced here (``keras/applications/imagenet_utils.py``, 'caffe' mode used by
ResNet50): images are RGB in [0, 255], channels last; preprocessing flips them to BGR and subtracts the
ImageNet channel means, with no scaling.  ``decode_predictions`` reads the class index from a local
``imagenet_class_index.json`` when one exists (``~/.keras/models``, or ``$KERAS_HOME/models``), else
labels classes by their index -- there is no download.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Tuple

import numpy as np
import torch

# BGR channel means of the ImageNet training set (Keras 'caffe' preprocessing)
IMAGENET_BGR_MEAN = (103.939, 116.779, 123.68)


def ResNet50(*args, **kwargs):  # noqa: N802
    from ..models.resnet50 import ResNet50 as _R

    return _R(*args, **kwargs)


def preprocess_input(x, data_format: Optional[str] = None):
    """'caffe' preprocessing: RGB -> BGR, minus the ImageNet BGR means (numpy arrays are returned as
    new float32 arrays, torch tensors as new float tensors; integer inputs are widened first)."""
    channels_first = data_format == "channels_first"
    mean = IMAGENET_BGR_MEAN
    if isinstance(x, torch.Tensor):
        t = x.float() if not torch.is_floating_point(x) else x.clone()
        t = t.flip(1 if channels_first else -1)
        shape = [1] * t.dim()
        shape[1 if channels_first else -1] = 3
        return t - torch.tensor(mean, dtype=t.dtype, device=t.device).reshape(shape)
    a = np.asarray(x)
    a = a.astype(np.float32) if not np.issubdtype(a.dtype, np.floating) else a.copy()
    a = np.flip(a, axis=1 if channels_first else -1)
    shape = [1] * a.ndim
    shape[1 if channels_first else -1] = 3
    return np.ascontiguousarray(a - np.asarray(mean, dtype=a.dtype).reshape(shape))


_CLASS_INDEX: Optional[dict] = None


def _class_index() -> Optional[dict]:
    global _CLASS_INDEX
    if _CLASS_INDEX is None:
        home = os.environ.get("KERAS_HOME", os.path.join(os.path.expanduser("~"), ".keras"))
        path = os.path.join(home, "models", "imagenet_class_index.json")
        if os.path.isfile(path):
            with open(path) as f:
                _CLASS_INDEX = json.load(f)
    return _CLASS_INDEX


def decode_predictions(preds, top: int = 5) -> List[List[Tuple[str, str, float]]]:
    """Per sample, the ``top`` classes as ``(class_id, class_name, score)``, best first (Keras order);
    ``preds`` is [N][classes] (numpy or torch)."""
    p = preds.detach().float().cpu().numpy() if isinstance(preds, torch.Tensor) else np.asarray(preds, np.float32)
    if p.ndim != 2:
        raise ValueError(f"decode_predictions expects a batch of predictions (2-D), got shape {p.shape}")
    idx = _class_index()
    out = []
    for row in p:
        best = np.argsort(-row, kind="stable")[:top]
        out.append([(tuple(idx[str(int(i))])[0], tuple(idx[str(int(i))])[1], float(row[i])) if idx and str(int(i)) in idx
                    else (str(int(i)), f"class_{int(i)}", float(row[i])) for i in best])
    return out


class resnet50:  # noqa: N801
    """``tf.keras.applications.resnet50`` module namespace."""

    ResNet50 = staticmethod(ResNet50)
    preprocess_input = staticmethod(preprocess_input)
    decode_predictions = staticmethod(decode_predictions)
