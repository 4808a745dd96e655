"""tf.keras.applications (architectures only; weights=None, no downloads offline)."""
from __future__ import annotations


def ResNet50(*args, **kwargs):  # noqa: N802
    from ..models.resnet50 import ResNet50 as _R

    return _R(*args, **kwargs)


class resnet50:  # noqa: N801
    ResNet50 = staticmethod(ResNet50)
