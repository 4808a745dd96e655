"""``import tensorflow_datasets as tfds`` stand-in (offline; the MNIST builder of data/tfds.py).

Besides ``load`` / ``DatasetInfo`` / the progress-bar switches the reference script touches
(tf_dist_example.py:24-26), the small part of the tfds surface a training script commonly uses:
``as_numpy`` (a dataset, or a dict / tuple of datasets, as numpy iterables), ``list_builders`` and
``builder(name).info`` / ``.as_dataset(split, as_supervised)``.
"""
from __future__ import annotations

from ..data.tfds import DatasetInfo, disable_progress_bar, enable_progress_bar, load  # noqa: F401

_BUILDERS = ("mnist",)


def list_builders():
    return list(_BUILDERS)


def as_numpy(ds):
    """tfds.as_numpy: a Dataset -> an iterable of numpy structures; dicts / tuples / lists of datasets
    map element-wise; a tensor (or a structure of tensors) -> numpy arrays."""
    import torch

    from ..data.dataset import Dataset

    if isinstance(ds, Dataset):
        return ds.as_numpy_iterator()
    if isinstance(ds, dict):
        return {k: as_numpy(v) for k, v in ds.items()}
    if isinstance(ds, (tuple, list)):
        return type(ds)(as_numpy(v) for v in ds)
    if isinstance(ds, torch.Tensor):
        return ds.detach().cpu().numpy()
    return ds


class _Builder:
    def __init__(self, name: str, data_dir=None):
        if name not in _BUILDERS:
            raise ValueError(f"tfds (offline): unknown dataset {name!r}; available: {list(_BUILDERS)}")
        self.name, self.data_dir = name, data_dir
        self._info = None

    @property
    def info(self) -> DatasetInfo:
        if self._info is None:
            self._info = load(self.name, with_info=True, data_dir=self.data_dir)[1]
        return self._info

    def download_and_prepare(self, *args, **kwargs):  # nothing to download offline
        return None

    def as_dataset(self, split=None, as_supervised: bool = False, **kwargs):
        return load(self.name, split=split, as_supervised=as_supervised, data_dir=self.data_dir)


def builder(name: str, data_dir=None) -> _Builder:
    return _Builder(name, data_dir)
