"""``import tensorflow_datasets as tfds`` stand-in (offline; see data/tfds.py)."""
from ..data.tfds import DatasetInfo, disable_progress_bar, enable_progress_bar, load  # noqa: F401
