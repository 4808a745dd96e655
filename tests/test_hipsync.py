"""TDL_HIP_SCHEDULE parsing (utils/hipsync.py): unknown or unset modes are no-ops; without a GPU
the supported modes report False and change nothing."""
import pytest

from tensorflow_distributed_learning_amd.utils import hipsync


def test_unset_and_unknown_modes_are_noops(monkeypatch):
    monkeypatch.delenv("TDL_HIP_SCHEDULE", raising=False)
    before = hipsync.applied
    assert hipsync.configure("") is False
    assert hipsync.configure("busy") is False
    assert hipsync.applied == before


@pytest.mark.parametrize("mode", ["spin", "yield", "auto", "SPIN"])
def test_known_modes_without_gpu(mode):
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    assert hipsync.configure(mode) is False
