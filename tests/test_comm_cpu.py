"""Communicator selection rules that do not need a GPU."""
import torch

from tensorflow_distributed_learning_amd.parallel import xgmi
from tensorflow_distributed_learning_amd.parallel.communicator import Communicator, LocalCommunicator


def test_xgmi_env_defaults(monkeypatch):
    monkeypatch.delenv("TDL_XGMI", raising=False)
    monkeypatch.delenv("TDL_XGMI_MAX_BYTES", raising=False)
    assert xgmi.enabled_by_env()
    assert xgmi.max_bytes() == 4 << 20
    monkeypatch.setenv("TDL_XGMI", "0")
    assert not xgmi.enabled_by_env()


def test_base_communicator_has_no_fused_sgd():
    c = LocalCommunicator(torch.device("cpu"))
    g, w = torch.ones(8), torch.zeros(8)
    assert c.all_reduce_sgd(g, w, torch.tensor([0.1])) is False
    assert torch.equal(w, torch.zeros(8))
    c.prepare_all_reduce(8, 16)  # no-op
    c.check_health()
    assert isinstance(c, Communicator)
