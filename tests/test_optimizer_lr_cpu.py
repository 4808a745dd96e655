"""The device learning rate follows schedule steps and assignments, and a constant rate is written
once (no fill launch in front of every graph replay)."""
import torch

from tensorflow_distributed_learning_amd.keras import optimizers, schedules


def _fills(opt, monkeypatch):
    n = [0]
    real = torch.Tensor.fill_

    def counting(self, v):
        if self is opt.lr_dev:
            n[0] += 1
        return real(self, v)

    monkeypatch.setattr(torch.Tensor, "fill_", counting)
    return n


def test_constant_lr_is_written_once(monkeypatch):
    opt = optimizers.SGD(learning_rate=0.05)
    opt.build(8, torch.device("cpu"))
    n = _fills(opt, monkeypatch)
    for _ in range(5):
        opt._sync_lr()
    assert n[0] == 0 and abs(float(opt.lr_dev) - 0.05) < 1e-8
    opt.learning_rate = 0.01
    opt._sync_lr()
    opt._sync_lr()
    assert n[0] == 1 and abs(float(opt.lr_dev) - 0.01) < 1e-9


def test_schedule_updates_device_lr():
    sch = schedules.PiecewiseConstantDecay([2, 4], [0.1, 0.01, 0.001])
    opt = optimizers.SGD(learning_rate=sch)
    opt.build(8, torch.device("cpu"))
    seen = []
    for it in range(6):
        opt.iterations = it
        opt._sync_lr()
        seen.append(round(float(opt.lr_dev), 6))
    assert seen == [0.1, 0.1, 0.1, 0.01, 0.01, 0.001]


def test_rebuilt_device_copy_is_rewritten():
    opt = optimizers.SGD(learning_rate=0.05)
    opt.build(8, torch.device("cpu"))
    opt.build(16, torch.device("cpu"))  # a new lr_dev tensor
    opt.lr_dev.zero_()
    opt._lr_synced = None
    opt._sync_lr()
    assert abs(float(opt.lr_dev) - 0.05) < 1e-8
