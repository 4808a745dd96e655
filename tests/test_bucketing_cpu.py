"""Size/topology-aware all-reduce plan (parallel/bucketing.py) and
CommunicationOptions plumbing (bytes_per_pack, all_reduce_dtype)."""
import pytest

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.parallel import bucketing

RESNET50 = 25_557_032
MNIST = 225_034


def test_resnet50_plan_at_8_gpus():
    p = bucketing.plan(RESNET50, 8)
    assert p.links_used == 7 and p.n_buckets == 4 and p.wire_bytes == 4 * RESNET50
    assert abs(p.bucket_bytes - 4 * RESNET50 / 4) < 4
    # 2(R-1)/R * 25.6 MB over 7 links at 60% of 153.6 GB/s, plus 25 us per call
    wire_us = 1.75 * p.bucket_bytes / (0.6 * 153.6e9 * 7) * 1e6
    assert p.per_bucket_us == pytest.approx(25.0 + wire_us)
    bf = bucketing.plan(RESNET50, 8, wire_dtype="bfloat16")
    assert bf.wire_bytes * 2 == p.wire_bytes and bf.n_buckets == 4 and bf.total_us < p.total_us


def test_plan_small_messages_and_explicit_packs():
    assert bucketing.plan(MNIST, 8).n_buckets == 1  # 900 KB: one all-reduce, latency-bound
    assert bucketing.plan(RESNET50, 8, bytes_per_pack=8 << 20).n_buckets == -(-4 * RESNET50 // (8 << 20))
    assert bucketing.plan(RESNET50, 1).total_us == 0.0
    # fewer GPUs use fewer direct links: one link at R = 2, so the same bucket takes longer
    assert bucketing.plan(RESNET50, 2).links_used == 1
    assert bucketing.ring_allreduce_us(1 << 24, 2) > bucketing.ring_allreduce_us(1 << 24, 8)
    with pytest.raises(ValueError):
        bucketing.plan(MNIST, 2, wire_dtype="int8")


def test_communication_options_plumbing():
    with pytest.raises(ValueError):
        tdl.distribute.experimental.CommunicationOptions(all_reduce_dtype="int8")
    o = tdl.distribute.experimental.CommunicationOptions(bytes_per_pack=1 << 20, all_reduce_dtype="bfloat16")
    s = tdl.distribute.MirroredStrategy(devices=["/cpu:0"], communication_options=o)
    assert s.extended.communication_options.bytes_per_pack == 1 << 20
    assert s.extended.communication_options.all_reduce_dtype == "bfloat16"
    from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

    with s.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(0.1))
    m.build((None, 28, 28, 1))
    tr = m._get_trainer()
    # the plan is always computed and reported; a CPU replica keeps f32 on the wire
    assert tr.plan.world == 1 and tr.plan.wire_dtype == "float32" and MNIST <= tr.plan.grad_numel < MNIST + 256


class _FakeRccl:
    """A world-2 'rccl' communicator that records the bucket all-reduces (identity sums)."""
    name = "rccl"
    algorithm = "rccl"
    world_size = 2
    rank = 0
    capturable = False

    def __init__(self):
        self.calls = 0

    def all_reduce_async(self, t, op="sum"):
        self.calls += 1

        class _Work:
            def wait(self):
                return None

        return _Work()

    def all_reduce(self, t, op="sum"):
        return t

    def check_health(self):
        pass


def test_bucket_hooks_follow_rebuilt_leaves():
    """evaluate()/predict() rebuild the trainer's autograd leaves (GenericTrainer._make_leaves);
    the per-bucket all-reduce hooks must move to the new leaves, or the next eager step would
    launch no bucket all-reduce and fail with 'hooks did not fire' (advisor finding, round 1)."""
    import torch

    import tensorflow_distributed_learning_amd as tdl

    tdl.keras.backend.clear_session()
    tdl.keras.utils.set_random_seed(0)
    strategy = tdl.distribute.OneDeviceStrategy("/cpu:0")
    with strategy.scope():
        inp = tdl.keras.layers.Input(shape=(6,))
        h = tdl.keras.layers.Dense(8, activation="relu")(inp)
        out = tdl.keras.layers.Dense(4)(h)
        m = tdl.keras.Model(inp, out)
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(0.1), bucket_bytes=64)
    tr = m._get_trainer()
    assert tr.kind == "generic"
    fake = _FakeRccl()
    tr.comm = fake
    tr._buckets = tr._make_buckets()
    assert tr._buckets is not None and len(tr._bucket_ranges) >= 2
    x, y = torch.randn(16, 6), torch.randint(0, 4, (16,))
    tr.train_step((x, y), 16)
    first = fake.calls
    assert first == len(tr._bucket_ranges)
    old = list(tr._leaves)
    tr._make_leaves()  # what evaluate() / predict() do
    assert all(a is not b for a, b in zip(old, tr._leaves))
    tr.train_step((x, y), 16)  # raised 'gradient bucket hooks did not fire' before the fix
    assert fake.calls == 2 * first
