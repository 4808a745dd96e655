"""Property-based tests (SURVEY.md §4.2 T-unit): sharding / rebatch invariants, the TF_CONFIG chief
rule, flat-slab layout and the native buffered shuffle, on randomly generated cases."""
import json
import types

import numpy as np
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.cluster.tf_config import parse_tf_config
from tensorflow_distributed_learning_amd.data import dataset as D
from tensorflow_distributed_learning_amd.engine.slab import SlabLayout
from tensorflow_distributed_learning_amd.parallel import input_lib

SETTINGS = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])


@SETTINGS
@given(n=st.integers(0, 10_000), parts=st.integers(1, 64))
def test_split_sizes_partition(n, parts):
    s = input_lib.split_sizes(n, parts)
    assert len(s) == parts and sum(s) == n and max(s) - min(s) <= 1 and s == sorted(s, reverse=True)


def _fake_strategy(R, rank):
    ext = types.SimpleNamespace(rank=rank, communicator=None, device=torch.device("cpu"))
    return types.SimpleNamespace(num_replicas_in_sync=R, extended=ext)


@SETTINGS
@given(n=st.integers(1, 300), B=st.integers(1, 40), R=st.integers(1, 6), buf=st.integers(1, 400),
       drop=st.booleans())
def test_data_sharding_sees_every_element_once(monkeypatch, n, B, R, buf, drop):
    """DATA auto-shard: the replicas' slices of each (identically shuffled) global batch partition it,
    so over one epoch every element is seen exactly once across the R replicas."""
    monkeypatch.setattr(input_lib, "shared_seed", lambda strategy: 1234)
    opts = tdl.data.Options()
    opts.experimental_distribute.auto_shard_policy = tdl.data.AutoShardPolicy.DATA
    ds = D.Dataset.range(n).shuffle(buf).batch(B, drop_remainder=drop).with_options(opts)
    seen = []
    for r in range(R):
        dd = input_lib.DistributedDataset(ds, _fake_strategy(R, r))
        for batch in dd:
            assert len(batch) <= -(-B // R)  # a replica's slice of a global batch
            seen.extend(int(v) for v in batch)
    full = (n // B) * B if drop else n
    assert len(seen) == full
    assert len(set(seen)) == full and all(0 <= v < n for v in seen)


roles = st.fixed_dictionaries({
    "chief": st.integers(0, 1), "worker": st.integers(0, 4), "ps": st.integers(0, 2), "evaluator": st.integers(0, 1)})


@SETTINGS
@given(counts=roles, data=st.data())
def test_chief_rule(counts, data):
    if counts["chief"] + counts["worker"] == 0:
        counts["worker"] = 1
    port = iter(range(20000, 20100))
    cluster = {r: [f"127.0.0.1:{next(port)}" for _ in range(k)] for r, k in counts.items() if k}
    tasks = [(r, i) for r, k in counts.items() for i in range(k)]
    ttype, tidx = data.draw(st.sampled_from(tasks))
    cfg = parse_tf_config(json.dumps({"cluster": cluster, "task": {"type": ttype, "index": tidx}}))
    chief = ("chief", 0) if counts["chief"] else ("worker", 0)
    assert cfg.is_chief == ((ttype, tidx) == chief)
    training = [(t.type, t.index) for t in cfg.cluster.training_tasks()]
    assert all(t in ("chief", "worker") for t, _ in training)
    assert len(training) == counts["chief"] + counts["worker"]
    assert cfg.is_training_task == (ttype in ("chief", "worker"))


@SETTINGS
@given(shapes=st.lists(st.lists(st.integers(1, 9), min_size=0, max_size=4), min_size=1, max_size=12),
       align=st.sampled_from([1, 4, 16, 64]))
def test_slab_layout_aligned_disjoint(shapes, align):
    layout = SlabLayout.from_shapes([(f"v{i}", s) for i, s in enumerate(shapes)], align=align)
    ends = 0
    for spec, off in zip(layout.specs, layout.offsets):
        assert off % align == 0 and off >= ends
        ends = off + spec.size
    assert layout.total >= ends
    flat = torch.arange(layout.total, dtype=torch.float32)
    views = layout.views(flat)
    covered = torch.zeros(layout.total, dtype=torch.int32)
    for v, off in zip(views, layout.offsets):
        assert v.numel() == 0 or int(v.reshape(-1)[0]) == off
        covered[off:off + v.numel()] += 1
    assert int(covered.max()) <= 1


@SETTINGS
@given(n=st.integers(1, 3000), buf=st.integers(1, 4000), seed=st.integers(0, 2**31 - 1))
def test_native_buffered_shuffle_matches_python(n, buf, seed):
    src = np.arange(n)
    a = D._shuffle_indices(n, buf, np.random.default_rng(seed))
    s64 = int(np.random.default_rng(seed).integers(0, 1 << 63))
    b = D._shuffle_indices_py(src, n, buf, D._splitmix64_stream(s64, n))
    assert np.array_equal(a, b)
    assert sorted(a.tolist()) == list(range(n))
