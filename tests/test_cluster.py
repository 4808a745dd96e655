"""TF_CONFIG parsing / validation / chief rule (README.md:31-61)."""
import json

import pytest

from tensorflow_distributed_learning_amd.cluster import (ClusterConfigError, TaskSpec, TFConfigClusterResolver,
                                                         make_tf_config, parse_tf_config)

README_EXAMPLE = {"cluster": {"chief": ["host1:1"], "worker": ["host2:2", "host3:3"], "ps": ["host4:4"],
                              "evaluator": ["host5:5"]}, "task": {"type": "worker", "index": 0}}


def test_absent_or_empty_is_local():
    assert parse_tf_config(environ={}) is None
    assert parse_tf_config("") is None
    assert parse_tf_config("{}") is None


def test_readme_example_roles_and_chief():
    cfg = parse_tf_config(json.dumps(README_EXAMPLE))
    assert cfg.chief_task == TaskSpec("chief", 0)
    assert not cfg.is_chief  # worker/0 is not chief when a chief exists
    assert cfg.num_training_tasks == 3  # ps/evaluator excluded from the collective group
    assert cfg.task_rank == 1
    assert cfg.chief_address == ("host1", 1)
    assert [str(t) for t in cfg.cluster.training_tasks()] == ["/job:chief/task:0", "/job:worker/task:0",
                                                              "/job:worker/task:1"]


def test_first_worker_is_chief_without_chief():
    cfg = parse_tf_config(make_tf_config(["a:1", "b:2"], 0))
    assert cfg.is_chief and cfg.task_rank == 0 and cfg.chief_address == ("a", 1)
    cfg1 = parse_tf_config(make_tf_config(["a:1", "b:2"], 1))
    assert not cfg1.is_chief and cfg1.task_rank == 1


def test_single_worker_degrades():
    assert parse_tf_config(make_tf_config(["a:1"], 0)).is_single_worker


def test_reference_tf_config():
    s = json.dumps({"cluster": {"worker": ["172.16.16.5:12345", "172.16.16.6:12345"]},
                    "task": {"type": "worker", "index": 1}})
    cfg = parse_tf_config(s)
    assert cfg.task == TaskSpec("worker", 1) and cfg.task_address == ("172.16.16.6", 12345)


@pytest.mark.parametrize("bad", [
    "not json",
    json.dumps({"cluster": {"worker": ["a:1"]}, "task": {"type": "worker", "index": 3}}),   # not in cluster
    json.dumps({"cluster": {"worker": ["a:1"]}, "task": {"type": "worker", "index": -1}}),  # 0-based
    json.dumps({"cluster": {"worker": ["a"]}, "task": {"type": "worker", "index": 0}}),     # no port
    json.dumps({"cluster": {"chief": ["a:1", "b:2"]}}),                                      # two chiefs
    json.dumps({"cluster": {"worker": ["a:1", "a:1"]}}),                                     # duplicate address
    json.dumps({"cluster": {"master": ["a:1"]}}),                                            # unknown role
    json.dumps({"cluster": {"worker": ["a:1"]}, "task": {"type": "boss", "index": 0}}),
    json.dumps({"cluster": {"worker": ["a:1"]}, "bogus": 1}),
])
def test_invalid_configs_rejected(bad):
    with pytest.raises(ClusterConfigError):
        parse_tf_config(bad)


def test_ps_task_not_training():
    d = dict(README_EXAMPLE, task={"type": "ps", "index": 0})
    cfg = parse_tf_config(json.dumps(d))
    assert not cfg.is_training_task
    with pytest.raises(ClusterConfigError):
        _ = cfg.task_rank


def test_resolver(monkeypatch):
    monkeypatch.setenv("TF_CONFIG", json.dumps(README_EXAMPLE))
    r = TFConfigClusterResolver()
    assert r.task_type == "worker" and r.task_id == 0
    assert r.master() == "grpc://host2:2"
    assert r.cluster_spec().num_tasks("worker") == 2
    assert r.master("chief", 0) == "grpc://host1:1"
