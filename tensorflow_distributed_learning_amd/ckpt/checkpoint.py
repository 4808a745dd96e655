"""Checkpoints and SavedModel-shaped model directories (README.md:51: the chief saves them).

Tensor bundle (``<prefix>.index`` + ``<prefix>.data-00000-of-00001``):
  * ``.data`` – raw little-endian tensor bytes, 64-byte aligned, in variable order;
  * ``.index`` – TensorFlow's own format: a LevelDB-format table of ``BundleHeaderProto`` /
    ``BundleEntryProto`` records (ckpt/tensor_bundle.py), with TF variable names and layouts (HWIO
    conv kernels, [in,out] dense kernels).  ``TDL_CKPT_INDEX=json`` writes the round-1/2 JSON index
    ``{"format": "tdl-bundle-v1", ...}`` instead; both are read.

Model directory (``model.save(path)``)::

    path/saved_model.json                       architecture + compile config
    path/saved_model.pb                         TF1-format SavedModel: serving graph, variables, V2 saver,
                                                signature (ckpt/saved_model_pb.py, ckpt/graph_def.py)
    path/variables/variables.index
    path/variables/variables.data-00000-of-00001
    path/assets/

Multi-worker protocol (TF's): only the chief writes to the real path; other workers write to
``<dir>/workertemp_<task_id>`` and delete it, so every worker runs the same code path.
"""
from __future__ import annotations

import json
import os
import re
import shutil
from typing import Dict, List, Optional

import numpy as np
import torch

from ..utils.events import crc32c
from . import tensor_bundle as TB

FORMAT = "tdl-bundle-v1"
_DT = {torch.float32: "float32", torch.float64: "float64", torch.float16: "float16", torch.bfloat16: "bfloat16",
       torch.int32: "int32", torch.int64: "int64", torch.int8: "int8", torch.uint8: "uint8", torch.bool: "bool"}
_DT_INV = {v: k for k, v in _DT.items()}


def write_bundle(prefix: str, tensors: Dict[str, torch.Tensor]) -> None:
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    index = {"format": FORMAT, "tensors": {}}
    tmp_data = prefix + ".data-00000-of-00001.tmp"
    off = 0
    with open(tmp_data, "wb") as f:
        for name, t in tensors.items():
            t = torch.as_tensor(t).detach().cpu().contiguous()
            raw = t.view(torch.uint8).numpy().tobytes() if t.dtype == torch.bfloat16 else t.numpy().tobytes()
            pad = (-off) % 64
            if pad:
                f.write(b"\0" * pad)
                off += pad
            f.write(raw)
            index["tensors"][name] = {"dtype": _DT[t.dtype], "shape": list(t.shape), "offset": off,
                                      "nbytes": len(raw), "crc32c": crc32c(raw)}
            off += len(raw)
    os.replace(tmp_data, prefix + ".data-00000-of-00001")
    if os.environ.get("TDL_CKPT_INDEX", "tf") == "json":
        with open(prefix + ".index.tmp", "w") as f:
            json.dump(index, f)
    else:
        TB.write_index(prefix + ".index.tmp", index["tensors"])
    os.replace(prefix + ".index.tmp", prefix + ".index")


def _read_index(prefix: str) -> dict:
    path = prefix + ".index"
    if TB.is_table(path):
        return {"format": "tf-tensor-bundle", "tensors": TB.read_index(path)}
    with open(path) as f:
        index = json.load(f)
    if index.get("format") != FORMAT:
        raise ValueError(f"{path} is neither a TF tensor-bundle index nor a {FORMAT} index")
    return index


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, torch.Tensor]:
    index = _read_index(prefix)
    out = {}
    with open(prefix + ".data-00000-of-00001", "rb") as f:
        data = f.read()
    for name, e in index["tensors"].items():
        if e["dtype"] not in _DT_INV:
            if name == "_CHECKPOINTABLE_OBJECT_GRAPH":
                continue  # a TF2 object-graph proto (string tensor): not a variable
            raise ValueError(f"{prefix}: tensor {name!r} has dtype {e['dtype']}, which this reader does not "
                             "support (numeric tensors only)")
        raw = data[e["offset"] : e["offset"] + e["nbytes"]]
        if verify and crc32c(raw) != e["crc32c"]:
            raise ValueError(f"checksum mismatch for {name} in {prefix}")
        dt = _DT_INV[e["dtype"]]
        if dt == torch.bfloat16:
            t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).view(torch.bfloat16)
        else:
            t = torch.from_numpy(np.frombuffer(raw, dtype=np.dtype(e["dtype"])).copy())
        out[name] = t.reshape(e["shape"])
    return out


def list_variables(prefix: str):
    return [(n, tuple(e["shape"])) for n, e in _read_index(prefix)["tensors"].items()]


# ------------------------------------------------------------------------------------------------
def _strategy_of(obj=None):
    from ..parallel.strategy import get_strategy

    s = getattr(obj, "_distribution_strategy", None) if obj is not None else None
    return s or get_strategy()


def write_dirpath(dirpath: str, strategy=None) -> str:
    """Chief writes to dirpath; non-chief workers to a temporary sibling (TF protocol)."""
    strategy = strategy or _strategy_of()
    if strategy is None or strategy.extended.is_chief:
        return dirpath
    tid = strategy.extended.rank
    base = os.path.dirname(dirpath.rstrip("/")) or "."
    return os.path.join(base, f"workertemp_{tid}", os.path.basename(dirpath.rstrip("/")))


def remove_temp_dirpath(dirpath: str, strategy=None):
    strategy = strategy or _strategy_of()
    if strategy is not None and not strategy.extended.is_chief:
        base = os.path.dirname(os.path.dirname(dirpath.rstrip("/")))
        tmp = os.path.dirname(dirpath.rstrip("/"))
        if os.path.basename(tmp).startswith("workertemp_"):
            shutil.rmtree(tmp, ignore_errors=True)
        del base


# ------------------------------------------------------------------------------------------------
def model_tensors(model) -> Dict[str, torch.Tensor]:
    return {v.name: v.read_value() for v in model.weights}


def model_tensors_are_float32(tensors: Dict[str, torch.Tensor], model) -> bool:
    """The serving graph declares every variable DT_FLOAT (the Keras default variable dtype)."""
    return all(tensors[v.name].dtype == torch.float32 for v in model.weights if v.name in tensors)


def save_model(model, path: str, overwrite: bool = True, include_optimizer: bool = True) -> None:
    """model.save(path): SavedModel-shaped directory (written by the chief only)."""
    strategy = _strategy_of(model)
    real = path
    path = write_dirpath(path, strategy)
    if os.path.exists(path) and not overwrite:
        raise FileExistsError(path)
    os.makedirs(os.path.join(path, "variables"), exist_ok=True)
    os.makedirs(os.path.join(path, "assets"), exist_ok=True)
    tensors = model_tensors(model)
    if include_optimizer and getattr(model, "optimizer", None) is not None:
        st = model.optimizer.state_dict()
        tensors["optimizer/iterations"] = torch.tensor(st["iterations"], dtype=torch.int64)
        for k, v in st["slots"].items():
            tensors[f"optimizer/slots/{k}"] = v
    write_bundle(os.path.join(path, "variables", "variables"), tensors)
    cfg = {"format": "tdl-saved-model-v1", "model": model.get_config_full()}
    if getattr(model, "_compile_config", None):
        cfg["compile"] = model._compile_config
    with open(os.path.join(path, "saved_model.json"), "w") as f:
        json.dump(cfg, f, indent=1, default=str)
    # saved_model.pb: the serving graph (inference ops, resource variables, V2 saver over
    # variables/) + tags + serving signature; header-only for a layer with no TF op mapping
    from . import graph_def as GD
    from . import saved_model_pb as SMP

    try:
        spec = SMP.model_signature(model)
    except Exception as e:  # the header is auxiliary: a model whose signature cannot be derived still saves
        import warnings

        warnings.warn(f"model.save: saved_model.pb skipped ({type(e).__name__}: {e})")
        spec = None
    if spec is not None:
        graph = None
        if model_tensors_are_float32(tensors, model):
            try:
                graph = GD.build_graph(model, SMP.GRAPH_PRODUCER)
            except Exception as e:  # noqa: BLE001 - the graph is best effort; variables/ is written
                import warnings

                why = str(e) if isinstance(e, GD.UnsupportedLayer) else f"{type(e).__name__}: {e}"
                warnings.warn(f"model.save: saved_model.pb without a TF graph ({why})")
        with open(os.path.join(path, "saved_model.pb"), "wb") as f:
            f.write(SMP.encode_saved_model(*spec, graph=graph))
    remove_temp_dirpath(path, strategy) if path != real else None


def load_model(path: str, compile: bool = True):
    from ..keras.models import model_from_config

    with open(os.path.join(path, "saved_model.json")) as f:
        cfg = json.load(f)
    model = model_from_config(cfg["model"])
    tensors = read_bundle(os.path.join(path, "variables", "variables"))
    model.load_named_tensors(tensors)
    if compile and cfg.get("compile"):
        model.compile_from_config(cfg["compile"])
        if "optimizer/iterations" in tensors and model.optimizer is not None:
            model.optimizer.load_state_dict({
                "iterations": int(tensors["optimizer/iterations"]),
                "slots": {k.split("/", 2)[2]: v for k, v in tensors.items() if k.startswith("optimizer/slots/")}})
    return model


# ------------------------------------------------------------------------------------------------
def _trackable_tensors(name: str, obj) -> Dict[str, torch.Tensor]:
    out = {}
    if hasattr(obj, "weights") and hasattr(obj, "get_config_full"):  # a model
        for v in obj.weights:
            out[f"{name}/{v.name}"] = v.read_value()
    elif hasattr(obj, "state_dict") and hasattr(obj, "apply_flat"):  # an optimizer
        st = obj.state_dict()
        out[f"{name}/iterations"] = torch.tensor(st["iterations"], dtype=torch.int64)
        for k, v in st["slots"].items():
            out[f"{name}/slots/{k}"] = v
    elif hasattr(obj, "read_value"):  # a variable
        out[name] = obj.read_value()
    elif isinstance(obj, torch.Tensor):
        out[name] = obj
    elif isinstance(obj, (int, float)):
        out[name] = torch.tensor(obj)
    elif isinstance(obj, dict):
        for k, v in obj.items():
            out.update(_trackable_tensors(f"{name}/{k}", v))
    return out


def _restore_into(name: str, obj, tensors: Dict[str, torch.Tensor]):
    if hasattr(obj, "weights") and hasattr(obj, "get_config_full"):
        sub = {k[len(name) + 1 :]: v for k, v in tensors.items() if k.startswith(name + "/")}
        obj.load_named_tensors(sub)
    elif hasattr(obj, "state_dict") and hasattr(obj, "apply_flat"):
        if f"{name}/iterations" in tensors:
            obj.load_state_dict({"iterations": int(tensors[f"{name}/iterations"]),
                                 "slots": {k.split("/slots/", 1)[1]: v for k, v in tensors.items()
                                           if k.startswith(name + "/slots/")}})
    elif hasattr(obj, "assign") and name in tensors:
        obj.assign(tensors[name])
    elif isinstance(obj, torch.Tensor) and name in tensors:
        with torch.no_grad():
            obj.copy_(tensors[name].reshape(obj.shape))
    elif isinstance(obj, dict):
        for k, v in obj.items():
            _restore_into(f"{name}/{k}", v, tensors)


class Checkpoint:
    """tf.train.Checkpoint(**objects): save()/restore()/write()/read()."""

    def __init__(self, **objects):
        self._objects = objects
        self.save_counter = 0

    def __getattr__(self, k):
        objs = self.__dict__.get("_objects", {})
        if k in objs:
            return objs[k]
        raise AttributeError(k)

    def _tensors(self):
        out = {"save_counter": torch.tensor(self.save_counter, dtype=torch.int64)}
        for k, v in self._objects.items():
            out.update(_trackable_tensors(k, v))
        return out

    def write(self, file_prefix: str) -> str:
        strategy = _strategy_of(next(iter(self._objects.values()), None))
        d = os.path.dirname(file_prefix) or "."
        wd = write_dirpath(d, strategy)
        target = os.path.join(wd, os.path.basename(file_prefix))
        write_bundle(target, self._tensors())
        if wd != d:
            remove_temp_dirpath(wd, strategy)
        return file_prefix

    def save(self, file_prefix: str) -> str:
        self.save_counter += 1
        path = f"{file_prefix}-{self.save_counter}"
        self.write(path)
        strategy = _strategy_of(next(iter(self._objects.values()), None))
        if strategy.extended.is_chief:
            _update_checkpoint_state(os.path.dirname(path) or ".", os.path.basename(path))
        return path

    def read(self, save_path: str):
        tensors = read_bundle(save_path)
        for k, v in self._objects.items():
            _restore_into(k, v, tensors)
        if "save_counter" in tensors:
            self.save_counter = int(tensors["save_counter"])
        return _LoadStatus()

    restore = read


class _LoadStatus:
    def assert_consumed(self):
        return self

    def expect_partial(self):
        return self

    def assert_existing_objects_matched(self):
        return self


def _state_file(directory: str) -> str:
    return os.path.join(directory, "checkpoint")


def _update_checkpoint_state(directory: str, latest: str, all_paths: Optional[List[str]] = None):
    paths = list(all_paths) if all_paths is not None else _read_state(directory)[1]
    if latest not in paths:
        paths.append(latest)
    with open(_state_file(directory) + ".tmp", "w") as f:
        f.write(f'model_checkpoint_path: "{latest}"\n')
        for p in paths:
            f.write(f'all_model_checkpoint_paths: "{p}"\n')
    os.replace(_state_file(directory) + ".tmp", _state_file(directory))


def _read_state(directory: str):
    fp = _state_file(directory)
    if not os.path.exists(fp):
        return None, []
    latest, allp = None, []
    for line in open(fp):
        m = re.match(r'(\w+): "(.*)"', line.strip())
        if not m:
            continue
        if m.group(1) == "model_checkpoint_path":
            latest = m.group(2)
        else:
            allp.append(m.group(2))
    return latest, allp


def latest_checkpoint(checkpoint_dir: str) -> Optional[str]:
    latest, _ = _read_state(checkpoint_dir)
    if latest is None:
        return None
    p = latest if os.path.isabs(latest) else os.path.join(checkpoint_dir, latest)
    return p if os.path.exists(p + ".index") else None


class CheckpointManager:
    """tf.train.CheckpointManager(checkpoint, directory, max_to_keep)."""

    def __init__(self, checkpoint: Checkpoint, directory: str, max_to_keep: Optional[int] = 5,
                 checkpoint_name: str = "ckpt"):
        self.checkpoint = checkpoint
        self.directory = directory
        self.max_to_keep = max_to_keep
        self.checkpoint_name = checkpoint_name
        os.makedirs(directory, exist_ok=True)
        _, allp = _read_state(directory)
        self._checkpoints = [os.path.join(directory, p) for p in allp]
        # continue numbering after the checkpoints already in the directory
        nums = [int(m.group(1)) for p in allp if (m := re.search(r"-(\d+)$", p))]
        if nums:
            checkpoint.save_counter = max(checkpoint.save_counter, max(nums))

    @property
    def latest_checkpoint(self) -> Optional[str]:
        return latest_checkpoint(self.directory)

    @property
    def checkpoints(self) -> List[str]:
        return list(self._checkpoints)

    def save(self, checkpoint_number: Optional[int] = None) -> str:
        ck = self.checkpoint
        if checkpoint_number is not None:
            ck.save_counter = int(checkpoint_number) - 1
        ck.save_counter += 1
        path = os.path.join(self.directory, f"{self.checkpoint_name}-{ck.save_counter}")
        ck.write(path)
        strategy = _strategy_of(next(iter(ck._objects.values()), None))
        if strategy.extended.is_chief:
            self._checkpoints = [p for p in self._checkpoints if p != path] + [path]
            if self.max_to_keep is not None:
                while len(self._checkpoints) > self.max_to_keep:
                    old = self._checkpoints.pop(0)
                    for suf in (".index", ".data-00000-of-00001"):
                        try:
                            os.remove(old + suf)
                        except FileNotFoundError:
                            pass
            _update_checkpoint_state(self.directory, os.path.basename(path),
                                     [os.path.basename(p) for p in self._checkpoints])
        return path

    def restore_or_initialize(self):
        p = self.latest_checkpoint
        if p:
            self.checkpoint.restore(p)
            return p
        return None
