"""Keras models: ``Sequential`` (tf_dist_example.py:40-48), functional ``Model(inputs, outputs)``,
subclassed models; ``compile`` / ``fit`` / ``evaluate`` / ``predict`` / ``save`` (ex:49-59).

Distribution: a model created inside ``strategy.scope()`` remembers its strategy (ex:56-59 call
``fit`` outside the scope, quirk Q9).  Its variables become views into ONE flat slab per replica
(engine/slab.py), initialised on the chief and broadcast to every replica.
``fit`` picks the fused MI355X engine for the reference CNN (engine/fused.py) and the generic
autograd engine otherwise (engine/trainer.py).
"""
from __future__ import annotations

import math
import os
import sys
import time
import warnings
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ..data import dataset as D
from ..engine.slab import SlabLayout, VarSpec
from ..parallel.values import Variable
from . import callbacks as cbks
from . import losses as _losses
from . import metrics as _metrics
from . import optimizers as _opt
from .layers import InputLayer, KerasTensor, Layer, Node, _flat, _map

_GLOBAL_POLICY = ["float32"]


_CONV_BN_STATS = os.environ.get("TDL_CONV_BN_STATS", "1") == "1"
_FUSE_CPU = [False]  # tests: apply the training-graph fusion plan to CPU tensors too


def _map_outputs(fn, y):
    """Apply fn to every tensor of a model output structure (tensor, list / tuple, dict)."""
    if isinstance(y, dict):
        return {k: _map_outputs(fn, v) for k, v in y.items()}
    if isinstance(y, (list, tuple)):
        return type(y)(_map_outputs(fn, v) for v in y)
    return fn(y)


def _concat_outputs(batches):
    """Concatenate per-batch output structures along the batch axis into numpy arrays."""
    first = batches[0]
    if isinstance(first, dict):
        return {k: _concat_outputs([b[k] for b in batches]) for k in first}
    if isinstance(first, (list, tuple)):
        return [_concat_outputs([b[i] for b in batches]) for i in range(len(first))]
    return torch.cat(batches).numpy()


class Model(Layer):
    def __init__(self, inputs=None, outputs=None, name: Optional[str] = None, **kw):
        from ..parallel.strategy import get_strategy, has_strategy

        trainable = kw.pop("trainable", True)
        super().__init__(name=name, trainable=trainable, **kw)
        self._distribution_strategy = get_strategy() if has_strategy() else None
        self._functional = inputs is not None and outputs is not None
        self.optimizer = None
        self.loss = None
        self.compiled_metrics: List[_metrics.Metric] = []
        self._loss_tracker = None
        self._compile_config = None
        self._trainer = None
        self._W = self._G = self._NT = None
        self._layout = None
        self._slab_vars_sig = None
        self._steps_per_execution = 1
        self._bucket_bytes = 0
        self.stop_training = False
        self.history = None
        self._built_input_shape = None
        self._current_epoch = 0
        self._initial_epoch_override = None
        if self._functional:
            self._init_graph(inputs, outputs)

    # ------------------------------------------------------------------ layer tracking
    def __setattr__(self, k, v):
        if isinstance(v, Layer) and k not in ("_trainer",) and not k.startswith("__"):
            layers = self.__dict__.get("_layers")
            if layers is not None and v not in layers and v is not self:
                layers.append(v)
        super().__setattr__(k, v)

    @property
    def layers(self) -> List[Layer]:
        return [l for l in self._layers if not isinstance(l, InputLayer)]

    def get_layer(self, name=None, index=None):
        if index is not None:
            return self.layers[index]
        for l in self.layers:
            if l.name == name:
                return l
        raise ValueError(f"no layer named {name}")

    # ------------------------------------------------------------------ functional graph
    def _init_graph(self, inputs, outputs):
        self._inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        self._outputs = outputs
        out_list = _flat(outputs)
        order: List[Node] = []
        seen = set()

        def visit(t: KerasTensor):
            node = t._node
            if node is None or id(node) in seen:
                return
            if node.inputs is not None:
                for it in _flat(node.inputs):
                    visit(it)
            seen.add(id(node))
            order.append(node)

        for t in out_list:
            visit(t)
        self._nodes = [n for n in order if n.inputs is not None]
        for n in self._nodes:
            if n.layer not in self._layers:
                self._layers.append(n.layer)
        self._built_input_shape = self._inputs[0].shape if len(self._inputs) == 1 else [i.shape for i in self._inputs]
        self.built = True

    def _fusion(self):
        fp = self.__dict__.get("_fusion_plan")
        if fp is None or fp[0] is not self._nodes:
            from . import fusion

            fp = (self._nodes, fusion.plan(self._nodes, self._outputs))
            self.__dict__["_fusion_plan"] = fp
        return fp[1]

    def _run_graph(self, inputs, training):
        xs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        vals = {id(k): v for k, v in zip(self._inputs, xs)}
        fp = None
        if training and isinstance(xs[0], torch.Tensor) and (xs[0].is_cuda or _FUSE_CPU[0]):
            fp = self._fusion()  # keras/fusion.py: conv-bias/BN/ReLU/Add groups (training, GPU)
            if not fp.groups and not fp.pool_pad and not fp.conv_box and not fp.conv_pool:
                fp = None
        boxes = {}  # id(tensor) -> GradBox of its two consumers' backward contributions
        self.__dict__["_grad_boxes"] = boxes
        from ..utils import checksums as _ck

        ck = _ck.enabled()
        for n in self._nodes:
            if fp is not None:
                nid = id(n)
                if nid in fp.skip:
                    continue
                g = fp.groups.get(nid)
                if g is not None:
                    from .fusion import run_group

                    run_group(g, vals, training, fp.taps.get(nid), boxes)
                    if ck:
                        tag = f"group:{g.bn_node.layer.name}"
                        _ck.record(tag, vals[id(g.out)])
                        _ck.hook_grad(tag, vals[id(g.out)])
                    continue
            kw = {k: v for k, v in n.kwargs.items() if k != "training"}
            src = n.inputs
            if fp is not None:
                if id(n) in fp.conv_nobias:
                    kw["_fold_bias"] = True
                    if _CONV_BN_STATS:
                        kw["_bn_stats"] = True  # its BN's statistics come from the conv epilogue
                pp = fp.pool_pad.get(id(n))
                if pp is not None:  # fused ZeroPadding2D: read the padding layer's input
                    src = pp[0]
                    kw["_zero_pad"] = pp[1]
                cpn = fp.conv_pool.get(id(n))
                if cpn is not None:  # Conv2D -> MaxPooling2D(2): the pool runs inside the conv's call
                    kw["_pool"] = cpn.layer
            if fp is not None and (id(n) in fp.conv_box or id(n) in fp.taps):
                from ..ops.conv import GradBox, grad_tap

                if id(n) in fp.conv_box:
                    kw["_grad_box"] = boxes.setdefault(fp.conv_box[id(n)], GradBox())
                tapped = fp.taps.get(id(n), ())
                args = _map(lambda t: grad_tap(vals[id(t)], boxes.setdefault(id(t), GradBox()))
                            if id(t) in tapped else vals[id(t)], src)
            else:
                args = _map(lambda t: vals[id(t)], src)
            out = n.layer(args, training=training, **kw)
            if ck:
                _ck.record_tree(f"node:{n.layer.name}", out)
                if isinstance(out, torch.Tensor):
                    _ck.hook_grad(f"node:{n.layer.name}", out)
            if isinstance(n.outputs, list):
                for t, o in zip(n.outputs, out):
                    vals[id(t)] = o
            else:
                vals[id(n.outputs)] = out
            if fp is not None and id(n) in fp.conv_pool:  # (the conv's own output is read by the pool only)
                vals[id(fp.conv_pool[id(n)].outputs)] = out
        return _map(lambda t: vals[id(t)], self._outputs)

    # ------------------------------------------------------------------ build / call
    def build(self, input_shape):
        if self._functional:
            return
        self._built_input_shape = tuple(input_shape) if not isinstance(input_shape, list) else input_shape
        dummy = torch.zeros((1,) + tuple(d if d is not None else 1 for d in tuple(input_shape)[1:]))
        with torch.no_grad():
            self.call(dummy, training=False)
        self.built = True

    def call(self, inputs, training=None):
        if self._functional:
            return self._run_graph(inputs, training)
        raise NotImplementedError("subclassed models must implement call()")

    def __call__(self, inputs, training=None, **kw):
        if not self.built:
            shapes = _map(lambda t: (None,) + tuple(t.shape[1:]), inputs) if not isinstance(inputs, KerasTensor) \
                else inputs.shape
            self.build(shapes)
        return super().__call__(inputs, training=training, **kw)

    def compute_output_shape(self, input_shape):
        if self._functional:
            return _map(lambda t: t.shape, self._outputs)
        return super().compute_output_shape(input_shape)

    # ------------------------------------------------------------------ distribution / slabs
    def _get_strategy(self):
        from ..parallel.strategy import get_strategy

        return self._distribution_strategy or get_strategy()

    def _is_chief(self) -> bool:
        return self._get_strategy().extended.is_chief

    @property
    def _trainable_vars(self) -> List[Variable]:
        return self.trainable_weights

    def _ensure_slabs(self):
        """Bind every variable to a view of this replica's flat slab(s)."""
        ws = self.weights
        sig = tuple(id(w) for w in ws) + tuple(w.trainable for w in ws)
        if self._slab_vars_sig == sig and self._W is not None:
            return
        strategy = self._get_strategy()
        dev = strategy.extended.device
        tv = [w for w in ws if w.trainable and w.dtype.is_floating_point]
        ntv = [w for w in ws if w not in tv]
        self._layout = SlabLayout([VarSpec(w.name, w.shape) for w in tv])
        W = torch.zeros(self._layout.total, dtype=torch.float32, device=dev)
        for v, view in zip(tv, self._layout.views(W)):
            v._bind(view)
        ntl = SlabLayout([VarSpec(w.name, w.shape) for w in ntv]) if ntv else None
        NT = torch.zeros(ntl.total, dtype=torch.float32, device=dev) if ntl else None
        if ntl:
            for v, view in zip(ntv, ntl.views(NT)):
                if v.dtype == torch.float32:
                    v._bind(view)
                else:
                    v._value = v._value.to(dev)
        comm = strategy.extended.communicator
        if comm.world_size > 1 and not getattr(comm, "threaded", False):
            # every replica starts from the chief's initial values (TF: broadcast from worker 0;
            # replica threads of one process got replica 0's values with their clone instead)
            comm.broadcast(W, 0)
            if NT is not None:
                comm.broadcast(NT, 0)
        self._W, self._G, self._NT, self._nt_layout = W, torch.zeros_like(W), NT, ntl
        self._slab_vars_sig = sig
        self._trainer = None

    def _regularization_loss(self):
        total = None
        for v in self.trainable_weights:
            r = getattr(v, "_regularizer", None)
            if r is not None:
                term = r(v.value)
                total = term if total is None else total + term
        return total

    def _dtype_policy(self) -> str:
        return _GLOBAL_POLICY[0]

    # ------------------------------------------------------------------ compile
    def compile(self, optimizer="rmsprop", loss=None, metrics=None, loss_weights=None, weighted_metrics=None,
                run_eagerly=None, steps_per_execution=1, jit_compile=None, bucket_bytes=None, **kw):
        strategy = self._get_strategy()
        with strategy.scope():
            self.optimizer = _opt.get(optimizer)
            self.loss = _losses.get(loss) if loss is not None else None
            ms = metrics or []
            if isinstance(ms, dict):
                ms = [m for v in ms.values() for m in (v if isinstance(v, list) else [v])]
            self.compiled_metrics = [_metrics.get(m, self.loss) for m in ms]
            self._loss_tracker = _metrics.Mean(name="loss")
        self._steps_per_execution = int(steps_per_execution or 1)
        # RCCL all-reduce bucket size for overlap with backward (0 = one all-reduce per step,
        # None = the strategy's CommunicationOptions.bytes_per_pack, else the size/topology plan
        # of parallel/bucketing.py)
        self._bucket_bytes = None if bucket_bytes is None else int(bucket_bytes)
        self._run_eagerly = bool(run_eagerly)
        self._trainer = None
        self._compile_config = {
            "optimizer": _opt.serialize(self.optimizer),
            "loss": self.loss.name if self.loss is not None else None,
            "loss_config": self.loss.get_config() if self.loss is not None else None,
            "metrics": [m.name for m in self.compiled_metrics],
            "steps_per_execution": self._steps_per_execution,
        }

    def compile_from_config(self, cfg):
        loss = None
        if cfg.get("loss"):
            loss = _losses.get(cfg["loss"])
            for k, v in (cfg.get("loss_config") or {}).items():
                if k == "from_logits":
                    loss.from_logits = v
        self.compile(optimizer=_opt.get(cfg["optimizer"]), loss=loss, metrics=cfg.get("metrics") or None,
                     steps_per_execution=cfg.get("steps_per_execution", 1))

    @property
    def metrics(self):
        return ([self._loss_tracker] if self._loss_tracker else []) + list(self.compiled_metrics)

    @property
    def metrics_names(self):
        return [m.name for m in self.metrics]

    def _get_trainer(self):
        from ..engine import fused
        from ..engine.trainer import GenericTrainer

        if self.optimizer is None:
            raise RuntimeError("You must compile() the model before training it")
        if self.loss is None:
            raise RuntimeError("compile() needs a loss to train")
        self._ensure_slabs()
        t = self._trainer
        if getattr(self._get_strategy(), "_local_group", None) is not None:
            if self._outer_local_group() is not None:
                # single-process multi-device MirroredStrategy, the user's thread: ONE training loop
                # over every local replica (engine/mirrored.py)
                if t is None or not getattr(t, "is_group", False):
                    from ..engine import mirrored

                    self._trainer = t = mirrored.make_group_trainer(self)
                return t
            if getattr(t, "is_group", False):  # inside a replica region: this replica's own engine
                return t.replica_trainer(self)
        if t is None:
            reason = fused.eligible(self)
            self._trainer = fused.FusedMnistTrainer(self) if reason is None else GenericTrainer(self)
            self._fused_reason = reason
        return self._trainer

    # ------------------------------------------------------------------ data adaptation
    def _adapt(self, x, y, batch_size, shuffle, sample_weight=None):
        from ..parallel.input_lib import DistributedDataset, DistributedDatasetFromFunction

        if isinstance(x, (DistributedDataset, DistributedDatasetFromFunction)):
            return x.dataset
        if isinstance(x, D.Dataset):
            if y is not None:
                raise ValueError("y must not be given when x is a Dataset")
            return x
        if x is None:
            raise ValueError("fit/evaluate need x")
        if hasattr(x, "__iter__") and not isinstance(x, (np.ndarray, torch.Tensor, list, tuple, dict)):
            return D.Dataset.from_generator(lambda: x)
        xs = x
        parts = (xs,) if y is None else (xs, y)
        if sample_weight is not None:
            parts = parts + (sample_weight,)
        ds = D.Dataset.from_tensor_slices(parts if len(parts) > 1 else parts[0])
        n = ds.cardinality()
        if shuffle:
            ds = ds.shuffle(max(1, n))
        return ds.batch(batch_size or 32)

    def _peek_build(self, ds):
        if self.built:
            return
        el = next(iter(ds))
        x = el[0] if isinstance(el, (tuple, list)) else el
        self.build((None,) + tuple(x.shape[1:]))

    # ------------------------------------------------------------------ single-process replicas
    def _outer_local_group(self):
        """The LocalReplicaGroup of a single-process multi-device MirroredStrategy when called
        from outside its replica threads (then fit / evaluate / predict run once per replica)."""
        g = getattr(self._get_strategy(), "_local_group", None)
        return g if g is not None and not g.in_region() else None

    def _local_replicas(self):
        """Replica models 0..G-1 of a single-process MirroredStrategy: replica 0 is this model, replicas
        1..G-1 are clones built in their replica's scope (device r), compiled alike, holding this
        model's current weights (parallel/local_replicas.py)."""
        strategy = self._get_strategy()
        g = strategy._local_group
        clones = getattr(self, "_local_clones", None)
        weights = self.get_weights()
        if clones is None or len(clones) != g.G - 1:
            if not self._functional and not isinstance(self, Sequential):
                raise NotImplementedError(
                    "single-process multi-device MirroredStrategy needs a Sequential or functional model (a "
                    "subclassed model cannot be cloned per device); launch one process per GPU instead: "
                    "python -m tensorflow_distributed_learning_amd.launch --nproc-per-node N script.py")
            cfg = self.get_config_full()
            clones = []
            for r in range(1, g.G):
                view = strategy._replica_strategy(r)
                with view.scope():
                    m = model_from_config(cfg)
                    if not m.built and self._built_input_shape:
                        m.build(tuple(self._built_input_shape))
                    if getattr(self, "_compile_config", None) is not None:
                        m.compile_from_config(self._compile_config)
                        m._bucket_bytes = self._bucket_bytes
                m._distribution_strategy = view
                clones.append(m)
            self._local_clones = clones
        for m in clones:  # every replica starts from replica 0's current values (mirrored variables)
            m.set_weights(weights)
        return [self] + clones

    def _local_run(self, name: str, kwargs: dict):
        """Run ``name`` (fit / evaluate / predict) once per local replica concurrently; replica 0 (this
        model, the caller's thread) keeps the callbacks and the output, the clones run silently."""
        g = self._get_strategy()._local_group
        x = kwargs.get("x")
        if not self.built and x is not None:  # build replica 0 so the clones get its shapes
            self._peek_build(x if isinstance(x, D.Dataset) else
                             self._adapt(x, kwargs.get("y"), kwargs.get("batch_size"), False))
        models = self._local_replicas()

        def one(r):
            kw = dict(kwargs)
            if r > 0:
                kw["verbose"] = 0
                if "callbacks" in kw:
                    kw["callbacks"] = None
            return getattr(models[r], f"_{name}_impl")(**kw)

        return g.run(one)[0]

    # ------------------------------------------------------------------ fit
    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose="auto", callbacks=None, validation_split=0.0,
            validation_data=None, shuffle=True, class_weight=None, sample_weight=None, initial_epoch=0,
            steps_per_epoch=None, validation_steps=None, validation_batch_size=None, validation_freq=1,
            max_queue_size=10, workers=1, use_multiprocessing=False):
        kw = dict(x=x, y=y, batch_size=batch_size, epochs=epochs, verbose=verbose, callbacks=callbacks,
                  validation_split=validation_split, validation_data=validation_data, shuffle=shuffle,
                  class_weight=class_weight, sample_weight=sample_weight, initial_epoch=initial_epoch,
                  steps_per_epoch=steps_per_epoch, validation_steps=validation_steps,
                  validation_batch_size=validation_batch_size, validation_freq=validation_freq)
        # (single-process multi-device MirroredStrategy: the same ONE loop; its trainer drives every
        # local replica, engine/mirrored.py)
        return self._fit_impl(**kw)

    def _fit_impl(self, x=None, y=None, batch_size=None, epochs=1, verbose="auto", callbacks=None,
                  validation_split=0.0, validation_data=None, shuffle=True, class_weight=None, sample_weight=None,
                  initial_epoch=0, steps_per_epoch=None, validation_steps=None, validation_batch_size=None,
                  validation_freq=1):
        strategy = self._get_strategy()
        if validation_split and not isinstance(x, D.Dataset):
            n = len(x)
            cut = int(n * (1 - validation_split))
            validation_data = (x[cut:], y[cut:])
            x, y = x[:cut], y[:cut]
        ds = self._adapt(x, y, batch_size, shuffle, sample_weight)
        self._peek_build(ds)
        trainer = self._get_trainer()
        group = getattr(trainer, "is_group", False)
        if group:
            trainer.broadcast_from_primary()  # weights / optimizer state set since the last fit
        handler = trainer.prepare(ds) if hasattr(trainer, "prepare") else None
        if handler is None:
            if trainer.kind == "fused":
                # pipeline not lowerable to the device: generic engine (host data path)
                if group:
                    from ..engine.mirrored import ThreadedGroupTrainer, _models_and_group

                    self._trainer = trainer = ThreadedGroupTrainer(self, *_models_and_group(self))
                else:
                    from ..engine.trainer import GenericTrainer

                    self._trainer = trainer = GenericTrainer(self)
                self._fused_reason = "input pipeline is not device-resident"
            if hasattr(trainer, "host_handler"):
                handler = trainer.host_handler(ds)
            else:
                from ..engine.trainer import HostDataHandler

                handler = HostDataHandler(ds, strategy)
        if verbose == "auto":
            verbose = 1
        steps = steps_per_epoch
        if steps is None:
            c = handler.dist.cardinality() if hasattr(handler, "dist") else _lowered_steps(handler)
            steps = c if c is not None and c >= 0 else None
        history = cbks.History()
        cb_list = cbks.CallbackList(list(callbacks or []) + [cbks.ProgbarLogger(), history], model=self,
                                    params={"epochs": epochs, "steps": steps, "verbose": verbose if self._is_chief() else 0})
        self.stop_training = False
        self._initial_epoch_override = None
        cb_list.on_train_begin()
        if group:
            trainer.broadcast_from_primary()  # e.g. BackupAndRestore restored replica 0
        if self._initial_epoch_override is not None:
            initial_epoch = max(initial_epoch, self._initial_epoch_override)
        want_batch = cb_list.wants_batch_logs or (verbose == 1 and sys.stdout.isatty())
        # replica-consistency checks (one 2-word collective each, parallel/consistency.py): every
        # TDL_CHECK_REPLICAS_EVERY epochs (default 1) and every TDL_CHECK_REPLICAS_EXECUTIONS
        # executions (default 100), plus once at the end of fit; 0 disables either
        check_epochs = int(os.environ.get("TDL_CHECK_REPLICAS_EVERY", "1") or 0)
        check_exec = int(os.environ.get("TDL_CHECK_REPLICAS_EXECUTIONS", "100") or 0)
        self._executions = getattr(self, "_executions", 0)
        K = max(1, self._steps_per_execution)
        persistent = steps_per_epoch is not None  # Q5: one iterator across epochs
        handler.new_iterator()
        exhausted = False
        logs = {}
        from ..utils import fault as _fault

        for epoch in range(initial_epoch, epochs):
            self._current_epoch = epoch
            trainer.reset_metrics()
            if not persistent and epoch > initial_epoch:
                handler.new_iterator()
            cb_list.on_epoch_begin(epoch)
            done = 0
            while steps is None or done < steps:
                n = K if steps is None else min(K, steps - done)
                if want_batch:
                    cb_list.on_train_batch_begin(done)
                got = _run_guarded(trainer, handler, n, strategy, self)
                done += got
                self._executions += 1
                if check_exec > 0 and self._executions % check_exec == 0:
                    self._check_replicas(trainer)
                if want_batch and got:
                    cb_list.on_train_batch_end(done - 1, _LazyLogs(trainer))
                if got < n:
                    if steps is not None and persistent:
                        exhausted = True
                    break
                if self.stop_training:
                    break
            cb_list.params["seen_steps"] = done
            _fault.note_progress(busy=True)  # the log read waits on the device and on peers
            logs = dict(trainer.logs())
            _fault.note_progress(busy=False)  # callbacks (chief checkpoints, validation) run now
            if validation_data is not None and (epoch + 1) % validation_freq == 0:
                val = self.evaluate(validation_data if isinstance(validation_data, D.Dataset) else
                                    validation_data[0], None if isinstance(validation_data, D.Dataset) else
                                    validation_data[1], batch_size=validation_batch_size or batch_size,
                                    steps=validation_steps, verbose=0, return_dict=True, _internal=True)
                logs.update({f"val_{k}": v for k, v in val.items()})
                trainer = self._get_trainer()
            cb_list.on_epoch_end(epoch, logs)
            if check_epochs > 0 and (epoch + 1) % check_epochs == 0:
                self._check_replicas(trainer)
            if exhausted:
                if self._is_chief():
                    warnings.warn("Your input ran out of data; interrupting training. Make sure that your dataset "
                                  "can generate at least `steps_per_epoch * epochs` batches (use .repeat()).")
                break
            if self.stop_training:
                break
        trainer.finish()
        _fault.note_progress(busy=False)
        if hasattr(handler, "close"):  # stop an index producer, commit the epochs it consumed
            handler.close()
        if os.environ.get("TDL_CHECK_REPLICAS", "1") == "1":
            self._check_replicas(trainer)
        cb_list.on_train_end(logs)
        self.history = history
        return history

    def _check_replicas(self, trainer):
        """Collective: the mirrored parameters must be bit-identical on every replica
        (README.md:15-17).  On a mismatch rank 0's copy is broadcast and the trainer drops its
        custom all-reduce path (parallel/consistency.py)."""
        from ..parallel import consistency

        if hasattr(trainer, "check_replicas"):  # one process, G replicas: compared in-process
            trainer.check_replicas()
            return
        comm = self._get_strategy().extended.communicator
        if comm.world_size == 1 or self._W is None:
            return
        if not consistency.check_and_repair(comm, self._W):
            if hasattr(trainer, "on_replica_divergence"):
                trainer.on_replica_divergence()

    # ------------------------------------------------------------------ evaluate / predict
    def evaluate(self, x=None, y=None, batch_size=None, verbose="auto", sample_weight=None, steps=None,
                 callbacks=None, return_dict=False, _internal=False, **kw):
        args = dict(x=x, y=y, batch_size=batch_size, verbose=verbose, sample_weight=sample_weight, steps=steps,
                    callbacks=callbacks, return_dict=return_dict, _internal=_internal)
        if self._outer_local_group() is not None:
            tr = self._trainer
            if (getattr(tr, "is_group", False) and tr.kind == "fused" and sample_weight is None and
                    os.environ.get("TDL_FUSED_EVAL", "1") == "1"):
                # every replica's slice on its own device from this thread (engine/mirrored.py)
                ds = self._adapt(x, y, batch_size, False, None)
                out = tr.evaluate(ds, steps)
                if out is not None:
                    return self._eval_result(out, verbose, return_dict, _internal)
            return self._local_run("evaluate", args)
        return self._evaluate_impl(**args)

    def _eval_result(self, out, verbose, return_dict, _internal):
        if verbose and verbose != "auto" and self._is_chief() and not _internal:
            from ..utils.progbar import format_logs

            print(format_logs(out))
        if return_dict:
            return out
        vals = [out[k] for k in ["loss"] + [m.name for m in self.compiled_metrics]]
        return vals if len(vals) > 1 else vals[0]

    def _replica_engine(self):
        """This replica's own engine (the group trainer's replica-0 engine for the user's model of a
        single-process multi-device MirroredStrategy), or None."""
        t = self._trainer
        if getattr(t, "is_group", False):
            return t.replica_trainer(self)
        return t

    def _evaluate_impl(self, x=None, y=None, batch_size=None, verbose="auto", sample_weight=None, steps=None,
                       callbacks=None, return_dict=False, _internal=False):
        from ..engine.trainer import GenericTrainer, HostDataHandler

        ds = self._adapt(x, y, batch_size, False, sample_weight)
        self._peek_build(ds)
        if self.optimizer is None:
            raise RuntimeError("compile() the model before evaluate()")
        if sample_weight is None and os.environ.get("TDL_FUSED_EVAL", "1") == "1":
            tr = self._get_trainer()
            out = tr.evaluate(ds, steps) if tr.kind == "fused" else None
            if out is not None:  # forward-only pass on the MI355X kernels (engine/fused.py)
                return self._eval_result(out, verbose, return_dict, _internal)
        keep = self._trainer
        prev = self._replica_engine()
        self._ensure_slabs()
        ev = GenericTrainer.__new__(GenericTrainer)
        ev.model, ev.strategy = self, self._get_strategy()
        ev.device = ev.strategy.extended.device
        ev.comm = ev.strategy.extended.communicator
        ev.loss, ev.metrics = self.loss, self.compiled_metrics
        ev.loss_tracker = self._loss_tracker
        for v in self._trainable_vars:
            v._leaf = None
        saved = None
        if prev is not None and prev.kind == "fused":
            saved = prev.metrics_dev.clone()
        ev.reset_metrics()
        h = HostDataHandler(ds, ev.strategy)
        h.new_iterator()
        ev.run_test(h, steps)
        out = ev.logs()
        self._trainer = keep
        if prev is not None and prev.kind == "generic":
            prev._make_leaves()
        if saved is not None:
            prev.metrics_dev.copy_(saved)
        return self._eval_result(out, verbose, return_dict, _internal)

    def predict(self, x, batch_size=None, verbose="auto", steps=None, callbacks=None, **kw):
        args = dict(x=x, batch_size=batch_size, verbose=verbose, steps=steps, callbacks=callbacks)
        # (single-process multi-device MirroredStrategy too: inference is replica-independent, so
        # replica 0 predicts every sample on its own device)
        return self._predict_impl(**args)

    @torch.no_grad()
    def _predict_impl(self, x, batch_size=None, verbose="auto", steps=None, callbacks=None):
        dev = self._get_strategy().extended.device
        if isinstance(x, D.Dataset):
            ds = x
        else:
            ds = D.Dataset.from_tensor_slices(x).batch(batch_size or 32)
        self._peek_build(ds)
        tr = self._trainer
        if tr is None and self.optimizer is not None and self.loss is not None:
            tr = self._get_trainer()
        if tr is not None and tr.kind == "fused" and os.environ.get("TDL_FUSED_EVAL", "1") == "1":
            out = tr.predict(ds, steps)
            if out is not None:  # forward-only pass on the MI355X kernels (engine/fused.py)
                return out
        if self._W is not None:
            for v in self._trainable_vars:
                v._leaf = None
        outs = []
        for k, b in enumerate(ds):
            if steps is not None and k >= steps:
                break
            xb = b[0] if isinstance(b, (tuple, list)) else b
            outs.append(_map_outputs(lambda t: t.cpu(), self(xb.to(dev), training=False)))
        rt = self._replica_engine()
        if rt is not None and rt.kind == "generic":
            rt._make_leaves()
        # (a multi-output model returns one array per output, in its output structure, as Keras does)
        return _concat_outputs(outs)

    def predict_on_batch(self, x):
        return self.predict(x, batch_size=len(x))

    def train_on_batch(self, x, y=None, sample_weight=None, return_dict=False, **kw):
        ds = D.Dataset.from_tensor_slices((x, y)).batch(len(x))
        h = self.fit(ds, epochs=1, verbose=0)
        out = {k: v[-1] for k, v in h.history.items()}
        return out if return_dict else list(out.values())

    # ------------------------------------------------------------------ weights
    def get_weights(self):
        return [w.numpy() for w in self.weights]

    def set_weights(self, weights):
        Layer.set_weights(self, weights)

    def load_named_tensors(self, tensors: Dict[str, torch.Tensor], strict: bool = True):
        missing = []
        ws = self.weights
        names = [w.name for w in ws]
        cand = [(k, t) for k, t in tensors.items() if not k.startswith("optimizer/")]
        if not any(n in tensors or n[:-2] in tensors for n in names) and len(cand) == len(ws) and \
                all(tuple(t.shape) == tuple(w.shape) for (_, t), w in zip(cand, ws)):
            # object-graph order matching (TF checkpoints match objects, not layer names)
            for (_, t), w in zip(cand, ws):
                w.assign(t)
            return
        by_name = {w.name: w for w in ws}
        for name, v in by_name.items():
            key = name if name in tensors else name[:-2] if name.endswith(":0") and name[:-2] in tensors else None
            if key is None:
                missing.append(name)
                continue
            v.assign(tensors[key])
        if strict and missing:
            raise ValueError(f"checkpoint is missing variables: {missing}")

    def save_weights(self, filepath, overwrite=True, save_format=None, options=None):
        from ..ckpt import checkpoint as ck

        import os

        d = os.path.dirname(filepath) or "."
        wd = ck.write_dirpath(d, self._get_strategy())
        ck.write_bundle(os.path.join(wd, os.path.basename(filepath)), ck.model_tensors(self))
        if self._is_chief():
            ck._update_checkpoint_state(d, os.path.basename(filepath))
        if wd != d:
            ck.remove_temp_dirpath(wd, self._get_strategy())

    def load_weights(self, filepath, by_name=False, skip_mismatch=False, options=None):
        from ..ckpt import checkpoint as ck

        import os

        if os.path.isdir(filepath):
            p = ck.latest_checkpoint(filepath)
            if p is None:
                p = os.path.join(filepath, "variables", "variables")
            filepath = p
        tensors = ck.read_bundle(filepath)
        if not self.built:
            raise ValueError("build the model before load_weights()")
        self.load_named_tensors(tensors, strict=not (by_name or skip_mismatch))
        return self

    def save(self, filepath, overwrite=True, include_optimizer=True, save_format=None, **kw):
        from ..ckpt.checkpoint import save_model

        save_model(self, str(filepath), overwrite=overwrite, include_optimizer=include_optimizer)

    # ------------------------------------------------------------------ config / summary
    def get_config_full(self):
        if isinstance(self, Sequential):
            return {"class_name": "Sequential", "config": {
                "name": self.name,
                "build_input_shape": list(self._built_input_shape) if self._built_input_shape else None,
                "layers": [{"class_name": type(l).__name__, "config": l.get_config()} for l in self.layers]}}
        if self._functional:
            layers = []
            for n in self._nodes:
                ins = [[t._node.layer.name, t._index] for t in _flat(n.inputs)]
                layers.append({"class_name": type(n.layer).__name__, "config": n.layer.get_config(),
                               "name": n.layer.name, "inbound": ins,
                               "list_input": isinstance(n.inputs, (list, tuple))})
            return {"class_name": "Functional", "config": {
                "name": self.name,
                "inputs": [{"name": t.name, "shape": list(t.shape[1:])} for t in self._inputs],
                "layers": layers,
                "outputs": [[t._node.layer.name, t._index] for t in _flat(self._outputs)]}}
        return {"class_name": type(self).__name__, "config": {"name": self.name}, "subclassed": True}

    def get_config(self):
        return self.get_config_full()["config"]

    def summary(self, line_length=80, print_fn=None):
        pf = print_fn or print
        pf(f'Model: "{self.name}"')
        pf("_" * line_length)
        pf(f"{'Layer (type)':<34}{'Output Shape':<28}{'Param #':>12}")
        pf("=" * line_length)
        shape = self._built_input_shape
        for l in self.layers:
            try:
                shape = l.compute_output_shape(shape) if shape is not None and not self._functional else None
            except Exception:
                shape = None
            pf(f"{l.name + ' (' + type(l).__name__ + ')':<34}{str(shape):<28}{l.count_params():>12,}")
        pf("=" * line_length)
        tp = sum(math.prod(w.shape) for w in self.trainable_weights)
        ntp = sum(math.prod(w.shape) for w in self.non_trainable_weights)
        pf(f"Total params: {tp + ntp:,}")
        pf(f"Trainable params: {tp:,}")
        pf(f"Non-trainable params: {ntp:,}")
        pf("_" * line_length)


class _LazyLogs:
    def __new__(cls, trainer):
        from ..engine.trainer import LazyLogs

        return LazyLogs(trainer.logs)


def _lowered_steps(handler):
    lp = getattr(handler, "lp", None)
    if lp is None or lp.repeat is None:
        return None
    B = lp.batch_size
    per = lp.n // B if lp.drop_remainder else -(-lp.n // B)
    return per * lp.repeat if not lp.batch_crosses_epochs else (lp.n * lp.repeat) // B


class Sequential(Model):
    def __init__(self, layers=None, name=None, **kw):
        super().__init__(name=name, **kw)
        self._seq: List[Layer] = []
        for l in layers or []:
            self.add(l)

    @property
    def layers(self):
        return list(self._seq)

    def add(self, layer: Layer):
        if isinstance(layer, KerasTensor):
            layer = layer._node.layer
        if isinstance(layer, InputLayer):
            self._batch_input_shape = layer._batch_input_shape
            self._seq_input = layer
        else:
            self._seq.append(layer)
            if layer not in self._layers:
                self._layers.append(layer)
        first_shape = self._batch_input_shape or (self._seq[0]._batch_input_shape if self._seq else None)
        if first_shape is not None:
            self._build_layers(first_shape)

    def pop(self):
        l = self._seq.pop()
        self._layers.remove(l)
        self.built = False
        return l

    def _build_layers(self, input_shape):
        shape = tuple(input_shape)
        for l in self._seq:
            if not l.built:
                l._maybe_build(shape)
            shape = l.compute_output_shape(shape)
        self._built_input_shape = tuple(input_shape)
        self._output_shape = shape
        self.built = True

    def build(self, input_shape=None):
        if input_shape is None:
            input_shape = self._batch_input_shape or self._seq[0]._batch_input_shape
        self._build_layers(input_shape)

    def call(self, x, training=None):
        seq, i = self._seq, 0
        fuse = bool(training) and isinstance(x, torch.Tensor) and x.is_cuda
        while i < len(seq):
            if fuse and i + 1 < len(seq):
                from .layers import conv_pool_pair

                if conv_pool_pair(seq[i], seq[i + 1]):
                    # Conv2D -> MaxPooling2D(2): one forward launch on the generic f32 path (Conv2D.call)
                    x = seq[i](x, training=training, _pool=seq[i + 1])
                    i += 2
                    continue
            x = seq[i](x, training=training)
            i += 1
        return x

    def compute_output_shape(self, s):
        for l in self._seq:
            s = l.compute_output_shape(s)
        return s


def model_from_config(cfg):
    from .layers import LAYER_CLASSES, Input

    cls = cfg["class_name"]
    c = cfg["config"]
    if cls == "Sequential":
        layers = []
        for lc in c["layers"]:
            k = LAYER_CLASSES[lc["class_name"]]
            layers.append(k.from_config(_clean_cfg(lc["config"])))
        m = Sequential(layers, name=c.get("name"))
        if not m.built and c.get("build_input_shape"):
            m.build(tuple(c["build_input_shape"]))
        return m
    if cls == "Functional":
        tensors = {}
        inputs = []
        for i in c["inputs"]:
            t = Input(shape=tuple(i["shape"]), name=i["name"])
            tensors[(i["name"], 0)] = t
            inputs.append(t)
        for lc in c["layers"]:
            layer = LAYER_CLASSES[lc["class_name"]].from_config(_clean_cfg(lc["config"]))
            args = [tensors[(n, i)] for n, i in lc["inbound"]]
            out = layer(args if lc.get("list_input") else args[0])
            for j, t in enumerate(out if isinstance(out, list) else [out]):
                tensors[(lc["name"], j)] = t
        outs = [tensors[(n, i)] for n, i in c["outputs"]]
        return Model(inputs, outs[0] if len(outs) == 1 else outs, name=c.get("name"))
    raise ValueError(f"cannot rebuild a {cls} model from its config (subclassed models: use save_weights)")


def _clean_cfg(c):
    from . import activations, initializers

    c = dict(c)
    c.pop("trainable", None)
    for k in ("kernel_initializer", "bias_initializer"):
        if isinstance(c.get(k), dict):
            c[k] = initializers.get(c[k])
    if "batch_input_shape" in c:
        c["batch_input_shape"] = tuple(c["batch_input_shape"])
    for k in ("kernel_size", "strides", "pool_size", "dilation_rate"):
        if isinstance(c.get(k), list):
            c[k] = tuple(c[k])
    return c


def load_model(path, compile=True, custom_objects=None):
    from ..ckpt.checkpoint import load_model as _lm

    return _lm(path, compile=compile)


def clone_model(model):
    return model_from_config(model.get_config_full())


def _run_guarded(trainer, handler, n, strategy, model=None):
    """One execution of ``n`` steps with failure detection (utils/fault.py): a collective that
    fails because a peer died is re-raised as PeerLostError with the watchdog's diagnosis, and the
    fault-injection hook runs at the execution boundary."""
    from ..utils import fault
    from ..utils.tracing import trace_range

    wd = getattr(strategy.extended, "watchdog", None)
    fault.note_progress(busy=True)
    try:
        with trace_range(f"tdl.execution[{n} steps]"):
            got = trainer.run_train(handler, n)
    except Exception as e:
        if wd is not None:
            deadline = time.monotonic() + 3 * wd.interval + 1.0
            while wd.reason is None and time.monotonic() < deadline:
                time.sleep(wd.interval / 4)
            if wd.reason is not None:
                wd.acknowledged = True
                raise fault.PeerLostError(f"{wd.reason} (collective failed: {e})") from e
        raise
    fault.note_progress(count=int(trainer.optimizer.iterations))
    fault.check()
    fault.maybe_inject(strategy.extended.rank, int(trainer.optimizer.iterations))
    if model is not None:
        fault.maybe_corrupt(strategy.extended.rank, int(trainer.optimizer.iterations), getattr(model, "_W", None))
    return got
