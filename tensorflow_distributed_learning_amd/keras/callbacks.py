"""Keras callbacks.  ``fit`` always adds History + ProgbarLogger (tf_dist_example.py:59); the
chief-only side effects of README.md:51 are ModelCheckpoint / BackupAndRestore (checkpoints) and
TensorBoard (event files): non-chief workers run the same code but write to temporary paths
(ckpt/checkpoint.py) or not at all."""
from __future__ import annotations

import csv
import json
import math
import os
import time
from typing import Dict, List, Optional

from ..utils.progbar import Progbar


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None): ...
    def on_train_end(self, logs=None): ...
    def on_epoch_begin(self, epoch, logs=None): ...
    def on_epoch_end(self, epoch, logs=None): ...
    def on_train_batch_begin(self, batch, logs=None): ...
    def on_train_batch_end(self, batch, logs=None): ...
    def on_test_begin(self, logs=None): ...
    def on_test_end(self, logs=None): ...
    def on_test_batch_begin(self, batch, logs=None): ...
    def on_test_batch_end(self, batch, logs=None): ...
    def on_predict_begin(self, logs=None): ...
    def on_predict_end(self, logs=None): ...
    def on_predict_batch_begin(self, batch, logs=None): ...
    def on_predict_batch_end(self, batch, logs=None): ...

    # which hooks need per-batch logs (forces a host sync per step when True)
    @property
    def _wants_batch_logs(self) -> bool:
        c = type(self)
        return c.on_train_batch_end is not Callback.on_train_batch_end or \
            c.on_train_batch_begin is not Callback.on_train_batch_begin


class CallbackList:
    def __init__(self, callbacks: Optional[List[Callback]] = None, model=None, params=None):
        self.callbacks = list(callbacks or [])
        self.params = params if params is not None else {}
        params = self.params  # shared dict: later updates (seen_steps) reach every callback
        for c in self.callbacks:
            if model is not None:
                c.set_model(model)
            if params is not None:
                c.set_params(params)

    def append(self, cb):
        self.callbacks.append(cb)

    def __iter__(self):
        return iter(self.callbacks)

    def _call(self, name, *args):
        for c in self.callbacks:
            getattr(c, name)(*args)

    def __getattr__(self, name):
        if name.startswith("on_"):
            return lambda *a: self._call(name, *a)
        raise AttributeError(name)

    @property
    def wants_batch_logs(self):
        return any(c._wants_batch_logs for c in self.callbacks if not isinstance(c, (ProgbarLogger, History)))


class History(Callback):
    def __init__(self):
        super().__init__()
        self.history: Dict[str, List[float]] = {}
        self.epoch: List[int] = []

    def on_train_begin(self, logs=None):
        self.epoch = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(float(v))
        if self.model is not None:
            self.model.history = self


class ProgbarLogger(Callback):
    def __init__(self, count_mode="steps", stateful_metrics=None):
        super().__init__()
        self.verbose = 1
        self.epochs = 1
        self._bar = None

    def set_params(self, params):
        super().set_params(params)
        self.verbose = params.get("verbose", 1)
        self.epochs = params.get("epochs", 1)

    def _active(self):
        return self.verbose and (self.model is None or self.model._is_chief())

    def on_epoch_begin(self, epoch, logs=None):
        if self._active():
            if self.epochs > 1 or self.verbose == 1:
                print(f"Epoch {epoch + 1}/{self.epochs}", flush=True)
            self._bar = Progbar(self.params.get("steps"), verbose=self.verbose)

    def on_train_batch_end(self, batch, logs=None):
        if self._active() and self._bar is not None and logs is not None:
            self._bar.update(batch + 1, logs, finalize=False)

    def on_epoch_end(self, epoch, logs=None):
        if self._active() and self._bar is not None:
            logs = logs or {}
            self._bar.update(self.params.get("seen_steps", self._bar._seen) or self._bar._seen, logs, finalize=True)


class LambdaCallback(Callback):
    def __init__(self, on_epoch_begin=None, on_epoch_end=None, on_batch_begin=None, on_batch_end=None,
                 on_train_begin=None, on_train_end=None, **kw):
        super().__init__()
        if on_epoch_begin:
            self.on_epoch_begin = on_epoch_begin
        if on_epoch_end:
            self.on_epoch_end = on_epoch_end
        if on_batch_begin:
            self.on_train_batch_begin = on_batch_begin
        if on_batch_end:
            self.on_train_batch_end = on_batch_end
        if on_train_begin:
            self.on_train_begin = on_train_begin
        if on_train_end:
            self.on_train_end = on_train_end
        self._lambda_batch = bool(on_batch_begin or on_batch_end)

    @property
    def _wants_batch_logs(self):
        return self._lambda_batch


class EarlyStopping(Callback):
    def __init__(self, monitor="val_loss", min_delta=0, patience=0, verbose=0, mode="auto", baseline=None,
                 restore_best_weights=False, start_from_epoch=0):
        super().__init__()
        self.monitor, self.min_delta, self.patience = monitor, abs(min_delta), patience
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.baseline, self.restore_best_weights = baseline, restore_best_weights
        self.start_from_epoch = start_from_epoch
        self.stopped_epoch = 0

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.best = math.inf if self.mode == "min" else -math.inf
        self.best_weights = None

    def _better(self, a, b):
        return a < b - self.min_delta if self.mode == "min" else a > b + self.min_delta

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None or epoch < self.start_from_epoch:
            return
        if self._better(cur, self.best):
            self.best, self.wait = cur, 0
            if self.restore_best_weights:
                self.best_weights = self.model.get_weights()
        else:
            self.wait += 1
            if self.wait >= self.patience:
                self.stopped_epoch = epoch
                self.model.stop_training = True
                if self.restore_best_weights and self.best_weights is not None:
                    self.model.set_weights(self.best_weights)


class TerminateOnNaN(Callback):
    def on_epoch_end(self, epoch, logs=None):
        v = (logs or {}).get("loss")
        if v is not None and (math.isnan(v) or math.isinf(v)):
            print(f"Epoch {epoch}: invalid loss, terminating training")
            self.model.stop_training = True


class LearningRateScheduler(Callback):
    def __init__(self, schedule, verbose=0):
        super().__init__()
        self.schedule, self.verbose = schedule, verbose

    def on_epoch_begin(self, epoch, logs=None):
        opt = self.model.optimizer
        try:
            lr = self.schedule(epoch, opt.current_lr())
        except TypeError:
            lr = self.schedule(epoch)
        opt.learning_rate = float(lr)
        if self.verbose and self.model._is_chief():
            print(f"\nEpoch {epoch + 1}: LearningRateScheduler setting learning rate to {lr}.")

    def on_epoch_end(self, epoch, logs=None):
        if logs is not None:
            logs["lr"] = self.model.optimizer.current_lr()


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="val_loss", factor=0.1, patience=10, verbose=0, mode="auto", min_delta=1e-4,
                 cooldown=0, min_lr=0):
        super().__init__()
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.min_delta, self.cooldown, self.min_lr = min_delta, cooldown, min_lr

    def on_train_begin(self, logs=None):
        self.wait, self.cd = 0, 0
        self.best = math.inf if self.mode == "min" else -math.inf

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None:
            return
        better = cur < self.best - self.min_delta if self.mode == "min" else cur > self.best + self.min_delta
        if self.cd > 0:
            self.cd -= 1
            self.wait = 0
        if better:
            self.best, self.wait = cur, 0
        elif self.cd == 0:
            self.wait += 1
            if self.wait >= self.patience:
                opt = self.model.optimizer
                opt.learning_rate = max(opt.current_lr() * self.factor, self.min_lr)
                self.cd, self.wait = self.cooldown, 0


class CSVLogger(Callback):
    def __init__(self, filename, separator=",", append=False):
        super().__init__()
        self.filename, self.sep, self.append = filename, separator, append
        self._keys = None

    def on_train_begin(self, logs=None):
        if not self.model._is_chief():
            self._f = None
            return
        self._f = open(self.filename, "a" if self.append else "w", newline="")
        self._w = None

    def on_epoch_end(self, epoch, logs=None):
        if self._f is None:
            return
        logs = logs or {}
        if self._w is None:
            self._keys = sorted(logs)
            self._w = csv.writer(self._f, delimiter=self.sep)
            if not self.append or self._f.tell() == 0:
                self._w.writerow(["epoch"] + self._keys)
        self._w.writerow([epoch] + [logs.get(k) for k in self._keys])
        self._f.flush()

    def on_train_end(self, logs=None):
        if self._f is not None:
            self._f.close()


class ModelCheckpoint(Callback):
    """Chief saves to ``filepath`` (formatted with epoch/logs); other workers to a temp dir."""

    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False, save_weights_only=False,
                 mode="auto", save_freq="epoch", initial_value_threshold=None):
        super().__init__()
        self.filepath, self.monitor, self.verbose = str(filepath), monitor, verbose
        self.save_best_only, self.save_weights_only = save_best_only, save_weights_only
        self.mode = mode if mode != "auto" else ("max" if "acc" in monitor else "min")
        self.save_freq = save_freq
        self.best = initial_value_threshold
        self._batches = 0

    def _save(self, epoch, logs):
        logs = logs or {}
        if self.save_best_only:
            cur = logs.get(self.monitor)
            if cur is None:
                return
            if self.best is not None and not (cur < self.best if self.mode == "min" else cur > self.best):
                return
            self.best = cur
        path = self.filepath.format(epoch=epoch + 1, **logs)
        if self.save_weights_only:
            self.model.save_weights(path)
        else:
            self.model.save(path)
        if self.verbose and self.model._is_chief():
            print(f"\nEpoch {epoch + 1}: saving model to {path}")

    def on_epoch_end(self, epoch, logs=None):
        if self.save_freq == "epoch":
            self._save(epoch, logs)

    def on_train_batch_end(self, batch, logs=None):
        if isinstance(self.save_freq, int):
            self._batches += 1
            if self._batches % self.save_freq == 0:
                self._save(self.model._current_epoch, logs)

    @property
    def _wants_batch_logs(self):
        return isinstance(self.save_freq, int)


class BackupAndRestore(Callback):
    """Fault tolerance (tf.keras.callbacks.BackupAndRestore): back up model + optimizer + epoch at
    every epoch end; on restart ``fit`` resumes from the last completed epoch."""

    def __init__(self, backup_dir, save_freq="epoch", delete_checkpoint=True):
        super().__init__()
        self.backup_dir = backup_dir
        self.save_freq = save_freq
        self.delete_checkpoint = delete_checkpoint
        self._batches = 0

    def _ckpt(self):
        from ..ckpt.checkpoint import Checkpoint

        return Checkpoint(model=self.model, optimizer=self.model.optimizer,
                          training_state={"epoch": self.model._current_epoch_tensor})

    def on_train_begin(self, logs=None):
        from ..ckpt.checkpoint import latest_checkpoint

        self.model._current_epoch_tensor = __import__("torch").tensor(-1, dtype=__import__("torch").int64)
        p = latest_checkpoint(self.backup_dir)
        if p:
            self._ckpt().restore(p)
            self.model._initial_epoch_override = int(self.model._current_epoch_tensor) + 1

    def on_epoch_end(self, epoch, logs=None):
        from ..ckpt.checkpoint import CheckpointManager

        self.model._current_epoch_tensor.fill_(epoch)
        CheckpointManager(self._ckpt(), self.backup_dir, max_to_keep=1).save()

    def on_train_end(self, logs=None):
        import shutil

        if self.delete_checkpoint and self.model._is_chief() and not getattr(self.model, "stop_training_error", False):
            shutil.rmtree(self.backup_dir, ignore_errors=True)


class TensorBoard(Callback):
    """Chief writes scalar summaries to ``log_dir/train`` (and ``/validation``) as tfevents."""

    def __init__(self, log_dir="logs", histogram_freq=0, write_graph=True, write_images=False, update_freq="epoch",
                 profile_batch=0, **kw):
        super().__init__()
        self.log_dir = log_dir
        self.update_freq = update_freq
        self._writers = {}
        self._step = 0

    def _writer(self, sub):
        from ..utils.events import EventFileWriter

        if sub not in self._writers:
            self._writers[sub] = EventFileWriter(os.path.join(self.log_dir, sub))
        return self._writers[sub]

    def on_train_batch_end(self, batch, logs=None):
        self._step += 1
        if isinstance(self.update_freq, int) and self.model._is_chief() and self._step % self.update_freq == 0 and logs:
            self._writer("train").scalars({f"batch_{k}": v for k, v in logs.items()}, self._step)

    @property
    def _wants_batch_logs(self):
        return isinstance(self.update_freq, int)

    def on_epoch_end(self, epoch, logs=None):
        if not self.model._is_chief():
            return
        logs = logs or {}
        tr = {f"epoch_{k}": v for k, v in logs.items() if not k.startswith("val_")}
        va = {f"epoch_{k[4:]}": v for k, v in logs.items() if k.startswith("val_")}
        self._writer("train").scalars(tr, epoch)
        if va:
            self._writer("validation").scalars(va, epoch)
        for w in self._writers.values():
            w.flush()

    def on_train_end(self, logs=None):
        for w in self._writers.values():
            w.close()
        self._writers = {}
