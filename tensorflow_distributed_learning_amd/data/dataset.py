"""tf.data-style input pipelines (tf_dist_example.py:20-37, README.md:113-129).

A :class:`Dataset` is an immutable description of a pipeline; iterating it yields elements
(nested tuples / dicts of ``torch.Tensor``).  Implemented transformations: ``from_tensor_slices``,
``from_tensors``, ``from_generator``, ``range``, ``zip``, ``list_files``, ``TextLineDataset``,
``map``, ``filter``, ``cache``, ``shuffle``, ``batch``, ``unbatch``, ``repeat``, ``take``,
``skip``, ``shard``, ``prefetch``, ``with_options``, ``concatenate``, ``enumerate``, ``apply``,
``reduce``, ``as_numpy_iterator``.

Columnar fast path: pipelines whose data is in memory (``from_tensor_slices``, a materialised
``cache()``) are kept as whole columns; ``shuffle`` then permutes *indices* (TF's buffered
shuffle algorithm on indices) and ``batch`` gathers rows with one ``index_select`` per column.
An element-wise ``map`` over columns is executed once on the whole column when it verifiably
equals the per-element result (Options.experimental_optimization.map_vectorization).
These columnar sources are also what ``Model.fit`` lowers to a device-resident dataset in HBM
(data/device.py), so the reference's ``map(scale).cache().shuffle().batch()`` pipeline costs no
host work or H2D copies in the training loop.
"""
from __future__ import annotations

import glob as _glob
import os
import queue
import threading
import warnings
from typing import Any, Callable, Iterator, List, Optional, Sequence

import numpy as np
import torch

from .options import AutoShardPolicy, Options

AUTOTUNE = -1
INFINITE_CARDINALITY = -1
UNKNOWN_CARDINALITY = -2


# ------------------------------------------------------------------------------------------------
# structure helpers
def _to_tensor(x):
    if isinstance(x, torch.Tensor):
        return x
    if isinstance(x, np.ndarray):
        if x.dtype == np.object_ or x.dtype.kind in "US":
            return x
        return torch.from_numpy(np.ascontiguousarray(x))
    if isinstance(x, (bool, int, float)):
        return torch.tensor(x)
    if isinstance(x, (bytes, str)):
        return x
    if isinstance(x, (list, tuple)) and x and not isinstance(x[0], (list, tuple, dict, np.ndarray, torch.Tensor)):
        return torch.as_tensor(np.asarray(x))
    return torch.as_tensor(x)


def map_structure(fn, *structs):
    s0 = structs[0]
    if isinstance(s0, dict):
        return {k: map_structure(fn, *[s[k] for s in structs]) for k in s0}
    if isinstance(s0, tuple) and hasattr(s0, "_fields"):
        return type(s0)(*[map_structure(fn, *xs) for xs in zip(*structs)])
    if isinstance(s0, (tuple, list)):
        return type(s0)(map_structure(fn, *xs) for xs in zip(*structs))
    return fn(*structs)


def flatten(s) -> List[Any]:
    if isinstance(s, dict):
        out = []
        for k in s:
            out += flatten(s[k])
        return out
    if isinstance(s, (tuple, list)):
        out = []
        for x in s:
            out += flatten(x)
        return out
    return [s]


def _normalize_input(x):
    if isinstance(x, dict):
        return {k: _normalize_input(v) for k, v in x.items()}
    if isinstance(x, tuple):
        return tuple(_normalize_input(v) for v in x)
    if isinstance(x, list) and x and isinstance(x[0], (np.ndarray, torch.Tensor, list, tuple)):
        # a list of arrays is one tensor (TF converts nested lists) unless heterogeneous
        try:
            return _to_tensor(np.asarray(x))
        except Exception:
            return tuple(_normalize_input(v) for v in x)
    return _to_tensor(x)


def _apply(fn, elem):
    if isinstance(elem, tuple) and not hasattr(elem, "_fields"):
        return fn(*elem)
    return fn(elem)


def _stack(elems: List[Any]):
    return map_structure(lambda *xs: torch.stack([_to_tensor(x) for x in xs]) if isinstance(xs[0], torch.Tensor)
                         else list(xs), *elems)


def _take_rows(cols, idx: torch.Tensor):
    n = int(idx.numel())
    lo = int(idx[0]) if n else 0
    # a contiguous run of rows (unshuffled batch) is a view, not a gather
    contiguous = n > 0 and int(idx[-1]) - lo == n - 1 and bool(torch.all(idx[1:] - idx[:-1] == 1))

    def take(c):
        if not isinstance(c, torch.Tensor):
            return [c[i] for i in idx.tolist()]
        if contiguous:
            return c.narrow(0, lo, n)
        return c.index_select(0, idx.to(c.device))

    return map_structure(take, cols)


def _num_rows(cols) -> int:
    leaves = flatten(cols)
    return len(leaves[0]) if leaves else 0


class _SeedState(threading.local):
    override: Optional[int] = None


_seed_state = _SeedState()
_global_seed: Optional[int] = None


def set_global_seed(seed: Optional[int]):
    global _global_seed
    _global_seed = seed


# ------------------------------------------------------------------------------------------------
class Dataset:
    """Base class.  Subclasses implement ``_iter()`` and optionally ``_columns()``."""

    _inputs: Sequence["Dataset"] = ()

    # --------------------------------------------------------------------- construction
    @staticmethod
    def from_tensor_slices(tensors) -> "Dataset":
        return TensorSliceDataset(_normalize_input(tensors))

    @staticmethod
    def from_tensors(tensors) -> "Dataset":
        return TensorDataset(_normalize_input(tensors))

    @staticmethod
    def from_generator(generator, output_types=None, output_shapes=None, args=None, output_signature=None):
        return GeneratorDataset(generator, args or ())

    @staticmethod
    def range(*args, dtype=torch.int64) -> "Dataset":
        return RangeDataset(*args, dtype=dtype)

    @staticmethod
    def zip(*datasets) -> "Dataset":
        if len(datasets) == 1 and isinstance(datasets[0], (tuple, list, dict)):
            datasets = datasets[0]
        return ZipDataset(datasets)

    @staticmethod
    def list_files(file_pattern, shuffle=None, seed=None) -> "Dataset":
        pats = [file_pattern] if isinstance(file_pattern, str) else list(file_pattern)
        files = sorted({f for p in pats for f in _glob.glob(p)})
        if not files:
            raise ValueError(f"no files match {file_pattern}")
        ds = FileListDataset(files)
        if shuffle is None or shuffle:
            ds = ds.shuffle(len(files), seed=seed)
        return ds

    # --------------------------------------------------------------------- transformations
    def map(self, map_func: Callable, num_parallel_calls=None, deterministic=None, name=None) -> "Dataset":
        return MapDataset(self, map_func)

    def filter(self, predicate: Callable, name=None) -> "Dataset":
        return FilterDataset(self, predicate)

    def cache(self, filename: str = "", name=None) -> "Dataset":
        return CacheDataset(self, filename)

    def shuffle(self, buffer_size: int, seed: Optional[int] = None, reshuffle_each_iteration: Optional[bool] = None,
                name=None) -> "Dataset":
        return ShuffleDataset(self, buffer_size, seed, True if reshuffle_each_iteration is None else reshuffle_each_iteration)

    def batch(self, batch_size: int, drop_remainder: bool = False, num_parallel_calls=None, deterministic=None,
              name=None) -> "Dataset":
        return BatchDataset(self, int(batch_size), bool(drop_remainder))

    def unbatch(self, name=None) -> "Dataset":
        return UnbatchDataset(self)

    def repeat(self, count: Optional[int] = None, name=None) -> "Dataset":
        return RepeatDataset(self, count)

    def take(self, count: int, name=None) -> "Dataset":
        return TakeDataset(self, int(count))

    def skip(self, count: int, name=None) -> "Dataset":
        return SkipDataset(self, int(count))

    def shard(self, num_shards: int, index: int, name=None) -> "Dataset":
        if not 0 <= index < num_shards:
            raise ValueError("shard index must be in [0, num_shards)")
        return ShardDataset(self, int(num_shards), int(index))

    def prefetch(self, buffer_size: int = AUTOTUNE, name=None) -> "Dataset":
        return PrefetchDataset(self, buffer_size)

    def with_options(self, options: Options, name=None) -> "Dataset":
        return OptionsDataset(self, options)

    def concatenate(self, dataset: "Dataset", name=None) -> "Dataset":
        return ConcatenateDataset(self, dataset)

    def enumerate(self, start: int = 0, name=None) -> "Dataset":
        return ZipDataset((RangeDataset(start, None), self))

    def apply(self, transformation_func: Callable) -> "Dataset":
        return transformation_func(self)

    def rebatch(self, batch_size, drop_remainder=False, name=None) -> "Dataset":
        return self.unbatch().batch(batch_size, drop_remainder)

    def reduce(self, initial_state, reduce_func):
        state = initial_state
        for e in self:
            state = reduce_func(state, e)
        return state

    # --------------------------------------------------------------------- introspection
    def options(self) -> Options:
        o = Options()
        for inp in self._inputs:
            o = o.merge(inp.options())
        return o

    def cardinality(self) -> int:
        return UNKNOWN_CARDINALITY

    def __len__(self):
        c = self.cardinality()
        if c < 0:
            raise TypeError("dataset length is infinite or unknown")
        return c

    @property
    def element_spec(self):
        e = next(iter(self.take(1)))
        return map_structure(lambda t: TensorSpec(tuple(t.shape), t.dtype) if isinstance(t, torch.Tensor) else type(t), e)

    def source_files(self) -> Optional[List[str]]:
        for inp in self._inputs:
            f = inp.source_files()
            if f is not None:
                return f
        return None

    def _columns(self):
        """In-memory columns (structure of tensors with a common leading dim) or None."""
        return None

    def _index_stream(self, cols_len: int) -> Optional[Iterator[int]]:
        """For columnar pipelines: the order in which rows are produced (None = not columnar).
        Consumes one iteration (a shuffle draws its next epoch's order)."""
        return None

    def _identity_order(self) -> bool:
        """Columnar AND rows come out in storage order (no shuffle below)."""
        return False

    def __iter__(self) -> Iterator:
        return iter(self._iter())

    def _iter(self):
        raise NotImplementedError

    def as_numpy_iterator(self):
        for e in self:
            yield map_structure(lambda t: t.numpy() if isinstance(t, torch.Tensor) else t, e)

    def __repr__(self):
        return f"<{type(self).__name__}>"


class TensorSpec:
    def __init__(self, shape, dtype):
        self.shape, self.dtype = shape, dtype

    def __repr__(self):
        return f"TensorSpec(shape={self.shape}, dtype={self.dtype})"


# ------------------------------------------------------------------------------------------------
class TensorSliceDataset(Dataset):
    def __init__(self, cols):
        n = {len(x) for x in flatten(cols)}
        if len(n) != 1:
            raise ValueError(f"from_tensor_slices: all components need the same leading dimension, got {n}")
        self._cols = cols
        self._n = n.pop()

    def _columns(self):
        return self._cols

    def _index_stream(self, n):
        return iter(range(self._n))

    def _identity_order(self):
        return True

    def cardinality(self):
        return self._n

    def _iter(self):
        cols = self._cols
        for i in range(self._n):
            yield map_structure(lambda c: c[i], cols)


class TensorDataset(Dataset):
    def __init__(self, value):
        self._v = value

    def cardinality(self):
        return 1

    def _iter(self):
        yield self._v


class RangeDataset(Dataset):
    def __init__(self, *args, dtype=torch.int64):
        if len(args) == 2 and args[1] is None:
            self.start, self.stop, self.step = args[0], None, 1
        else:
            r = range(*args)
            self.start, self.stop, self.step = r.start, r.stop, r.step
        self.dtype = dtype

    def cardinality(self):
        if self.stop is None:
            return INFINITE_CARDINALITY
        return len(range(self.start, self.stop, self.step))

    def _columns(self):
        if self.stop is None:
            return None
        return torch.arange(self.start, self.stop, self.step, dtype=self.dtype)

    def _index_stream(self, n):
        return None if self.stop is None else iter(range(self.cardinality()))

    def _identity_order(self):
        return self.stop is not None

    def _iter(self):
        i = self.start
        while self.stop is None or (i < self.stop if self.step > 0 else i > self.stop):
            yield torch.tensor(i, dtype=self.dtype)
            i += self.step


class GeneratorDataset(Dataset):
    def __init__(self, gen, args):
        self._gen, self._args = gen, args

    def _iter(self):
        for e in self._gen(*self._args):
            yield _normalize_input(e)


class FileListDataset(Dataset):
    def __init__(self, files: List[str]):
        self.files = list(files)

    def source_files(self):
        return self.files

    def cardinality(self):
        return len(self.files)

    def _iter(self):
        for f in self.files:
            yield f


class TextLineDataset(Dataset):
    """tf.data.TextLineDataset(filenames): one element (str) per line; file based (FILE sharding)."""

    def __init__(self, filenames, compression_type=None, buffer_size=None):
        if isinstance(filenames, Dataset):
            self._files_ds = filenames
        else:
            self._files_ds = FileListDataset([filenames] if isinstance(filenames, str) else list(filenames))
        self._inputs = (self._files_ds,)

    def _iter(self):
        for f in self._files_ds:
            with open(f, "r") as fh:
                for line in fh:
                    yield line.rstrip("\n")


class ZipDataset(Dataset):
    def __init__(self, datasets):
        self._structure = datasets
        self._inputs = tuple(flatten(datasets)) if not isinstance(datasets, dict) else tuple(datasets.values())

    def cardinality(self):
        cs = [d.cardinality() for d in self._inputs]
        fin = [c for c in cs if c >= 0]
        if fin:
            return min(fin)
        return INFINITE_CARDINALITY if all(c == INFINITE_CARDINALITY for c in cs) else UNKNOWN_CARDINALITY

    def _iter(self):
        its = [iter(d) for d in self._inputs]
        while True:
            try:
                vals = [next(i) for i in its]
            except StopIteration:
                return
            if isinstance(self._structure, dict):
                yield dict(zip(self._structure.keys(), vals))
            else:
                yield tuple(vals)


class ConcatenateDataset(Dataset):
    def __init__(self, a, b):
        self._inputs = (a, b)

    def cardinality(self):
        a, b = (d.cardinality() for d in self._inputs)
        if a == INFINITE_CARDINALITY or b == INFINITE_CARDINALITY:
            return INFINITE_CARDINALITY
        if a < 0 or b < 0:
            return UNKNOWN_CARDINALITY
        return a + b

    def _iter(self):
        for d in self._inputs:
            yield from d


class MapDataset(Dataset):
    def __init__(self, inp, fn):
        self._inputs = (inp,)
        self.fn = fn
        self._vec = None  # cached vectorised columns (or False)

    def cardinality(self):
        return self._inputs[0].cardinality()

    def _columns(self):
        if self._vec is None:
            self._vec = self._try_vectorize()
        return self._vec if self._vec is not False else None

    def _index_stream(self, n):
        return self._inputs[0]._index_stream(n) if self._columns() is not None else None

    def _identity_order(self):
        return self._columns() is not None

    def _try_vectorize(self):
        inp = self._inputs[0]
        if not self.options().experimental_optimization.map_vectorization:
            return False
        # only identity-ordered in-memory sources (a shuffle below would change which row is which)
        if not inp._identity_order():
            return False
        cols = inp._columns()
        if cols is None:
            return False
        n = _num_rows(cols)
        if n == 0:
            return False
        try:
            with torch.no_grad():
                out = _apply(self.fn, cols)
            out = map_structure(lambda t: t if isinstance(t, torch.Tensor) else _to_tensor(t), out)
            if any(not isinstance(t, torch.Tensor) or t.dim() == 0 or len(t) != n for t in flatten(out)):
                return False
            for i in sorted({0, n // 2, n - 1}):
                ref = _apply(self.fn, map_structure(lambda c: c[i], cols))
                got = map_structure(lambda c: c[i], out)
                for r, g in zip(flatten(ref), flatten(got)):
                    r = _to_tensor(r)
                    if r.shape != g.shape or r.dtype != g.dtype or not torch.equal(r, g):
                        return False
            return out
        except Exception:
            return False

    def _iter(self):
        cols = self._columns()
        if cols is not None:
            for i in range(_num_rows(cols)):
                yield map_structure(lambda c: c[i], cols)
            return
        fn = self.fn
        for e in self._inputs[0]:
            yield _normalize_output(_apply(fn, e))


def _normalize_output(x):
    if isinstance(x, (torch.Tensor, str, bytes)):
        return x
    if isinstance(x, dict):
        return {k: _normalize_output(v) for k, v in x.items()}
    if isinstance(x, tuple):
        return tuple(_normalize_output(v) for v in x)
    return _to_tensor(x)


class FilterDataset(Dataset):
    def __init__(self, inp, pred):
        self._inputs = (inp,)
        self.pred = pred

    def _iter(self):
        for e in self._inputs[0]:
            if bool(_apply(self.pred, e)):
                yield e


class CacheDataset(Dataset):
    """In-memory cache (filename='') or an on-disk cache file (torch.save of the columns)."""

    def __init__(self, inp, filename=""):
        self._inputs = (inp,)
        self.filename = filename
        self._cache: Optional[list] = None
        self._cols = None

    def cardinality(self):
        return len(self._cache) if self._cache is not None else self._inputs[0].cardinality()

    def materialize(self):
        if self._cols is not None or self._cache is not None:
            return
        if self.filename and os.path.exists(self.filename + ".tdlcache"):
            self._cols = torch.load(self.filename + ".tdlcache", weights_only=True)
            return
        inp = self._inputs[0]
        cols = inp._columns()
        if cols is not None and inp._identity_order():
            self._cols = cols
        elif cols is not None and (order := inp._index_stream(_num_rows(cols))) is not None:
            # cache below a shuffle freezes the first epoch's order (TF semantics)
            self._cols = _take_rows(cols, torch.as_tensor(list(order), dtype=torch.long))
        else:
            elems = list(self._inputs[0])
            try:
                self._cols = _stack(elems) if elems else None
            except Exception:
                self._cols = None
            if self._cols is None:
                self._cache = elems
        if self.filename and self._cols is not None:
            torch.save(self._cols, self.filename + ".tdlcache")

    def _columns(self):
        self.materialize()
        return self._cols

    def _index_stream(self, n):
        self.materialize()
        return iter(range(_num_rows(self._cols))) if self._cols is not None else None

    def _identity_order(self):
        self.materialize()
        return self._cols is not None

    def _iter(self):
        self.materialize()
        if self._cols is not None:
            cols = self._cols
            for i in range(_num_rows(cols)):
                yield map_structure(lambda c: c[i], cols)
        else:
            yield from self._cache


_MASK64 = (1 << 64) - 1


def _splitmix64_stream(seed: int, n: int) -> np.ndarray:
    """The 62-bit random stream r[k] of the buffered shuffle: splitmix64(seed) outputs >> 2."""
    with np.errstate(over="ignore"):
        k = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(2)).astype(np.int64)


def _shuffle_indices(n: int, buffer_size: int, rng: np.random.Generator, source_order=None) -> np.ndarray:
    """TF's buffered shuffle on indices: fill a buffer, emit a random slot, refill it.  One 64-bit
    seed is drawn from ``rng``; the per-element random stream is splitmix64 of that seed, so the
    native implementation (csrc/native, GIL released) and the Python one give the same order."""
    src = np.arange(n) if source_order is None else np.asarray(source_order)
    seed = int(rng.integers(0, 1 << 63))
    N = _native_or_none()
    if N is not None:
        return N.buffered_shuffle(torch.from_numpy(np.ascontiguousarray(src, dtype=np.int64)), int(buffer_size),
                                  seed).numpy()
    return _shuffle_indices_py(src, n, buffer_size, _splitmix64_stream(seed, n))


def _native_or_none():
    from .. import ops

    try:
        return ops.native()
    except Exception:
        return None


def _shuffle_indices_py(src, n, buffer_size, r):
    out = np.empty(n, dtype=np.int64)
    buf = list(src[:buffer_size])
    nxt = min(buffer_size, n)
    for k in range(n):
        j = int(r[k] % len(buf))
        out[k] = buf[j]
        if nxt < n:
            buf[j] = src[nxt]
            nxt += 1
        else:
            buf[j] = buf[-1]
            buf.pop()
    return out


class ShuffleDataset(Dataset):
    def __init__(self, inp, buffer_size, seed, reshuffle):
        if buffer_size is None or (buffer_size <= 0 and buffer_size != AUTOTUNE):
            raise ValueError("shuffle buffer_size must be > 0")
        self._inputs = (inp,)
        self.buffer_size = int(buffer_size) if buffer_size != AUTOTUNE else 1 << 30
        self.seed = seed
        self.reshuffle = reshuffle
        self._epoch = 0
        self._base = None

    def cardinality(self):
        return self._inputs[0].cardinality()

    def _rng_at(self, epoch: int, seed_override: Optional[int] = None):
        """The shuffle RNG of iteration ``epoch`` (pure: no counter advances).  ``seed_override``
        stands in for an unset ``seed`` (synchronised DATA sharding, parallel/input_lib.reseed)."""
        seed = _seed_state.override if _seed_state.override is not None else self.seed
        if seed is None:
            seed = seed_override
        if seed is None and _global_seed is not None:
            seed = _global_seed
        if seed is None:
            if self._base is None:
                self._base = int(np.random.SeedSequence().entropy % (1 << 63))
            seed = self._base
        ep = epoch if self.reshuffle else 0
        return np.random.default_rng([int(seed) & ((1 << 63) - 1), ep])

    def _rng(self):
        r = self._rng_at(self._epoch)
        self._epoch += 1
        return r

    def _columns(self):
        return self._inputs[0]._columns()

    def _index_stream(self, n):
        inp = self._inputs[0]
        cols = inp._columns()
        if cols is None:
            return None
        rows = _num_rows(cols)
        order = inp._index_stream(rows)
        if order is None:
            return None
        return iter(_shuffle_indices(rows, self.buffer_size, self._rng(), list(order)).tolist())

    def _iter(self):
        stream = self._index_stream(0)
        if stream is not None:
            cols = self._columns()
            for i in stream:
                yield map_structure(lambda c: c[i], cols)
            return
        rng = self._rng()
        buf = []
        for e in self._inputs[0]:
            if len(buf) < self.buffer_size:
                buf.append(e)
                continue
            j = int(rng.integers(len(buf)))
            yield buf[j]
            buf[j] = e
        while buf:
            j = int(rng.integers(len(buf)))
            buf[j], buf[-1] = buf[-1], buf[j]
            yield buf.pop()


class BatchDataset(Dataset):
    def __init__(self, inp, batch_size, drop_remainder):
        if batch_size <= 0:
            raise ValueError("batch_size must be > 0")
        self._inputs = (inp,)
        self.batch_size = batch_size
        self.drop_remainder = drop_remainder

    def cardinality(self):
        c = self._inputs[0].cardinality()
        if c < 0:
            return c
        return c // self.batch_size if self.drop_remainder else -(-c // self.batch_size)

    def _iter(self):
        inp = self._inputs[0]
        cols = inp._columns()
        stream = inp._index_stream(_num_rows(cols)) if cols is not None else None
        B = self.batch_size
        if stream is not None:
            order = np.fromiter(stream, dtype=np.int64)
            n = len(order)
            end = (n // B) * B if self.drop_remainder else n
            idx_all = torch.from_numpy(order)
            for s in range(0, end, B):
                yield _take_rows(cols, idx_all[s : s + B])
            return
        buf = []
        for e in inp:
            buf.append(e)
            if len(buf) == B:
                yield _stack(buf)
                buf = []
        if buf and not self.drop_remainder:
            yield _stack(buf)


class UnbatchDataset(Dataset):
    def __init__(self, inp):
        self._inputs = (inp,)

    def _iter(self):
        for b in self._inputs[0]:
            n = len(flatten(b)[0])
            for i in range(n):
                yield map_structure(lambda c: c[i], b)


class RepeatDataset(Dataset):
    def __init__(self, inp, count):
        self._inputs = (inp,)
        self.count = None if count is None or count < 0 else int(count)

    def cardinality(self):
        c = self._inputs[0].cardinality()
        if self.count is None:
            return INFINITE_CARDINALITY if c != 0 else 0
        return c * self.count if c >= 0 else c

    def _iter(self):
        k = 0
        while self.count is None or k < self.count:
            empty = True
            for e in self._inputs[0]:
                empty = False
                yield e
            if empty:
                return
            k += 1


class TakeDataset(Dataset):
    def __init__(self, inp, n):
        self._inputs = (inp,)
        self.n = n

    def cardinality(self):
        c = self._inputs[0].cardinality()
        if self.n < 0:
            return c
        if c == INFINITE_CARDINALITY:
            return self.n
        return min(c, self.n) if c >= 0 else UNKNOWN_CARDINALITY

    def _iter(self):
        if self.n == 0:
            return
        for k, e in enumerate(self._inputs[0]):
            yield e
            if self.n >= 0 and k + 1 >= self.n:
                return


class SkipDataset(Dataset):
    def __init__(self, inp, n):
        self._inputs = (inp,)
        self.n = n

    def cardinality(self):
        c = self._inputs[0].cardinality()
        if c < 0:
            return c
        return max(0, c - self.n) if self.n >= 0 else 0

    def _iter(self):
        for k, e in enumerate(self._inputs[0]):
            if self.n < 0:
                return
            if k >= self.n:
                yield e


class ShardDataset(Dataset):
    def __init__(self, inp, num_shards, index):
        self._inputs = (inp,)
        self.num_shards, self.index = num_shards, index

    def cardinality(self):
        c = self._inputs[0].cardinality()
        if c < 0:
            return c
        return c // self.num_shards + (1 if self.index < c % self.num_shards else 0)

    def source_files(self):
        f = self._inputs[0].source_files()
        return f[self.index :: self.num_shards] if f is not None else None

    def _iter(self):
        for k, e in enumerate(self._inputs[0]):
            if k % self.num_shards == self.index:
                yield e


class PrefetchDataset(Dataset):
    """Background-thread prefetch of up to ``buffer_size`` elements (AUTOTUNE = 2)."""

    def __init__(self, inp, buffer_size):
        self._inputs = (inp,)
        self.buffer_size = 2 if buffer_size in (None, AUTOTUNE) or buffer_size < 1 else int(buffer_size)

    def cardinality(self):
        return self._inputs[0].cardinality()

    def _columns(self):
        return self._inputs[0]._columns()

    def _index_stream(self, n):
        return self._inputs[0]._index_stream(n)

    def _identity_order(self):
        return self._inputs[0]._identity_order()

    def _iter(self):
        q: "queue.Queue" = queue.Queue(self.buffer_size)
        done = object()
        stop = threading.Event()
        err = []
        seed_override = _seed_state.override

        def worker():
            _seed_state.override = seed_override
            try:
                for e in self._inputs[0]:
                    while not stop.is_set():
                        try:
                            q.put(e, timeout=0.1)
                            break
                        except queue.Full:
                            continue
                    if stop.is_set():
                        return
            except BaseException as ex:  # propagate to the consumer
                err.append(ex)
            finally:
                while not stop.is_set():
                    try:
                        q.put(done, timeout=0.1)
                        break
                    except queue.Full:
                        continue

        t = threading.Thread(target=worker, daemon=True)
        t.start()
        try:
            while True:
                e = q.get()
                if e is done:
                    if err:
                        raise err[0]
                    return
                yield e
        finally:
            stop.set()


class OptionsDataset(Dataset):
    def __init__(self, inp, options):
        self._inputs = (inp,)
        self._opts = options

    def options(self):
        return self._inputs[0].options().merge(self._opts)

    def cardinality(self):
        return self._inputs[0].cardinality()

    def _columns(self):
        return self._inputs[0]._columns()

    def _index_stream(self, n):
        return self._inputs[0]._index_stream(n)

    def _identity_order(self):
        return self._inputs[0]._identity_order()

    def _iter(self):
        return iter(self._inputs[0])


class _SeedOverride:
    """Context: every unseeded shuffle uses ``seed`` (synchronised DATA sharding)."""

    def __init__(self, seed):
        self.seed = seed

    def __enter__(self):
        self.prev = _seed_state.override
        _seed_state.override = self.seed

    def __exit__(self, *a):
        _seed_state.override = self.prev


def seed_override(seed):
    return _SeedOverride(seed)


def reset_iteration_state(ds: Dataset):
    """Restart per-iteration epoch counters (used after re-seeding)."""
    if isinstance(ds, ShuffleDataset):
        ds._epoch = 0
    for i in ds._inputs:
        reset_iteration_state(i)


def auto_shard(ds: Dataset, num_workers: int, index: int, policy: AutoShardPolicy) -> Dataset:
    """FILE auto-shard: rewrite the file source so worker `index` reads every num_workers-th file."""
    if policy != AutoShardPolicy.FILE and policy != AutoShardPolicy.AUTO:
        return ds
    files = ds.source_files()
    if files is None:
        if policy == AutoShardPolicy.FILE:
            raise ValueError("AutoShardPolicy.FILE needs a file-based dataset (list_files / TextLineDataset); "
                             "use DATA or OFF for in-memory datasets")
        return ds
    if len(files) < num_workers:
        if policy == AutoShardPolicy.FILE:
            raise ValueError(f"AutoShardPolicy.FILE: {len(files)} files cannot be sharded over {num_workers} workers")
        return ds
    return _rewrite_file_source(ds, num_workers, index)


def _rewrite_file_source(ds, n, i):
    import copy

    if isinstance(ds, FileListDataset):
        return FileListDataset(ds.files[i::n])
    new = copy.copy(ds)
    new._inputs = tuple(_rewrite_file_source(x, n, i) for x in ds._inputs)
    if isinstance(new, TextLineDataset):
        new._files_ds = new._inputs[0]
    return new
