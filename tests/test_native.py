"""C++ runtime: KV store, ring collectives (vs exact oracle), CRC-32C."""
import threading

import numpy as np
import pytest
import torch

from tensorflow_distributed_learning_amd import ops

N = ops.native()


def test_kv_store_ops():
    s = N.KVServer("127.0.0.1", 0)
    try:
        c = N.KVClient("127.0.0.1", s.port, 5000, "t")
        c.set("k", b"v")
        assert c.get("k", 1000) == b"v"
        assert c.get("missing", 50) is None
        assert c.add("n", 5) == 5 and c.add("n", -2) == 3
        assert c.compare_set("slot", b"", b"A") == b"A"
        assert c.compare_set("slot", b"", b"B") == b"A"  # already claimed
        assert c.compare_set("slot", b"A", b"C") == b"C"
        assert c.check(["k", "n"]) and not c.check(["k", "zz"])
        c.append("log", b"ab")
        c.append("log", b"cd")
        assert c.get("log", 100) == b"abcd"
        assert c.delete("k") and not c.check(["k"])
        # blocking get released by another client's set
        c2 = N.KVClient("127.0.0.1", s.port, 5000, "u")
        out = []
        th = threading.Thread(target=lambda: out.append(c2.get("later", 5000)))
        th.start()
        c.set("later", b"x")
        th.join()
        assert out == [b"x"]
        assert c.wait(["later"], 100) and not c.wait(["never"], 50)
        assert "t" in s.heartbeat_ages()
    finally:
        s.stop()


def _ring(W):
    rings = [N.RingComm(r, W, "127.0.0.1", 10000) for r in range(W)]
    ports = [r.port for r in rings]
    ts = [threading.Thread(target=rings[r].connect, args=("127.0.0.1", ports[(r + 1) % W])) for r in range(W)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    return rings


def _par(fns):
    ts = [threading.Thread(target=f) for f in fns]
    [t.start() for t in ts]
    [t.join() for t in ts]


@pytest.mark.parametrize("W", [2, 3, 4])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64])
def test_ring_allreduce_exact(W, dtype):
    rings = _ring(W)
    n = 1000 + W  # not divisible by W
    xs = [torch.randint(-100, 100, (n,)).to(dtype) for _ in range(W)]
    ref = sum(x.clone() for x in xs)
    _par([lambda r=r: rings[r].all_reduce(xs[r], "sum") for r in range(W)])
    for x in xs:
        assert torch.equal(x, ref)
    xs = [torch.randint(-100, 100, (n,)).to(dtype) for _ in range(W)]
    ref = torch.stack(xs).amax(0)
    _par([lambda r=r: rings[r].all_reduce(xs[r], "max") for r in range(W)])
    assert all(torch.equal(x, ref) for x in xs)
    for r in rings:
        r.close()


def test_ring_float_identical_across_ranks_and_bcast_gather():
    W = 3
    rings = _ring(W)
    xs = [torch.randn(300001) for _ in range(W)]
    _par([lambda r=r: rings[r].all_reduce(xs[r], "sum") for r in range(W)])
    assert torch.equal(xs[0], xs[1]) and torch.equal(xs[1], xs[2])  # bit-identical on every rank
    bs = [torch.full((2_500_000,), float(r)) for r in range(W)]
    _par([lambda r=r: rings[r].broadcast(bs[r], 1) for r in range(W)])
    assert all(torch.all(b == 1).item() for b in bs)
    outs = [torch.zeros(W * 4, dtype=torch.int64) for _ in range(W)]
    _par([lambda r=r: rings[r].all_gather(torch.full((4,), r, dtype=torch.int64), outs[r]) for r in range(W)])
    assert all(torch.equal(o, torch.arange(W).repeat_interleave(4)) for o in outs)
    _par([lambda r=r: rings[r].barrier() for r in range(W)])


def test_crc32c():
    assert N.crc32c(b"123456789", 0) == 0xE3069283
    from tensorflow_distributed_learning_amd.utils.events import _crc32c_py

    d = np.random.bytes(1000)
    assert _crc32c_py(d) == N.crc32c(d, 0)


def test_crash_trace_names_the_aborting_native_thread(tmp_path):
    """A thread that calls abort() with no Python frame on top (the round-4 failure mode) is named
    with its native backtrace before faulthandler's Python stacks, and the process still dies with
    SIGABRT (csrc/native/crash_trace.cpp)."""
    import os
    import subprocess
    import sys
    import textwrap

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "abort.py"
    f.write_text(textwrap.dedent("""
        import ctypes, faulthandler, threading
        faulthandler.enable(all_threads=True)
        from tensorflow_distributed_learning_amd import ops
        assert ops.native().install_crash_trace()
        libc = ctypes.CDLL(None)
        libc.pthread_setname_np.argtypes = [ctypes.c_ulong, ctypes.c_char_p]
        libc.pthread_self.restype = ctypes.c_ulong
        def worker():
            libc.pthread_setname_np(libc.pthread_self(), b"tdl-test-worker")
            libc.abort()
        t = threading.Thread(target=worker)
        t.start()
        t.join()
    """))
    r = subprocess.run([sys.executable, str(f)], env=dict(os.environ, PYTHONPATH=root), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == -6, (r.returncode, r.stderr[-2000:])
    assert "[tdl crash trace] signal 6" in r.stderr and "name 'tdl-test-worker'" in r.stderr, r.stderr[-3000:]
    assert "[tdl crash trace] end" in r.stderr
    assert "Fatal Python error" in r.stderr  # faulthandler still runs after it (chained)
