import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: multi-second multi-process tests")
    # evidence for a native-thread abort: the faulting thread's id, name and
    # native backtrace before faulthandler's Python stacks (csrc/native/crash_trace.cpp), and MIOpen's
    # own warnings/errors (its log level 3) in the suite's output
    os.environ.setdefault("MIOPEN_LOG_LEVEL", "3")
    try:
        from tensorflow_distributed_learning_amd import ops

        if ops.native_available():
            ops.native().install_crash_trace()
    except Exception:  # noqa: BLE001 - diagnostics only
        pass


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
