import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _no_leaked_process_group():
    """Tests that initialise torch.distributed in the pytest process itself (TP=1 in-process
    paths) must not leak the group into the next test of the same (xdist) worker."""
    yield
    import torch.distributed as dist

    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    ps.destroy_model_parallel()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
