import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "reference: compares against the read-only reference code")


def pytest_collection_modifyitems(config, items):
    """``-m gpu`` tests need a HIP device: on a CPU-only host they are skipped, not failed."""
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU (HIP device) available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from llm_driven_multi_factor_model_amd import _native
    _native.lib()  # fail loudly if the kernel library is missing
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def ab_lib(cuda):
    """Tests of kernel variants that lost their A/B measurements: they live only in the A/B
    library (``python -m llm_driven_multi_factor_model_amd._build --ab``, loaded through
    ``MFA_HIP_LIB=.../_lib/ab/libmfa_hip.so``); the production library skips them."""
    from llm_driven_multi_factor_model_amd import _native
    if not _native.ab_build():
        pytest.skip("A/B kernel variant: not in the production library (build --ab)")
    return _native.lib()


@pytest.fixture(scope="session")
def ref():
    from tests._refshim import load_reference
    r = load_reference()
    if r is None:
        pytest.skip("reference repository not mounted")
    return r
