"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures, host logic, C-ABI load/export.
`-m gpu` runs on an MI355X: the HIP kernels through the C ABI vs the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Restatement

    return Restatement()


@pytest.fixture(scope="session")
def reference():
    from oracle.oracle import Reference

    try:
        return Reference()
    except (FileNotFoundError, OSError):
        pytest.skip("oracle/_ref not built (reference sources absent)")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test collected but no GPU is visible (run -m 'not gpu' on CPU hosts)")
    import lampi_amd

    lampi_amd.lib()  # the HIP library must load: no fallback
    return torch.device("cuda:0")
