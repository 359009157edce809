import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def _ensure_oracle():
    lib = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session")
def oracle():
    _ensure_oracle()
    from tests import oracle_binding
    return oracle_binding.Oracle()


@pytest.fixture(scope="session")
def orc_bin():
    _ensure_oracle()
    return os.path.join(ROOT, "oracle", "_build", "orc")


@pytest.fixture(scope="session")
def gpu_lib():
    # torch's bundled HIP runtime must initialise before the system runtime
    # our library links, or torch sees no GPU (tools/mix_probe.py)
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from unipeak_amd import capi
    capi.load_library()  # raises loudly if the HIP library is missing
    if capi.device_count() < 1:
        pytest.fail("no HIP device visible for a gpu-marked test")
    return capi
