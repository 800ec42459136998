"""Shared test setup: import paths, the `gpu` marker, scene fixtures."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "optix-renderer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    import nori_hip as nh
    nh.configure_runtime()  # before any test touches HIP: one hardware queue per path pool (nh_env.py)


@pytest.fixture(scope="session")
def scene_dir(tmp_path_factory):
    import scenegen
    return scenegen.materialize(str(tmp_path_factory.mktemp("scenes")))


@pytest.fixture(scope="session")
def gpu():
    """The HIP path must run on the GPU box: no device is a failure, not a skip."""
    import nori_hip as nh
    n = nh.device_count()
    assert n > 0, "no GPU visible to the HIP runtime"
    return 0
