"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libdvo_hip.so")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


_FRAME_CACHE = {}


def synth_frames(w, h, idxs):
    """Seeded synthetic frames (rendered once per session on the CPU)."""
    from droplet_visual_odometry_amd.synth import SceneStream
    key = (w, h)
    st = _FRAME_CACHE.setdefault(key, (SceneStream(w, h), {}))
    stream, cache = st
    out = []
    for i in idxs:
        if i not in cache:
            cache[i] = stream.render(i).numpy()
        out.append(cache[i])
    return np.stack(out), stream.K


@pytest.fixture(scope="session")
def frames_640():
    return synth_frames(640, 480, range(4))


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from droplet_visual_odometry_amd._native import Context
    return Context.default(0)
