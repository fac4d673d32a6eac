import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmgicp.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(autouse=True)
def _no_target_cache_across_engines(request):
    """r05 target cache: the library keeps a destroyed engine's target for the next engine that sets the
    same points.  GPU tests compare engines built on purpose with different forms, so by default their
    engines neither adopt nor leave targets ("target_cache" 0); tests/test_target_cache.py turns it on
    for the engines it checks, and the C++ adapter replay runs with the library default (on)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from leica_point_cloud_processing_amd.engine import GICPEngine

    GICPEngine.DEFAULT_OPTIONS = {"target_cache": 0}
    GICPEngine.release_cache()
    yield
    GICPEngine.release_cache()


@pytest.fixture(scope="session")
def cube_clouds():
    """The reference unit-test fixture (test_gicp_alignment.cpp:32-47): 5000 glibc-rand()
    samples of cube.ply and their Rz(0.175) rotation."""
    from leica_point_cloud_processing_amd import synth

    src, tgt, T = synth.cube_fixture(os.path.join(GOLDEN, "cube.ply"))
    return src, tgt, T


@pytest.fixture(scope="session")
def part_small():
    """A 20k/20k scan-vs-CAD case of the synthetic aero part (seeded)."""
    from leica_point_cloud_processing_amd import synth

    scan, cad, T = synth.scan_vs_cad(20000, 20000)
    return scan, cad, T


class heartbeat:
    """Context manager: a line on the real stderr every `every` seconds while a long step (the
    full-size CPU oracle) runs, so a supervisor watching the output does not take it for a hang."""

    def __init__(self, what: str, every: float = 30.0):
        self.what, self.every = what, every

    def __enter__(self):
        import threading
        import time

        self._stop = threading.Event()
        t0 = time.time()

        def beat():
            while not self._stop.wait(self.every):
                sys.__stderr__.write(f"[heartbeat] {self.what}: {time.time() - t0:.0f} s\n")
                sys.__stderr__.flush()

        self._t = threading.Thread(target=beat, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join(timeout=5)


def frob(a, b) -> float:
    return float(np.linalg.norm(np.asarray(a, np.float64) - np.asarray(b, np.float64)))
