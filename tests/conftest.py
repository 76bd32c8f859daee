import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "unnamed-rust-sdr_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running full-size checks")


def rms_rel_err(y, ref):
    """Parity metric of SURVEY.md 8c / BASELINE.md: (max |y-ref| / rms(ref), ||y-ref||/||ref||)."""
    y = np.asarray(y, dtype=np.complex128 if np.iscomplexobj(y) else np.float64)
    ref = np.asarray(ref, dtype=np.complex128 if np.iscomplexobj(ref) else np.float64)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    if ref.size == 0:
        return 0.0, 0.0
    d = np.abs(y - ref)
    rms = np.sqrt(np.mean(np.abs(ref) ** 2))
    nrm = np.linalg.norm(ref.ravel())
    if rms == 0:
        return float(d.max()), float(np.linalg.norm(d.ravel()))
    return float(d.max() / rms), float(np.linalg.norm(d.ravel()) / nrm)


TOL = 1e-5  # north_star: within 1e-5 relative on f32 (RMS-normalised)


def assert_parity(y, ref, tol=TOL, what=""):
    mx, l2 = rms_rel_err(y, ref)
    assert mx <= tol and l2 <= tol, f"{what}: max/rms={mx:.3e} l2={l2:.3e} tol={tol:.1e}"


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def sdr():
    import sdrgpu
    return sdrgpu
