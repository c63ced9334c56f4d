import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'ofdm-lte_amd')
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden', 'golden.npz')
GOLDEN_MIMO = os.path.join(ROOT, 'tests', 'golden', 'golden_mimo.npz')
GOLDEN_TM4 = os.path.join(ROOT, 'tests', 'golden', 'golden_tm4.npz')
GOLDEN_SCFDM = os.path.join(ROOT, 'tests', 'golden', 'golden_scfdm.npz')
GOLDEN_IMAGE = os.path.join(ROOT, 'tests', 'golden', 'golden_image.npz')
GOLDEN_BF = os.path.join(ROOT, 'tests', 'golden', 'golden_bf.npz')
GOLDEN_R2 = os.path.join(ROOT, 'tests', 'golden', 'golden_r2.npz')
GOLDEN_R3 = os.path.join(ROOT, 'tests', 'golden', 'golden_r3.npz')
FIXTURE_CURVE = os.path.join(ROOT, 'tests', 'golden', 'fixture_ber_curve.npz')
FIXTURE_CURVE_C4 = os.path.join(ROOT, 'tests', 'golden', 'fixture_ber_curve_c4.npz')
GOLDEN_CODING_R2 = os.path.join(ROOT, 'tests', 'golden', 'golden_coding_r2.npz')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU; runs the HIP path')


def _gpu_present():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_present() or os.environ.get('LTE_REQUIRE_GPU'):
        return
    skip = pytest.mark.skip(reason='no GPU in this container (run with -m gpu on an MI355X)')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope='session')
def golden():
    return np.load(GOLDEN, allow_pickle=False)


@pytest.fixture(scope='session')
def golden_mimo():
    return np.load(GOLDEN_MIMO, allow_pickle=False)


@pytest.fixture(scope='session')
def golden_tm4():
    return np.load(GOLDEN_TM4, allow_pickle=False)


@pytest.fixture(scope='session')
def golden_scfdm():
    return np.load(GOLDEN_SCFDM, allow_pickle=False)


@pytest.fixture(scope='session')
def golden_image():
    return np.load(GOLDEN_IMAGE, allow_pickle=False)


@pytest.fixture(scope='session')
def golden_bf():
    return np.load(GOLDEN_BF, allow_pickle=False)


@pytest.fixture(scope='session')
def golden_r2():
    return np.load(GOLDEN_R2, allow_pickle=False)


@pytest.fixture(scope='session')
def golden_coding():
    import json
    meta = json.load(open(GOLDEN_CODING_R2.replace('.npz', '_meta.json')))
    return np.load(GOLDEN_CODING_R2, allow_pickle=False), meta


@pytest.fixture(scope='session')
def golden_r3():
    return np.load(GOLDEN_R3, allow_pickle=False)


@pytest.fixture(scope='session')
def fixture_curve():
    return np.load(FIXTURE_CURVE, allow_pickle=False)


@pytest.fixture(scope='session')
def fixture_curve_c4():
    return np.load(FIXTURE_CURVE_C4, allow_pickle=False)


@pytest.fixture(scope='session')
def bf_oracle():
    from oracle import bf_oracle
    return bf_oracle


@pytest.fixture(scope='session')
def tm4_oracle():
    from oracle import tm4_oracle
    return tm4_oracle


@pytest.fixture(scope='session')
def mimo_oracle():
    from oracle import mimo_oracle
    return mimo_oracle


@pytest.fixture(scope='session')
def oracle():
    from oracle import lte_oracle
    lte_oracle.lib()
    return lte_oracle


def unpack(a, n=None):
    b = np.unpackbits(np.asarray(a, dtype=np.uint8))
    return b if n is None else b[:n]


GOLDEN_R5 = os.path.join(ROOT, 'tests', 'golden', 'golden_r5.npz')


@pytest.fixture(scope='session')
def golden_r5():
    return np.load(GOLDEN_R5, allow_pickle=False)
