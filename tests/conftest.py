import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run on the GPU box with -m gpu)')
    config.addinivalue_line('markers', 'slow: long CPU test')


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope='session')
def demo_pop():
    return load_golden('demo_population.npz')


@pytest.fixture(scope='session')
def demo_pairs():
    return load_golden('demo_hic_pairs.npz')


@pytest.fixture(scope='session')
def g1():
    return load_golden('actdist_golden.npz')


@pytest.fixture(scope='session')
def g2():
    return load_golden('actdist_edge.npz')


@pytest.fixture(scope='session')
def mstep_inputs():
    return load_golden('mstep_inputs.npz')


def make_pairs(i, j, pwish, plast):
    from igm_amd._lib import pair_dtype
    a = np.zeros(len(i), pair_dtype)
    a['i'] = i
    a['j'] = j
    a['pwish'] = pwish
    a['plast'] = plast
    return a


def expand_per_pair(nrows, dist, prob):
    """per-pair golden -> per-row dist/prob (rows of a pair share dist/prob)."""
    nrows = np.asarray(nrows, np.int64)
    return np.repeat(dist[nrows > 0], nrows[nrows > 0]), np.repeat(prob[nrows > 0], nrows[nrows > 0])


@pytest.fixture
def heartbeat(request):
    """For a GPU test that runs minutes inside one native call (the fp64 oracle on a
    full protocol): a thread appends a line every 30 s to gpurun_out/heartbeat.txt, so a
    runner that takes minutes without output for a hang sees the test alive (pytest
    captures the test's own stdout and stderr)."""
    import threading
    import time
    d = os.path.join(os.environ.get('GRAFT_REPO_ROOT', ROOT), 'gpurun_out')
    os.makedirs(d, exist_ok=True)
    stop = threading.Event()

    def beat():
        while not stop.wait(30.0):
            with open(os.path.join(d, 'heartbeat.txt'), 'a') as fh:
                fh.write('%s %s alive\n' % (time.strftime('%H:%M:%S'), request.node.name))
                fh.flush()
            sys.stderr.flush()

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
    th.join(timeout=5)
