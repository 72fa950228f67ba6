"""The world>1 branches of AMIteration actually running: two and four ranks on
cuda:0 over gloo (torch.distributed.run, host-staged collectives) against one rank
doing everything.  The A-step rows gathered in CSR order, every structure's Hi-C
bonds, final coordinates, optimisation info and violation records, and the
population violation score must be byte-identical: structures are independent
(ModelingStep.py:164-573) and the pair shards are contiguous CSR ranges."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import dist_am_inputs as I

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize('world', [2, 3, 4])
def test_gpu_ranks_equal_one_rank(tmp_path, world):
    """(world 3: 8 structures split 2/3/3 -- uneven shards, padded all-gather)"""
    env = dict(os.environ, IGM_DIST_OUT=str(tmp_path), OMP_NUM_THREADS='2')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=%d' % world,
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(HERE, 'dist_am_worker.py')]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-4000:]
    parts = [np.load(str(tmp_path / ('rank%d.npz' % k))) for k in range(world)]
    inp = I.inputs()
    it = I.iteration(inp, 'cuda:0', 0, inp['xyz'].shape[0])
    it.astep()
    rows = it.rows[:it.nrows * 16].cpu().numpy()
    it.mstep()
    score = it.violation_score()
    for p in parts:  # every rank holds the whole gathered row list
        assert p['rows'].tobytes() == rows.tobytes()
    ptr = it.hic_ptr.cpu().numpy()
    bonds = it.hic_bonds[:it.nbonds * 16].cpu().numpy()
    xyz = it.xyz.cpu().numpy()
    info = it.info.cpu().numpy()
    stats = it.stats.cpu().numpy()
    rec = info.size // xyz.shape[0]
    for p in parts:
        s0, s1 = int(p['s0']), int(p['s1'])
        assert np.array_equal(p['xyz'], xyz[s0:s1])
        assert np.array_equal(p['stats'], stats[s0:s1])
        assert p['info'].tobytes() == info[s0 * rec:s1 * rec].tobytes()
        assert p['bonds'].tobytes() == bonds[ptr[s0] * 16:ptr[s1] * 16].tobytes()
        assert np.array_equal(p['ptr'], ptr[s0:s1 + 1] - ptr[s0])
        assert float(p['score']) == score
        assert np.array_equal(p['restored'], xyz[s0:s1])  # checkpoint after a step, resumed per rank
    assert len(rows) > 1000 and ptr[-1] > 1000


def test_gpu_rccl_collectives_one_rank():
    """The RCCL ('nccl') path of the collective helpers and a whole AMIteration.step() with its
    N > 1 exchanges run on device tensors, the step byte-equal to one without them (one rank:
    RCCL refuses two ranks on one GPU; the two-rank equality above runs over gloo)."""
    env = dict(os.environ, OMP_NUM_THREADS='2')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(HERE, 'rccl_worker.py')]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0 and 'RCCL-OK' in r.stdout, r.stdout[-4000:]

