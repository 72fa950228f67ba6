"""Host-side helpers of bench.py (no GPU): the warmup protocol of the config C block and the
force-evaluation count the roofline's algorithmic bytes are priced on."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from igm_amd import model as M  # noqa: E402
from igm_amd import synthetic as syn  # noqa: E402


@pytest.fixture
def prm():
    return M.params_from_cfg({'optimization': {'optimizer_options': syn.DEMO_PROTOCOL}}, [((5500.0,) * 3, 1.0)])


def test_scaled_prm_scales_md_steps_only(prm):
    w = bench._scaled_prm(prm, 0.1)
    cap = syn.DEMO_PROTOCOL['custom_annealing_protocol']
    assert w.nstages == prm.nstages == len(cap['mdsteps'])
    assert [w.mdsteps[k] for k in range(w.nstages)] == [round(n * 0.1) for n in cap['mdsteps']]
    assert w.relax_steps == round(cap['relax']['mdsteps'] * 0.1)
    # the original is untouched (the timed iteration runs it) and everything else is copied
    assert [prm.mdsteps[k] for k in range(prm.nstages)] == cap['mdsteps']
    assert bytes(bench._scaled_prm(prm, 1.0)) == bytes(prm)
    for name, _ in type(prm)._fields_:
        if name not in ('mdsteps', 'relax_steps'):
            a, b = getattr(w, name), getattr(prm, name)
            assert (bytes(a) == bytes(b)) if hasattr(a, '_length_') else a == b, name


def test_scaled_prm_keeps_one_step(prm):
    w = bench._scaled_prm(prm, 1e-6)
    assert all(w.mdsteps[k] == 1 for k in range(w.nstages)) and w.relax_steps == 1


def test_evaluations_counts_setup_steps(prm):
    # every run (relax + stage) evaluates its forces nsteps + 1 times (Verlet::setup + steps)
    cap = syn.DEMO_PROTOCOL['custom_annealing_protocol']
    n = sum(s + 1 for s in cap['mdsteps']) + len(cap['mdsteps']) * (cap['relax']['mdsteps'] + 1)
    assert bench._evaluations(prm) == n


def test_bench_defaults(monkeypatch):
    monkeypatch.setattr(sys, 'argv', ['bench.py'])
    a = bench.parse()
    assert a.gpus == 1 and a.c_warmup == 1 and a.c_warmup_scale == 0.1 and a.c_shard == 125
    assert a.protocol_scale == 1.0 and a.config == 'B' and a.nstruct == 1000
