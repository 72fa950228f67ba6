"""Checkpoint / resume of the device-resident A/M loop through the native .hss writer
(AMIteration.checkpoint / restore, SURVEY 5 checkpoint row and 8(f)2): a run
interrupted after one iteration and resumed from its .hss continues bitwise like the
uninterrupted run (the kernels are deterministic), and the checkpoint is a .hss the
Step layer reads as a population."""
import numpy as np
import pytest

import h5_inspect
from dist_am_inputs import inputs, iteration


@pytest.mark.gpu
def test_resume_from_checkpoint_is_bitwise_the_uninterrupted_run(tmp_path):
    from igm_amd import hss
    from igm_amd import steps as ST
    from igm_amd._lib import row_dtype
    inp = inputs(nstruct=4)
    path = str(tmp_path / 'ckpt.hss')
    a = iteration(inp, 'cuda:0', 0, 4)
    a.step()
    a.checkpoint(path)
    h5_inspect.inspect(path)
    a.step()
    xa = a.xyz.cpu().numpy()
    ra = a.rows[:a.nrows * row_dtype.itemsize].cpu().numpy().tobytes()
    b = iteration(inp, 'cuda:0', 0, 4)
    b.restore(path)
    assert b.step_no == 1
    b.step()
    assert b.nrows == a.nrows
    assert b.rows[:b.nrows * row_dtype.itemsize].cpu().numpy().tobytes() == ra
    assert np.array_equal(b.xyz.cpu().numpy(), xa)
    assert b.violation_score() == a.violation_score()
    # the checkpoint is a population the Step layer can run from
    store = ST.PopulationStore(path)
    assert store.nstruct == 4 and np.array_equal(store.copy_ptr, inp['pop']['copy_ptr'])
    h = hss.Hss(path)
    assert np.isfinite(h.violation)


@pytest.mark.gpu
def test_restore_a_shard_whose_first_structure_is_not_zero(tmp_path):
    """A single-rank shard of structures 4..7 (first_sid 4, as bench.py's ranks pass):
    the checkpoint holds its 4 structures in columns 0..3, and restore() reads them
    back from there (not from column first_sid)."""
    inp = inputs(nstruct=8)
    path = str(tmp_path / 'ckpt.hss')
    a = iteration(inp, 'cuda:0', 4, 8)
    a.step()
    a.checkpoint(path)
    b = iteration(inp, 'cuda:0', 4, 8)
    b.restore(path)
    assert np.array_equal(b.xyz.cpu().numpy(), a.xyz.cpu().numpy())
    assert b.step_no == a.step_no
