"""One rank of tests/test_distributed_gpu.py::test_gpu_rccl_collectives_one_rank: the
product's collective helpers (igm_amd.pipeline) on device tensors through an RCCL
('nccl') process group, then a whole AMIteration.step() with its N > 1 exchanges forced
on (collective=True).  RCCL refuses two ranks on one device, so on a one-GPU box the
group has one rank: every all_gather / all_reduce call of the N > 1 path runs as an
RCCL kernel on HBM tensors of the path's dtypes and shapes."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from igm_amd import pipeline as P  # noqa: E402

dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
dist.init_process_group('nccl', device_id=dev)
assert dist.get_backend() == 'nccl' and dist.get_world_size() == 1
g = torch.Generator(device='cpu').manual_seed(5)
xyz = torch.randn(7, 3009, 3, generator=g).to(dev)
out = P.gather_population(xyz)
assert out.is_cuda and torch.equal(out, xyz)
rows = torch.randint(0, 255, (16 * 1000,), dtype=torch.uint8, generator=g).to(dev)
got, n = P.gather_rows(rows, 900, 16, 1000)
assert got.is_cuda and n == 900 and torch.equal(got, rows[:900 * 16])
vals = [1.5, -2.25, 1e-3]
red = P.reduce_sum_f64(vals, dev)
assert [float(x) for x in red] == vals, red
# one whole AMIteration.step() with every exchange of the N > 1 path (population all-gather,
# row gather, shard-count check, violation-score all-reduce, checkpoint gathers) through RCCL,
# byte-equal to the same step without collectives
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import dist_am_inputs as I  # noqa: E402

inp = I.inputs()
S = inp['xyz'].shape[0]
res = {}
for coll in (True, False):
    it = I.iteration(inp, 'cuda:0', 0, S, collective=coll)
    assert it.coll is coll
    it.step()
    res[coll] = dict(rows=it.rows[:it.nrows * 16].cpu().numpy(), xyz=it.xyz.cpu().numpy(), info=it.info.cpu().numpy(),
                     stats=it.stats.cpu().numpy(), score=it.violation_score(), nrows=it.nrows)
    if coll:
        it.checkpoint(os.path.join(os.environ.get('TMPDIR', '/tmp'), 'rccl_ckpt_%d.hss' % os.getpid()))
a, b = res[True], res[False]
assert a['nrows'] == b['nrows'] > 1000 and a['rows'].tobytes() == b['rows'].tobytes()
assert np.array_equal(a['xyz'], b['xyz']) and a['info'].tobytes() == b['info'].tobytes()
assert np.array_equal(a['stats'], b['stats']) and a['score'] == b['score']
torch.cuda.synchronize()
dist.destroy_process_group()
print('RCCL-OK')
