"""One rank of tests/test_distributed_gpu.py (launched by torch.distributed.run): the
world>1 branches of igm_amd.pipeline.AMIteration -- population all-gather, pair-sharded
A-step, rows gathered in CSR order, M-step of the rank's structure shard, violation
score summed over the ranks -- on cuda:0 over gloo (host-staged collectives).  Saves
the rank's results to $IGM_DIST_OUT/rank<r>.npz."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import dist_am_inputs as I  # noqa: E402
from igm_amd import pipeline  # noqa: E402


def main():
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    try:
        inp = I.inputs()
        S = inp['xyz'].shape[0]
        s0, s1 = pipeline.shard(S, rank, world)
        it = I.iteration(inp, 'cuda:0', s0, s1, rank, world)
        it.astep()
        rows = it.rows[:it.nrows * 16].cpu().numpy()
        it.mstep()
        score = it.violation_score()
        # checkpoint after a step is a collective (the violation score is summed over
        # the ranks before rank 0 writes); every rank then resumes its own block
        ck = os.path.join(os.environ['IGM_DIST_OUT'], 'ckpt.hss')
        it.checkpoint(ck)
        dist.barrier()
        back = I.iteration(inp, 'cuda:0', s0, s1, rank, world)
        back.restore(ck)
        restored = back.xyz.cpu().numpy()
        np.savez(os.path.join(os.environ['IGM_DIST_OUT'], 'rank%d.npz' % rank), rows=rows,
                 ptr=it.hic_ptr.cpu().numpy(), bonds=it.hic_bonds[:it.nbonds * 16].cpu().numpy(),
                 xyz=it.xyz.cpu().numpy(), stats=it.stats.cpu().numpy(), score=np.float64(score),
                 info=it.info.cpu().numpy(), s0=s0, s1=s1, restored=restored)
    finally:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
