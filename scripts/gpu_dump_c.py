"""Anneal 4 config C (200 kb) structures through two A/M iterations (full protocol) and
save the final coordinates (tuning/planning data: domain/halo statistics for a
domain-decomposed engine).  -> gpurun_out/configC_final.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    args = bench.parse()
    args.config, args.nstruct, args.sigma = 'C', 4, 0.01
    inp = bench.build_inputs(args, 0)
    from igm_amd.pipeline import AMIteration
    pop = inp['pop']
    it = AMIteration(torch.device('cuda', 0), inp['xyz'], inp['atoms'], inp['chrom'], pop['copy_ptr'],
                     pop['copy_idx'], inp['pairs'], inp['prm'], inp['poly'])
    it.step()  # the first M-step from the random territories ends frustrated (E ~ 1e4 per bead)
    it.step()  # the second, the bench's timed iteration, relaxes to E ~ 0
    x = it.xyz.cpu().numpy()[:, :inp['atoms'].nbead]
    os.makedirs('gpurun_out', exist_ok=True)
    np.savez_compressed('gpurun_out/configC_final.npz', xyz=x, radii=inp['atoms'].radii[:inp['atoms'].nbead],
                        chrom=pop['chrom'])
    print('saved', x.shape, 'rebuilds', it.info_host()['nrebuild'])


if __name__ == '__main__':
    main()
