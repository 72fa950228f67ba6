"""Diagnostic (not product): one config C A/M iteration on 4 structures; the reported
optimisation info against the energies of the returned coordinates (GPU f64 forces and
the fp64 oracle, with the structure's own Hi-C bonds)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    import oracle
    from igm_amd import mstep
    from igm_amd._lib import bond_dtype
    args = bench.parse()
    args.config, args.nstruct, args.sigma = 'C', 4, 0.01
    if os.environ.get('DIAG_SCALE'):
        args.protocol_scale = float(os.environ['DIAG_SCALE'])
    inp = bench.build_inputs(args, 0)
    from igm_amd.pipeline import AMIteration
    pop = inp['pop']
    it = AMIteration(torch.device('cuda', 0), inp['xyz'], inp['atoms'], inp['chrom'], pop['copy_ptr'],
                     pop['copy_idx'], inp['pairs'], inp['prm'], inp['poly'])
    it.step()
    info = it.info_host()
    x = it.xyz.cpu().numpy()
    ptr = it.hic_ptr.cpu().numpy()
    bonds = it.hic_bonds.cpu().numpy().view(bond_dtype)[:ptr[-1]]
    at = inp['atoms']
    print('info final/pair/bond/einitial/temp/cg_iters/stop/nrebuild')
    for s in range(4):
        print(s, info['final_energy'][s], info['pair_energy'][s], info['bond_energy'][s], info['einitial'][s],
              info['temp'][s], info['cg_iters'][s], info['stop_reason'][s], info['nrebuild'][s])
    fg, eg = mstep.forces(inp['prm'], x, at.radii, at.flags, inp['poly'], ptr, bonds, 1.0, 1.0)
    fo, eo = oracle.mstep_forces(inp['prm'], x, at.radii, at.flags, inp['poly'], ptr, bonds, 1.0, 1.0)
    print('GPU forces energies', eg[:, :4])
    print('oracle energies', eo[:, :4])


if __name__ == '__main__':
    main()
