"""Inputs of the multi-rank AMIteration test (tests/test_distributed_gpu.py and its
worker): 8 demo structures (2 Mb), demo Hi-C pairs with p >= 0.05, a shortened demo
protocol."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden')


def inputs(nstruct=8):
    from igm_amd import model as M
    from igm_amd import synthetic as syn
    from igm_amd._lib import pair_dtype
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    hic = np.load(os.path.join(GOLDEN, 'demo_hic_pairs.npz'))
    keep = np.where(hic['p'] >= 0.05)[0]
    pairs = np.zeros(len(keep), pair_dtype)
    pairs['i'], pairs['j'], pairs['pwish'] = hic['i'][keep], hic['j'][keep], hic['p'][keep]
    atoms = M.Atoms(pop['radii'])
    xyz = np.zeros((nstruct, atoms.n, 3), np.float32)
    xyz[:, :atoms.nbead] = pop['coordinates'][:, :nstruct].transpose(1, 0, 2)
    proto = json.loads(json.dumps(syn.DEMO_PROTOCOL))
    proto['custom_annealing_protocol']['mdsteps'] = [100, 100, 100, 100]
    proto['custom_annealing_protocol']['relax']['mdsteps'] = 20
    prm = M.params_from_cfg({'optimization': {'optimizer_options': proto}}, [((5500.0,) * 3, 1.0)])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    chrom = np.concatenate([pop['chrom'], [-1]]).astype(np.int32)
    return dict(pop=pop, pairs=pairs, atoms=atoms, xyz=xyz, prm=prm, poly=poly, chrom=chrom)


def iteration(inp, device, s0, s1, rank=0, world=1, collective=None):
    from igm_amd.pipeline import AMIteration
    pop = inp['pop']
    return AMIteration(device, inp['xyz'][s0:s1], inp['atoms'], inp['chrom'], pop['copy_ptr'], pop['copy_idx'],
                       inp['pairs'], inp['prm'], inp['poly'], first_sid=s0, rank=rank, world=world,
                       collective=collective)
