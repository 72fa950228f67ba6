"""`optimization/kernel = 'hip'`: the drop-in for lammps.optimize
(igm/model/kernel/lammps.py:361-492) selected by Model.optimize
(igm/model/model.py:130-137).

Same contract: mutates model.particles[i].pos in place (lammps.py:467-468) and
returns the info dict {final-energy, pair-energy, bond-energy, md-time, thermo}.
A failing GPU call raises RuntimeError (lammps.py:453-457).  One structure per
call here; the batched path (igm_amd.pipeline) is what the engine is built for.
"""
import time

import numpy as np

from . import model as M
from . import mstep


def optimize(model, cfg, ctx=None):
    lm = M.from_igm_model(model)
    prm = M.params_from_cfg(cfg, lm.envelopes, evfactor=lm.evfactor)
    opt = cfg['optimization']['optimizer_options']
    # cfg.get('runtime/step_no', 1) as lammps.py:435 reads it (Config keypath get)
    step_no = cfg.get('runtime', {}).get('step_no', 1) if hasattr(cfg, 'get') else 1
    seeds = M.lammps_seeds(opt.get('seed', 6535), [lm.id], step_no)
    t0 = time.time()
    x, info = mstep.run(prm, lm.xyz[None], lm.radii, lm.flags, lm.bonds, None, None, seeds, ctx=ctx)
    dt = time.time() - t0
    for i, p in enumerate(model.particles):
        p.pos = x[0, lm.imap[i]].copy()
    ienv = info['env_energy'][0]
    thermo = {'Temp': float(info['temp'][0]), 'E_pair': float(info['pair_energy'][0]),
              'E_bond': float(info['bond_energy'][0])}
    for e in range(len(lm.envelopes)):
        thermo['f_envelope%d' % e] = float(ienv[e])
    return {'final-energy': float(info['final_energy'][0]), 'pair-energy': float(info['pair_energy'][0]),
            'bond-energy': float(info['bond_energy'][0]), 'md-time': dt, 'thermo': thermo}
