"""Shared M-step inputs built from the golden fixtures (demo population, the
reference's own restraint selection and LAMMPS inputs)."""
import json
import os

import numpy as np

from conftest import GOLDEN

from igm_amd.synthetic import DEMO_PROTOCOL  # noqa: E402  (demo/config_file.json optimizer_options)


def load():
    pop = np.load(os.path.join(GOLDEN, 'demo_population.npz'))
    g3 = np.load(os.path.join(GOLDEN, 'mstep_inputs.npz'))
    return pop, g3


def demo_model(pop, protocol=None, envelope=((5500.0, 5500.0, 5500.0), 1.0)):
    """Atoms (3008 beads + the static envelope centre), polymer bonds, params."""
    from igm_amd import model as M
    atoms = M.Atoms(pop['radii'])
    poly = M.polymer_bonds(pop['chrom'], pop['copy'], pop['radii'], 2.0, 1.0)
    prm = M.params_from_cfg({'optimization': {'optimizer_options': protocol or DEMO_PROTOCOL}}, [envelope])
    chrom = np.concatenate([pop['chrom'], [-1]]).astype(np.int32)
    return atoms, poly, prm, chrom


def struct_major(pop, sids, natom):
    crd = pop['coordinates']
    x = np.zeros((len(sids), natom, 3), np.float32)
    x[:, :crd.shape[0]] = crd[:, sids, :].transpose(1, 0, 2)
    return x


def golden_bonds(g3, sid):
    """The reference LammpsModel bond list of structure sid (G3): (i, j, r0, k)."""
    from igm_amd._lib import bond_dtype
    b = g3['bonds_%d' % sid]
    bt = g3['bond_types_%d' % sid]
    out = np.zeros(len(b), bond_dtype)
    out['i'] = b[:, 0]
    out['j'] = b[:, 1]
    out['r0'] = bt[b[:, 2], 2]
    out['k'] = bt[b[:, 2], 1]
    return out


def hic_bonds_from_golden(g3, radii, sid, cr=2.0, k=1.0):
    """Hi-C bonds of the reference selection G4 (inter rows first, then intra)."""
    from igm_amd._lib import bond_dtype
    from igm_amd import model as M
    sel = np.concatenate([g3['sel_inter_%d' % sid], g3['sel_intra_%d' % sid]])
    b = np.zeros(len(sel), bond_dtype)
    b['i'] = sel[:, 0]
    b['j'] = sel[:, 1]
    b['r0'] = M.r0_contact(cr, radii[sel[:, 0]], radii[sel[:, 1]]).astype(np.float32)
    b['k'] = k
    cls = np.concatenate([np.full(len(g3['sel_inter_%d' % sid]), M.CLASS_INTER_HIC),
                          np.full(len(g3['sel_intra_%d' % sid]), M.CLASS_INTRA_HIC)]).astype(np.int32)
    return b, cls
