"""M-step violation records -> the reference's per-structure `violation_stats` and the
population `summary`.

  restraint_key      -- repr(restraint) the reference uses as the vstat key
                        (restraints/restraint.py:95-96 type name; Envelope
                        envelope.py:65-66; ExpEnvelope genenvelope.py:60-61)
  vstat_from_record  -- ModelingStep.task's vstat dict (ModelingStep.py:519-557) from one
                        structure's igm_mstep_violations record (counts[101],
                        violated_restr, n_violations, n_imposed per restraint class)
  PopulationSummary  -- ModelingStep.setup_poller / set_structure / teardown_poller
                        (ModelingStep.py:578-725): the summary JSON of the .hss and
                        runtime/violation_score = sum(n_violations) / sum(n_imposed)
"""
import json

import numpy as np

DEFAULT_HIST_BINS = 100  # ModelingStep.py:27-28
DEFAULT_HIST_MAX = 0.1


def restraint_key(kind, **kw):
    if kind == 'Envelope':
        return 'Envelope[shape={},k={},a={},b={},c={}]'.format(kw['shape'], kw['k'], kw['a'], kw['b'], kw['c'])
    if kind == 'ExpEnvelope':
        return 'ExpEnvelope[shape={},map={},k={}]'.format(kw.get('shape', 'exp_map'), kw['volume_file'], kw['k'])
    return kind  # Polymer, interHiC, intraHiC, Damid, Sprite, Fish, ...: type(self).__name__


def _edges(nbins=DEFAULT_HIST_BINS, vmax=1):
    e = np.histogram([], bins=nbins, range=(0, vmax))[1]
    return np.concatenate([e, [np.inf]])


def vstat_from_record(rec, names):
    """rec: (ncls, 104) int64 of igm_mstep_violations; names: the vstat key per class."""
    rec = np.asarray(rec)
    edges = _edges().tolist()
    out = {}
    for c, name in enumerate(names):
        if name is None:  # a record class the configuration does not monitor
            continue
        out[name] = {'histogram': {'edges': edges, 'counts': [int(x) for x in rec[c, :101]]},
                     'violated_restr': int(rec[c, 101]), 'n_violations': int(rec[c, 102]),
                     'n_imposed': int(rec[c, 103])}
    return out


class PopulationSummary(object):
    """The poller's accumulation over the structures of one M-step."""

    def __init__(self, population_size):
        n = int(population_size)
        self.n = n
        self.data = {
            'n_imposed': 0.0, 'n_violations': 0.0, 'violated_restr': 0.0,
            'histogram': {'counts': np.zeros(DEFAULT_HIST_BINS + 1),
                          'edges': np.arange(0, DEFAULT_HIST_MAX, DEFAULT_HIST_MAX / DEFAULT_HIST_BINS).tolist()
                          + [DEFAULT_HIST_MAX, np.inf]},
            'bystructure': {k: np.zeros(n, dtype=np.float32) for k in
                            ('n_imposed', 'n_violations', 'violated_restr', 'total_energies', 'pair_energies',
                             'bond_energies')},
            'byrestraint': {},
        }
        self.data['bystructure']['thermo'] = {}

    def set_structure(self, i, vstat, optinfo=None):
        """ModelingStep.set_structure (py:611-700) for structure i."""
        d = self.data
        n_tot = n_vio = ex_vio = 0
        hist_tot = np.zeros(DEFAULT_HIST_BINS + 1)
        for k, cstat in vstat.items():
            if k not in d['byrestraint']:
                d['byrestraint'][k] = {'histogram': {'counts': np.zeros(DEFAULT_HIST_BINS + 1)}, 'n_violations': 0,
                                       'violated_restr': 0, 'n_imposed': 0,
                                       'viol_by_struct': np.zeros(self.n, dtype=np.float32),
                                       'imposed_by_struct': np.zeros(self.n, dtype=np.float32)}
            r = d['byrestraint'][k]
            n_tot += cstat.get('n_imposed', 0)
            n_vio += cstat.get('n_violations', 0)
            ex_vio += cstat.get('violated_restr', 0)
            hist_tot += cstat['histogram']['counts']
            r['n_violations'] += cstat.get('n_violations', 0)
            r['n_imposed'] += cstat.get('n_imposed', 0)
            r['violated_restr'] += cstat.get('violated_restr', 0)
            r['viol_by_struct'][i] = cstat.get('n_violations', 0)
            r['imposed_by_struct'][i] = cstat.get('n_imposed', 0)
            r['histogram']['counts'] += cstat['histogram']['counts']
        d['n_imposed'] += n_tot
        d['n_violations'] += n_vio
        d['violated_restr'] += ex_vio
        d['histogram']['counts'] += hist_tot
        bs = d['bystructure']
        bs['n_imposed'][i], bs['n_violations'][i], bs['violated_restr'][i] = n_tot, n_vio, ex_vio
        if optinfo is not None:
            bs['total_energies'][i] = optinfo['final-energy']
            bs['pair_energies'][i] = optinfo['pair-energy']
            bs['bond_energies'][i] = optinfo['bond-energy']
            for k, v in optinfo.get('thermo', {}).items():
                bs['thermo'].setdefault(k, np.zeros(self.n))[i] = v

    def violation_score(self):
        """teardown_poller (py:703-716)."""
        tot = self.data['n_imposed']
        return 0 if tot == 0 else self.data['n_violations'] / tot

    def to_json(self):
        return json.dumps(self.data, default=lambda a: a.tolist())
