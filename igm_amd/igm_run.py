"""The igm-run pipeline body on the Step layer (bin/igm-run:50-325): the
start-up steps, then A/M iterations until every data set's threshold list is used
up with an acceptable violation score, or max_iterations unsuccessful iterations.

  start-up   starting_coordinates copied, or RandomInit [+ PolymerAssignmentStep when
             the chain is modelled by distance distributions] + RelaxInit (:50-82)
  iteration  PolymerAssignmentStep (restraints/polymer), ActivationDistanceStep
             (Hi-C), FishAssignmentStep (FISH), SpriteAssignmentStep (sprite),
             DamidActivationDistanceStep (DamID), ModelingStep (:105-167), in that order
  control    is_acceptable = runtime/violation_score < optimization/max_violations;
             the threshold lists advance together when acceptable and no further
             iteration is forced (min_iterations, force_last_iteration,
             force_minimum_iterations_hic_cutoff), else opt_iter += 1 (:169-325)

Unsupported sections (tracing, nuclDamID, nucleolus) raise where the reference would
run them.  Preprocess (genome/index, .hss allocation) is the caller's: the population
file must exist.  No email notifications, no control socket.
"""
import os
import shutil

from . import steps as ST


def startup_steps(cfg):
    """bin/igm-run:50-82"""
    start = ST.cget(cfg, 'model/starting_coordinates', '')
    if start:
        if ST.cget(cfg, 'optimization/clean_restart', False) or \
                not os.path.isfile(ST.cget(cfg, 'parameters/step_db', 'stepdb.sqlite')):
            out = cfg['optimization']['structure_output']
            if os.path.abspath(start) != os.path.abspath(out):
                shutil.copyfile(start, out)
        return []
    steps = [ST.RandomInit]
    if 'polymer' not in cfg['model']['restraints']:
        steps.append(ST.PolymerAssignmentStep)
    steps.append(ST.RelaxInit)
    return steps


def iteration_steps(cfg):
    """bin/igm-run:105-161"""
    R = cfg.get('restraints', {})
    for key in ('nuclDamID', 'tracing'):
        if key in R:
            raise NotImplementedError('restraints/%s is not implemented on the hip kernel' % key)
    steps = []
    if 'polymer' in R:
        steps.append(ST.PolymerAssignmentStep)
    if 'Hi-C' in R:
        steps.append(ST.ActivationDistanceStep)
    if 'FISH' in R:
        steps.append(ST.FishAssignmentStep)
    if 'sprite' in R:
        steps.append(ST.SpriteAssignmentStep)
    if 'DamID' in R:
        steps.append(ST.DamidActivationDistanceStep)
    steps.append(ST.ModelingStep)
    return steps


def _remaining(cfg, section, key):
    return section in cfg.get('restraints', {}) and len(ST.cget(cfg, 'runtime/%s/%s' % (section, key), [])) != 0


def run_pipeline(cfg, on_iteration=None):
    """Run the pipeline; returns 'completed' or 'max_iterations'.  on_iteration(cfg,
    opt_iter, steps) is called after every A/M iteration (tests, logging)."""
    rt = cfg.setdefault('runtime', {})
    for k in cfg.get('restraints', {}):  # Config.__init__ gives every restraint a runtime section
        rt.setdefault(k, {})
    for S in startup_steps(cfg):
        S(cfg).run()
    opt_iter = 0
    min_iter = ST.cget(cfg, 'optimization/min_iterations', 5)
    max_iter = ST.cget(cfg, 'optimization/max_iterations', 12)
    while True:
        rt['opt_iter'] = opt_iter
        steps = iteration_steps(cfg)
        for S in steps:
            S(cfg).run()
        if on_iteration is not None:
            on_iteration(cfg, opt_iter, steps)
        acceptable = ST.cget(cfg, 'runtime/violation_score') < ST.rget(cfg, 'optimization/max_violations', 0.01)
        hic_inc = 'Hi-C' in cfg.get('restraints', {}) and (
            len(ST.cget(cfg, 'runtime/Hi-C/intra_sigma_list', [])) != 0 or
            len(ST.cget(cfg, 'runtime/Hi-C/inter_sigma_list', [])) != 0)
        damid_inc = _remaining(cfg, 'DamID', 'sigma_list')
        fish_inc = _remaining(cfg, 'FISH', 'tol_list')
        sprite_inc = _remaining(cfg, 'sprite', 'volume_fraction_list')
        all_done = not (hic_inc or damid_inc or fish_inc or sprite_inc)
        force = (opt_iter < min_iter - 1) and (opt_iter != 0)
        if ST.cget(cfg, 'optimization/force_last_iteration', False) and all_done and opt_iter == 0:
            force = True
        if 'Hi-C' in cfg.get('restraints', {}) and opt_iter == 0 and \
                ST.cget(cfg, 'runtime/Hi-C/intra_sigma') <= ST.cget(cfg, 'optimization/force_minimum_iterations_hic_cutoff',
                                                                  0.0):
            force = True
        if acceptable and not force:
            if hic_inc:
                del rt['Hi-C']['intra_sigma']
                del rt['Hi-C']['inter_sigma']
                opt_iter = 0
            if damid_inc:
                del rt['DamID']['sigma']
                opt_iter = 0
            if fish_inc:
                del rt['FISH']['tol']
                opt_iter = 0
            if sprite_inc:
                del rt['sprite']['volume_fraction']
                opt_iter = 0
            if all_done:
                open(os.path.join(ST.cget(cfg, 'parameters/workdir', '.'), 'completed'), 'w').close()
                return 'completed'
        else:
            opt_iter += 1
            if max_iter is not None and opt_iter >= max_iter:
                return 'max_iterations'
