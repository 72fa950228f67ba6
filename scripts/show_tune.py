import glob, json, sys
for f in sorted(glob.glob('gpurun_out/tune_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l); b = d['breakdown']; p = d.get('profile')
            s = '%-28s value %8.2f anneal_ms %9.1f cg_ms %7.1f rebuilds %7.1f frac %.3f' % (
                f, d['value'], b['anneal_ms'], b['cg_ms'], b.get('mean_rebuilds', -1), d['roofline']['frac'])
            if p:
                tot = p['build_cycles'] + p['force_cycles'] + p['rest_cycles']
                s += ' | cyc/eval %.0f build %.2f force %.2f rest %.2f' % (tot / p['evaluations'], p['build_cycles'] / tot,
                                                                       p['force_cycles'] / tot, p['rest_cycles'] / tot)
                if p.get('walk_cycles'):
                    s += ' walk %.2f cyc/build %.0f' % (p['walk_cycles'] / tot, p['build_cycles'] / max(p['builds'], 1))
            print(s)
