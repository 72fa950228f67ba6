"""Append the breakdowns of gpu_variants.sh runs (gpurun_out/<tag>/v*.log) to profiles/r04_ab/ab_runs.jsonl.
usage: python scripts/ab_collect.py TAG [TAG ...]"""
import glob
import json
import os
import sys

out = os.path.join(os.path.dirname(__file__), '..', 'profiles', 'r04_ab', 'ab_runs.jsonl')
with open(out, 'a') as f:
    for tag in sys.argv[1:]:
        for log in sorted(glob.glob('gpurun_out/%s/v*.log' % tag), key=lambda p: int(p.rsplit('v', 1)[1][:-4])):
            lines = [l for l in open(log) if l.startswith('{')]
            if not lines:
                continue
            b = json.loads(lines[-1])['breakdown']
            f.write(json.dumps({'run': '%s/%s' % (tag, os.path.basename(log)), 'anneal_ms': b['anneal_ms'],
                                'cg_ms': b['cg_ms'], 'mean_rebuilds': b['mean_rebuilds'],
                                'violation_score': b['violation_score']}) + '\n')
