"""Same-box A/B of the frustrated shard and the config E M-step blocks of bench.py under the
environment settings in VARIANTS ("K=V K2=V2;K=V ..."), blocks in BLOCKS (frustrated,D,E), one JSON
line per variant."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402
import bench  # noqa: E402

variants = [v for v in os.environ.get('VARIANTS', '').split(';') if v.strip()]
blocks = os.environ.get('BLOCKS', 'frustrated,E').split(',')
sys.argv = [sys.argv[0], '--gpus', '1']
args = bench.parse()
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
for v in variants:
    env = dict(kv.split('=', 1) for kv in v.split())
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        out = {'variant': v}
        if 'frustrated' in blocks:
            r = bench.bench_frustrated(args, dev, 125)
            out['frustrated'] = {k: r[k] for k in ('mstep_s', 'anneal_ms', 'cg_ms', 'mean_rebuilds')}
        for cfg in ('D', 'E'):
            if cfg in blocks:
                r = bench.bench_mstep_de(args, dev, cfg, 125)
                out[cfg] = {k: r[k] for k in ('mstep_s', 'anneal_ms', 'cg_ms', 'mean_rebuilds')}
        print(json.dumps(out), flush=True)
    finally:
        for k, val in old.items():
            if val is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = val
        torch.cuda.empty_cache()
