"""A/B of libctg.so builds (variants/libctg_<name>.so) on the BASELINE workloads.

usage: ab_variants.py <workload>[,<workload>...] <variant> [<variant> ...]
  workloads: b512 (configs[1]), b1024c5 (configs[4]), nn1024 / lr1024 (configs[3]),
             b2048 (configs[2]);  variant "base" = cluster_tools_amd/libctg.so
Each (variant, workload) runs in its own child process: 2 warm-up calls, 5
timed calls; one JSON line with the per-phase device ms and a result checksum
(edges, sum of counts, sum of means) so that variants can be compared.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = {'b512': (512, 10, None), 'b1024c5': (1024, 5, None), 'nn1024': (1024, 10, 'nn'), 'lr1024': (1024, 10, 'lr'),
     'b2048': (2048, 16, None), 'lr512': (512, 10, 'lr')}

if len(sys.argv) > 1 and sys.argv[1] == '--child':
    sys.path.insert(0, ROOT)
    import torch
    from cluster_tools_amd import rag, synthetic
    wl = sys.argv[2]
    S, cell, aff = W[wl]
    lab, bnd = rag.synth_volume((S, S, S), cell=cell)
    data, off = bnd, None
    if aff:
        off = synthetic.NN_OFFSETS if aff == 'nn' else synthetic.LR_OFFSETS
        data = rag.synth_affinities(bnd, off)
        del bnd
    torch.cuda.synchronize()
    r = None
    for _ in range(2):
        if r:
            r.free()
        r = rag.rag_features_handle(lab, data, offsets=off)
    rag.set_profiling(True)
    ts = []
    for _ in range(5):
        r.free()
        r = rag.rag_features_handle(lab, data, offsets=off)
        ts.append(rag.last_timings())
    f = r.features_torch()
    out = {'lib': os.path.basename(os.environ.get('CTG_LIB', 'libctg.so')), 'workload': wl,
           'env': {k: v for k, v in os.environ.items() if k.startswith('CTG_') and k != 'CTG_LIB'},
           'records': r.info()[0], 'direct': r.info()[1], 'edges': r.n_edges,
           'sum_count': float(f[:, 9].sum().item()), 'sum_mean': float(f[:, 0].sum().item()),
           'sum_q50': float(f[:, 5].sum().item())}
    out.update({k: round(sum(t[k] for t in ts) / len(ts), 4) for k in ts[0]})
    print(json.dumps(out), flush=True)
else:
    wls = sys.argv[1].split(',')
    for wl in wls:
        for spec in sys.argv[2:]:
            # "<variant>[@ENV=val[,ENV=val...]]"
            var, _, envs = spec.partition('@')
            env = dict(os.environ)
            for kv in filter(None, envs.split(',')):
                k, _, v = kv.partition('=')
                env[k] = v
            if var != 'base':
                env['CTG_LIB'] = os.path.join(ROOT, 'variants', 'libctg_%s.so' % var)
            subprocess.run([sys.executable, os.path.abspath(__file__), '--child', wl], env=env, check=True,
                           timeout=300)
