"""Timing of the face scan under CTG_ABLATE values given on the command line
(each in a child process; stderr carries the s_memtime stamp line for 256)."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == '--child':
    sys.path.insert(0, ROOT)
    import torch
    from cluster_tools_amd import rag
    S = int(os.environ.get('CTG_PROF_SIZE', '512'))
    lab, bnd = rag.synth_volume((S, S, S), cell=int(os.environ.get('CTG_PROF_CELL', '10')))
    torch.cuda.synchronize()
    r = None
    for i in range(3):
        if r: r.free()
        r = rag.rag_features_handle(lab, bnd)
    rag.set_profiling(True)
    ts = []
    for i in range(5):
        r.free(); r = rag.rag_features_handle(lab, bnd); ts.append(rag.last_timings())
    print(json.dumps({'lib': os.path.basename(os.environ.get('CTG_LIB', 'libctg.so')),
                      'ablate': os.environ.get('CTG_ABLATE', '0'),
                      'check': os.environ.get('CTG_CHECK_PLANES', '-'), 'tz': os.environ.get('CTG_TILE_Z', '-'), 'records': r.info()[0],
                      **{k: round(sum(t[k] for t in ts) / len(ts), 4) for k in ts[0]}}), flush=True)
else:
    # spec: "<variant>@<ablate>[@<check_planes>[@<tile_z>]]" (variant -> variants/libctg_<variant>.so)
    for spec in sys.argv[1:]:
        parts = spec.split('@')
        var, ab = (parts[0], parts[1]) if len(parts) > 1 else ('', parts[0])
        env = dict(os.environ, CTG_ABLATE=ab or '0')
        if len(parts) > 2 and parts[2]:
            env['CTG_CHECK_PLANES'] = parts[2]
        if len(parts) > 3 and parts[3]:
            env['CTG_TILE_Z'] = parts[3]
        if var:
            env['CTG_LIB'] = os.path.join(ROOT, 'variants', 'libctg_%s.so' % var)
        subprocess.run([sys.executable, os.path.abspath(__file__), '--child'], env=env, check=True)
