import os, sys, time, json, subprocess
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1:
    import torch
    from cluster_tools_amd import rag
    S = 512
    lab, bnd = rag.synth_volume((S, S, S), cell=10)
    torch.cuda.synchronize()
    mode = sys.argv[1]
    out = {}
    for name, d in (('graph', None), ('boundary', bnd)):
        r = None
        for i in range(3):
            if r: r.free()
            r = rag.rag_features_handle(lab, d)
        rag.set_profiling(True)
        ts = []
        for i in range(5):
            r.free(); r = rag.rag_features_handle(lab, d); ts.append(rag.last_timings())
        rag.set_profiling(False)
        out[name] = {k: round(sum(t[k] for t in ts) / len(ts), 4) for k in ts[0]}
        r.free()
    print(json.dumps({'ablate': mode, **out}), flush=True)
else:
    for ab in ['0', '8', '32', '64', '128']:
        env = dict(os.environ, CTG_ABLATE=ab)
        subprocess.run([sys.executable, __file__, ab], env=env, check=True)
