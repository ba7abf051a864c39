"""Where the 12-channel long-range affinity scan spends its time: the scan's
device ms for channel subsets of test_mws.py:26-29's offsets on the same
1024^3 volume (NN only, NN + the z / y / x long-range channels, all 12), each
with and without the Bloom prefilter's probes (CTG_ABLATE=512 needs a
CTG_DIAG build: CTG_LIB=variants/libctg_diag.so)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cluster_tools_amd import rag, synthetic  # noqa: E402

S = int(os.environ.get('CTG_PROF_SIZE', '1024'))
lab, bnd = rag.synth_volume((S, S, S), cell=10)
off = synthetic.LR_OFFSETS
affs = rag.synth_affinities(bnd, off)
del bnd
subsets = {'nn': [0, 1, 2], 'nn+z': [0, 1, 2, 3, 6, 9], 'nn+y': [0, 1, 2, 4, 7, 10], 'nn+x': [0, 1, 2, 5, 8, 11],
           'all': list(range(12))}
rag.set_profiling(True)
for name, idx in subsets.items():
    if name == 'all' and os.environ.get('CTG_ABLATE') == '512':
        continue   # without the probes the x / y channels' non-edge records exceed the workspace
    a = affs if len(idx) == 12 else affs[idx].contiguous()
    o = [off[i] for i in idx]
    ts = []
    for it in range(4):
        r = rag.rag_features_handle(lab, a, offsets=o)
        if it:
            ts.append(rag.last_timings())
        info = r.info()
        r.free()
    del a
    torch.cuda.empty_cache()
    print(json.dumps({'subset': name, 'ablate': os.environ.get('CTG_ABLATE', '0'), 'records': info[0],
                      **{k: round(sum(t[k] for t in ts) / len(ts), 3) for k in ('scan', 'sort', 'reduce', 'total')}}),
          flush=True)
