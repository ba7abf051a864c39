"""Single-GPU cost model of the z-slab distributed step (cluster_tools_amd/dist.py):
times the rank-local pieces that do not need a second GPU - the local
keep_stats call, the device copies/packing of the partial rows and the merge
of (all) of them - next to the plain single-GPU call."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cluster_tools_amd import dist as D  # noqa: E402
from cluster_tools_amd import rag  # noqa: E402

S = int(os.environ.get('CTG_PROF_SIZE', '512'))
lab, bnd = rag.synth_volume((S + 1, S, S), cell=10)
own = (1, 0, 0)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def plain():
    r = rag.rag_features_handle(lab, bnd, own_begin=own)
    r.free()


be = D.HipBackend()
state = {}


def local():
    state['loc'] = be.local(lab, bnd, None, own, None, False, (0.0, 1.0))


def pack():
    k, s, r, n, i, f = state['loc']
    state['rows'] = D.pack_rows(k, s, r)


def merge():
    k, s, r = D.unpack_rows(state['rows'])
    be.merge(k, s, r, (0.0, 1.0))


out = {'plain_ms': timed(plain), 'local_keep_stats_ms': timed(local), 'pack_ms': timed(pack),
       'merge_all_rows_ms': timed(merge), 'rows': int(state['rows'].shape[0])}
print(json.dumps(out))
