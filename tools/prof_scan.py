"""Run the hot path a few times on a resident synthetic volume (for rocprofv3).

usage: prof_scan.py [boundary|graph|nn|lr]   (CTG_PROF_SIZE, CTG_PROF_CELL,
CTG_PROF_ITERS select the cube edge, cell size and repetitions;
CTG_PROF_CHANNELS="0,1,2,..." a subset of the affinity channels)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cluster_tools_amd import rag, synthetic  # noqa: E402

S = int(os.environ.get('CTG_PROF_SIZE', '512'))
mode = sys.argv[1] if len(sys.argv) > 1 else 'boundary'
lab, bnd = rag.synth_volume((S, S, S), cell=int(os.environ.get('CTG_PROF_CELL', '10')))
data, offsets = bnd, None
if mode in ('nn', 'lr'):
    offsets = synthetic.NN_OFFSETS if mode == 'nn' else synthetic.LR_OFFSETS
    data = rag.synth_affinities(bnd, offsets)
    del bnd
    if os.environ.get('CTG_PROF_CHANNELS'):
        idx = [int(c) for c in os.environ['CTG_PROF_CHANNELS'].split(',')]
        data, offsets = data[idx].contiguous(), [offsets[i] for i in idx]
        torch.cuda.empty_cache()
elif mode == 'graph':
    data = None
torch.cuda.synchronize()
for _ in range(int(os.environ.get('CTG_PROF_ITERS', '3'))):
    r = rag.rag_features_handle(lab, data, offsets=offsets)
    n_rec, n_direct = r.info()
    r.free()
torch.cuda.synchronize()
# records x (8-B key + 128-B body): the scan's nominal record writes, to set
# beside its WRITE_SIZE
print('done', mode, 'records=%d direct_faces=%d record_bytes=%d' % (n_rec, n_direct, n_rec * 136))
