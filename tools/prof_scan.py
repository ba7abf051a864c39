"""Run the hot path a few times on the 512^3 bench volume (for rocprofv3)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cluster_tools_amd import rag  # noqa: E402

S = int(os.environ.get('CTG_PROF_SIZE', '512'))
mode = sys.argv[1] if len(sys.argv) > 1 else 'boundary'
lab, bnd = rag.synth_volume((S, S, S), cell=int(os.environ.get('CTG_PROF_CELL', '10')))
torch.cuda.synchronize()
for _ in range(int(os.environ.get('CTG_PROF_ITERS', '3'))):
    r = rag.rag_features_handle(lab, bnd if mode == 'boundary' else None)
    r.free()
torch.cuda.synchronize()
print('done', mode)
