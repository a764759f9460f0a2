import os, sys
sys.path.insert(0, os.getcwd())
if sys.argv[1] == 'torch':
    import torch
    torch.cuda.set_device(0)
    x = torch.zeros(10, device='cuda')
from reporter_amd import matcher as M
from reporter_amd.tools import gen
path = gen.graph_path('metro', 'build/graphs')
M.configure(M.default_config(path, turn_penalty_factor=0))
tr = gen.make_traces(path, 300, 100, 15, 10.0, 2)
m = M.Matcher()
r = m.match_batch(tr, copy_out=False)
print(sys.argv[1], 'status', r.status)
