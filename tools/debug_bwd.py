import sys, numpy as np, torch
sys.path[:0] = ['3dgs_study_amd', 'tests', '.']
from helpers import case, run_hip, run_oracle, rel_l2, random_dL
from oracle import oracle
dev = torch.device('cuda:0')
for P, W, H in ((1, 32, 32), (3, 32, 32), (50, 64, 64), (2000, 128, 128)):
    cam, g = case(P, W, H, 0, seed=1, radius=0.5, scale_range=(0.02, 0.05))
    dL = random_dL(H, W)
    h = run_hip(cam, g, dev, dL=dL)
    r = run_oracle(oracle, cam, g)
    rb = oracle.backward(r, dL)
    print(P, 'I', h['num_rendered'], r['num_rendered'], 'maxc', h['tile_max_contrib'].max())
    for n in ('dcolors', 'dopacity', 'dmeans2D'):
        print('  ', n, rel_l2(h['grads'][n], rb[n]))
    if P <= 3:
        print('  hip dcolors', h['grads']['dcolors'][:3])
        print('  ref dcolors', rb['dcolors'][:3])
        print('  hip dop', h['grads']['dopacity'][:3].ravel(), 'ref', rb['dopacity'][:3].ravel())
