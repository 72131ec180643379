"""Diagnostic: full-step parity errors (values + parameter gradients) vs the reference fixture."""
import os, sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))] + [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), d) for d in ('tests', 'tests/golden')]
import numpy as np, torch
import test_gpu_parity as T
import common as G
for which in ('fusion', 'mono'):
    cfg_fn, fixture, seed = (G.step_cfg, 'step_small.npz', 5) if which == 'fusion' else (G.mono_cfg, 'mono_small.npz', 6)
    cfg, fx, algo, inputs, outputs, losses = T._step(cfg_fn, fixture, seed)
    named = {f'{m}.{p}': q for m, mod in algo.models.items() for p, q in mod.named_parameters()}
    for key in [k for k in fx.files if k.startswith('grad__')]:
        a = named[key[6:]].grad.detach().double().cpu().numpy(); b = fx[key].astype(np.float64)
        print(which, key[6:], 'max/scale %.3g' % (np.abs(a-b).max()/np.abs(b).max()), 'fro %.3g' % (np.linalg.norm(a-b)/np.linalg.norm(b)), flush=True)
    got = outputs[('cam', 0)][('reproj_mask', 0)].detach().cpu()
    print(which, 'automask flips cam0:', int(((got != 0) != (torch.tensor(fx['c0_reproj_mask_0']) != 0)).sum()))
    for k in [k for k in fx.files if k.startswith('loss_')]:
        print(which, k, float(losses[k[5:]]), float(fx[k]))
