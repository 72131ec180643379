"""Diagnostic: stage-by-stage comparison of the GPU full step with the CPU oracle step on the
same weights / inputs / noise: the depth net's 1/8 aggregation (conv1x1 output), the decoder's
fused-feature input, the encoder skips and the disparity — forward values and gradients."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import common as G  # noqa: E402
from oracle import vfd_oracle as O  # noqa: E402
from vfdepth_amd import synth  # noqa: E402
from vfdepth_amd.layers import seeded_state_dict  # noqa: E402
from vfdepth_amd.network import FusedDepthNet, FusedPoseNet  # noqa: E402
from vfdepth_amd.vfdepth import VFDepthAlgo  # noqa: E402


def attach(dnet, st):
    def keep(name, t):
        st[name] = t
        if t.requires_grad:
            t.register_hook(lambda g: st.__setitem__('d_' + name, g))

    dnet.conv1x1.register_forward_hook(lambda m, i, o: keep('agg', o))            # CPU oracle path
    dnet.fusion_net.register_forward_pre_hook(lambda m, args: keep('agg', args[1]))  # GPU (fused aggregate)

    def pre(m, args):
        feats = args[0]
        keep('proj', feats[-1])
        for i, f in enumerate(feats[:-1]):
            keep(f'skip{i}', f)
    dnet.decoder.register_forward_pre_hook(pre)
    dnet.decoder.register_forward_hook(lambda m, i, o: keep('disp', o[('disp', 0)]))


fx = np.load(os.path.join(ROOT, 'tests', 'golden', 'step_small.npz'))
cfg = G.step_cfg()
N = cfg['data']['num_cams']
noise = torch.stack([torch.tensor(fx[f'noise_c{c}']) for c in range(N)])
inputs = synth.make_batch(cfg, seed=5, with_depth=True)
cpu_inputs = {k: v.clone() if torch.is_tensor(v) else v for k, v in inputs.items()}

algo = VFDepthAlgo(cfg, 0)
for m in algo.models.values():
    m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
algo.set_train()
sg = {}
attach(algo.models['depth_net'], sg)
_, lg = algo.process_batch(inputs, 0, noise=noise.cuda())
lg['total_loss'].backward()
torch.cuda.synchronize()

torch.set_num_threads(16)
dn, pn = FusedDepthNet(cfg), FusedPoseNet(cfg)
dn.load_state_dict(seeded_state_dict(dn, seed=G.STEP_SEED))
pn.load_state_dict(seeded_state_dict(pn, seed=G.STEP_SEED))
dn.train()
pn.train()
sc = {}
attach(dn, sc)
_, lc = O.process_batch(O.nets_from_modules(dn, pn), cpu_inputs, cfg, [n for n in noise])
lc['total_loss'].backward()
print('total loss gpu %.9f cpu %.9f fixture %.9f' % (float(lg['total_loss']), float(lc['total_loss']),
                                                      float(fx['loss_total_loss'])))
for k in sorted(k for k in sc if k in sg):
    a, b = sg[k].detach().double().cpu(), sc[k].detach().double()
    if a.shape != b.shape:
        a = a.reshape(b.shape)
    print('%-8s fwd/grad max/scale %.3g  fro %.3g  (scale %.3g)' % (
        k, float((a - b).abs().max() / b.abs().max()), float((a - b).norm() / b.norm()), float(b.abs().max())))
gnamed = dict(algo.models['depth_net'].named_parameters())
for k, p in dn.named_parameters():
    a, b = gnamed[k].grad.double().cpu(), p.grad.double()
    r = float((a - b).norm() / max(b.norm(), 1e-30))
    if r > 5e-4:
        print('param %-55s grad fro %.3g' % (k, r))
