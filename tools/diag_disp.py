"""Diagnostic: d(total loss)/d(disp) of the GPU step vs the CPU oracle's loss path evaluated on
the GPU's own disparities and poses (isolates the view-synthesis + loss backward from the nets),
plus per-camera decision mismatches (auto-mask, colour / overlap masks)."""
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
from vfdepth_amd.vfdepth import VFDepthAlgo  # noqa: E402

fx = np.load(os.path.join(ROOT, 'tests', 'golden', 'step_small.npz'))
cfg = G.step_cfg()
algo = VFDepthAlgo(cfg, 0)
for m in algo.models.values():
    m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
algo.set_train()
inputs = synth.make_batch(cfg, seed=5, with_depth=True)
cpu_inputs = {k: v.clone() if torch.is_tensor(v) else v for k, v in inputs.items()}
N = cfg['data']['num_cams']
noise = torch.stack([torch.tensor(fx[f'noise_c{c}']) for c in range(N)])
outputs, losses = algo.process_batch(inputs, 0, noise=noise.cuda())
disp = outputs['_disp_all'][0]
disp.retain_grad()
losses['total_loss'].backward()
torch.cuda.synchronize()
g_gpu = disp.grad.detach().cpu().double()

# oracle loss path on the GPU's disparities / poses
ci = dict(cpu_inputs)
ci['extrinsics_inv'] = torch.inverse(ci['extrinsics'])
d_leaf = disp.detach().cpu().clone().requires_grad_(True)
total = 0.0
cam_outs = []
for c in range(N):
    co = {('disp', 0): d_leaf[:, c:c + 1]}
    co[('depth', 0)] = O.to_depth(co[('disp', 0)], ci[('K', 0)][:, c], cfg)
    for f in cfg['training']['frame_ids'][1:]:
        co[('cam_T_cam', 0, f)] = outputs[('cam', c)][('cam_T_cam', 0, f)].detach().cpu()
    rp = O.relative_poses(ci, co, c, cfg)
    O.view_rendering(ci, co, c, rp, cfg)
    cl, _ = O.cam_loss(ci, co, c, cfg, noise[c])
    total = total + cl
    cam_outs.append(co)
total = total / N
total.backward()
g_ref = d_leaf.grad.double()
print('total gpu %.9f oracle-on-gpu-disp %.9f' % (float(losses['total_loss']), float(total)))
scale = g_ref.abs().max()
print('d disp: max/scale %.3g fro %.3g' % (float((g_gpu - g_ref).abs().max() / scale),
                                           float((g_gpu - g_ref).norm() / g_ref.norm())))
for c in range(N):
    e = (g_gpu[:, c] - g_ref[:, c]).abs()
    bad = e > 1e-3 * scale
    msg = [f'cam {c}: d disp fro %.3g, {int(bad.sum())} px > 1e-3 max' % float(e.norm() / g_ref[:, c].norm())]
    go, co = outputs[('cam', c)], cam_outs[c]
    for key in [('reproj_mask', 0), ('color_mask', -1, 0), ('color_mask', 1, 0), ('overlap_mask', 0, 0),
                ('overlap_mask', -1, 0), ('overlap_mask', 1, 0)]:
        if key in go and key in co:
            a, b = go[key].detach().cpu(), co[key].detach()
            msg.append(f'{key[0]}{key[1:]} mism {int((a != b).sum())}')
    for key in [('color', -1, 0), ('overlap', 0, 0)]:
        if key in go:
            msg.append(f'{key} maxerr %.2g' % float((go[key].detach().cpu() - cam_outs[c][key].detach()).abs().max()))
    print('; '.join(msg))
