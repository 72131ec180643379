"""Where does d loss / d disp of the full-resolution GPU step differ from the CPU oracle's
(test_full_step_gradient_chain[full], stage 1)?  Two halves:

    python tools/diag_gradchain.py gpu OUT.npz     # on the GPU box: the GPU step, its disparities,
                                                   # poses, their gradients and warp masks
    python tools/diag_gradchain.py nets OUT.npz [--fp64]  # here: stage 2, the GPU's upstream gradients
                                                   # through the oracle step (fp32, or fp64 to
                                                   # price the fp32 oracle's own rounding)
    python tools/diag_gradchain.py cpu OUT.npz [--cells]  # here: the oracle's loss path on those
                                                   # disparities / poses, and an error breakdown
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]


def setup():
    import common as G
    from conftest import golden
    from vfdepth_amd import synth
    fx = golden('step_full.npz')
    cfg = G.full_cfg()
    t = cfg['training']
    noise = torch.stack(G.full_noise(fx, (t['batch_size'], len(t['frame_ids']) - 1, t['height'], t['width'])))
    inputs = synth.make_batch(cfg, seed=G.FULL_SEED, with_depth=True)
    return G, cfg, noise, inputs


def gpu(out):
    G, cfg, noise, inputs = setup()
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    dev = torch.device('cuda:0')
    N, frames = cfg['data']['num_cams'], cfg['training']['frame_ids']
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    from vfdepth_amd import kernels as KN
    held, orig = {}, KN.ProjConv.apply

    def proj_conv(*a):            # K3C's output (the activated, reflect-padded reduce_dim[0] map)
        out = orig(*a)
        held['y0'] = out.detach()
        return out
    KN.ProjConv.apply = proj_conv
    outputs, losses = algo.process_batch(inputs, 0, noise=noise.to(dev))
    KN.ProjConv.apply = orig
    disp = outputs['_disp_all'][0]
    disp.retain_grad()
    P_all = outputs['_cam_T_cam']
    for t in P_all.values():
        t.retain_grad()
    losses['total_loss'].backward()
    res = {'disp': disp.detach().cpu().numpy(), 'disp_grad': disp.grad.cpu().numpy(),
           'total_loss': float(losses['total_loss'])}
    if 'y0' in held:             # its LeakyReLU decisions (interior, NCHW), as bits
        y0 = held['y0'][:, :, 1:-1, 1:-1].contiguous()
        res['y0_pos_bits'] = np.packbits((y0 > 0).cpu().numpy().reshape(-1))
        res['y0_shape'] = np.array(y0.shape)
    for f in frames[1:]:
        res[f'P_{f}'] = P_all[f].detach().cpu().numpy()
        res[f'P_grad_{f}'] = P_all[f].grad.cpu().numpy()
    for c in range(N):
        go = outputs[('cam', c)]
        for key, v in go.items():
            if isinstance(key, tuple) and key[0] in ('color_mask', 'overlap_mask', 'reproj_mask'):
                res[f'c{c}_' + '_'.join(map(str, key))] = v.detach().cpu().numpy()
            if isinstance(key, tuple) and key[0] in ('color', 'overlap') and c == 0:
                res[f'c{c}_' + '_'.join(map(str, key))] = v.detach().cpu().numpy()
    for mname in ('depth_net', 'pose_net'):
        for n, p in algo.models[mname].named_parameters():
            if not n.startswith('encoder.') and p.grad is not None and p.numel() <= 600000:   # (gpurun_out cap)
                res[f'grad:{mname}:{n}'] = p.grad.cpu().numpy()
    np.savez_compressed(out, **res)
    print('saved', out, 'total_loss', res['total_loss'], flush=True)


def cpu(path):
    G, cfg, noise, inputs = setup()
    from oracle import vfd_oracle as O
    from test_gpu_parity import _near_decisions
    fx = np.load(path)
    N, frames = cfg['data']['num_cams'], cfg['training']['frame_ids']
    ci = dict(inputs)
    ci['extrinsics_inv'] = torch.inverse(ci['extrinsics'])
    d_leaf = torch.from_numpy(fx['disp']).requires_grad_(True)
    T_leaf = {(c, f): torch.from_numpy(fx[f'P_{f}'][:, c]).clone().requires_grad_(True)
              for c in range(N) for f in frames[1:]}
    total = 0.0
    near = torch.zeros_like(d_leaf, dtype=torch.bool)
    cos = []
    for c in range(N):
        co = {('disp', 0): d_leaf[:, c:c + 1]}
        co[('depth', 0)] = O.to_depth(co[('disp', 0)], ci[('K', 0)][:, c], cfg)
        for f in frames[1:]:
            co[('cam_T_cam', 0, f)] = T_leaf[(c, f)]
        rp = O.relative_poses(ci, co, c, cfg)
        O.view_rendering(ci, co, c, rp, cfg)
        total = total + O.cam_loss(ci, co, c, cfg, noise[c])[0]
        go = {}
        for k in fx.files:
            if k.startswith(f'c{c}_'):
                parts = k[len(f'c{c}_'):].split('_')
                nums = []
                while parts and parts[-1].lstrip('-').isdigit():
                    nums.insert(0, int(parts.pop()))
                go[('_'.join(parts), *nums)] = torch.from_numpy(fx[k])
        near[:, c] = _near_decisions(O, ci, co, go, c, frames, noise[c], rp if '--cells' in sys.argv else None)[:, 0]
        cos.append(co)
    print('oracle total', float(total / N), 'gpu total', float(fx['total_loss']), flush=True)
    (total / N).backward()
    g_gpu = torch.from_numpy(fx['disp_grad']).double()
    g_ref = d_leaf.grad.double()
    keep = ~near
    err = (g_gpu - g_ref).abs()
    scale = float(g_ref.abs().max())
    print(f'near {int(near.sum())} px; fro outside near {float((g_gpu - g_ref)[keep].norm() / g_ref[keep].norm()):.3g}'
          f' max {float(err[keep].max()) / scale:.3g}')
    for c in range(N):
        e = err[:, c][keep[:, c]]
        r = g_ref[:, c][keep[:, c]]
        print(f'cam {c}: fro {float(e.norm() / r.norm()):.3g} max {float(e.max()) / scale:.3g} '
              f'|g| max {float(r.abs().max()):.3g}')
    e = (err * keep).squeeze(2)     # [B, N, H, W]
    flat = e.flatten()
    top = torch.topk(flat, 20).indices
    B, Nn, H, W = e.shape
    for i in top.tolist():
        b, rem = divmod(i, Nn * H * W)
        c, rem = divmod(rem, H * W)
        y, x = divmod(rem, W)
        print(f'  cam {c} y {y} x {x}: gpu {float(g_gpu[b, c, y, x]):.4g} ref {float(g_ref[b, c, y, x]):.4g} '
              f'disp {float(fx["disp"][b, c, y, x]):.4g}')
    # error mass by distance to the image border and by the masks
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing='ij')
    bd = torch.minimum(torch.minimum(yy, H - 1 - yy), torch.minimum(xx, W - 1 - xx))
    tot = float((e ** 2).sum())
    for lo, hi in ((0, 1), (1, 2), (2, 4), (4, 16), (16, 10000)):
        m = (bd >= lo) & (bd < hi)
        print(f'border dist [{lo},{hi}): {float((e[..., m] ** 2).sum()) / tot:.3f} of the squared error, '
              f'{float(m.float().mean()):.3f} of the px')
    for f in frames[1:]:
        for c in range(N):
            a, b = torch.from_numpy(fx[f'P_grad_{f}'][:, c]).double(), T_leaf[(c, f)].grad.double()
            print(f'd loss / d cam_T_cam (cam {c}, frame {f}): fro {float((a - b).norm() / b.norm()):.3g}')
    np.savez_compressed(path.replace('.npz', '_cpu.npz'), ref=g_ref.float().numpy(), near=near.numpy())


def nets(path):
    G, cfg, noise, inputs = setup()
    from oracle import vfd_oracle as O
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.network import FusedDepthNet, FusedPoseNet
    fx = np.load(path)
    N, frames = cfg['data']['num_cams'], cfg['training']['frame_ids']
    dt = torch.float64 if '--fp64' in sys.argv else torch.float32
    dn, pn = FusedDepthNet(cfg), FusedPoseNet(cfg)
    dn.load_state_dict(seeded_state_dict(dn, seed=G.STEP_SEED))
    pn.load_state_dict(seeded_state_dict(pn, seed=G.STEP_SEED))
    dn.train().to(dt)
    pn.train().to(dt)
    ci = {k: v.to(dt) if torch.is_tensor(v) and v.is_floating_point() else v for k, v in inputs.items()}
    held = {}
    hook = dn.decoder.register_forward_hook(lambda m, i, o: held.__setitem__('disp', o[('disp', 0)]))

    def keep_z0(m, i, o):      # called once per camera ([B, O, h, w] each)
        held.setdefault('z0', []).append(o)
        j = len(held['z0']) - 1
        o.register_hook(lambda gz: held.setdefault('gz0', {}).__setitem__(j, gz))
    hook0 = dn.fusion_net.reduce_dim[0].register_forward_hook(keep_z0)
    o_out, _ = O.process_batch(O.nets_from_modules(dn, pn), ci, cfg, [n.to(dt) for n in noise])
    hook.remove()
    hook0.remove()
    keys = [(c, f) for c in range(N) for f in frames[1:]]
    tensors = [held['disp']] + [o_out[('cam', c)][('cam_T_cam', 0, f)] for (c, f) in keys]
    grads = [torch.from_numpy(fx['disp_grad']).reshape(held['disp'].shape).to(dt)]
    grads += [torch.from_numpy(fx[f'P_grad_{f}'][:, c]).to(dt) for (c, f) in keys]
    torch.autograd.backward(tensors, grads)
    tag = 'fp64' if dt == torch.float64 else 'fp32'
    res = {}
    if 'y0_pos_bits' in fx.files and 'gz0' in held:
        # d reduce_dim[0].bias under the oracle's LeakyReLU decisions vs under the GPU's: the
        # oracle's gradient at the activation output, g_a = gz0 / lrelu'(z0)
        n_c = len(held['z0'])
        z0 = torch.stack([z.detach() for z in held['z0']], 1).flatten(0, 1)          # [B*N, O, h, w]
        gz0 = torch.stack([held['gz0'][j].detach() for j in range(n_c)], 1).flatten(0, 1)
        shp = tuple(fx['y0_shape'])
        gpos = torch.from_numpy(np.unpackbits(fx['y0_pos_bits'])[:int(np.prod(shp))].reshape(shp).astype(bool))
        opos = z0 > 0
        ga = gz0 / torch.where(opos, torch.ones_like(z0), torch.full_like(z0, 0.1))
        db_o = gz0.sum((0, 2, 3))
        db_g = (ga * torch.where(gpos, torch.ones_like(z0), torch.full_like(z0, 0.1))).sum((0, 2, 3))
        flips = gpos != opos
        k = 'grad:depth_net:fusion_net.reduce_dim.0.bias'
        gd = torch.from_numpy(fx[k]).double()
        print(f'LeakyReLU decisions of reduce_dim[0]: {int(flips.sum())} of {flips.numel()} differ '
              f'(|z0| at flips max {float(z0[flips].abs().max()) if flips.any() else 0:.3g}, '
              f'|z0| median {float(z0.abs().median()):.3g})')
        print(f'd bias: oracle-{tag} decisions vs GPU grad fro {float((gd - db_o.double()).norm() / db_o.double().norm()):.3g}; '
              f'GPU decisions vs GPU grad fro {float((gd - db_g.double()).norm() / db_g.double().norm()):.3g}')
    for mname, net in (('depth_net', dn), ('pose_net', pn)):
        for n, p in net.named_parameters():
            k = f'grad:{mname}:{n}'
            if k in fx.files:
                res[k] = p.grad.double().numpy()
                a, b = fx[k].astype(np.float64), res[k]
                print(f'{mname}.{n}: gpu vs oracle-{tag} fro {np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300):.3g}')
    np.savez_compressed(path.replace('.npz', f'_nets_{tag}.npz'), **res)


if __name__ == '__main__':
    {'gpu': gpu, 'cpu': cpu, 'nets': nets}[sys.argv[1]](sys.argv[2])
