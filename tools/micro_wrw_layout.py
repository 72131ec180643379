import os, sys, torch
ROOT = os.environ.get('GRAFT_REPO_ROOT', '/root/repo')
sys.path.insert(0, ROOT)
os.environ.setdefault('MIOPEN_USER_DB_PATH', os.path.join(ROOT, 'miopen_db'))
def timed(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3
cb = torch.ops.aten.convolution_backward
dev = 'cuda:0'
DT = torch.bfloat16 if '--bf16' in sys.argv else torch.float32
F = torch.nn.functional
for (N, C, H, W, K, s) in ((12, 64, 96, 160, 64, 1), (12, 128, 48, 80, 128, 1), (12, 256, 24, 40, 256, 1), (12, 512, 12, 20, 512, 1)) if DT == torch.bfloat16 else ((6, 64, 96, 160, 64, 1), (6, 128, 48, 80, 128, 1), (6, 256, 24, 40, 256, 1), (6, 512, 12, 20, 512, 1), (6, 64, 96, 160, 128, 2)):
    x = torch.randn(N, C, H, W, device=dev, dtype=DT); w = torch.randn(K, C, 3, 3, device=dev, dtype=DT)
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    dy = torch.randn(N, K, Ho, Wo, device=dev, dtype=DT)
    args = (None, [s, s], [1, 1], [1, 1], False, [0, 0], 1)
    t_w = timed(lambda: cb(dy, x, w, *args, [False, True, False]))
    t_d = timed(lambda: cb(dy, x, w, *args, [True, False, False]))
    t_wd = timed(lambda: cb(dy, x, w, *args, [True, True, False]))
    xc, dyc, wc = (t.contiguous(memory_format=torch.channels_last) for t in (x, dy, w))
    t_wc = timed(lambda: cb(dyc, xc, wc, *args, [False, True, False]))
    t_dc = timed(lambda: cb(dyc, xc, wc, *args, [True, False, False]))
    t_conv = timed(lambda: (x.contiguous(memory_format=torch.channels_last), dy.contiguous(memory_format=torch.channels_last)))
    t_f = timed(lambda: F.conv2d(x, w, None, s, 1))
    t_fc = timed(lambda: F.conv2d(xc, wc, None, s, 1))
    print(f'{DT} {N}x{C}x{H}x{W}->{K} s{s}: NCHW fwd {t_f:6.1f} wgrad {t_w:6.1f} dgrad {t_d:6.1f} both {t_wd:6.1f} | '
          f'NHWC fwd {t_fc:6.1f} wgrad {t_wc:6.1f} dgrad {t_dc:6.1f} | x,dy->NHWC copies {t_conv:6.1f} us', flush=True)
