"""Which multi-stream HIP-graph capture patterns does this HIP runtime end cleanly?  Each pattern
runs in its own child process (a crash in hipStreamEndCapture is a segfault); prints one line per
pattern with its exit code.

    python tools/diag_capture_patterns.py [--from P3] # the patterns in order, stopping at the first crash
    python tools/diag_capture_patterns.py --one P3   # one pattern in this process
"""
import os
import subprocess
import sys

import torch


def k(x):
    return x.mul_(1.0001).add_(1.0)


def p1_fork_join():
    """cap forks B once (B waits on cap), work on B, cap joins B."""
    x = torch.ones(1024, device='cuda')
    B = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        B.wait_stream(cap)
        with torch.cuda.stream(B):
            k(x)
        cap.wait_stream(B)
        k(x)
    g.replay()


def p2_fork_join_twice():
    """the same side stream forked and joined twice in one capture."""
    x, y = torch.ones(1024, device='cuda'), torch.ones(1024, device='cuda')
    B = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        for _ in range(2):
            B.wait_stream(cap)
            with torch.cuda.stream(B):
                k(x)
            k(y)
            cap.wait_stream(B)
    g.replay()


def p3_side_used_before():
    """B used eagerly (events recorded) before the capture forks it."""
    x = torch.ones(1024, device='cuda')
    B = torch.cuda.Stream()
    B.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(B):
        k(x)
    torch.cuda.current_stream().wait_stream(B)
    torch.cuda.synchronize()
    p1_body(x, B)


def p1_body(x, B):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        B.wait_stream(cap)
        with torch.cuda.stream(B):
            k(x)
        cap.wait_stream(B)
    g.replay()


def p4_autograd_branch():
    """a branch of the forward on B; autograd runs its backward on B (engine syncs)."""
    lin1, lin2 = torch.nn.Linear(64, 64).cuda(), torch.nn.Linear(64, 64).cuda()
    x = torch.randn(32, 64, device='cuda')
    B = torch.cuda.Stream()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())

    def step():
        cap = torch.cuda.current_stream()
        B.wait_stream(cap)
        with torch.cuda.stream(B):
            a = lin1(x)
        b = lin2(x)
        cap.wait_stream(B)
        (a * b).sum().backward()
        cap.wait_stream(B)
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        step()
    g.replay()


def p5_event_across():
    """an event recorded on B in the forward, waited on by cap later (FusionPlan.ready)."""
    x, y = torch.ones(1024, device='cuda'), torch.ones(1024, device='cuda')
    B = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        B.wait_stream(cap)
        with torch.cuda.stream(B):
            k(x)
            ev = torch.cuda.Event()
            ev.record(B)
            k(x)
        k(y)
        cap.wait_event(ev)
        k(y)
        cap.wait_stream(B)
    g.replay()


def p6_nested():
    """cap forks B, B forks C, C joins B, B joins cap."""
    x = torch.ones(1024, device='cuda')
    B, C = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        B.wait_stream(cap)
        with torch.cuda.stream(B):
            C.wait_stream(B)
            with torch.cuda.stream(C):
                k(x)
            B.wait_stream(C)
        cap.wait_stream(B)
    g.replay()


def p7_cap_waits_then_side_waits():
    """ping-pong: cap forks B, cap waits B, B waits cap again (B still in the capture), cap joins."""
    x, y = torch.ones(1024, device='cuda'), torch.ones(1024, device='cuda')
    B = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        B.wait_stream(cap)
        with torch.cuda.stream(B):
            k(x)
        cap.wait_stream(B)
        k(y)
        B.wait_stream(cap)
        with torch.cuda.stream(B):
            k(x)
        cap.wait_stream(B)
    g.replay()


def p8_capture_on_named_stream():
    """capture on a user stream (torch.cuda.graph(stream=S)) that forks B."""
    x = torch.ones(1024, device='cuda')
    S, B = torch.cuda.Stream(), torch.cuda.Stream()
    S.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=S):
        B.wait_stream(S)
        with torch.cuda.stream(B):
            k(x)
        S.wait_stream(B)
    g.replay()


PATTERNS = {n: f for n, f in globals().items() if n[:1] == 'p' and n[1:2].isdigit() and callable(f)}


def main():
    if '--one' in sys.argv:
        name = sys.argv[sys.argv.index('--one') + 1]
        fn = next(f for n, f in PATTERNS.items() if n.split('_')[0] == name.lower())
        fn()
        torch.cuda.synchronize()
        print(f'{name} ok', flush=True)
        return 0
    start = sys.argv[sys.argv.index('--from') + 1].lower() if '--from' in sys.argv else 'p0'
    for n in sorted(PATTERNS):
        if n.split('_')[0] < start:
            continue
        tag = n.split('_')[0].upper()
        rc = subprocess.call([sys.executable, os.path.abspath(__file__), '--one', tag], timeout=120)
        print(f'{tag:4s} {n:34s} rc={rc}', flush=True)
        if rc != 0:          # a crashed child: nothing more on the GPU in this run
            return rc
    return 0


if __name__ == '__main__':
    sys.exit(main())
