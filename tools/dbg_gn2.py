"""Debug: two streams running mdx_groupnorm concurrently on different
tensors / workspaces; count results that differ from serial ones."""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd._lib import call

P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
S = lambda st: ctypes.c_void_p(st.cuda_stream)  # noqa: E731
for dt, tdt in ((1, torch.float16), (0, torch.float32)):
    C, G = 256, 32
    cases = []
    for k, (N, H, W, fuse) in enumerate(((4, 14, 16, 0), (4, 28, 32, 2), (4, 56, 64, 2), (4, 112, 128, 2))):
        g = torch.Generator().manual_seed(k)
        x = (torch.randn(N, H, W, C, generator=g) * 3 + 1).to(tdt).cuda()
        up = torch.randn(N, max(H // 2, 1), max(W // 2, 1), C, generator=g).to(tdt).cuda()
        gam = (torch.rand(C, generator=g) + 0.5).cuda(); bet = torch.randn(C, generator=g).cuda()
        wsa = torch.empty(call("mdx_groupnorm_workspace_bytes", N, H, W, G) // 4 + 16, device="cuda")
        wsb = torch.empty_like(wsa)
        ref = torch.empty_like(x)
        call("mdx_groupnorm", P(x), N, H, W, C, G, 1e-5, P(gam), P(bet), P(up), fuse, dt, P(ref), P(wsa),
             S(torch.cuda.current_stream()))
        cases.append((N, H, W, fuse, x, up, gam, bet, wsa, wsb, ref))
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    bad = [0] * len(cases)
    for r in range(100):
        outs = []
        for i, (N, H, W, fuse, x, up, gam, bet, wsa, wsb, ref) in enumerate(cases):
            oa, ob = torch.empty_like(x), torch.empty_like(x)
            call("mdx_groupnorm", P(x), N, H, W, C, G, 1e-5, P(gam), P(bet), P(up), fuse, dt, P(oa), P(wsa), S(sa))
            j = (i + 1 + r) % len(cases)
            c2 = cases[j]
            ob = torch.empty_like(c2[4])
            call("mdx_groupnorm", P(c2[4]), c2[0], c2[1], c2[2], C, G, 1e-5, P(c2[6]), P(c2[7]), P(c2[5]), c2[3], dt,
                 P(ob), P(c2[9]), S(sb))
            outs.append((i, oa, j, ob))
        torch.cuda.synchronize()
        for i, oa, j, ob in outs:
            bad[i] += int(not torch.equal(oa, cases[i][10]))
            bad[j] += int(not torch.equal(ob, cases[j][10]))
    print("dtype", dt, "GN vs GN mismatches per case (of 200):", bad, flush=True)
