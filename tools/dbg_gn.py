"""Debug: mdx_groupnorm repeated on stream A while convolutions run on stream
B; count outputs that differ from the first (serial) result."""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mdx_pkg
mdx_pkg.load()
from moseq2_detectron_extract_amd._lib import call

P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731


def S(st):
    return ctypes.c_void_p(st.cuda_stream)


for dt, tdt in ((1, torch.float16), (0, torch.float32)):
    for (N, H, W, fuse) in ((4, 14, 16, 0), (4, 28, 32, 2), (4, 112, 128, 2)):
        C, G = 256, 32
        g = torch.Generator().manual_seed(1)
        x = (torch.randn(N, H, W, C, generator=g) * 3 + 1).to(tdt).cuda()
        up = (torch.randn(N, H // 2, W // 2, C, generator=g)).to(tdt).cuda()
        gam = (torch.rand(C, generator=g) + 0.5).cuda(); bet = torch.randn(C, generator=g).cuda()
        wsb = call("mdx_groupnorm_workspace_bytes", N, H, W, G)
        ws = torch.empty(wsb // 4 + 16, device="cuda")
        ref = torch.empty_like(x)
        cur = torch.cuda.current_stream()
        call("mdx_groupnorm", P(x), N, H, W, C, G, 1e-5, P(gam), P(bet), P(up), fuse, dt, P(ref), P(ws), S(cur))
        torch.cuda.synchronize()
        # background load: a big conv on stream B
        bx = torch.randn(8, 112, 128, 256).to(tdt).cuda()
        bw = torch.randn(256, 3 * 3 * 256).to(tdt).cuda() * 0.02
        bo = torch.empty(8, 112, 128, 256, dtype=tdt, device="cuda")
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        bad = 0
        outs = [torch.empty_like(x) for _ in range(4)]
        for r in range(200):
            call("mdx_conv2d", P(bx), 8, 112, 128, 256, P(bw), None, 256, 3, 3, 1, 1, None, 0, 0, dt, dt, P(bo), S(sb))
            o = outs[r % 4]
            call("mdx_groupnorm", P(x), N, H, W, C, G, 1e-5, P(gam), P(bet), P(up), fuse, dt, P(o), P(ws), S(sa))
            if r % 4 == 3:
                torch.cuda.synchronize()
                for oo in outs:
                    bad += int(not torch.equal(oo, ref))
        print("dtype", dt, (N, H, W, fuse), "mismatching GN outputs:", bad, "/ 200", flush=True)
