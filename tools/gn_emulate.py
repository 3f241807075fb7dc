"""CPU restatement of the GroupNorm statistics kernels (k_gn_partial,
k_gn_final in csrc/model_ops.hip) in the exact operation order of the
packed-FP32 build (unfused multiply / add, IEEE divisions), for the
workspace dumps of tools/dbg_race.py (DBG_DUMP=...npz): which of the serial
and the pipelined workspace is the arithmetic of the code, and where the
other one departs from it.

Usage: python tools/gn_emulate.py dump.npz"""
import sys

import numpy as np

f32, f64 = np.float32, np.float64
CHUNK = 64  # GN_CHUNK_PIX


def partials(x, G):
    """x: (N, HW, C) fp16 -> part (N, G, nch, 3) float32, lane order of the kernel."""
    N, HW, C = x.shape
    CV = C // 8
    rows = 256 // CV
    opg = (C // G) // 8
    nch = (HW + CHUNK - 1) // CHUNK
    part = np.zeros((N, G, nch, 3), f32)
    xf = x.astype(f32)
    for n in range(N):
        for ch in range(nch):
            p0 = ch * CHUNK
            s_n = np.zeros(256, f32)
            s_m = np.zeros(256, f32)
            s_q = np.zeros(256, f32)
            for t in range(256):
                cv, pr = t % CV, t // CV
                if pr >= rows or p0 + pr >= HW:
                    continue
                S = Q = sh = f32(0)
                cnt = f32(0)
                first = True
                for p in range(p0 + pr, min(p0 + CHUNK, HW), rows):
                    v = xf[n, p, cv * 8:cv * 8 + 8]
                    if first:
                        sh, first = v[0], False
                    for k in range(8):
                        d = f32(v[k] - sh)
                        S = f32(S + d)
                        Q = f32(Q + f32(d * d))
                    cnt = f32(cnt + f32(8))
                q = f32(S / cnt)
                s_n[t] = cnt
                s_m[t] = f32(sh + q)
                s_q[t] = max(f32(Q - f32(S * q)), f32(0))
            for g in range(G):
                Nn = M = Qq = f32(0)
                for r in range(rows):
                    for o in range(opg):
                        t = r * CV + g * opg + o
                        nb = s_n[t]
                        if nb == 0:
                            continue
                        tot = f32(Nn + nb)
                        d = f32(s_m[t] - M)
                        M = f32(M + f32(d * f32(nb / tot)))
                        Qq = f32(Qq + f32(s_q[t] + f32(f32(d * d) * f32(f32(Nn * nb) / tot))))
                        Nn = tot
                part[n, g, ch] = (Nn, M, Qq)
    return part


def _merge(a, b):
    N, M, Q = a
    nb, mb, qb = b
    tot = N + nb
    if tot <= 0:
        return a
    d = mb - M
    M = M + d * (nb / tot)
    Q = Q + (qb + d * d * (N * nb / tot))
    return (tot, M, Q)


def final(part, eps):
    N, G, nch, _ = part.shape
    stats = np.zeros((N, G, 2), f32)
    for n in range(N):
        for g in range(G):
            lanes = [(f64(0), f64(0), f64(0))] * 64
            for c in range(nch):  # lane c takes chunk c (nch <= 64 here)
                nb, mb, qb = (f64(v) for v in part[n, g, c])
                lanes[c % 64] = _merge(lanes[c % 64], (nb, mb, qb)) if nb != 0 else lanes[c % 64]
            off = 32
            while off >= 1:
                lanes = [_merge(lanes[l], lanes[l ^ off]) for l in range(64)]
                off //= 2
            Nt, M, Q = lanes[0]
            var = f32(Q / Nt)
            stats[n, g] = (f32(M), f32(f32(1) / np.sqrt(f32(var + f32(eps)))))
    return stats


def main():
    z = np.load(sys.argv[1])
    x = z["lat_ref"]
    N, H, W, C = x.shape
    G = 32
    assert np.array_equal(x.view(np.uint16), z["lat_rep"].view(np.uint16)), "GN inputs differ"
    part = partials(x.reshape(N, H * W, C), G)
    nch = part.shape[2]
    ns = 2 * N * G
    for tag in ("ws_ref", "ws_rep"):
        ws = z[tag].reshape(-1)
        wp = ws[ns:ns + part.size].reshape(part.shape)
        bad = np.argwhere(wp.view(np.uint32) != part.view(np.uint32))
        print(tag, "partials differing from the restatement:", len(bad), bad[:8].tolist())
        st = final(wp, 1e-5)
        sb = np.argwhere(ws[:ns].reshape(N, G, 2).view(np.uint32) != st.view(np.uint32))
        print(f"  {tag} stats vs final(own partials):", len(sb), sb[:8].tolist())
    a, b = z["ws_ref"].reshape(-1), z["ws_rep"].reshape(-1)
    pa = a[ns:ns + part.size].reshape(part.shape)
    pb = b[ns:ns + part.size].reshape(part.shape)
    d = np.argwhere(pa.view(np.uint32) != pb.view(np.uint32))
    print("serial vs pipelined partials differing (n, g, chunk, field):", len(d), d[:16].tolist())
    for i in d[:6].tolist():
        print("   ", i, "serial", pa[tuple(i)], "pipelined", pb[tuple(i)], "restated", part[tuple(i)])
    print("nch", nch, "rep", int(z["rep"]))


if __name__ == "__main__":
    main()
