"""LDS cost of lstm_grads_body's per-tile staging and MFMA operand reads vs the transposed-image row
pitch LDR (bf16; rows must stay 16-byte aligned for the b128 reads)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sim import cycles, ideal


def analyze(H, Din, LDR, DZRP=72, ldx=None, seq_fast=True):
    ldx = ldx or Din
    res = {}
    NWV = 4

    def add(name, kind, fn, waves=range(NWV), valid=None):
        c = i = 0
        for w in waves:
            addrs = []
            for l in range(64):
                t = w * 64 + l
                addrs.append(fn(t, l) if (valid is None or valid(t)) else None)
            if all(a is None for a in addrs):
                continue
            c += cycles(kind, addrs); i += ideal(kind)
        res[name] = (c, i)
    # dzT[zc + j][rr] bf16x2, zc = (tid & 15) * 4, rr = 2 (tid >> 4)
    zr = (lambda t: t & 15) if seq_fast else (lambda t: t >> 4)
    zc = (lambda t: 4 * (t >> 4)) if seq_fast else (lambda t: 4 * (t & 15))
    pair = (lambda it, nq: it & 15) if seq_fast else (lambda it, nq: it // nq)
    quad = (lambda it, nq: it >> 4) if seq_fast else (lambda it, nq: it % nq)
    for j in range(4):
        add(f"dzT_st{j}", "w32", lambda t, l, j=j: 2 * ((zc(t) + j) * LDR + 2 * zr(t)))
    # dzR[rr][zc] bf16x4 (8 B)
    add("dzR_st0", "w64", lambda t, l: 2 * ((2 * zr(t)) * DZRP + zc(t)))
    # xT[d0 + q][rr] bf16x2, it = tid: rr = 2 (it / nq), d0 = 4 (it % nq)
    nq = ldx // 4; nit = 16 * nq
    for q in range(4):
        add(f"xT_st{q}", "w32", lambda t, l, q=q: 2 * ((4 * quad(t, nq) + q) * LDR + 2 * pair(t, nq)), valid=lambda t: t < nit)
    # hT[k0 + q][rr]: it = tid, rr = 2 (it / (H / 4)), k0 = 4 (it % (H / 4))
    nh = 16 * H // 4
    for q in range(4):
        for i in range((nh + 255) // 256):
            add(f"hT_st{q}_{i}", "w32", lambda t, l, q=q, i=i: 2 * ((4 * quad(t + 256 * i, H // 4) + q) * LDR + 2 * pair(t + 256 * i, H // 4)),
                valid=lambda t, i=i: t + 256 * i < nh)
    add("dzT_rd", "r128", lambda t, l: 2 * ((16 * (t >> 6) + (l & 15)) * LDR + 8 * (l >> 4)))
    DT = (Din + 1 + 15) // 16
    for d in range(DT):
        add(f"xT_rd{d}", "r128", lambda t, l, d=d: 2 * ((16 * d + (l & 15)) * LDR + 8 * (l >> 4)))
    for k in range(H // 16):
        add(f"hT_rd{k}", "r128", lambda t, l, k=k: 2 * ((16 * k + (l & 15)) * LDR + 8 * (l >> 4)))
    return res


if __name__ == "__main__":
    for LDR, sf in ((40, False), (40, True), (48, True), (56, True)):
        tot = ti = 0
        det = {}
        for H, Din in ((128, 64), (64, 64), (64, 32), (16, 20), (32, 16)):
            r = analyze(H, Din, LDR, seq_fast=sf)
            for k, (c, i) in r.items():
                tot += c; ti += i
                det[k.split("_")[0] + "_" + k.split("_")[1][:2]] = det.get(k.split("_")[0] + "_" + k.split("_")[1][:2], 0) + c - i
        print(LDR, "seq_fast" if sf else "channel_fast", tot, ti, det)
